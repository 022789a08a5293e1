# The reference's default mode through the whole system: 1080p JPEG frames -> distributor ->
# GPU workers in JPEG mode -> in-order release, every result checked
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_pipe_jpeg.jsonl
for w in 1 2; do
  timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers $w --gpus 1 --size 1080p --batch 32 --frames 4096 --policy pull --out gpurun_out/r2_pipe_jpeg.jsonl > gpurun_out/r2_pipe_jpeg_$w.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe_jpeg_$w.log; exit 1; }
done
timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers 1 --gpus 1 --size 4k --batch 16 --frames 1024 --policy shard --out gpurun_out/r2_pipe_jpeg.jsonl > gpurun_out/r2_pipe_jpeg_4k.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe_jpeg_4k.log; exit 1; }
cut -c1-600 gpurun_out/r2_pipe_jpeg.jsonl
