# JPEG worker form: 3 / 4 / 5 batches in flight
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_jpeg_depth2.jsonl
for size in 1080p 480p; do
  for m in async3 async4 async5; do
    timeout -k 10 100 python -u tools/jpeg_modes.py $size $m >> gpurun_out/r2_jpeg_depth2.jsonl 2>> gpurun_out/r2_jpeg_depth2.err || { echo FAILED; tail -20 gpurun_out/r2_jpeg_depth2.err; exit 1; }
  done
done
cat gpurun_out/r2_jpeg_depth2.jsonl
