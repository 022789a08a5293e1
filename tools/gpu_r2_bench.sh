# Round 2: the bench line (N=1) and the JPEG host->host forms with warm codecs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r2_bench2.json 2> gpurun_out/r2_bench2.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench2.log; exit 1; }
cut -c1-300 gpurun_out/r2_bench2.json
rm -f gpurun_out/r2_jpeg_modes3.jsonl
for s in 480p 1080p 4k; do
  timeout -k 10 300 python -u tools/jpeg_modes.py $s >> gpurun_out/r2_jpeg_modes3.jsonl 2> gpurun_out/r2_jpeg_modes3_$s.err || { echo MODES_FAILED $s; tail -20 gpurun_out/r2_jpeg_modes3_$s.err; exit 1; }
done
cat gpurun_out/r2_jpeg_modes3.jsonl
