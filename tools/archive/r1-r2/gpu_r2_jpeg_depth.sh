# JPEG: batches in flight (2 vs 3) in the worker form, and the 2-thread form gated / ungated
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_jpeg_depth.jsonl
for size in 480p 1080p 4k; do
  for m in async async3; do
    timeout -k 10 100 python -u tools/jpeg_modes.py $size $m >> gpurun_out/r2_jpeg_depth.jsonl 2>> gpurun_out/r2_jpeg_depth.err || { echo FAILED; tail -20 gpurun_out/r2_jpeg_depth.err; exit 1; }
  done
  for g in 0 1; do
    echo "{\"VF_JPEG_GATE\": $g}" >> gpurun_out/r2_jpeg_depth.jsonl
    VF_JPEG_GATE=$g timeout -k 10 100 python -u tools/jpeg_modes.py $size 2threads >> gpurun_out/r2_jpeg_depth.jsonl 2>> gpurun_out/r2_jpeg_depth.err || { echo FAILED; tail -20 gpurun_out/r2_jpeg_depth.err; exit 1; }
  done
done
cat gpurun_out/r2_jpeg_depth.jsonl
