# JPEG worker form: batches in flight 3 / 4 / 5 and batch 32 / 64, interleaved, 1080p and 4K
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/depth4.jsonl
for rep in 1 2; do
for sz in 1080p 4k; do
for m in "async3 32" "async4 32" "async5 32" "async3 64" "async2 64"; do
  timeout -k 10 120 python -u tools/jpeg_modes.py $sz $m >> gpurun_out/depth4.jsonl 2>> gpurun_out/depth4.err || { echo MODES_FAILED; tail -20 gpurun_out/depth4.err; exit 1; }
done
done
done
cat gpurun_out/depth4.jsonl
