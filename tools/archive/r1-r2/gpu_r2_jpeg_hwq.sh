# JPEG worker form after the engine creates its streams lazily: 4 (default) vs 8 hardware
# queues x compute gate on / off, all three sizes; then the host-path parity tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_jpeg_hwq2.jsonl
for size in 1080p 480p 4k; do
  for q in 4 8; do
    for g in 1 0; do
      echo "{\"size\": \"$size\", \"GPU_MAX_HW_QUEUES\": $q, \"VF_JPEG_GATE\": $g}" >> gpurun_out/r2_jpeg_hwq2.jsonl
      GPU_MAX_HW_QUEUES=$q VF_JPEG_GATE=$g timeout -k 10 100 python -u tools/jpeg_modes.py $size async >> gpurun_out/r2_jpeg_hwq2.jsonl 2>> gpurun_out/r2_jpeg_hwq2.err || { echo HWQ_FAILED; tail -20 gpurun_out/r2_jpeg_hwq2.err; exit 1; }
    done
  done
done
cat gpurun_out/r2_jpeg_hwq2.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jpeg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_hwq_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_hwq_tests.log; exit 1; }
tail -1 gpurun_out/r2_hwq_tests.log
