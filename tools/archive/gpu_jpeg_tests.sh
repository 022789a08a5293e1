# JPEG GPU tests only (the working tree's library).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/jt.log 2>&1 || { echo PYTEST_JPEG_FAILED; grep -E "FAILED|Error|error" gpurun_out/jt.log | head -20; tail -30 gpurun_out/jt.log; exit 1; }
grep -E "span_sync|passed|failed" gpurun_out/jt.log | tail -12
