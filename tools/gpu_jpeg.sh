# GPU box: JPEG parity tests first (new code), then the rest of the GPU suite and smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo JPEG_FAILED; tail -80 gpurun_out/pytest_jpeg.log; exit 1; }
tail -3 gpurun_out/pytest_jpeg.log
