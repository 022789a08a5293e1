# JPEG + plumbing GPU tests only (after codec changes).  Usage: bash tools/gpu_jpeg_quick2.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plumbing.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -60 gpurun_out/pytest_gpu_jpeg.log; exit 1; }
tail -5 gpurun_out/pytest_gpu_jpeg.log
