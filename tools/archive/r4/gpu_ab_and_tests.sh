# pipeline A/B (tools/r4/gpu_pipe_ab.sh), then the GPU test suite
set -o pipefail
bash tools/r4/gpu_pipe_ab.sh || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
