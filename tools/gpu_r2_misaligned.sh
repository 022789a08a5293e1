# Round 2: the shifting (misaligned) and descriptor kernels: parity, then HBM rates.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2_pytest_parity.log 2>&1 || { echo PYTEST_FAILED; tail -60 gpurun_out/r2_pytest_parity.log; exit 1; }
tail -2 gpurun_out/r2_pytest_parity.log
timeout -k 10 120 python -u tools/misaligned_probe.py > gpurun_out/r2_misaligned.jsonl 2> gpurun_out/r2_misaligned.err || { echo PROBE_FAILED; tail -20 gpurun_out/r2_misaligned.err; exit 1; }
cat gpurun_out/r2_misaligned.jsonl
