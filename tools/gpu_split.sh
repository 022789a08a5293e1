# split-launch parity + configs[4] sweep after the sub-launch change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_parity.log; exit 1; }
tail -3 gpurun_out/pytest_parity.log
rm -f gpurun_out/c5_a.jsonl
timeout -k 10 300 python -u tools/sweep.py --c5-only --out gpurun_out/c5_a.jsonl > gpurun_out/c5_a.log 2>&1 || { echo C5A_FAILED; tail -20 gpurun_out/c5_a.log; exit 1; }
cat gpurun_out/c5_a.jsonl
