# Confirmation on a fresh box of what the driver runs at round end: GPU tests, smoke, default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6c_pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r6c_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r6c_pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c_smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/r6c_smoke.log; exit 1; }
tail -3 gpurun_out/r6c_smoke.log
S=$(date +%s)
BENCH_DETAIL=gpurun_out/r6c_bench_detail.json timeout -k 10 500 python -u bench.py > gpurun_out/r6c_bench.json 2> gpurun_out/r6c_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6c_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - S )) s"
echo CONFIRM_OK
