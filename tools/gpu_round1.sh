set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
timeout -k 10 120 ./tools/tune_invert > gpurun_out/tune2.txt 2>&1 && cat gpurun_out/tune2.txt
