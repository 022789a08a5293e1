# Round 2 full check: GPU tests, smoke, the bench line (N=1), an N=2 rehearsal on the one
# card, and the rocprof kernel summary of the headline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2_pytest_gpu_full.log 2>&1 || { echo PYTEST_FAILED; tail -80 gpurun_out/r2_pytest_gpu_full.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/r2_smoke.log; exit 1; }
tail -2 gpurun_out/r2_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench.log; exit 1; }
cat gpurun_out/r2_bench.json | cut -c1-600
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/r2_bench_n2_rehearsal.json 2> gpurun_out/r2_bench_n2.log || { echo BENCH_N2_FAILED; tail -30 gpurun_out/r2_bench_n2.log; exit 1; }
cut -c1-400 gpurun_out/r2_bench_n2_rehearsal.json
rm -rf gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 300 --warmup 30 --no-traffic --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep --cpu-seconds 0 > gpurun_out/r2_bench_under_rocprof.json 2> gpurun_out/r2_bench_rocprof.log || { echo ROCPROF_FAILED; tail -20 gpurun_out/r2_bench_rocprof.log; exit 1; }
grep -h invert_stream gpurun_out/prof_bench/bench_kernel_stats.csv | cut -c1-300
