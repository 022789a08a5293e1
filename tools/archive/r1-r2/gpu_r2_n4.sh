# Round 2: GPU suite + smoke, then an N=4 rehearsal of the bench on ONE card (4 ranks + 4
# workers share GPU 0; --no-sweep: 4 x 51 GB would not fit one card).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2_pytest_gpu_full2.log 2>&1 || { echo PYTEST_FAILED; tail -80 gpurun_out/r2_pytest_gpu_full2.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu_full2.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke2.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/r2_smoke2.log; exit 1; }
tail -1 gpurun_out/r2_smoke2.log
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 100 --warmup 10 --no-sweep > gpurun_out/r2_bench_n4_rehearsal.json 2> gpurun_out/r2_bench_n4.log || { echo BENCH_N4_FAILED; tail -30 gpurun_out/r2_bench_n4.log; exit 1; }
cut -c1-300 gpurun_out/r2_bench_n4_rehearsal.json
