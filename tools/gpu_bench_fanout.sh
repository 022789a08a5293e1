# bench line at N=1 (with the configs[2]/[3] distributor leg), then an N=2 rehearsal on one
# card (2 ranks, gloo barrier, 2 workers sharing GPU 0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 --no-jpeg --no-e2e > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo BENCH2_FAILED; tail -30 gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
