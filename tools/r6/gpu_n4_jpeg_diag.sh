# The N=4 one-card bench's JPEG legs (every other leg off), to see why they stop.
set -o pipefail
mkdir -p gpurun_out
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo BENCH_DETAIL=gpurun_out/r6_n4diag_detail.json timeout -k 10 600 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 4 --steps 20 --warmup 5 --no-sweep --no-sizes --no-e2e --no-per-frame --no-traffic --cpu-seconds 0 --dist-reps 1 \
    > gpurun_out/r6_n4diag.json 2> gpurun_out/r6_n4diag.err
echo "rc $?"
grep "distributor .* run" gpurun_out/r6_n4diag.err | cut -c1-600
