#!/bin/bash
# N=4 rehearsal of the driver's multi-GPU bench on one card (4 ranks + 4 workers share the GPU;
# per-GPU numbers are therefore not the 8-GPU node's): the torchrun path and the distributor legs
# at 4 workers with the native control plane.
set -o pipefail
mkdir -p gpurun_out
S=$(date +%s)
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/bench_n4.json 2> gpurun_out/bench_n4.err || { echo BENCH_N4_FAILED; tail -40 gpurun_out/bench_n4.err; exit 1; }
echo "bench n4 wall $(( $(date +%s) - S )) s"
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/bench_n4.json").read().splitlines() if x.startswith("{")][-1]
d = json.loads(l)
print("n_gpus", d["n_gpus"], "value", d["value"])
for k, v in d["distributor"].items():
    if isinstance(v, dict):
        print(k, {x: v.get(x) for x in ("fps", "fps_per_gpu", "workers", "of_worker_form", "evictions", "frames_lost", "n_errors", "error", "wall_s")})
PY
