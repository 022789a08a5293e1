#!/bin/bash
# N=2 rehearsal of the driver's multi-GPU bench on one card (2 ranks + 2 workers share the GPU, so
# per-GPU numbers are not an 8-GPU node's): the torchrun path, the compact headline at N=2 and the
# distributor legs at 2 workers with the native control plane.
set -o pipefail
mkdir -p gpurun_out
S=$(date +%s)
VF_DEVICE=0 BENCH_DIST_BACKEND=gloo BENCH_DETAIL=gpurun_out/r6_bench_n2_detail.json timeout -k 10 900 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
    bench.py --gpus 2 --steps 20 --warmup 5 --no-sweep > gpurun_out/r6_bench_n2.json 2> gpurun_out/r6_bench_n2.err \
    || { echo BENCH_N2_FAILED; tail -40 gpurun_out/r6_bench_n2.err; exit 1; }
echo "bench n2 wall $(( $(date +%s) - S )) s"
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r6_bench_n2.json").read().splitlines() if x.startswith("{")][-1]
print("headline bytes", len(l.encode()))
d = json.loads(l)
print("n_gpus", d["n_gpus"], "value", d["value"], "scaling", d.get("scaling"))
for k, v in d["distributor"].items():
    if isinstance(v, dict):
        print(k, {x: v.get(x) for x in ("fps", "fps_per_gpu", "workers", "of_worker_form", "evictions", "frames_lost", "n_errors", "error", "wall_s")})
PY
