#!/bin/bash
# SpanLane (k_syncg's lane without a bit buffer) vs the buffered step: JPEG GPU parity, then
# k_syncg per-kernel means on hard 1080p and 4K scenes (tools/r5/gpu_kernel_ab.sh).
# VARIANTS overrides the libraries compared.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_jpeg.py \
    > gpurun_out/spanlane_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/spanlane_pytest.log; exit 1; }
tail -3 gpurun_out/spanlane_pytest.log
V=${VARIANTS:-"base=tools/exp/libvf_base.so new=distributed-video-filter_amd/vfilter/libvfilter_hip.so"}
VARIANTS="$V" KERNELS="k_syncg" SIZES=1080p CONTENT=hard REPS="1 2" bash tools/r5/gpu_kernel_ab.sh || exit 1
for t in $(echo "$V" | tr ' ' '\n' | cut -d= -f1); do for r in 1 2; do
  python3 - "$t" "$r" <<'PY'
import csv, sys
t, r = sys.argv[1:]
rows = sorted((x for x in csv.DictReader(open(f"gpurun_out/prof_kab_{t}_{r}/ks_kernel_trace.csv")) if "k_syncg" in x["Kernel_Name"]),
              key=lambda x: int(x["Start_Timestamp"]))
d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in rows]
p0, p1 = d[0::4][2:], d[1::4][2:]
print(f"{t} rep {r} hard 1080p k_syncg pass 0 {sum(p0)/len(p0):.1f} us, pass 1 {sum(p1)/len(p1):.1f} us")
PY
done; done
mkdir -p gpurun_out/hard_ab && mv gpurun_out/prof_kab_* gpurun_out/kab_* gpurun_out/hard_ab/
VARIANTS="$V" KERNELS="k_syncg" SIZES=4k CONTENT=scene REPS="1" bash tools/r5/gpu_kernel_ab.sh || exit 1
