#!/bin/bash
# Span-sync warm-up length A/B on hard 1080p (VF_JPEG_SYNC_WARM), k_syncg pass 0 / pass 1 means.
set -o pipefail
mkdir -p gpurun_out
L=distributed-video-filter_amd/vfilter/libvfilter_hip.so
V=${VARIANTS:-"auto=$L w1024=$L@VF_JPEG_SYNC_WARM=1024 w1536=$L@VF_JPEG_SYNC_WARM=1536 w3072=$L@VF_JPEG_SYNC_WARM=3072 w4096=$L@VF_JPEG_SYNC_WARM=4096"}
VARIANTS="$V" KERNELS="k_syncg" SIZES=${SIZES:-1080p} CONTENT=${CONTENT:-hard} REPS="${REPS:-1}" bash tools/r5/gpu_kernel_ab.sh || exit 1
for r in ${REPS:-1}; do for t in $(echo "$V" | tr ' ' '\n' | cut -d= -f1); do
  python3 - "$t" "$r" <<'PY'
import csv, sys, json
t, r = sys.argv[1:]
rows = sorted((x for x in csv.DictReader(open(f"gpurun_out/prof_kab_{t}_{r}/ks_kernel_trace.csv")) if "k_syncg" in x["Kernel_Name"]),
              key=lambda x: int(x["Start_Timestamp"]))
d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in rows]
j = json.loads(open(f"gpurun_out/kab_{t}_{r}.jsonl").readline())
np_ = int(j["stages_ms"]["sync_passes"])
ps = [d[k::np_][2:] for k in range(np_)]
print(f"{t} rep {r}: sync {j['stages_ms']['huffman_sync']} ms, passes {np_}: " + ", ".join(f"{sum(p)/len(p):.1f}" for p in ps) + " us")
PY
done; done
