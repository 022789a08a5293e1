#!/bin/bash
# Speculative sync vs the auto choice (SIZES, CONTENT: default hard 1080p q95), rocprof kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in auto spec; do
  tag=hard_$mode
  rm -rf gpurun_out/prof_$tag
  VF_JPEG_SYNC=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o ks -- \
      python3 tools/jpeg_bench.py --sizes ${SIZES:-1080p} --batch 32 --iters 10 --cpu-seconds 0 --resident-only --content ${CONTENT:-hard} \
      --out gpurun_out/$tag.jsonl > gpurun_out/$tag.log 2>&1 || { echo PROF_FAILED $tag; tail -30 gpurun_out/$tag.log; exit 1; }
  VF_JPEG_SYNC=$mode VF_JPEG_SYNC_STATS=1 timeout -k 10 120 python3 tools/jpeg_bench.py --sizes ${SIZES:-1080p} --batch 32 --iters 1 \
      --cpu-seconds 0 --resident-only --content ${CONTENT:-hard} > gpurun_out/${tag}_stats.log 2>&1 || { echo STATS_FAILED; tail -20 gpurun_out/${tag}_stats.log; exit 1; }
  grep -m2 "spec:" gpurun_out/${tag}_stats.log
done
python3 - <<'PY'
import collections, csv, glob, json, re
for mode in ("auto", "spec"):
    tag = f"hard_{mode}"
    for d in [json.loads(l) for l in open(f"gpurun_out/{tag}.jsonl")]:
        print(f"{mode}: {d.get('size')} resident {d['gpu_resident_fps']} parity {d['parity_vs_oracle']} sync mode {d.get('huffman_sync_mode')} stages {json.dumps(d['stages_ms'])}")
    f = glob.glob(f"gpurun_out/prof_{tag}/**/*kernel_stats.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    print("   " + ", ".join(f"{re.sub(r'[<(].*', '', r['Name'].replace('(anonymous namespace)::', '')).split('::')[-1]} {float(r['AverageNs'])/1e3:.1f}us x{r['Calls']}" for r in rows[:10]))
PY
