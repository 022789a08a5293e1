#!/bin/bash
# k_syncg pass anatomy on hard 1080p x 32 (tools/build_syncg_stats.sh build): round 0 vs the
# chain rounds per workgroup, lanes re-decoding per round.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VFILTER_LIB=tools/variants/libv_syncg_stats.so VF_SYNCG_STATS=1 timeout -k 10 200 python3 tools/jpeg_bench.py \
  --sizes 1080p --batch 32 --iters 2 --cpu-seconds 0 --resident-only --content hard \
  --out gpurun_out/r6_syncg_stats.jsonl > gpurun_out/r6_syncg_stats.log 2>&1 || { echo FAILED; tail -20 gpurun_out/r6_syncg_stats.log; exit 1; }
grep "\[syncg\]" gpurun_out/r6_syncg_stats.log | tail -12
tail -1 gpurun_out/r6_syncg_stats.jsonl
