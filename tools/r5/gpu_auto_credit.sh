#!/bin/bash
# The JPEG worker's adaptive request size (--batch 0, vfilter.inverter.auto_credit) against fixed
# 32 and 64, 512² and 1080p through distributor + worker (ring slices sized for 64), 2 reps.
set -o pipefail
mkdir -p gpurun_out
P=gpurun_out/r5_auto_credit.jsonl; rm -f $P
for rep in ${REPS:-1 2}; do
for sz in ${SIZES:-512sq 1080p}; do
for wb in ${WBS:-32 64 0}; do
  n=65536; [ $sz = 1080p ] && n=16384
  timeout -k 10 200 python tools/pipeline_bench.py --workers 1 --jpeg --size $sz --batch 64 --worker-batch $wb --policy pull --frames $n --out $P > /dev/null 2>> gpurun_out/r5_auto_credit.err || { echo FAILED; tail -20 gpurun_out/r5_auto_credit.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$P')][-1]; print(d['size'], 'worker batch', d['worker_batch'], d['fps'], d['n_errors'], 'lat_ms', d.get('latency_ms_mean'))"
done
done
done
