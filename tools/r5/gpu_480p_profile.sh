#!/bin/bash
# 480p vs 512² JPEG system legs, 2 reps each, the second with the thread sampler (tools/sampler.py).
set -o pipefail
mkdir -p gpurun_out
P=gpurun_out/r5_480p.jsonl; rm -f $P
for rep in 1 2; do
for sz in 480p 512sq; do
  prof=""; [ $rep = 2 ] && prof="--profile gpurun_out/r5_prof_$sz"
  timeout -k 10 200 python tools/pipeline_bench.py --workers 1 --jpeg --size $sz --batch 32 --policy pull --frames 65536 $prof --out $P > /dev/null 2>> gpurun_out/r5_480p.err || { echo FAILED; tail -20 gpurun_out/r5_480p.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$P')][-1]; print(d['size'], d['fps'], d['n_errors'], 'lat', d.get('latency_ms_mean'), 'jpeg B', d.get('jpeg_bytes_in_mean'), 'slots', d.get('ring_slots_per_worker'))"
done
done
for sz in 480p 512sq; do timeout -k 10 120 python3 tools/jpeg_modes.py $sz async3 2>&1 | tail -1; done
