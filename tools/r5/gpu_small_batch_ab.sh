#!/bin/bash
# JPEG system legs at the reference app's frame sizes with worker batches of 32 / 64 / 96, 2 reps.
set -o pipefail
mkdir -p gpurun_out
P=gpurun_out/r5_small_batch.jsonl; rm -f $P
for rep in 1 2; do
for sz in 512sq 480p; do
for b in 32 64 96; do
  timeout -k 10 200 python tools/pipeline_bench.py --workers 1 --jpeg --size $sz --batch $b --policy pull --frames 98304 --out $P > /dev/null 2>> gpurun_out/r5_small_batch.err || { echo FAILED; tail -20 gpurun_out/r5_small_batch.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$P')][-1]; print(d['size'], 'batch', d['batch'], d['fps'], d['n_errors'], 'lat_ms', d.get('latency_ms_mean'))"
done
done
done
