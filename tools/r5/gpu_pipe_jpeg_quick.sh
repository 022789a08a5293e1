#!/bin/bash
# JPEG legs through pipeline_bench only (no bench line): consumer batch and inline vs pooled
# verification at 1 and 2 workers (2 share the card).  Run from the repo root under gpurun.
set -o pipefail
mkdir -p gpurun_out
P=gpurun_out/r5_pipe_quick.jsonl
rm -f $P
run() { timeout -k 10 200 python tools/pipeline_bench.py "$@" --out $P > /dev/null 2>> gpurun_out/r5_pipe_quick.err || { echo "FAILED: $*"; tail -20 gpurun_out/r5_pipe_quick.err; exit 1; }; python3 -c "import json,sys; d=[json.loads(l) for l in open('$P')][-1]; print(d['size'], d['workers'], 'consume', d['consume'], 'pool', d['verify_pool'], d['fps'], d['n_errors'], d.get('frames_lost'))"; }
for rep in 1 2; do
for v in "--consume 64 --verify-pool 0" "--consume 64 --verify-pool 1" "--consume 256 --verify-pool 0" "--consume 256 --verify-pool 1"; do
run --workers 1 --jpeg --size 480p --batch 32 --policy pull --frames 32768 $v
done
done
for v in "--consume 64 --verify-pool 0" "--consume 256 --verify-pool 1"; do
run --workers 2 --jpeg --size 480p --batch 32 --policy pull --frames 65536 $v
run --workers 1 --jpeg --size 1080p --batch 32 --policy pull --frames 12288 $v
done
