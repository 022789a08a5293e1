#!/bin/bash
# Round 5: the distributor legs through pipeline_bench (native control plane, batch consumer),
# then the full bench line.  Run from the repo root under gpurun.
set -o pipefail
mkdir -p gpurun_out
P=gpurun_out/r5_pipe.jsonl
run() { timeout -k 10 200 python tools/pipeline_bench.py "$@" --out $P > /dev/null 2>> gpurun_out/r5_pipe.err || { echo "FAILED: $*"; tail -20 gpurun_out/r5_pipe.err; exit 1; }; tail -1 $P | cut -c1-400; }
run --workers 1 --jpeg --size 512sq --batch 32 --policy pull --frames 32768
run --workers 1 --jpeg --size 480p --batch 32 --policy pull --frames 32768
run --workers 1 --jpeg --size 1080p --batch 32 --policy pull --frames 12288
run --workers 1 --jpeg --content hard --size 1080p --batch 32 --policy pull --frames 1536
run --workers 1 --size 4k --batch 16 --policy shard --producer copy --frames 768
run --workers 1 --size mixed --batch 16 --policy pull --producer copy --frames 1152
timeout -k 10 900 python bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { echo "bench failed"; tail -30 gpurun_out/r5_bench.err; exit 1; }
cut -c1-600 gpurun_out/r5_bench.json
