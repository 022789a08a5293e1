#!/bin/bash
# Round 5: the worker's ring-batch form on the GPU -- plumbing + JPEG suites, then the small-frame
# JPEG system legs (and a sampled profile of the 512 x 512 one).  Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_plumbing.py tests/test_gpu_jpeg.py -x -q --timeout 240 \
    --timeout-method thread > gpurun_out/r5_ring_pytest.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r5_ring_pytest.log; exit 1; }
tail -2 gpurun_out/r5_ring_pytest.log
P=gpurun_out/r5_ring_pipe.jsonl
run() { timeout -k 10 200 python tools/pipeline_bench.py "$@" --out $P > /dev/null 2>> gpurun_out/r5_ring_pipe.err || { echo "FAILED: $*"; tail -20 gpurun_out/r5_ring_pipe.err; exit 1; }; python -c "import json,sys; d=[json.loads(l) for l in open('$P')][-1]; print(d['size'], d.get('content'), d['fps'], d['n_errors'])"; }
run --workers 1 --jpeg --size 512sq --batch 32 --policy pull --frames 32768
run --workers 1 --jpeg --size 480p --batch 32 --policy pull --frames 32768
run --workers 1 --jpeg --size 1080p --batch 32 --policy pull --frames 12288
run --workers 1 --size 4k --batch 16 --policy shard --producer copy --frames 768
run --workers 1 --jpeg --size 512sq --batch 32 --policy pull --frames 32768 --profile gpurun_out/r5_prof512
