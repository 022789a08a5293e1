#!/bin/bash
# Round 5: GPU suite + the distributor control plane (native and Python engines) on a GPU box's
# CPU share.  Run from the repo root under gpurun.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r5_control_plane.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5_pytest_gpu.log 2>&1 || { echo "GPU suite failed"; tail -30 gpurun_out/r5_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5_pytest_gpu.log
for w in 1 2 4 8; do
  timeout -k 10 150 python tools/distributor_overhead.py --workers $w --no-copy --frames 300000 --out $OUT | tail -1 || exit 1
  timeout -k 10 150 python tools/distributor_overhead.py --workers $w --no-copy --bytes 24883200 --batch 16 \
      --policy shard --frames 150000 --out $OUT | tail -1 || exit 1
  timeout -k 10 150 python tools/distributor_overhead.py --workers $w --no-copy --mixed --batch 16 \
      --frames 150000 --out $OUT | tail -1 || exit 1
done
timeout -k 10 150 python tools/distributor_overhead.py --workers 8 --no-copy --frames 100000 --engine python \
    --out $OUT | tail -1 || exit 1
