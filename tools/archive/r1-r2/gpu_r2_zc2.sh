#!/bin/bash
# Zero-copy host->host path: parity, then sync / pipelined rates against the slot ring
# (VF_ZEROCOPY=0), then the configs[2] fan-out through the distributor.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_zc_parity.log 2>&1 || { echo PARITY_FAILED; tail -30 gpurun_out/r2_zc_parity.log; exit 1; }
tail -3 gpurun_out/r2_zc_parity.log
rm -f gpurun_out/r2_e2e_zc.jsonl gpurun_out/r2_pipe_zc.jsonl
for r in 1 2; do
  for z in 1 0; do
    VF_ZEROCOPY=$z timeout -k 10 120 python -u tools/e2e_probe.py >> gpurun_out/r2_e2e_zc.jsonl 2> gpurun_out/r2_e2e_zc_$z.err || { echo E2E_FAILED $z; tail -20 gpurun_out/r2_e2e_zc_$z.err; exit 1; }
  done
done
cat gpurun_out/r2_e2e_zc.jsonl
for z in 1 0; do
  VF_ZEROCOPY=$z timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --gpus 1 --size 4k --batch 16 --frames 512 --policy shard --producer copy --out gpurun_out/r2_pipe_zc.jsonl > gpurun_out/r2_pipe_zc_$z.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe_zc_$z.log; exit 1; }
  VF_ZEROCOPY=$z timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --gpus 1 --size 4k --batch 16 --frames 512 --policy shard --producer resident --out gpurun_out/r2_pipe_zc.jsonl > gpurun_out/r2_pipe_zc_r$z.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe_zc_r$z.log; exit 1; }
done
cut -c1-420 gpurun_out/r2_pipe_zc.jsonl
