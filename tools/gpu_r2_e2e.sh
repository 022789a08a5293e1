# Round 2: NUMA placement A/B for the host->host paths, and the configs[2]/[3] fan-out with
# verification off the consumer path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_e2e_numa.jsonl gpurun_out/r2_pipe2.jsonl
for r in 1 2; do
  for n in 1 0; do
    VF_NUMA=$n timeout -k 10 120 python -u tools/e2e_probe.py >> gpurun_out/r2_e2e_numa.jsonl 2> gpurun_out/r2_e2e_$n.err || { echo E2E_FAILED $n; tail -20 gpurun_out/r2_e2e_$n.err; exit 1; }
  done
done
cat gpurun_out/r2_e2e_numa.jsonl
for p in copy resident; do
  timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --gpus 1 --size 4k --batch 16 --frames 512 --policy shard --producer $p --out gpurun_out/r2_pipe2.jsonl > gpurun_out/r2_pipe2_$p.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe2_$p.log; exit 1; }
done
timeout -k 10 200 python -u tools/pipeline_bench.py --workers 2 --gpus 1 --size mixed --batch 16 --frames 768 --policy pull --producer copy --out gpurun_out/r2_pipe2.jsonl > gpurun_out/r2_pipe2_mixed.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe2_mixed.log; exit 1; }
cut -c1-420 gpurun_out/r2_pipe2.jsonl
