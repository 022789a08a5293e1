# Round 2: full GPU suite, then the configs[2] fan-out rehearsed on one card.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -80 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r2_pytest_gpu.log
df -h /dev/shm | tail -1
for w in 1 8; do
  timeout -k 10 240 python -u tools/pipeline_bench.py --workers $w --gpus 1 --size 4k --batch 16 --frames $((128*w)) --policy shard --producer copy --out gpurun_out/r2_pipeline.jsonl > gpurun_out/r2_pipe_$w.log 2>&1 || { echo PIPE_FAILED $w; tail -30 gpurun_out/r2_pipe_$w.log; exit 1; }
  tail -1 gpurun_out/r2_pipe_$w.log
done
