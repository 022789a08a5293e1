# configs[4] large-batch points, time-based warmup (>= 300 ms kernel time) and timing
# (>= 200 ms), each point in a fresh process; run twice to see the spread.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/c5_a.jsonl gpurun_out/c5_b.jsonl
timeout -k 10 300 python -u tools/sweep.py --c5-only --out gpurun_out/c5_a.jsonl > gpurun_out/c5_a.log 2>&1 || { echo C5A_FAILED; tail -20 gpurun_out/c5_a.log; exit 1; }
timeout -k 10 300 python -u tools/sweep.py --c5-only --out gpurun_out/c5_b.jsonl > gpurun_out/c5_b.log 2>&1 || { echo C5B_FAILED; tail -20 gpurun_out/c5_b.log; exit 1; }
cat gpurun_out/c5_a.jsonl gpurun_out/c5_b.jsonl
