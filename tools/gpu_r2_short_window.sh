# The headline at the driver's window (--steps 20 --warmup 5) several times, beside 300 steps
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/short_window.jsonl
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-traffic --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep --cpu-seconds 0 >> gpurun_out/short_window.jsonl 2>> gpurun_out/short_window.log || { echo BENCH_FAILED; tail -20 gpurun_out/short_window.log; exit 1; }
done
timeout -k 10 120 python -u bench.py --steps 300 --warmup 30 --no-traffic --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep --cpu-seconds 0 >> gpurun_out/short_window.jsonl 2>> gpurun_out/short_window.log || { echo BENCH_FAILED; tail -20 gpurun_out/short_window.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/short_window.jsonl'):
    d=json.loads(l); print(d['steps'], d['warmup'], d['value'], d['ms_per_step'], d['roofline']['mean_launch_ms'])"
