# configs[4] large-buffer behaviour: the sweep (fresh process per point, more steps) and the
# single-buffer experiment of tune_invert at 6.4 and 12.7 GB.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep.py --out gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1 || { echo SWEEP_FAILED; tail -20 gpurun_out/sweep.log; exit 1; }
timeout -k 10 200 tools/tune_invert large 12740198400 5 > gpurun_out/large_12g.txt 2>&1 || { echo LARGE_FAILED; tail gpurun_out/large_12g.txt; exit 1; }
grep '"kind": "kernel"' gpurun_out/sweep.jsonl; cat gpurun_out/large_12g.txt
