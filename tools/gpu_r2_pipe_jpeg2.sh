set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_pipe_jpeg2.jsonl
for w in 1 2; do
  timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers $w --gpus 1 --size 1080p --batch 32 --frames 8192 --policy pull --out gpurun_out/r2_pipe_jpeg2.jsonl > gpurun_out/r2_pipe_jpeg2_$w.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe_jpeg2_$w.log; exit 1; }
done
timeout -k 10 200 python -u tools/pipeline_bench.py --jpeg --workers 1 --gpus 1 --size 480p --batch 32 --frames 16384 --policy pull --out gpurun_out/r2_pipe_jpeg2.jsonl > gpurun_out/r2_pipe_jpeg2_480.log 2>&1 || { echo PIPE_FAILED; tail -20 gpurun_out/r2_pipe_jpeg2_480.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r2_pipe_jpeg2.jsonl'):
    d = json.loads(l); print(d['size'], d['workers'], d['fps'], d['latency_ms_mean'], d['n_errors'])
"
