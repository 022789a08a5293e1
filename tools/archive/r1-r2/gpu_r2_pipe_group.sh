set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_pipe_group.jsonl
run() { timeout -k 10 300 python -u tools/pipeline_bench.py "$@" --out gpurun_out/r2_pipe_group.jsonl > gpurun_out/r2_pipe_group_last.log 2>&1 || { echo PIPE_FAILED "$@"; tail -20 gpurun_out/r2_pipe_group_last.log; exit 1; }; }
run --jpeg --workers 1 --gpus 1 --size 480p --batch 32 --frames 32768 --policy pull
run --jpeg --workers 1 --gpus 1 --size 1080p --batch 32 --frames 8192 --policy pull
run --jpeg --workers 2 --gpus 1 --size 480p --batch 32 --frames 32768 --policy pull
run --workers 1 --gpus 1 --size mixed --batch 16 --frames 768 --policy pull --producer copy
python3 -c "
import json
for l in open('gpurun_out/r2_pipe_group.jsonl'):
    d = json.loads(l); print(d['kind'], d['size'], d['workers'], d['fps'], d['latency_ms_mean'], d['n_errors'], d['frames_lost'])
"
