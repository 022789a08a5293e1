set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_pipe_jpeg3.jsonl
run() { timeout -k 10 200 python -u tools/pipeline_bench.py "$@" --out gpurun_out/r2_pipe_jpeg3.jsonl > gpurun_out/r2_pipe_jpeg3_last.log 2>&1 || { echo PIPE_FAILED "$@"; tail -20 gpurun_out/r2_pipe_jpeg3_last.log; exit 1; }; }
run --jpeg --workers 1 --gpus 1 --size 1080p --batch 32 --frames 8192 --policy pull
run --jpeg --workers 1 --gpus 1 --size 4k --batch 16 --frames 2048 --policy shard
run --jpeg --workers 1 --gpus 1 --size 480p --batch 32 --frames 16384 --policy pull
run --workers 1 --gpus 1 --size mixed --batch 16 --frames 768 --policy pull --producer copy
run --workers 1 --gpus 1 --size 4k --batch 16 --frames 512 --policy shard --producer copy
python3 -c "
import json
for l in open('gpurun_out/r2_pipe_jpeg3.jsonl'):
    d = json.loads(l); print(d['kind'], d['size'], d['workers'], d['ring_slots_per_worker'], d['fps'], d['latency_ms_mean'], d['n_errors'])
"
