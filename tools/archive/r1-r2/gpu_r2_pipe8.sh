# 8 workers on the one GPU: JPEG 1080p and raw mixed through the distributor (N=8 rehearsal of
# the bench's distributor legs; rates are one card's)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_pipe8.jsonl
run() { timeout -k 10 300 python -u tools/pipeline_bench.py "$@" --out gpurun_out/r2_pipe8.jsonl > gpurun_out/r2_pipe8_last.log 2>&1 || { echo PIPE_FAILED "$@"; tail -20 gpurun_out/r2_pipe8_last.log; exit 1; }; }
run --jpeg --workers 8 --gpus 1 --size 1080p --batch 32 --frames 32768 --policy pull
run --workers 8 --gpus 1 --size mixed --batch 16 --frames 3072 --policy pull --producer copy
run --workers 8 --gpus 1 --size 4k --batch 16 --frames 2048 --policy shard --producer resident
python3 -c "
import json
for l in open('gpurun_out/r2_pipe8.jsonl'):
    d = json.loads(l); print(d['kind'], d['size'], d['workers'], d['producers'], d['ring_slots_per_worker'], d['fps'], d['latency_ms_mean'], d['n_errors'], d['frames_lost'])
"
