# pipeline tool with parallel producers: configs[2] 4K copy / resident (1 and 8 workers on the
# one GPU), configs[3] mixed, JPEG 1080p through the distributor
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_pipe2b.jsonl
run() { timeout -k 10 200 python -u tools/pipeline_bench.py "$@" --out gpurun_out/r2_pipe2b.jsonl > gpurun_out/r2_pipe2b_last.log 2>&1 || { echo PIPE_FAILED "$@"; tail -20 gpurun_out/r2_pipe2b_last.log; exit 1; }; }
run --workers 1 --gpus 1 --size 4k --batch 16 --frames 512 --policy shard --producer copy
run --workers 1 --gpus 1 --size 4k --batch 16 --frames 512 --policy shard --producer resident
run --workers 8 --gpus 1 --size 4k --batch 16 --frames 1024 --policy shard --producer copy
run --workers 1 --gpus 1 --size mixed --batch 16 --frames 768 --policy pull --producer copy
run --jpeg --workers 1 --gpus 1 --size 1080p --batch 32 --frames 4096 --policy pull
run --jpeg --workers 2 --gpus 1 --size 1080p --batch 32 --frames 4096 --policy pull
python3 -c "
import json
for l in open('gpurun_out/r2_pipe2b.jsonl'):
    d = json.loads(l); print(d['kind'], d['size'], d['workers'], d['producers'], d['producer'], d['fps'], d['GBps_each_way'], d['n_errors'], d['latency_ms_mean'])
"
