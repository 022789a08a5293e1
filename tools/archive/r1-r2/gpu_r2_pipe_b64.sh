# JPEG 1080p / 4K through distributor + one GPU worker: batch 32 vs 64, interleaved; then the
# bench's JPEG child (worker form at batch 32 and 64)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/pipe_b64.jsonl
for rep in 1 2; do
for sz in 1080p 4k; do
for b in 32 64; do
  n=4096; [ $sz = 4k ] && n=1024
  timeout -k 10 150 python -u tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch $b --policy pull --frames $n >> gpurun_out/pipe_b64.jsonl 2>> gpurun_out/pipe_b64.err || { echo PIPE_FAILED; tail -20 gpurun_out/pipe_b64.err; exit 1; }
done
done
done
timeout -k 10 200 python -u bench.py --jpeg-child 0 --batch 32 --cpu-seconds 0 > gpurun_out/jchild.json 2>> gpurun_out/pipe_b64.err || { echo CHILD_FAILED; tail -20 gpurun_out/pipe_b64.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/pipe_b64.jsonl'):
    d=json.loads(l); print(d.get('size'), d.get('batch'), d.get('fps'), d.get('verified', d.get('checked')))
d=json.load(open('gpurun_out/jchild.json')); print({k:v for k,v in d.items() if 'fps' in k})"
