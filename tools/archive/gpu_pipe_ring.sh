# JPEG 1080p through distributor + worker: ring slots per worker x batches in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rs in 160 256 384; do
  for inf in 3 4; do
    timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --jpeg --size 1080p --batch 32 --frames 3072 --policy pull --ring-slots $rs --inflight $inf > gpurun_out/pr.jsonl 2> gpurun_out/pr.log || { echo PIPE_FAILED; tail -20 gpurun_out/pr.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/pr.jsonl').read().strip().splitlines()[-1]); print('ring $rs inflight $inf', d['fps'], 'lat', d['latency_ms_mean'], 'depth', d['max_buffer_depth'], 'errors', d.get('n_errors'))"
  done
done
