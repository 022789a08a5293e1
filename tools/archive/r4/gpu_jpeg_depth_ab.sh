# Round-4 A/B of the JPEG batches kept in flight: the worker form (tools/jpeg_modes.py asyncN,
# one thread, N batches) and the system leg (tools/pipeline_bench.py --jpeg, one worker,
# --inflight N), N = 3, 4, 5, alternating, two reps.  Each batch in flight is one codec on its
# own stream; the process has GPU_MAX_HW_QUEUES (4) hardware queues.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for n in 3 4 5; do
    timeout -k 10 120 python3 tools/jpeg_modes.py 1080p async$n > gpurun_out/dab.json 2> gpurun_out/dab.err || { echo WORKER_FAILED; tail -20 gpurun_out/dab.err; exit 1; }
    echo "worker depth $n rep $rep $(tail -1 gpurun_out/dab.json)"
    timeout -k 10 150 python -u tools/pipeline_bench.py --jpeg --size 1080p --batch 32 --policy pull --frames 16384 --inflight $n > gpurun_out/dab_pipe.json 2> gpurun_out/dab_pipe.err || { echo PIPE_FAILED; tail -20 gpurun_out/dab_pipe.err; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/dab_pipe.json').read().splitlines()[-1]); print('system depth $n rep $rep', json.dumps({k:r.get(k) for k in ('fps','latency_ms_mean','n_errors','inflight_per_worker')}))"
  done
done
echo DEPTH_AB_OK
