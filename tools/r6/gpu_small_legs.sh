#!/bin/bash
# The JPEG system legs at the reference app's frame sizes (bench distributor.jpeg_512 / jpeg_480p:
# distributor + one worker process, batches of 64, pull), 3 reps each, interleaved; and the
# worker form beside them (tools/r6/worker_form_phases.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for sz in 512sq 480p; do
  timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch 64 --policy pull \
      --frames 98304 > gpurun_out/r6_leg_${sz}_$rep.json 2> gpurun_out/r6_leg_${sz}_$rep.err || { echo LEG_FAILED $sz; tail -20 gpurun_out/r6_leg_${sz}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r6_leg_${sz}_$rep.json') if l.startswith('{')][-1]); print('$sz rep $rep', d['fps'], 'errors', d['n_errors'], 'lat', d['latency_ms_mean'])"
done
done
for sz in 512sq 480p; do timeout -k 10 120 python3 tools/r6/worker_form_phases.py $sz 64; done
if [ "${PROFILE:-0}" = 1 ]; then
for sz in 512sq 480p; do
  timeout -k 10 200 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch 64 --policy pull \
      --frames 98304 --profile gpurun_out/r6_prof_$sz > gpurun_out/r6_leg_${sz}_prof.json 2> gpurun_out/r6_leg_${sz}_prof.err || { echo PROF_FAILED $sz; tail -20 gpurun_out/r6_leg_${sz}_prof.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r6_leg_${sz}_prof.json') if l.startswith('{')][-1]); print('$sz profiled', d['fps'])"
done
fi
