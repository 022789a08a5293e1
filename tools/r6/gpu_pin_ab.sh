# The JPEG system legs with the worker process pinned to its GPU's NUMA node (VF_WORKER_PIN=1, the
# default) or left to the scheduler (0), interleaved, 3 reps each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for sz in 480p 512sq 1080p; do
for pin in 0 1; do
  b=64; [ $sz = 1080p ] && b=32
  n=98304; [ $sz = 1080p ] && n=24576
  VF_WORKER_PIN=$pin timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch $b --policy pull \
      --frames $n > gpurun_out/r6_pin_${sz}_${pin}_$rep.json 2> gpurun_out/r6_pin_${sz}_${pin}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_pin_${sz}_${pin}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6_pin_${sz}_${pin}_$rep.json') if l.startswith('{')][-1]); print('$sz pin $pin rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'errors', d['n_errors'])"
done
done
done
