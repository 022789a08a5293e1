# The JPEG worker's batches in flight (--inflight 3, the default, vs 4 and 2) on the small system
# legs and 1080p, interleaved, 3 reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for sz in 512sq 480p 1080p; do
for k in 2 3 4; do
  b=64; n=98304
  [ $sz = 1080p ] && { b=32; n=24576; }
  timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch $b --policy pull \
      --frames $n --inflight $k > gpurun_out/r6_if_${sz}_${k}_$rep.json 2> gpurun_out/r6_if_${sz}_${k}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_if_${sz}_${k}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([x for x in open('gpurun_out/r6_if_${sz}_${k}_$rep.json') if x.startswith('{')][-1]); print('$sz inflight $k rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'errors', d['n_errors'])"
done
done
done
