# The JPEG codec's host task pool woken through a futex (this tree) or a condition variable (the
# pre-change library, tools/r6/ab/libvfilter_cv.so): jpeg_bench's host->host forms and the
# 480p / 512x512 / 1080p system legs, interleaved, 3 reps each.
set -o pipefail
mkdir -p gpurun_out
NEW=distributed-video-filter_amd/vfilter/libvfilter_hip.so
OLD=tools/r6/ab/libvfilter_cv.so
for rep in 1 2 3; do
for lib in cv futex; do
  L=$NEW; [ $lib = cv ] && L=$OLD
  VFILTER_LIB=$L timeout -k 10 120 python3 tools/jpeg_bench.py --sizes 480p,512sq,1080p --batch 64 --iters 40 --cpu-seconds 0 \
      > gpurun_out/r6_tp_jb_${lib}_$rep.jsonl 2> gpurun_out/r6_tp_jb_${lib}_$rep.err || { echo JB_FAILED; tail -20 gpurun_out/r6_tp_jb_${lib}_$rep.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r6_tp_jb_${lib}_$rep.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('jb $lib rep $rep', d.get('size'), d.get('host_to_host_fps'), d.get('host_to_host_2threads_fps'))"
done
for sz in 480p 512sq 1080p; do
for lib in cv futex; do
  L=$NEW; [ $lib = cv ] && L=$OLD
  b=64; [ $sz = 1080p ] && b=32
  n=98304; [ $sz = 1080p ] && n=24576
  VFILTER_LIB=$L timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $sz --batch $b --policy pull \
      --frames $n > gpurun_out/r6_tp_${sz}_${lib}_$rep.json 2> gpurun_out/r6_tp_${sz}_${lib}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_tp_${sz}_${lib}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6_tp_${sz}_${lib}_$rep.json') if l.startswith('{')][-1]); print('$sz $lib rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'errors', d['n_errors'])"
done
done
done
