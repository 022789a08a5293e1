# The JPEG codec's first output copy sized from its previous batch's output/input ratio
# (VF_JPEG_FETCH_LEARN=1, this tree's default) vs the fixed rule of 1.25x the input + 8 KB per frame (0):
# the JPEG GPU tests first, then jpeg_bench's host->host forms on hard 1080p content and the system legs,
# interleaved, 3 reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_fl_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r6_fl_pytest.log; exit 1; }
tail -2 gpurun_out/r6_fl_pytest.log
for rep in 1 2 3; do
for l in 0 1; do
  VF_JPEG_FETCH_LEARN=$l timeout -k 10 120 python3 tools/jpeg_bench.py --sizes 1080p --content hard --batch 32 --iters 20 --cpu-seconds 0 \
      > gpurun_out/r6_fl_jb_${l}_$rep.jsonl 2> gpurun_out/r6_fl_jb_${l}_$rep.err || { echo JB_FAILED; tail -20 gpurun_out/r6_fl_jb_${l}_$rep.err; exit 1; }
  python3 -c "
import json
for x in open('gpurun_out/r6_fl_jb_${l}_$rep.jsonl'):
    if x.startswith('{'):
        d=json.loads(x); print('jb hard learn $l rep $rep resident', d['gpu_resident_fps'], 'h2h', d['host_to_host_fps'], '2thr', d['host_to_host_2threads_fps'])"
done
for sz in 1080p_hard 1080p 512sq; do
for l in 0 1; do
  b=64; n=98304; extra=""
  case $sz in 1080p) b=32; n=24576;; 1080p_hard) b=32; n=4608; extra="--content hard";; esac
  s=$sz; [ $sz = 1080p_hard ] && s=1080p
  VF_JPEG_FETCH_LEARN=$l timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $s --batch $b --policy pull \
      --frames $n $extra > gpurun_out/r6_fl_${sz}_${l}_$rep.json 2> gpurun_out/r6_fl_${sz}_${l}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_fl_${sz}_${l}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([x for x in open('gpurun_out/r6_fl_${sz}_${l}_$rep.json') if x.startswith('{')][-1]); print('$sz learn $l rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'errors', d['n_errors'], 'lost', d['frames_lost'])"
done
done
done
