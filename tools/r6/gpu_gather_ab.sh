# The JPEG worker reading its ring slots in place (k_gather, VF_JPEG_INPUTS_HELD; VF_JPEG_GATHER=1, the
# default) vs staging them through the codec's page-locked buffer (VF_JPEG_GATHER=0): the held-input
# tests and the JPEG GPU suite first, then the system legs interleaved, 3 reps each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_gather_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r6_gather_pytest.log; exit 1; }
tail -2 gpurun_out/r6_gather_pytest.log
for rep in 1 2 3; do
for sz in 1080p_hard 1080p 512sq 480p; do
for g in 0 1; do
  b=64; n=98304; extra=""
  case $sz in 1080p) b=32; n=24576;; 1080p_hard) b=32; n=4608; extra="--content hard";; esac
  s=$sz; [ $sz = 1080p_hard ] && s=1080p
  VF_JPEG_GATHER=$g timeout -k 10 150 python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size $s --batch $b --policy pull \
      --frames $n $extra > gpurun_out/r6_ga_${sz}_${g}_$rep.json 2> gpurun_out/r6_ga_${sz}_${g}_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_ga_${sz}_${g}_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6_ga_${sz}_${g}_$rep.json') if l.startswith('{')][-1]); print('$sz gather $g rep $rep', d['fps'], 'lat', d['latency_ms_mean'], 'errors', d['n_errors'], 'lost', d['frames_lost'])"
done
done
done
