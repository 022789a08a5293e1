# Stage events only in the bench breakdown: head vs the working tree, resident and host forms
# (full tools/jpeg_bench.py) at 480p and 1080p, JPEG tests first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ev_pytest.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -30 gpurun_out/ev_pytest.log; exit 1; }
tail -1 gpurun_out/ev_pytest.log
for rep in 1 2; do
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  timeout -k 10 200 python3 tools/jpeg_bench.py --sizes 480p,1080p --batch 32 --iters 20 --cpu-seconds 0 > gpurun_out/ev_$v.jsonl 2> gpurun_out/ev_$v.log || { echo RUN_FAILED; tail -20 gpurun_out/ev_$v.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/ev_$v.jsonl'):
    d = json.loads(l)
    print('rep $rep $v', d['size'], 'resident', d['gpu_resident_fps'], 'h2h', d['host_to_host_fps'], '2threads', d['host_to_host_2threads_fps'], d['parity_vs_oracle'])"
done
done
for rep in 1 2 3; do
  timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --jpeg --size 1080p --batch 32 --frames 8192 --policy pull > gpurun_out/ev_pipe.jsonl 2> gpurun_out/ev_pipe.log || { echo PIPE_FAILED; tail -20 gpurun_out/ev_pipe.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/ev_pipe.jsonl').read().strip().splitlines()[-1]); print('pipe rep $rep jpeg 1080p', d['fps'], 'lat', d['latency_ms_mean'], 'errors', d.get('n_errors'))"
done
