# JPEG worker default of 3 batches in flight: plumbing tests + the bench's JPEG child
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_plumbing.py tests/test_gpu_jpeg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_if3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_if3_tests.log; exit 1; }
tail -1 gpurun_out/r2_if3_tests.log
timeout -k 10 200 python -u bench.py --jpeg-child 0 --batch 32 --cpu-seconds 0 > gpurun_out/r2_if3_child.json 2> gpurun_out/r2_if3_child.err || { echo CHILD_FAILED; tail -20 gpurun_out/r2_if3_child.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r2_if3_child.json').read().strip().splitlines()[-1]); print({k: v for k, v in d.items() if 'fps' in k})"
