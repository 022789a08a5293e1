set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu5.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_pytest_gpu5.log; exit 1; }
tail -1 gpurun_out/r2_pytest_gpu5.log
timeout -k 10 700 python -u bench.py > gpurun_out/r2_bench9.json 2> gpurun_out/r2_bench9.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench9.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r2_bench9.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['end_to_end']['pinned_GBps_each_way'], d['jpeg_mode']['host_to_host_worker_fps'], {k: (v.get('fps'), v.get('error')) for k, v in d['distributor'].items() if isinstance(v, dict)})"
