# Round-2 refresh: GPU suite, smoke, bench line, rocprof stats of the headline and of the JPEG pass
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu6.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_pytest_gpu6.log; exit 1; }
tail -1 gpurun_out/r2_pytest_gpu6.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke: OK')" > gpurun_out/r2_smoke6.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r2_smoke6.log; exit 1; }
tail -1 gpurun_out/r2_smoke6.log
timeout -k 10 700 python -u bench.py > gpurun_out/r2_bench10.json 2> gpurun_out/r2_bench10.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench10.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r2_bench10.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['mean_launch_ms'], d['end_to_end']['pinned_GBps_each_way'], d['jpeg_mode']['host_to_host_worker_fps'], {k: v.get('fps') for k, v in d['distributor'].items() if isinstance(v, dict)})"
rm -rf gpurun_out/prof_r2g
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r2g -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-traffic --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r2_bench10_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2_bench10_prof.log || { echo PROF_FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r2_bench10_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && bash tools/gpu_jpeg_stats.sh 1080p > gpurun_out/r2_jpeg_kstats_final2.txt && cat gpurun_out/r2_jpeg_kstats_final2.txt | head -12
