# Round-6 refresh: GPU tests, smoke, the default bench line, rocprof kernel stats of the bench kernel leg,
# the JPEG-mode bench at 480p / 1080p / 4K and rocprof kernel stats of the 1080p JPEG bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6_pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r6_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r6_pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/r6_smoke.log; exit 1; }
cat gpurun_out/r6_smoke.log
S=$(date +%s)
BENCH_DETAIL=gpurun_out/r6_bench_detail.json timeout -k 10 500 python -u bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r6_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - S )) s"
rm -rf gpurun_out/prof_bench
BENCH_DETAIL=gpurun_out/r6_bench_detail_under_rocprof.json timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --no-traffic --cpu-seconds 0 --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep > gpurun_out/r6_bench_under_rocprof.json 2> gpurun_out/r6_bench_prof.err || { echo PROF_FAILED; tail -30 gpurun_out/r6_bench_prof.err; exit 1; }
cp "$(find gpurun_out/prof_bench -name '*kernel_stats.csv' | head -1)" gpurun_out/r6_bench_kernel_stats.csv
rm -f gpurun_out/r6_jpeg_sizes.jsonl
timeout -k 10 300 python -u tools/jpeg_bench.py --sizes 480p,1080p,4k --batch 32 --iters 20 --cpu-seconds 5 --out gpurun_out/r6_jpeg_sizes.jsonl > gpurun_out/r6_jpeg.log 2>&1 || { echo JPEG_FAILED; tail -30 gpurun_out/r6_jpeg.log; exit 1; }
rm -rf gpurun_out/prof_js
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_js -o js -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 20 --cpu-seconds 0 --resident-only > gpurun_out/js.log 2>&1 || { echo JPEG_PROF_FAILED; tail -30 gpurun_out/js.log; exit 1; }
cp "$(find gpurun_out/prof_js -name '*kernel_stats.csv' | head -1)" gpurun_out/r6_jpeg_kernel_stats_1080p.csv
rm -rf gpurun_out/prof_jh
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_jh -o jh -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 20 --cpu-seconds 0 --resident-only --content hard > gpurun_out/jh.log 2>&1 || { echo JPEG_HARD_PROF_FAILED; tail -30 gpurun_out/jh.log; exit 1; }
cp "$(find gpurun_out/prof_jh -name '*kernel_stats.csv' | head -1)" gpurun_out/r6_jpeg_kernel_stats_1080p_hard.csv

echo REFRESH_OK
