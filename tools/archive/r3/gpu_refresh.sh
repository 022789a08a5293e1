# Round-3 refresh: tools/gpu_refresh.sh plus the per-frame drop-in probe (profiles/r03_per_frame.jsonl).
# GPU tests, smoke, the default bench line, rocprof kernel stats of the bench's kernel leg,
# the JPEG-mode bench at 480p / 1080p / 4K and rocprof kernel stats of the 1080p JPEG bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
S=$(date +%s)
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - S )) s"
rm -rf gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --no-traffic --cpu-seconds 0 --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo PROF_FAILED; tail -30 gpurun_out/bench_prof.err; exit 1; }
cp "$(find gpurun_out/prof_bench -name '*kernel_stats.csv' | head -1)" gpurun_out/bench_kernel_stats.csv
rm -f gpurun_out/jpeg.jsonl
timeout -k 10 300 python -u tools/jpeg_bench.py --sizes 480p,1080p,4k --batch 32 --iters 20 --cpu-seconds 5 --out gpurun_out/jpeg.jsonl > gpurun_out/jpeg.log 2>&1 || { echo JPEG_FAILED; tail -30 gpurun_out/jpeg.log; exit 1; }
rm -rf gpurun_out/prof_js
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_js -o js -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 20 --cpu-seconds 0 --resident-only > gpurun_out/js.log 2>&1 || { echo JPEG_PROF_FAILED; tail -30 gpurun_out/js.log; exit 1; }
cp "$(find gpurun_out/prof_js -name '*kernel_stats.csv' | head -1)" gpurun_out/jpeg_kernel_stats.csv

timeout -k 10 120 python -u tools/per_frame_probe.py > gpurun_out/per_frame.jsonl 2> gpurun_out/per_frame.log || { echo PERFRAME_FAILED; tail -20 gpurun_out/per_frame.log; exit 1; }
cat gpurun_out/per_frame.jsonl
echo REFRESH_OK
