# GPU box: full GPU suite + smoke, then the JPEG-mode bench with a rocprof kernel summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
rm -f gpurun_out/jpeg.jsonl
timeout -k 10 300 python -u tools/jpeg_bench.py --sizes 480p,1080p,4k --batch 32 --iters 20 --out gpurun_out/jpeg.jsonl > gpurun_out/jpeg_bench.log 2>&1 || { echo JPEG_BENCH_FAILED; tail -30 gpurun_out/jpeg_bench.log; exit 1; }
cat gpurun_out/jpeg_bench.log
rm -rf gpurun_out/prof_jpeg
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_jpeg -o jpeg -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 > gpurun_out/jpeg_prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/jpeg_prof.log; exit 1; }
find gpurun_out/prof_jpeg -name "*kernel_stats.csv" -exec cat {} \;
