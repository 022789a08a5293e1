# Round 2 JPEG: parity of the new k_idct / k_fdct LDS layouts, their SQ counters and kernel
# times, and the host->host forms the worker could use (tools/jpeg_modes.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -60 gpurun_out/r2_pytest_jpeg.log; exit 1; }
tail -2 gpurun_out/r2_pytest_jpeg.log
bash tools/gpu_jpeg_pmc.sh > gpurun_out/r2_jpeg_pmc_sq.txt 2>&1 || { echo PMC_FAILED; cat gpurun_out/r2_jpeg_pmc_sq.txt; exit 1; }
grep -E "k_idct|k_fdct|k_write|k_spec" gpurun_out/r2_jpeg_pmc_sq.txt
bash tools/gpu_jpeg_stats.sh 1080p > gpurun_out/r2_jpeg_kstats_1080p.txt 2>&1 || { echo STATS_FAILED; cat gpurun_out/r2_jpeg_kstats_1080p.txt; exit 1; }
grep -E "k_idct|k_fdct|k_color|k_write|k_spec" gpurun_out/r2_jpeg_kstats_1080p.txt
for s in 480p 1080p 4k; do
  timeout -k 10 300 python -u tools/jpeg_modes.py $s >> gpurun_out/r2_jpeg_modes.jsonl 2> gpurun_out/r2_jpeg_modes_$s.err || { echo MODES_FAILED $s; tail -20 gpurun_out/r2_jpeg_modes_$s.err; exit 1; }
done
cat gpurun_out/r2_jpeg_modes.jsonl
VF_JPEG_TRACE=1 timeout -k 10 120 python -u tools/jpeg_modes.py 1080p 2threads > /dev/null 2> gpurun_out/r2_jpeg_trace_2threads_1080p.txt || { echo TRACE_FAILED; exit 1; }
VF_JPEG_TRACE=1 timeout -k 10 120 python -u tools/jpeg_modes.py 1080p 1thread > /dev/null 2> gpurun_out/r2_jpeg_trace_1thread_1080p.txt || { echo TRACE_FAILED; exit 1; }
tail -8 gpurun_out/r2_jpeg_trace_2threads_1080p.txt
