# Round 2 JPEG, second pass: the async ticket API + fdct table-read fix: parity, kernel times,
# SQ counters, host->host forms.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_plumbing.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_pytest_jpeg2.log 2>&1 || { echo PYTEST_FAILED; tail -60 gpurun_out/r2_pytest_jpeg2.log; exit 1; }
tail -2 gpurun_out/r2_pytest_jpeg2.log
bash tools/gpu_jpeg_pmc.sh > gpurun_out/r2_jpeg_pmc_sq2.txt 2>&1 || { echo PMC_FAILED; cat gpurun_out/r2_jpeg_pmc_sq2.txt; exit 1; }
grep -E "k_idct|k_fdct" gpurun_out/r2_jpeg_pmc_sq2.txt
bash tools/gpu_jpeg_stats.sh 1080p > gpurun_out/r2_jpeg_kstats2_1080p.txt 2>&1 || { echo STATS_FAILED; cat gpurun_out/r2_jpeg_kstats2_1080p.txt; exit 1; }
grep -E "k_idct|k_fdct|k_color" gpurun_out/r2_jpeg_kstats2_1080p.txt
rm -f gpurun_out/r2_jpeg_modes2.jsonl
for s in 480p 1080p 4k; do
  timeout -k 10 300 python -u tools/jpeg_modes.py $s >> gpurun_out/r2_jpeg_modes2.jsonl 2> gpurun_out/r2_jpeg_modes2_$s.err || { echo MODES_FAILED $s; tail -20 gpurun_out/r2_jpeg_modes2_$s.err; exit 1; }
done
cat gpurun_out/r2_jpeg_modes2.jsonl
VF_JPEG_TRACE=1 timeout -k 10 120 python -u tools/jpeg_modes.py 1080p async > /dev/null 2> gpurun_out/r2_jpeg_trace_async_1080p.txt || { echo TRACE_FAILED; exit 1; }
tail -8 gpurun_out/r2_jpeg_trace_async_1080p.txt
