# JPEG host->host forms after lazy engine streams and the ungated default; then the full GPU
# suite, smoke and the bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_jpeg_modes2.jsonl
for size in 480p 1080p 4k; do
  timeout -k 10 200 python -u tools/jpeg_modes.py $size >> gpurun_out/r2_jpeg_modes2.jsonl 2>> gpurun_out/r2_jpeg_modes2.err || { echo MODES_FAILED; tail -20 gpurun_out/r2_jpeg_modes2.err; exit 1; }
done
cat gpurun_out/r2_jpeg_modes2.jsonl
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu3.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_pytest_gpu3.log; exit 1; }
tail -1 gpurun_out/r2_pytest_gpu3.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke: OK')" > gpurun_out/r2_smoke3.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r2_smoke3.log; exit 1; }
tail -1 gpurun_out/r2_smoke3.log
timeout -k 10 700 python -u bench.py > gpurun_out/r2_bench6.json 2> gpurun_out/r2_bench6.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench6.log; exit 1; }
cut -c1-200 gpurun_out/r2_bench6.json
