# Device timeline of the JPEG worker form (1080p, one host thread, two batches in flight):
# kernel + memory-copy trace, then the idle gaps between consecutive batches' GPU work.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_jg
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_jg -o jg -- python3 tools/jpeg_modes.py 1080p async > gpurun_out/jg.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/jg.log; exit 1; }
cat gpurun_out/jg.log | tail -2
python3 tools/jpeg_gaps.py gpurun_out/prof_jg > gpurun_out/r2_jpeg_gaps.txt && tail -60 gpurun_out/r2_jpeg_gaps.txt
rm -f gpurun_out/r2_e2e_scab.jsonl
for r in 1 2; do
  for sc in 1 0; do
    VF_SCATTER=$sc timeout -k 10 120 python -u tools/e2e_probe.py >> gpurun_out/r2_e2e_scab.jsonl 2> gpurun_out/r2_e2e_scab.err || { echo E2E_FAILED; tail -20 gpurun_out/r2_e2e_scab.err; exit 1; }
  done
done
cut -c1-120 gpurun_out/r2_e2e_scab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_jq_tests.log 2>&1 || { echo JPEG_TESTS_FAILED; tail -30 gpurun_out/r2_jq_tests.log; exit 1; }
tail -1 gpurun_out/r2_jq_tests.log
for r in 1 2; do timeout -k 10 120 python -u tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 20 --cpu-seconds 0 2>&1 | grep -v amdgpu.ids | cut -c1-400; done
