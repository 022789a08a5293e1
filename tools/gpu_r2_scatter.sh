# Staged (pageable) host path with the scatter thread: parity + engine tests, e2e rates,
# then the JPEG worker-form A/B (tools/jpeg_modes.py vs the bench's JPEG child) and the
# headline rocprof stats in csv.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plumbing.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_sc_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_sc_tests.log; exit 1; }
tail -2 gpurun_out/r2_sc_tests.log
rm -f gpurun_out/r2_e2e_sc.jsonl
for r in 1 2; do
  timeout -k 10 120 python -u tools/e2e_probe.py >> gpurun_out/r2_e2e_sc.jsonl 2> gpurun_out/r2_e2e_sc.err || { echo E2E_FAILED; tail -20 gpurun_out/r2_e2e_sc.err; exit 1; }
done
cut -c1-330 gpurun_out/r2_e2e_sc.jsonl
bash tools/gpu_r2_jpegab.sh
