# synchronous zero-copy from the calling thread: parity suite + per-frame latency + e2e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plumbing.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_rn_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r2_rn_tests.log; exit 1; }
tail -1 gpurun_out/r2_rn_tests.log
timeout -k 10 200 python -u tools/per_frame_probe.py > gpurun_out/r2_per_frame2.jsonl 2> gpurun_out/r2_per_frame2.err || { echo FAILED; tail -20 gpurun_out/r2_per_frame2.err; exit 1; }
cat gpurun_out/r2_per_frame2.jsonl
timeout -k 10 120 python -u tools/e2e_probe.py > gpurun_out/r2_e2e_rn.jsonl 2> gpurun_out/r2_e2e_rn.err || { echo E2E_FAILED; tail -20 gpurun_out/r2_e2e_rn.err; exit 1; }
cut -c1-300 gpurun_out/r2_e2e_rn.jsonl
