# The drop-in's pageable frame: gated launch vs copy-then-launch vs a pinned source, in one process
# (tools/r6/gated_ab.py), after the whole parity file (staged / zero-copy / gated / engine paths).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r6_gated_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6_gated_tests.log; exit 1; }
tail -1 gpurun_out/r6_gated_tests.log
timeout -k 10 200 python -u tools/r6/gated_ab.py 20 10 > gpurun_out/r6_gated_ab.jsonl 2>&1 || { cat gpurun_out/r6_gated_ab.jsonl; exit 1; }
timeout -k 10 200 python -u tools/r6/gated_ab.py 20 10 >> gpurun_out/r6_gated_ab.jsonl 2>&1 || { cat gpurun_out/r6_gated_ab.jsonl; exit 1; }
timeout -k 10 120 python -u tools/per_frame_probe.py > gpurun_out/r6_per_frame.jsonl 2>&1 || exit 1
cat gpurun_out/r6_gated_ab.jsonl gpurun_out/r6_per_frame.jsonl
