# one frame per call (the drop-in's shape): CPU numpy vs GPU pageable vs GPU pinned (zero-copy)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/per_frame_probe.py > gpurun_out/r2_per_frame.jsonl 2> gpurun_out/r2_per_frame.err || { echo FAILED; tail -20 gpurun_out/r2_per_frame.err; exit 1; }
cat gpurun_out/r2_per_frame.jsonl
