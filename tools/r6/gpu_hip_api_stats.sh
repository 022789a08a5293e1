# HIP API time of the JPEG invert path at 480p x 64 (jpeg_bench's host->host forms): how much of a
# batch's host time is launch and copy calls (the case for capturing a batch in a hipGraph).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/r6_hipapi -o run -- \
    python3 tools/jpeg_bench.py --sizes 480p --batch 64 --iters 40 --cpu-seconds 0 > gpurun_out/r6_hipapi.log 2>&1
rc=$?; tail -3 gpurun_out/r6_hipapi.log; find gpurun_out/r6_hipapi -name "*stats.csv" | head; exit $rc
