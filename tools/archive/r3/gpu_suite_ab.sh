# Round 3: the whole GPU suite on the working tree's library, then tools/r3/gpu_abn.sh's A/B
# (its own JPEG test run included) with the environment given.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/suite.log; exit 1; }
tail -1 gpurun_out/suite.log
bash tools/r3/gpu_abn.sh
