# Round 2: bench line with the configs[4] sweep and the torch-free JPEG child.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > gpurun_out/r2_bench3.json 2> gpurun_out/r2_bench3.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench3.log; exit 1; }
cut -c1-300 gpurun_out/r2_bench3.json
