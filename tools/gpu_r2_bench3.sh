# Round 2: bench line after the zero-copy host path, then the rocprof kernel stats of the headline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > gpurun_out/r2_bench4.json 2> gpurun_out/r2_bench4.log || { echo BENCH_FAILED; tail -30 gpurun_out/r2_bench4.log; exit 1; }
cut -c1-300 gpurun_out/r2_bench4.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-traffic --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r2_bench4_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2_bench4_prof.log || { echo PROF_FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r2_bench4_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof4 -name "*kernel_stats.csv" | head -3
