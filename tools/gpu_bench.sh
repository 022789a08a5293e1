# bench line + rocprof kernel stats of the same command (PMC passes off under the profiler)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --no-traffic --cpu-seconds 0 --no-e2e --no-jpeg --no-distributor --no-sizes > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo PROF_FAILED; tail -30 gpurun_out/bench_prof.err; exit 1; }
cat gpurun_out/bench_prof.json; cat gpurun_out/prof_bench/bench_kernel_stats.csv
