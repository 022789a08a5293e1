# Why the bench's JPEG child reports a lower worker-form rate than tools/jpeg_modes.py:
# both, twice, on one box; plus the headline rocprof stats in csv.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_jab.jsonl
for r in 1 2; do
  timeout -k 10 120 python -u tools/jpeg_modes.py 1080p async >> gpurun_out/r2_jab.jsonl 2>> gpurun_out/r2_jab.err || { echo MODES_FAILED; tail -20 gpurun_out/r2_jab.err; exit 1; }
  timeout -k 10 200 python -u bench.py --jpeg-child 0 --batch 32 --cpu-seconds 0 >> gpurun_out/r2_jab.jsonl 2>> gpurun_out/r2_jab.err || { echo CHILD_FAILED; tail -20 gpurun_out/r2_jab.err; exit 1; }
done
cut -c1-400 gpurun_out/r2_jab.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-traffic --no-e2e --no-jpeg --no-distributor --no-sizes --no-sweep --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r2_bench5_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2_bench5_prof.log || { echo PROF_FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r2_bench5_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof5 -name "*kernel_stats.csv"
