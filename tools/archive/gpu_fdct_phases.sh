# k_fdct phase timers (tools/build_fdct_phases.sh) at 1080p x 32, scene content, plus the plain
# library's kernel time beside it (the timers' own cost).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VF_FDCT_STATS=1 VFILTER_LIB=$PWD/tools/variants/libv_phases.so timeout -k 10 200 python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 5 --cpu-seconds 0 > gpurun_out/ph.log 2>&1 || { echo PH_FAILED; tail -20 gpurun_out/ph.log; exit 1; }
grep "fdct phases" gpurun_out/ph.log | tail -4
rm -rf gpurun_out/prof_ph
VFILTER_LIB=$PWD/tools/variants/libv_phases.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ph -o ks -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 > gpurun_out/ph2.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/ph2.log; exit 1; }
grep -h "k_fdct" $(find gpurun_out/prof_ph -name '*kernel_stats.csv') | cut -c1-200
