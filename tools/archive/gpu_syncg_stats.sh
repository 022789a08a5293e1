# k_syncg counters (tools/build_syncg_stats.sh) on hard 1080p and 4K scenes, G = 4 and 8.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 4 8; do
  for sc in "1080p hard" "4k scene"; do
    set -- $sc
    VF_SYNCG_STATS=1 VF_JPEG_SYNC_G=$g VFILTER_LIB=$PWD/tools/variants/libv_syncg_stats.so timeout -k 10 200 python3 tools/jpeg_bench.py --sizes $1 --content $2 --batch 32 --iters 2 --cpu-seconds 0 --resident-only > gpurun_out/sgs_${g}_$1.log 2>&1 || { echo STATS_FAILED; tail -20 gpurun_out/sgs_${g}_$1.log; exit 1; }
    echo "G $g $1 $2"; grep "\[syncg\]" gpurun_out/sgs_${g}_$1.log | tail -4
  done
done
