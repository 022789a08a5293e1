# k_fdct time split: timing-only ablations (tools/build_fdct_ablations_r3.sh) at 1080p x 32,
# two interleaved rounds; then the per-frame probe on the working tree.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in base noac nolist nofdct noquant nopix; do
  rm -rf gpurun_out/prof_abl
  VFILTER_LIB=$PWD/tools/variants/libv_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_abl -o ks -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 > gpurun_out/abl_$v.log 2>&1 || { echo ABL_FAILED $v; tail -20 gpurun_out/abl_$v.log; exit 1; }
  python3 - "$v" "$rep" <<'PY'
import csv, glob, re, sys
f = glob.glob("gpurun_out/prof_abl/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_fdct" in r["Name"]:
        print(f"rep {sys.argv[2]} {sys.argv[1]:8s} k_fdct {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
done
timeout -k 10 120 python -u tools/per_frame_probe.py > gpurun_out/r3_per_frame.jsonl 2> gpurun_out/r3_per_frame.log || { echo PERFRAME_FAILED; tail -20 gpurun_out/r3_per_frame.log; exit 1; }
cat gpurun_out/r3_per_frame.jsonl
