# k_fdct joint 4:2:2 pass 1: JPEG GPU tests, then k_fdct head vs new at 1080p scene and hard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/r3_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/r3_pytest_jpeg.log
for content in scene hard; do
for rep in 1 2; do
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  rm -rf gpurun_out/prof_j
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_j -o ks -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 --content $content --out gpurun_out/j_$v.jsonl > gpurun_out/j_$v.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/j_$v.log; exit 1; }
  python3 - "$v" "$rep" "$content" <<'PY'
import csv, glob, re, sys, json
f = glob.glob("gpurun_out/prof_j/**/*kernel_stats.csv", recursive=True)[0]
ks = {re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
d = json.loads(open(f"gpurun_out/j_{sys.argv[1]}.jsonl").read().splitlines()[-1])
print(sys.argv[3], "rep", sys.argv[2], sys.argv[1], "fps", d["gpu_resident_fps"], "parity", d["parity_vs_oracle"], "k_fdct %.1f k_spec %.1f k_wglink %.1f k_resolve %.1f" % (ks.get("k_fdct", 0), ks.get("k_spec", 0), ks.get("k_wglink", 0), ks.get("k_resolve", 0)), d["stages_ms"])
PY
done
done
done
