# rocprofv3 kernel stats of the JPEG-mode bench (one size); parsed per-kernel summary
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_js
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_js -o js -- python3 tools/jpeg_bench.py --sizes ${1:-1080p} --batch 32 --iters 10 --cpu-seconds 0 > gpurun_out/js.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/js.log; exit 1; }
python3 - <<'PY'
import csv, glob, re
f = glob.glob("gpurun_out/prof_js/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
    print(f"{n:34s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
