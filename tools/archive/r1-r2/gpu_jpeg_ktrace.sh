# kernel trace of the 1080p JPEG invert (per-dispatch durations, e.g. each sync pass)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_jk
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_jk -o jk -- python3 tools/jpeg_bench.py --sizes ${1:-1080p} --batch 32 --iters 3 --cpu-seconds 0 > gpurun_out/jk.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/jk.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_jk/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
import re
out = []
for r in rows[-60:]:
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("::")[-1][:28]
    out.append(f'{n:28s} {(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3:9.1f} us  grid {r.get("Grid_Size_X","")}x{r.get("Grid_Size_Y","")}  start {int(r["Start_Timestamp"])/1e3:.1f}')
print("\n".join(out))
PY
