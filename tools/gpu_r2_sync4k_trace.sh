# per-launch k_sync durations at 4K (pass-based sync): which pass costs what
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_s4k
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_s4k -o s4k -- python3 tools/jpeg_bench.py --sizes 4k --batch 32 --iters 3 --cpu-seconds 0 > gpurun_out/s4k.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/s4k.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_s4k/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = []
for r in rows:
    n = r["Kernel_Name"]
    if any(k in n for k in ("k_sync", "k_write", "k_unstuff_write", "k_idct")):
        seq.append((n.split("(")[0].split("::")[-1], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
for s in seq[-24:]:
    print(f"{s[0]:20s} {s[1]:8.1f}")
PY
