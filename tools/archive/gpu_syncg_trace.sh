# Per-dispatch k_syncg durations (kernel trace) on hard 1080p content for G = 4 / 8: which of the
# queued passes costs what.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in ${GS:-4 8}; do
  rm -rf gpurun_out/prof_sgt_$g
  VF_JPEG_SYNC_G=$g timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_sgt_$g -o kt -- python3 tools/jpeg_bench.py --sizes ${SIZE:-1080p} --content ${CONTENT:-hard} --batch 32 --iters 4 --cpu-seconds 0 --resident-only > gpurun_out/sgt_$g.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/sgt_$g.log; exit 1; }
  G=$g python3 - <<'PY'
import csv, glob, os, re
g = os.environ["G"]
f = glob.glob(f"gpurun_out/prof_sgt_{g}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = []
for r in rows:
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
    if "k_syncg" in n or "k_write" in n:
        seq.append((n[:12], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
# print the last 3 batches' sync sequences
out, cur = [], []
for n, d in seq:
    cur.append(f"{n} {d:.1f}")
    if n.startswith("k_write"):
        out.append(cur); cur = []
for b in out[-3:]:
    print("G", g, " | ".join(b))
PY
done
