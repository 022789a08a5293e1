# Kernel sums vs the GPU-resident batch time at the small frame sizes (512x512 and 480p, batches of
# 64): how much of a batch is launch gaps between its ~25 kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for sz in 512sq 480p; do
  rm -rf gpurun_out/prof_sk_$sz
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sk_$sz -o k -- python3 tools/jpeg_bench.py --sizes $sz --batch 64 --iters 40 --cpu-seconds 0 --resident-only --out gpurun_out/r6_sk_$sz.jsonl > gpurun_out/r6_sk_$sz.log 2>&1 || { tail -20 gpurun_out/r6_sk_$sz.log; exit 1; }
  python3 - "$sz" <<'PY'
import csv, json, sys, glob
sz = sys.argv[1]
d = [json.loads(l) for l in open(f"gpurun_out/r6_sk_{sz}.jsonl")][-1]
f = glob.glob(f"gpurun_out/prof_sk_{sz}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
# per launch sequence: group by kernel name counts; total kernel ns / number of batches
names = {}
for r in rows:
    names.setdefault(r["Kernel_Name"][:40], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
nb = max(len(v) for v in names.values())
tot = sum(sum(v) for v in names.values())
print(sz, "resident ms/batch", d["gpu_resident_ms_per_batch"], "stages", d.get("stages_ms"))
print(sz, "kernels:", len(names), "max calls", nb, "kernel ns per batch (approx)", round(tot / nb / 1e3, 1), "us")
for k, v in sorted(names.items(), key=lambda kv: -sum(kv[1]))[:30]:
    print("   %-40s calls %5d mean %7.1f us" % (k, len(v), sum(v) / len(v) / 1e3))
PY
done
