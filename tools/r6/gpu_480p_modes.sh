# The 480p JPEG system leg is bimodal run to run (115-120 k or 160-179 k fps): 4 runs, each under a
# rocprofv3 kernel trace (the worker process is traced with its parent), to compare the kernels of a
# slow run with a fast one.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  rm -rf gpurun_out/prof480_$rep
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof480_$rep -o k -- python3 tools/pipeline_bench.py --workers 1 --gpus 1 --jpeg --size 480p --batch 64 --policy pull \
      --frames 98304 > gpurun_out/r6_480m_$rep.json 2> gpurun_out/r6_480m_$rep.err || { echo LEG_FAILED; tail -20 gpurun_out/r6_480m_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6_480m_$rep.json') if l.startswith('{')][-1]); print('rep $rep', d['fps'], 'lat', d['latency_ms_mean'])"
  f=$(find gpurun_out/prof480_$rep -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("   %-28s calls %6s avg %8.1f us  share %.3f" % (r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / tot))
print("   total kernel ms", round(tot / 1e6, 1))
PY
done
