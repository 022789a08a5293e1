# SQ counters of the JPEG kernels (1080p batch): wave cycles split into active / issue-stall /
# parked, VALU and LDS instruction counts, LDS bank conflicts.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_j
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_j -o pmc -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 2 --cpu-seconds 0 > gpurun_out/pmc_j.log 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc_j.log; exit 1; }
python3 - <<'PY'
import csv, glob, re, collections
f = glob.glob("gpurun_out/pmc_j/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
    acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(n, r["Counter_Name"])] += 1
for n, d in acc.items():
    if d.get("SQ_WAVE_CYCLES", 0) < 1e6: continue
    wc = d["SQ_WAVE_CYCLES"]
    print(f"{n:20s} waves {d['SQ_WAVES']:.0f} wavecyc {wc:.3e} active {d['SQ_ACTIVE_INST_ANY']/wc:.2f} "
          f"issue-stall {d['SQ_WAIT_INST_ANY']/wc:.2f} parked {d['SQ_WAIT_ANY']/wc:.2f} "
          f"valu/wave {d['SQ_INSTS_VALU']/d['SQ_WAVES']:.0f} lds/wave {d['SQ_INSTS_LDS']/d['SQ_WAVES']:.0f} "
          f"ldsconf {d['SQ_LDS_BANK_CONFLICT']:.3e}")
PY
