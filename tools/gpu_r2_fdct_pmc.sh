# SQ counters of the JPEG kernels (1080p batch): the stall split pass and an instruction-mix pass
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_jpeg_pmc.sh || exit 1
rm -rf gpurun_out/pmc_j2
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_j2 -o pmc -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 2 --cpu-seconds 0 > gpurun_out/pmc_j2.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/pmc_j2.log; exit 1; }
python3 - <<'PY'
import csv, glob, re, collections
f = glob.glob("gpurun_out/pmc_j2/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
    acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
for n, d in acc.items():
    w = d.get("SQ_WAVES", 0)
    if w < 1e4: continue
    print(f"{n:20s} " + " ".join(f"{k[3:]} {v / w:.1f}" for k, v in sorted(d.items()) if k != "SQ_WAVES"))
PY
