#!/bin/bash
# Round 5: span width / occupancy of the pass-based sync on hard content.
# k_syncg's LDS per workgroup: G=4 50 KB -> 3 workgroups per CU; G=3 40.7 KB -> 4; G=2 32 KB -> 5
# (32-bit relative exits).  Span tests first, then rocprof kernel stats per G, two reps; plus the
# host's CPU / memory facts for DESIGN §7's node budget.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
lscpu > gpurun_out/r5_lscpu.txt 2>&1; head -3 /proc/meminfo >> gpurun_out/r5_lscpu.txt; numactl -H >> gpurun_out/r5_lscpu.txt 2>&1
grep -E "Model name|Socket|NUMA node\(s\)|^CPU\(s\)" gpurun_out/r5_lscpu.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 200 --timeout-method thread -k "span_sync or sync_modes or operating_points" \
    > gpurun_out/r5_syncg_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r5_syncg_pytest.log; exit 1; }
tail -1 gpurun_out/r5_syncg_pytest.log
for rep in 1 2; do
for g in 4 3 2; do
  tag=hard_g${g}_$rep
  rm -rf gpurun_out/prof_$tag
  VF_JPEG_SYNC_G=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o ks -- \
      python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 --resident-only --content hard \
      --out gpurun_out/$tag.jsonl > gpurun_out/$tag.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/$tag.log; exit 1; }
done
done
python3 - <<'PY'
import csv, glob, json, re
for rep in (1, 2):
    for g in (4, 3, 2):
        tag = f"hard_g{g}_{rep}"
        f = glob.glob(f"gpurun_out/prof_{tag}/**/*kernel_stats.csv", recursive=True)[0]
        ks = {re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]: float(r["AverageNs"]) / 1e3
              for r in csv.DictReader(open(f))}
        d = [json.loads(l) for l in open(f"gpurun_out/{tag}.jsonl")][-1]
        print(f"G={g} rep {rep}: resident {d['gpu_resident_fps']} fps parity {d['parity_vs_oracle']} sync {d['stages_ms']['huffman_sync']} ms "
              f"k_syncg avg {ks.get('k_syncg', 0):.1f} us")
PY
