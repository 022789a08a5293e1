# Round 3 JPEG A/B: the JPEG GPU tests on the working tree's library, then per-kernel rocprof
# stats of tools/libv_head.so (HEAD_REF build) vs the working tree at 1080p x 32, scene content
# and hard content (noisy q95), then the per-dispatch PMC pass on the working tree.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/r3_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/r3_pytest_jpeg.log
for content in scene hard; do
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  rm -rf gpurun_out/prof_ks_${v}_$content
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ks_${v}_$content -o ks -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 --content $content --out gpurun_out/ks_${v}_$content.jsonl > gpurun_out/ks_${v}_$content.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/ks_${v}_$content.log; exit 1; }
done
done
unset VFILTER_LIB
python3 - <<'PY'
import csv, glob, re, json
for content in ("scene", "hard"):
    st = {}
    for v in ("head", "new"):
        f = glob.glob(f"gpurun_out/prof_ks_{v}_{content}/**/*kernel_stats.csv", recursive=True)[0]
        for r in csv.DictReader(open(f)):
            n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
            st.setdefault(n, {})[v] = float(r["AverageNs"]) / 1e3
        for l in open(f"gpurun_out/ks_{v}_{content}.jsonl"):
            d = json.loads(l); print(content, v, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d['jpeg_bytes_in_mean'], d.get('stages_ms'))
    for n, d in sorted(st.items(), key=lambda x: -x[1].get("new", 0))[:12]:
        print(f"{content:6s} {n:34s} head {d.get('head', 0):9.1f}  new {d.get('new', 0):9.1f} us")
PY
rm -rf gpurun_out/pmc_b
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_b -o pmc -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 3 --cpu-seconds 0 > gpurun_out/pmc_b.log 2>&1 || { echo PMC_B_FAILED; tail -20 gpurun_out/pmc_b.log; exit 1; }
python3 tools/pmc_issue.py gpurun_out/pmc_b/pmc_counter_collection.csv --durations gpurun_out/prof_ks_new_scene/ks_kernel_stats.csv > gpurun_out/r3_jpeg_issue.json
python3 -c "
import json; d=json.load(open('gpurun_out/r3_jpeg_issue.json'))
for k in ('k_fdct','k_spec','k_idct','k_color','k_write','k_wglink','k_resolve'):
    if k in d: print(k, {x: d[k][x] for x in ('duration_us','valu_per_wave','valu_issue_frac','lds_issue_frac','clock_GHz') if x in d[k]})"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_pytest_parity.log 2>&1 || { echo PYTEST_PARITY_FAILED; tail -40 gpurun_out/r3_pytest_parity.log; exit 1; }
tail -1 gpurun_out/r3_pytest_parity.log
timeout -k 10 120 python -u tools/per_frame_probe.py > gpurun_out/r3_per_frame.jsonl 2> gpurun_out/r3_per_frame.log || { echo PERFRAME_FAILED; tail -20 gpurun_out/r3_per_frame.log; exit 1; }
cat gpurun_out/r3_per_frame.jsonl
