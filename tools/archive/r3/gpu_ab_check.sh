# Round 3: JPEG GPU tests on the working tree's library (24-bit DCT multiplies), the whole GPU
# suite and smoke, the per-kernel rocprof stats of head (tools/libv_head.so = last commit) vs
# the working tree at 1080p x 32, then one per-dispatch PMC pass (instruction counts, busy
# cycles, GRBM clock) with the kernel trace beside it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/r3_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/r3_pytest_jpeg.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -60 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3_pytest_gpu.log
grep -E "batch4096|async_in_flight|size_limit" gpurun_out/r3_pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  rm -rf gpurun_out/prof_ks_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ks_$v -o ks -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 --out gpurun_out/ks_$v.jsonl > gpurun_out/ks_$v.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/ks_$v.log; exit 1; }
done
unset VFILTER_LIB
python3 - <<'PY'
import csv, glob, re, json
st = {}
for v in ("head", "new"):
    f = glob.glob(f"gpurun_out/prof_ks_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
        st.setdefault(n, {})[v] = float(r["AverageNs"]) / 1e3
    for l in open(f"gpurun_out/ks_{v}.jsonl"):
        d = json.loads(l); print(v, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d.get('stages_ms'))
for n, d in sorted(st.items(), key=lambda x: -x[1].get("new", 0))[:14]:
    print(f"{n:34s} head {d.get('head', 0):9.1f}  new {d.get('new', 0):9.1f} us")
PY
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r3_counters.txt 2>&1 || echo LIST_FAILED
rm -rf gpurun_out/pmc_a
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_a -o pmc -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 3 --cpu-seconds 0 > gpurun_out/pmc_a.log 2>&1 || { echo PMC_A_FAILED; tail -20 gpurun_out/pmc_a.log; exit 1; }
ls gpurun_out/pmc_a/*/
timeout -k 10 120 python -u tools/per_frame_probe.py > gpurun_out/r3_per_frame.jsonl 2> gpurun_out/r3_per_frame.log || { echo PERFRAME_FAILED; tail -20 gpurun_out/r3_per_frame.log; exit 1; }
cat gpurun_out/r3_per_frame.jsonl
timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --size 4k --batch 16 --frames 256 --policy shard --producer copy > gpurun_out/r3_pipe_4k.jsonl 2> gpurun_out/r3_pipe_4k.log || { echo PIPE4K_FAILED; tail -20 gpurun_out/r3_pipe_4k.log; exit 1; }
cut -c1-700 gpurun_out/r3_pipe_4k.jsonl
timeout -k 10 200 python -u tools/pipeline_bench.py --workers 1 --jpeg --content hard --size 1080p --batch 32 --frames 1024 --policy pull > gpurun_out/r3_pipe_jpeg_hard.jsonl 2> gpurun_out/r3_pipe_jpeg_hard.log || { echo PIPEJH_FAILED; tail -20 gpurun_out/r3_pipe_jpeg_hard.log; exit 1; }
cut -c1-700 gpurun_out/r3_pipe_jpeg_hard.jsonl
