# Round 3 A/B: JPEG GPU tests on the working tree's library, then per-kernel rocprof stats of
# tools/libv_head.so (tools/build_head_lib.sh: HEAD or $HEAD_REF) vs the working tree at 1080p x 32
# (scene content; AB_CONTENT=hard for the noisy q95 set), two alternating repetitions.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${AB_CONTENT:-scene}
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/ab_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/ab_pytest_jpeg.log
for rep in 1 2; do
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  rm -rf gpurun_out/prof_ab_$v gpurun_out/ab_$v.jsonl
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab_$v -o ks -- python3 tools/jpeg_bench.py --sizes ${AB_SIZE:-1080p} --batch 32 --iters 10 --cpu-seconds 0 --content $C --out gpurun_out/ab_$v.jsonl > gpurun_out/ab_$v.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/ab_$v.log; exit 1; }
done
unset VFILTER_LIB
REP=$rep python3 - <<'PY'
import csv, glob, re, json, os
st = {}
for v in ("head", "new"):
    f = glob.glob(f"gpurun_out/prof_ab_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
        n = re.sub(r"^void ", "", n)
        n = re.sub(r"<.*", "", n)
        st.setdefault(n, {})[v] = float(r["AverageNs"]) / 1e3
    for l in open(f"gpurun_out/ab_{v}.jsonl"):
        d = json.loads(l); print("rep", os.environ["REP"], v, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d.get('stages_ms'))
for n, d in sorted(st.items(), key=lambda x: -x[1].get("new", 0))[:12]:
    print(f"rep {os.environ['REP']} {n:28s} head {d.get('head', 0):9.1f}  new {d.get('new', 0):9.1f} us")
PY
done
