# Round 3 A/B/n: JPEG GPU tests on the working tree's library, then per-kernel rocprof stats of
# each library in $LIBS ("name=path ...", "new" = the working tree's) at 1080p x 32, $REPS rounds
# alternating (AB_CONTENT=hard: the noisy q95 set; AB_SIZE: 480p / 1080p / 4k).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${AB_CONTENT:-scene}
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/ab_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/ab_pytest_jpeg.log
for rep in $(seq 1 ${REPS:-2}); do
for nv in ${LIBS:-head=tools/libv_head.so new=}; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ -n "$lib" ]; then export VFILTER_LIB=$PWD/$lib; else unset VFILTER_LIB; fi
  rm -rf gpurun_out/prof_ab_$v gpurun_out/ab_$v.jsonl
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab_$v -o ks -- python3 tools/jpeg_bench.py --sizes ${AB_SIZE:-1080p} --batch 32 --iters 10 --cpu-seconds 0 --content $C --resident-only --out gpurun_out/ab_$v.jsonl > gpurun_out/ab_$v.log 2>&1 || { echo PROF_FAILED $v; tail -30 gpurun_out/ab_$v.log; exit 1; }
done
unset VFILTER_LIB
REP=$rep NAMES="${LIBS:-head=tools/libv_head.so new=}" KERNELS="${KERNELS:-k_fdct k_spec k_wglink k_resolve k_sync k_write k_write4 k_idct}" python3 - <<'PY'
import csv, glob, re, json, os
names = [x.split("=")[0] for x in os.environ["NAMES"].split()]
st = {}
for v in names:
    f = glob.glob(f"gpurun_out/prof_ab_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
        n = re.sub(r"<.*", "", re.sub(r"^void ", "", n))
        st.setdefault(n, {})[v] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]))
    for l in open(f"gpurun_out/ab_{v}.jsonl"):
        d = json.loads(l)
        print("rep", os.environ["REP"], v, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d.get('stages_ms'))
for n in os.environ["KERNELS"].split():
    if n in st:
        print(f"rep {os.environ['REP']} {n:10s} " + "  ".join(f"{v} {st[n].get(v, (0, 0))[0]:8.1f}us x{st[n].get(v, (0, 0))[1]}" for v in names))
PY
done
