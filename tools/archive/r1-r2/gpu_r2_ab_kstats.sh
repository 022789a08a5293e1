# A/B of two library builds (tools/libv_head.so = last commit, in-tree = working tree): the JPEG
# GPU tests on the new build, the JPEG-mode bench twice each, then per-kernel rocprof stats of
# both at one size.   AB_SIZES (default 480p,1080p), KS_SIZE (default 1080p)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
rm -f gpurun_out/ab_*.jsonl
for rep in 1 2; do
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  timeout -k 10 200 python -u tools/jpeg_bench.py --sizes ${AB_SIZES:-480p,1080p} --batch 32 --iters 20 --cpu-seconds 0 --out gpurun_out/ab_$v.jsonl > gpurun_out/ab_$v.log 2>&1 || { echo JPEG_BENCH_FAILED $v; tail -30 gpurun_out/ab_$v.log; exit 1; }
done
done
python3 -c "
import json
for v in ('head','new'):
    for l in open('gpurun_out/ab_%s.jsonl'%v):
        d=json.loads(l); print(v, d['size'], d['gpu_resident_fps'], 'h2h', d.get('host_to_host_fps'), d.get('host_to_host_2threads_fps'), d['parity_vs_oracle'], d.get('stages_ms'))"
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  rm -rf gpurun_out/prof_ks_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ks_$v -o ks -- python3 tools/jpeg_bench.py --sizes ${KS_SIZE:-1080p} --batch 32 --iters 10 --cpu-seconds 0 > gpurun_out/ks_$v.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/ks_$v.log; exit 1; }
done
unset VFILTER_LIB
python3 - <<'PY'
import csv, glob, re
st = {}
for v in ("head", "new"):
    f = glob.glob(f"gpurun_out/prof_ks_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
        st.setdefault(n, {})[v] = float(r["AverageNs"]) / 1e3
for n, d in sorted(st.items(), key=lambda x: -x[1].get("new", 0)):
    print(f"{n:34s} head {d.get('head', 0):9.1f}  new {d.get('new', 0):9.1f} us")
PY
