# Round 3 iteration: JPEG tests on the working tree, k_fdct/k_idct stats head (HEAD_REF build)
# vs new at 1080p scene, hard content with the speculative sync forced vs auto, and the staged
# drop-in's host timeline at 3 / 6 / 12 pieces.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/r3_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/r3_pytest_jpeg.log
for v in head new; do
  if [ $v = head ]; then export VFILTER_LIB=$PWD/tools/libv_head.so; else unset VFILTER_LIB; fi
  rm -rf gpurun_out/prof_it_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_it_$v -o ks -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 10 --cpu-seconds 0 --out gpurun_out/it_$v.jsonl > gpurun_out/it_$v.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/it_$v.log; exit 1; }
done
unset VFILTER_LIB
python3 - <<'PY'
import csv, glob, re, json
st = {}
for v in ("head", "new"):
    f = glob.glob(f"gpurun_out/prof_it_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
        st.setdefault(n, {})[v] = float(r["AverageNs"]) / 1e3
    for l in open(f"gpurun_out/it_{v}.jsonl"):
        d = json.loads(l); print(v, d['gpu_resident_fps'], d['parity_vs_oracle'], d.get('stages_ms'))
for n in ("k_fdct", "k_idct", "k_color", "k_spec", "k_wglink", "k_resolve"):
    d = st.get(n, {})
    print(f"{n:12s} head {d.get('head', 0):8.1f}  new {d.get('new', 0):8.1f} us")
PY
for mode in auto; do
  VF_JPEG_SYNC=$mode timeout -k 10 200 python3 -u tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 5 --cpu-seconds 0 --content hard > gpurun_out/it_hard_$mode.jsonl 2> gpurun_out/it_hard_$mode.log || { echo HARD_FAILED $mode; tail -20 gpurun_out/it_hard_$mode.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/it_hard_$mode.jsonl').read().splitlines()[-1]); print('hard', '$mode', d['gpu_resident_fps'], d['parity_vs_oracle'], d['stages_ms'])"
done
for np_ in 1 2 3; do
  VF_STAGE_PIECES=$np_ timeout -k 10 120 python -u tools/per_frame_probe.py > gpurun_out/it_pf_$np_.jsonl 2> gpurun_out/it_pf_$np_.log || { echo PF_FAILED; tail -20 gpurun_out/it_pf_$np_.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/it_pf_$np_.jsonl'):
    d=json.loads(l); print('pieces $np_', d['size'], 'dropin', d['dropin_ms'], 'pageable', d['pageable_ms'], 'pinned', d['pinned_ms'])"
done
VF_STAGE_TRACE=1 timeout -k 10 60 python3 - > gpurun_out/it_trace.log 2>&1 <<'PY' || { echo TRACE_FAILED; tail -20 gpurun_out/it_trace.log; exit 1; }
import sys, numpy as np
sys.path[:0] = [".", "distributed-video-filter_amd"]
import vfilter
ctx = vfilter.Context(0, max_frame_bytes=6220800, max_batch=4)
f = np.random.default_rng(0).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
for _ in range(20):
    r = vfilter.bitwise_not(f, ctx=ctx)
assert np.array_equal(r, ~f)
PY
tail -5 gpurun_out/it_trace.log
