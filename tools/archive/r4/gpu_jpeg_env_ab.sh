# Round-4 JPEG A/B by environment switch: the JPEG GPU tests, then rocprof kernel stats of
# tools/jpeg_bench.py --resident-only at 1080p x 32 with VAR=A and VAR=B, alternating twice,
# on scene (and optionally hard) content; prints per-kernel averages and resident fps.
#   bash tools/r4/gpu_jpeg_env_ab.sh VF_JPEG_FUSE_IDCT 0 1 [scene,hard] [size]
set -o pipefail
VAR=$1; A=$2; B=$3; CONTENTS=${4:-scene}; SIZE=${5:-1080p}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest_jpeg.log 2>&1 || { echo PYTEST_JPEG_FAILED; tail -40 gpurun_out/ab_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/ab_pytest_jpeg.log
fi
for content in ${CONTENTS//,/ }; do
for rep in 1 2; do
for v in $A $B; do
  tag=${content}_${v}_$rep
  rm -rf gpurun_out/prof_ab_$tag
  env $VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab_$tag -o ks -- python3 tools/jpeg_bench.py --sizes $SIZE --batch 32 --iters 10 --cpu-seconds 0 --resident-only --content $content --out gpurun_out/ab_$tag.jsonl > gpurun_out/ab_$tag.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/ab_$tag.log; exit 1; }
done
done
done
python3 - "$VAR" "$A" "$B" "$CONTENTS" <<'PY'
import csv, glob, re, json, sys
var, A, B, contents = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4].split(",")
for content in contents:
    st = {}
    for rep in (1, 2):
        for v in (A, B):
            tag = f"{content}_{v}_{rep}"
            f = glob.glob(f"gpurun_out/prof_ab_{tag}/**/*kernel_stats.csv", recursive=True)[0]
            for r in csv.DictReader(open(f)):
                n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
                st.setdefault(n, {}).setdefault(v, []).append(float(r["AverageNs"]) / 1e3)
            for l in open(f"gpurun_out/ab_{tag}.jsonl"):
                d = json.loads(l)
                print(content, f"{var}={v}", rep, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d.get('stages_ms'))
    for n, d in sorted(st.items(), key=lambda x: -max(x[1].get(B, [0]) + x[1].get(A, [0])))[:14]:
        print(f"{content:6s} {n:34s} {var}={A}: {' '.join(f'{x:7.1f}' for x in d.get(A, []))}   {var}={B}: {' '.join(f'{x:7.1f}' for x in d.get(B, []))} us")
PY
