# Round-4 JPEG A/B between two builds of the library (Makefile `exp` target): rocprof kernel
# stats of tools/jpeg_bench.py --resident-only at 1080p x 32 with VFILTER_LIB=A and =B,
# alternating twice, per content; prints per-kernel averages and resident fps.  Timing only:
# an experiment library may produce wrong output (parity_vs_oracle says so).
#   bash tools/r4/gpu_jpeg_lib_ab.sh LIB_A LIB_B [scene,hard] [size]
set -o pipefail
A=$1; B=$2; CONTENTS=${3:-scene}; SIZE=${4:-1080p}
mkdir -p gpurun_out
export TMPDIR=/tmp
for content in ${CONTENTS//,/ }; do
for rep in 1 2; do
for v in A B; do
  lib=$A; [ $v = B ] && lib=$B
  tag=${content}_${v}_$rep
  rm -rf gpurun_out/prof_lab_$tag
  VFILTER_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lab_$tag -o ks -- python3 tools/jpeg_bench.py --sizes $SIZE --batch 32 --iters 10 --cpu-seconds 0 --resident-only --content $content --out gpurun_out/lab_$tag.jsonl > gpurun_out/lab_$tag.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/lab_$tag.log; exit 1; }
done
done
done
python3 - "$A" "$B" "$CONTENTS" <<'PY'
import csv, glob, re, json, sys
A, B, contents = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
for content in contents:
    st = {}
    for rep in (1, 2):
        for v in ("A", "B"):
            tag = f"{content}_{v}_{rep}"
            f = glob.glob(f"gpurun_out/prof_lab_{tag}/**/*kernel_stats.csv", recursive=True)[0]
            for r in csv.DictReader(open(f)):
                n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
                st.setdefault(n, {}).setdefault(v, []).append(float(r["AverageNs"]) / 1e3)
            for l in open(f"gpurun_out/lab_{tag}.jsonl"):
                d = json.loads(l)
                print(content, v, rep, d['size'], d['gpu_resident_fps'], d['parity_vs_oracle'], d.get('stages_ms'))
    print(f"A = {A}   B = {B}")
    for n, d in sorted(st.items(), key=lambda x: -max(x[1].get("B", [0]) + x[1].get("A", [0])))[:14]:
        print(f"{content:6s} {n:34s} A: {' '.join(f'{x:7.1f}' for x in d.get('A', []))}   B: {' '.join(f'{x:7.1f}' for x in d.get('B', []))} us")
PY
