#!/bin/bash
# Per-kernel timing A/B over libraries (VARIANTS="name=path[@VAR=VAL,...] ..."), rocprofv3 kernel trace of
# tools/jpeg_bench.py (SIZES, CONTENT, resident only, JB_ARGS extra arguments), REPS reps, means of the kernels in KERNELS.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export STAGES=${STAGES:-"color_invert fdct_huffman"} VARIANTS KERNELS=${KERNELS:-"k_idct_color422 k_fdct"} SIZES=${SIZES:-1080p} CONTENT=${CONTENT:-scene} REPS=${REPS:-"1 2"}
for rep in $REPS; do
for nv in $VARIANTS; do
  v=${nv%%=*}; lib=${nv#*=}
  envs=""; case "$lib" in *@*) envs=${lib#*@}; lib=${lib%%@*};; esac  # name=path@VAR=VAL,VAR=VAL
  tag=kab_${v}_$rep
  rm -rf gpurun_out/prof_$tag
  env ${envs//,/ } VFILTER_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o ks -- \
      python3 tools/jpeg_bench.py --sizes $SIZES --batch 32 --iters 10 --cpu-seconds 0 --resident-only --content $CONTENT \
      $JB_ARGS --out gpurun_out/$tag.jsonl > gpurun_out/$tag.log 2>&1 || { echo PROF_FAILED $tag; tail -30 gpurun_out/$tag.log; exit 1; }
done
done
python3 - <<'PY'
import collections, csv, glob, json, os, re
names = [nv.split("=")[0] for nv in os.environ["VARIANTS"].split()]
kern = os.environ["KERNELS"].split()
for rep in os.environ["REPS"].split():
    for v in names:
        tag = f"kab_{v}_{rep}"
        ds = [json.loads(l) for l in open(f"gpurun_out/{tag}.jsonl")]
        f = glob.glob(f"gpurun_out/prof_{tag}/**/*kernel_trace.csv", recursive=True)[0]
        dd = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            n = re.sub(r"\(.*", "", re.sub(r"<[^()]*>", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))).split("::")[-1]
            if n in kern:
                dd[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print(f"{v:10s} rep {rep}: " + "; ".join(f"{d.get('size')} resident {d['gpu_resident_fps']} parity {d['parity_vs_oracle']} "
              f"stages {json.dumps({k: d['stages_ms'][k] for k in os.environ.get('STAGES', 'color_invert fdct_huffman').split()})}" for d in ds)
              + " | " + ", ".join(f"{k} {sum(x)/len(x):.1f} us (n={len(x)})" for k, x in dd.items()))
PY
