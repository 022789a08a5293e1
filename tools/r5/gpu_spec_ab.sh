#!/bin/bash
# Round 5: overlapping k_spec workgroups by one subsequence (k_wglink deleted).
# JPEG GPU tests first (parity), then rocprof kernel stats of the speculative sync for each
# library in VARIANTS (name=path ...; default: this tree against tools/variants/libv_spec_wglink.so,
# the round-5 start), 1080p and 480p scenes, REPS reps; then VF_JPEG_SYNC_STATS diagnostics.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -x -q ${PYK:+-k "$PYK"} --timeout 300 --timeout-method thread \
    > gpurun_out/r5_spec_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r5_spec_pytest.log; exit 1; }
tail -1 gpurun_out/r5_spec_pytest.log
VARIANTS=${VARIANTS:-"new=$PWD/distributed-video-filter_amd/vfilter/libvfilter_hip.so old=$PWD/tools/variants/libv_spec_wglink.so"}
export VARIANTS
for rep in ${REPS:-1 2}; do
for nv in $VARIANTS; do
  v=${nv%%=*}; lib=${nv#*=}
  tag=spec_${v}_$rep
  rm -rf gpurun_out/prof_$tag
  VFILTER_LIB=$lib VF_JPEG_SYNC=spec timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o ks -- \
      python3 tools/jpeg_bench.py --sizes 1080p,480p --batch 32 --iters 10 --cpu-seconds 0 --resident-only \
      --out gpurun_out/$tag.jsonl > gpurun_out/$tag.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/$tag.log; exit 1; }
done
done
for nv in $VARIANTS; do
  v=${nv%%=*}; lib=${nv#*=}
  VFILTER_LIB=$lib VF_JPEG_SYNC=spec VF_JPEG_SYNC_STATS=1 timeout -k 10 120 python3 tools/jpeg_bench.py --sizes 1080p --batch 32 \
      --iters 1 --cpu-seconds 0 --resident-only > gpurun_out/spec_stats_$v.log 2>&1 || { echo STATS_FAILED; tail -30 gpurun_out/spec_stats_$v.log; exit 1; }
  echo "$v: $(grep -m1 'ended explicit' gpurun_out/spec_stats_$v.log)"
done
python3 - <<'PY'
import collections, csv, glob, json, os, re
names = [nv.split("=")[0] for nv in os.environ["VARIANTS"].split()]
for rep in [int(x) for x in os.environ.get("REPS", "1 2").split()]:
    for v in names:
        tag = f"spec_{v}_{rep}"
        for d in [json.loads(l) for l in open(f"gpurun_out/{tag}.jsonl")]:
            print(f"{v} rep {rep} {d.get('size')}: resident {d['gpu_resident_fps']} fps parity {d['parity_vs_oracle']} "
                  f"sync {d['stages_ms']['huffman_sync']} ms")
        f = glob.glob(f"gpurun_out/prof_{tag}/**/*kernel_trace.csv", recursive=True)[0]
        dd = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
            if n in ("k_spec", "k_wglink", "k_resolve", "k_finalize"):
                dd[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        # the first half of each kernel's launches is 1080p, the second 480p
        print("   kernel mean us 1080p | 480p: " + ", ".join(
            f"{k} {sum(x[:len(x)//2])/(len(x)//2):.1f} | {sum(x[len(x)//2:])/(len(x)-len(x)//2):.1f}" for k, x in dd.items()))
PY
