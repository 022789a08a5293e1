# k_spec's phases (VF_SPEC_PHASES build, tools/build_variants.sh phases:"-DVF_SPEC_PHASES=1"):
# wall ticks summed over workgroups to the end of part A (trajectory decodes), of part B (links),
# and of the walkers' serial continuations, at 512x512 x 64 and 1080p x 32.
set -o pipefail
mkdir -p gpurun_out
for sz in 512sq 1080p; do
  b=64; [ $sz = 1080p ] && b=32
  VF_JPEG_SYNC_STATS=1 VFILTER_LIB=tools/variants/libv_phases.so timeout -k 10 120 python3 tools/jpeg_bench.py --sizes $sz --batch $b --iters 3 --cpu-seconds 0 --resident-only --out gpurun_out/r6_ph_$sz.jsonl > gpurun_out/r6_ph_$sz.log 2>&1 || { tail -20 gpurun_out/r6_ph_$sz.log; exit 1; }
  echo "== $sz"; grep "k_spec phases" gpurun_out/r6_ph_$sz.log | tail -2; grep "spec: unres" gpurun_out/r6_ph_$sz.log | tail -1
done
