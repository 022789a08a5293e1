# kernel durations of the drop-in's gated launch vs the pinned zero-copy launch at 1080p
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in gated pinned; do
  rm -rf gpurun_out/prof_g_$m
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g_$m -o g -- python3 tools/r6/gated_ab.py 10 10 1080p $m > gpurun_out/r6_gated_prof_$m.log 2>&1 || { tail -20 gpurun_out/r6_gated_prof_$m.log; exit 1; }
  cat gpurun_out/r6_gated_prof_$m.log | grep size
  cat "$(find gpurun_out/prof_g_$m -name '*kernel_stats.csv' | head -1)"
done
