#!/bin/bash
# Warm-up length sweep on hard 1080p over several content seeds (tools/jpeg_bench.py --seed0).
set -o pipefail
L=distributed-video-filter_amd/vfilter/libvfilter_hip.so
V="auto=$L w2560=$L@VF_JPEG_SYNC_WARM=2560 w3072=$L@VF_JPEG_SYNC_WARM=3072 w4096=$L@VF_JPEG_SYNC_WARM=4096"
for sd in ${SEEDS:-100 200 300}; do
  echo "== seed0 $sd"
  JB_ARGS="--seed0 $sd" VARIANTS="$V" REPS=1 bash tools/r5/gpu_warm_ab.sh > gpurun_out/warm_s$sd.txt 2>&1 || { tail -20 gpurun_out/warm_s$sd.txt; exit 1; }
  grep "sync .* ms, passes" gpurun_out/warm_s$sd.txt
  mkdir -p gpurun_out/ws$sd && mv gpurun_out/prof_kab_* gpurun_out/kab_* gpurun_out/ws$sd/
done
