#!/bin/bash
# k_write occupancy A/B: the DC / chunk-mask stage at 4096 vs 2048 blocks (LDS 41.8 -> 29.6 KB) and
# amdgpu_waves_per_eu(4) (VGPRs 129 -> 81): JPEG GPU parity on the variant, then k_write means.
set -o pipefail
mkdir -p gpurun_out
V=${VARIANTS:-"cur=distributed-video-filter_amd/vfilter/libvfilter_hip.so st2k=tools/exp/libvf_st2k.so st2kw4=tools/exp/libvf_st2kw4.so"}
if [ -n "$PARITY_LIB" ]; then
  VFILTER_LIB=$PARITY_LIB timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_jpeg.py \
      > gpurun_out/writeocc_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/writeocc_pytest.log; exit 1; }
  tail -2 gpurun_out/writeocc_pytest.log
fi
VARIANTS="$V" KERNELS="k_write" SIZES=1080p CONTENT=scene REPS="1 2" bash tools/r5/gpu_kernel_ab.sh || exit 1
mkdir -p gpurun_out/w1080 && mv gpurun_out/prof_kab_* gpurun_out/kab_* gpurun_out/w1080/
VARIANTS="$V" KERNELS="k_write" SIZES=480p CONTENT=scene REPS="1 2" bash tools/r5/gpu_kernel_ab.sh || exit 1
