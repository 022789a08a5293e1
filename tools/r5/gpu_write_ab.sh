#!/bin/bash
# Write-pass reader A/B (write_span on aligned byte-swapped staged words vs the refilled bit buffer):
# JPEG GPU parity, then k_write on 1080p scenes and k_write4 on hard 1080p (tools/r5/gpu_kernel_ab.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_jpeg.py \
    > gpurun_out/write_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/write_pytest.log; exit 1; }
tail -2 gpurun_out/write_pytest.log
V=${VARIANTS:-"base=tools/exp/libvf_base.so new=distributed-video-filter_amd/vfilter/libvfilter_hip.so"}
VARIANTS="$V" KERNELS="k_write k_write4" SIZES=1080p CONTENT=scene REPS="1 2" bash tools/r5/gpu_kernel_ab.sh || exit 1
mkdir -p gpurun_out/wscene && mv gpurun_out/prof_kab_* gpurun_out/kab_* gpurun_out/wscene/
VARIANTS="$V" KERNELS="k_write k_write4" SIZES=1080p CONTENT=hard REPS="1 2" bash tools/r5/gpu_kernel_ab.sh || exit 1
