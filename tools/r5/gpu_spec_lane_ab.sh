#!/bin/bash
# k_spec on SpanLane (aligned byte-swapped staged words, no bit buffer) vs SyncLane: JPEG GPU
# parity, then k_spec means on 1080p and 480p scenes (tools/r5/gpu_kernel_ab.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_jpeg.py \
    > gpurun_out/speclane_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/speclane_pytest.log; exit 1; }
tail -2 gpurun_out/speclane_pytest.log
V=${VARIANTS:-"base=tools/exp/libvf_base.so new=distributed-video-filter_amd/vfilter/libvfilter_hip.so"}
VARIANTS="$V" KERNELS="k_spec k_resolve k_finalize" SIZES=1080p CONTENT=scene REPS="1 2 3" bash tools/r5/gpu_kernel_ab.sh || exit 1
mkdir -p gpurun_out/s1080 && mv gpurun_out/prof_kab_* gpurun_out/kab_* gpurun_out/s1080/
VARIANTS="$V" KERNELS="k_spec k_resolve k_finalize" SIZES=480p CONTENT=scene REPS="1 2" bash tools/r5/gpu_kernel_ab.sh || exit 1
