#!/bin/bash
# SpanLaneR (LSB-first span-sync lane): the sync parity tests, then hard 1080p timing with the
# lane on and off (VF_JPEG_SYNC_LSB), interleaved, 2 reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 200 --timeout-method thread \
    -k "span_sync or sync_modes or operating_points or golden" > gpurun_out/r6_syncr_pytest.log 2>&1 \
    || { echo PYTEST_FAILED; tail -40 gpurun_out/r6_syncr_pytest.log; exit 1; }
tail -2 gpurun_out/r6_syncr_pytest.log
L=distributed-video-filter_amd/vfilter/libvfilter_hip.so
KERNELS="k_syncg k_write4" CONTENT=hard STAGES='huffman_sync huffman_write' REPS='1 2' \
  VARIANTS="msb=$L@VF_JPEG_SYNC_LSB=0 lsb=$L" bash tools/r6/gpu_kernel_ab.sh
KERNELS="k_syncg" SIZES=4k CONTENT=scene STAGES='huffman_sync' REPS='1' \
  VARIANTS="msb4k=$L@VF_JPEG_SYNC_LSB=0 lsb4k=$L" bash tools/r6/gpu_kernel_ab.sh
