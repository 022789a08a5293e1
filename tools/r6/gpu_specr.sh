#!/bin/bash
# SpanLaneRT in k_spec (and k_syncg): the JPEG parity suite, then scene batches with the LSB-first
# lanes on / off (VF_JPEG_SYNC_LSB), 1080p and 480p, interleaved, 2 reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r6_specr_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r6_specr_pytest.log; exit 1; }
tail -2 gpurun_out/r6_specr_pytest.log
L=distributed-video-filter_amd/vfilter/libvfilter_hip.so
KERNELS="k_spec k_resolve" CONTENT=scene STAGES='huffman_sync' REPS='1 2' \
  VARIANTS="msb=$L@VF_JPEG_SYNC_LSB=0 lsb=$L" bash tools/r6/gpu_kernel_ab.sh
KERNELS="k_spec" SIZES=480p CONTENT=scene STAGES='huffman_sync' REPS='1' \
  VARIANTS="msb480=$L@VF_JPEG_SYNC_LSB=0 lsb480=$L" bash tools/r6/gpu_kernel_ab.sh
