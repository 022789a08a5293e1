#!/bin/bash
# k_idct_color422 / k_idct: the range limit folded into the row pass, dequantisation at the
# coefficient scatter; JPEG parity suite, then the working tree against the last commit
# (tools/libv_head.so), 1080p scenes, interleaved, 2 reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jpeg.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r6_idct_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r6_idct_pytest.log; exit 1; }
tail -2 gpurun_out/r6_idct_pytest.log
L=distributed-video-filter_amd/vfilter/libvfilter_hip.so
KERNELS="k_idct_color422 k_fdct" CONTENT=scene STAGES='color_invert fdct_huffman' REPS='1 2' \
  VARIANTS="head=tools/libv_head.so tree=$L" bash tools/r6/gpu_kernel_ab.sh
