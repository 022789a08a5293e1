set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_jpeg.py > gpurun_out/r6_scan_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_scan_tests.log; exit 1; }
tail -1 gpurun_out/r6_scan_tests.log
for sz in 512sq 1080p; do
  b=64; [ $sz = 1080p ] && b=32
  SIZES=$sz JB_ARGS="--batch $b --iters 30" STAGES="unstuff huffman_sync fdct_huffman stuffing" KERNELS="seg_apply seg_tile_sum" REPS="1 2" \
    VARIANTS="head=tools/libv_head.so tree=distributed-video-filter_amd/vfilter/libvfilter_hip.so" bash tools/r6/gpu_kernel_ab.sh || exit 1
done
