# Timing ablation: k_spec without the walkers' serial continuations (VF_SPEC_NOSERIAL=1; its outputs are wrong) vs the same tree.
set -o pipefail
SIZES=512sq JB_ARGS="--batch 64 --iters 30" STAGES="huffman_sync" KERNELS="k_spec k_resolve" REPS="1 2" \
  VARIANTS="base=tools/variants/libv_base.so noserial=tools/variants/libv_noserial.so" bash tools/r6/gpu_kernel_ab.sh || exit 1
SIZES=1080p JB_ARGS="--iters 30" STAGES="huffman_sync" KERNELS="k_spec k_resolve" REPS="1" \
  VARIANTS="base=tools/variants/libv_base.so noserial=tools/variants/libv_noserial.so" bash tools/r6/gpu_kernel_ab.sh || exit 1
