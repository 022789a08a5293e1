# Round-3 before / after: the library at the round's first refresh commit (7f820b8,
# tools/variants/libv_r3start.so) against the working tree, resident-only JPEG stages and kernel
# stats at 480p / 1080p / 4K scenes and 1080p hard content, 2 alternating reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="start=tools/variants/libv_r3start.so end=" KERNELS="k_fdct k_spec k_wglink k_resolve k_sync k_syncg k_write k_write4 k_idct k_color k_pack" REPS=2 AB_SIZE=1080p bash tools/r3/gpu_abn.sh || exit 1
for sz in 480p 4k; do
  LIBS="start=tools/variants/libv_r3start.so end=" KERNELS="k_fdct k_spec k_sync k_syncg k_write k_write4" REPS=1 AB_SIZE=$sz bash tools/r3/gpu_abn.sh | grep -v passed || exit 1
done
LIBS="start=tools/variants/libv_r3start.so end=" KERNELS="k_fdct k_sync k_syncg k_write4" REPS=1 AB_SIZE=1080p AB_CONTENT=hard bash tools/r3/gpu_abn.sh | grep -v passed || exit 1
