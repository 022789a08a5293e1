// vf_kernels.hip — gfx950 (CDNA4) kernels for the frame filter of
// kylemcdonald/distributed-video-filter: `cv2.bitwise_not(frame)` (inverter.py:41).
//
// The op is dst[i] = ~src[i] over bytes: no reuse, ~1 VALU op per 16 B, so it is bound by
// HBM (2 bytes moved per byte filtered) and LDS / MFMA are deliberately unused.  Design:
//   * 16 B per lane per access (global_load_dwordx4 / global_store_dwordx4): one
//     wave-instruction moves a contiguous, 1 KiB, fully coalesced span;
//   * U = 4 independent 16-B loads per lane in flight before the first store (memory-level
//     parallelism to cover the ~900-cycle HBM miss), chosen by tools/tune_invert.hip over
//     U = 1..8 with and without nontemporal hints (templates in vf_stream.h);
//   * grid-stride over whole tiles of 256 lanes x U vectors; the grid is capped at a
//     multiple of the CU count so each CU holds several workgroups for its whole life;
//   * frames of a batch are packed back to back, so a batch is ONE byte range and ONE
//     launch whatever its frame count or resolution mix;
//   * non-16-B-aligned heads and sub-16-B tails are done bytewise by block 0 inside the
//     same launch, so any pointer / size from the C ABI is legal.
// XCD-aware block remapping (guide T1) buys nothing here: no two workgroups touch the
// same line, so there is no L2 reuse to localise.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vf_internal.h"
#include "vf_stream.h"

namespace vf {

// src and dst misaligned relative to each other (their addresses differ mod 16): no common
// 16-B grid exists, so fall back to coalesced bytewise access (64 B per wave-instruction).
// Only reachable from vf_invert_device with caller pointers at unrelated offsets; the host
// entry points always stage into 16-B-aligned slot buffers.
__global__ __launch_bounds__(kBlock) void invert_bytes_kernel(const uint8_t *__restrict__ src,
                                                              uint8_t *__restrict__ dst,
                                                              uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    dst[i] = (uint8_t)~src[i];
}

// Descriptor-table form: blockIdx.y = frame, blockIdx.x strides within the frame.
__global__ __launch_bounds__(kBlock) void invert_frames_kernel(const uint8_t *const *srcs,
                                                               uint8_t *const *dsts,
                                                               const size_t *nbytes) {
  const uint32_t f = blockIdx.y;
  const uint8_t *s = srcs[f];
  uint8_t *d = dsts[f];
  const uint64_t n = nbytes[f];
  const uint32_t t = threadIdx.x;
  const uint64_t stride16 = (uint64_t)gridDim.x * kBlock;
  if ((((uintptr_t)s | (uintptr_t)d) & 15) == 0) {
    const uint64_t n16 = n >> 4;
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(s);
    u32x4 *d4 = reinterpret_cast<u32x4 *>(d);
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + t; i < n16; i += stride16)
      st16<true>(d4 + i, ~ld16<true>(s4 + i));
    const uint64_t tail0 = n16 << 4;
    if (blockIdx.x == 0 && tail0 + t < n) d[tail0 + t] = (uint8_t)~s[tail0 + t];
  } else {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + t; i < n; i += stride16)
      d[i] = (uint8_t)~s[i];
  }
}

// ---- launchers ----------------------------------------------------------------------

hipError_t launch_invert(const void *dsrc, void *ddst, size_t nbytes, const LaunchCfg &cfg,
                         hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  const uint8_t *s = static_cast<const uint8_t *>(dsrc);
  uint8_t *d = static_cast<uint8_t *>(ddst);
  if ((((uintptr_t)s ^ (uintptr_t)d) & 15) != 0) {
    uint64_t blocks = (nbytes + kBlock - 1) / kBlock;
    if (blocks > (uint64_t)cfg.max_blocks) blocks = (uint64_t)cfg.max_blocks;
    hipLaunchKernelGGL(invert_bytes_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, s,
                       d, (uint64_t)nbytes);
    return hipGetLastError();
  }
  return launch_stream<4, true, true>(s, d, nbytes, cfg.max_blocks, stream);
}

hipError_t launch_invert_frames(const void *const *dsrcs, void *const *ddsts,
                                const size_t *nbytes, int n, size_t total_bytes,
                                const LaunchCfg &cfg, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  // Spread one frame over enough blocks that the whole launch fills the chip.
  const uint64_t per_frame = (total_bytes / (uint64_t)n + 16ull * kBlock - 1) / (16ull * kBlock);
  uint64_t gx = per_frame ? per_frame : 1;
  const uint64_t cap = (uint64_t)cfg.max_blocks / (uint64_t)n + 1;
  if (gx > cap) gx = cap;
  hipLaunchKernelGGL(invert_frames_kernel, dim3((unsigned)gx, (unsigned)n), dim3(kBlock), 0,
                     stream, reinterpret_cast<const uint8_t *const *>(dsrcs),
                     reinterpret_cast<uint8_t *const *>(ddsts), nbytes);
  return hipGetLastError();
}

}  // namespace vf
