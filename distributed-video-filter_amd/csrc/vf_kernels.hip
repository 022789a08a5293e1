// vf_kernels.hip — gfx950 (CDNA4) kernels for the frame filter of
// kylemcdonald/distributed-video-filter: `cv2.bitwise_not(frame)` (inverter.py:41).
//
// The op is dst[i] = ~src[i] over bytes: no reuse, ~1 VALU op per 16 B, so it is bound by
// HBM (2 bytes moved per byte filtered) and LDS / MFMA are deliberately unused.  Design:
//   * 16 B per lane per access (global_load_dwordx4 / global_store_dwordx4): one
//     wave-instruction moves a contiguous, 1 KiB, fully coalesced span;
//   * U independent 16-B loads per lane in flight before the first store (memory-level
//     parallelism to cover the ~900-cycle HBM miss), U chosen by tools/tune_invert.hip;
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

namespace vf {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(u32x4 *p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Body: n16 aligned 16-B vectors at src/dst.  Head/tail: up to 15 bytes each, bytewise.
// CHUNK (tuning variant): block b takes the contiguous tiles [b * tpb, (b + 1) * tpb)
// instead of striding over the grid.
template <int U, bool NTL, bool NTS, bool CHUNK = false>
__global__ __launch_bounds__(kBlock) void invert_stream_kernel(
    const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t n16,
    const uint8_t *__restrict__ hsrc, uint8_t *__restrict__ hdst, uint32_t head,
    const uint8_t *__restrict__ tsrc, uint8_t *__restrict__ tdst, uint32_t tail, uint64_t tpb) {
  constexpr uint64_t TILE = (uint64_t)kBlock * U;
  const uint64_t stride = CHUNK ? TILE : (uint64_t)gridDim.x * TILE;
  const uint32_t t = threadIdx.x;
  uint64_t t0 = (uint64_t)blockIdx.x * (CHUNK ? tpb : 1) * TILE;  // wave-uniform tile start
  if (CHUNK) {
    const uint64_t e = t0 + tpb * TILE;
    n16 = e < n16 ? e : n16;
  }
  for (; t0 + TILE <= n16; t0 += stride) {
    const u32x4 *s = src + t0 + t;
    u32x4 *d = dst + t0 + t;
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld16<NTL>(s + j * kBlock);
#pragma unroll
    for (int j = 0; j < U; ++j) st16<NTS>(d + j * kBlock, ~v[j]);
  }
  if (t0 < n16) {  // the single partial tile, owned by whichever block reaches it
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t i = t0 + (uint64_t)j * kBlock + t;
      if (i < n16) st16<NTS>(dst + i, ~ld16<NTL>(src + i));
    }
  }
  if (blockIdx.x == 0) {
    if (t < head) hdst[t] = (uint8_t)~hsrc[t];
    if (t < tail) tdst[t] = (uint8_t)~tsrc[t];
  }
}

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

const char *variant_name(int v) {
  static const char *names[kVariantCount] = {"u4-nt", "u2-nt", "u8-nt", "u1-nt", "u4-ntl",
                                             "u4-nts", "u4", "u2", "u8", "u1", "u4-nt-chunk",
                                             "u8-nt-chunk"};
  return (v >= 0 && v < kVariantCount) ? names[v] : "?";
}

// Bodies above kSplitBytes are cut into equal sub-launches of at most kChunkBytes, issued
// back to back on the stream.  Measured (profiles/r01_large_buffers.txt, tools/tune_invert
// large): ONE grid-stride launch over 1.6-12.7 GB runs at 5.0-5.6 TB/s, the same bytes as
// 192-256 MiB launches at 6.2-6.3 TB/s (64 MiB: 5.7, the grid is then half empty; 1 GiB:
// 6.0).  Each sub-launch is 1.5-2 grid strides, so workgroups re-align at every launch
// boundary instead of drifting apart over tens of strides.
constexpr uint64_t kSplitBytes = 512ull << 20;
constexpr uint64_t kChunkBytes = 256ull << 20;

template <int U, bool NTL, bool NTS, bool CHUNK = false>
static hipError_t launch_stream(const uint8_t *src, uint8_t *dst, size_t nbytes, int max_blocks,
                                hipStream_t stream) {
  // Split [src, src+n) into head (bytes until 16-B alignment), body (whole vectors) and tail.
  const uint32_t head = (uint32_t)((16 - ((uintptr_t)src & 15)) & 15);
  const uint32_t h = head < nbytes ? head : (uint32_t)nbytes;
  const uint64_t rest = nbytes - h;
  const uint64_t n16 = rest >> 4;
  const uint32_t tail = (uint32_t)(rest & 15);
  constexpr uint64_t TILE = (uint64_t)kBlock * U;  // vectors per tile
  const uint64_t nchunks = (n16 << 4) > kSplitBytes ? ((n16 << 4) + kChunkBytes - 1) / kChunkBytes : 1;
  // whole tiles per chunk; the last chunk takes the remainder (including any partial tile)
  const uint64_t per = nchunks > 1 ? ((n16 + nchunks - 1) / nchunks + TILE - 1) / TILE * TILE : n16;
  const uint8_t *bs = src + h;
  uint8_t *bd = dst + h;
  for (uint64_t c0 = 0, k = 0; k == 0 || c0 < n16; c0 += per, ++k) {
    const uint64_t m = (n16 - c0) < per ? (n16 - c0) : per;
    const bool first = k == 0, last = c0 + m >= n16;
    const uint64_t tiles = (m + TILE - 1) / TILE;
    uint64_t blocks = tiles ? tiles : 1;
    if (blocks > (uint64_t)max_blocks) blocks = (uint64_t)max_blocks;
    const uint64_t tpb = (tiles + blocks - 1) / blocks;  // CHUNK: tiles per block
    if (CHUNK && tpb) blocks = (tiles + tpb - 1) / tpb;
    hipLaunchKernelGGL((invert_stream_kernel<U, NTL, NTS, CHUNK>), dim3((unsigned)blocks), dim3(kBlock), 0,
                       stream, reinterpret_cast<const u32x4 *>(bs) + c0,
                       reinterpret_cast<u32x4 *>(bd) + c0, m, src, dst, first ? h : 0u,
                       bs + (n16 << 4), bd + (n16 << 4), last ? tail : 0u, tpb);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (last) break;
  }
  return hipSuccess;
}

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
  const int mb = cfg.max_blocks;
  switch (cfg.variant) {
    case kVariantU4NT: return launch_stream<4, true, true>(s, d, nbytes, mb, stream);
    case kVariantU2NT: return launch_stream<2, true, true>(s, d, nbytes, mb, stream);
    case kVariantU8NT: return launch_stream<8, true, true>(s, d, nbytes, mb, stream);
    case kVariantU1NT: return launch_stream<1, true, true>(s, d, nbytes, mb, stream);
    case kVariantU4NTL: return launch_stream<4, true, false>(s, d, nbytes, mb, stream);
    case kVariantU4NTS: return launch_stream<4, false, true>(s, d, nbytes, mb, stream);
    case kVariantU4: return launch_stream<4, false, false>(s, d, nbytes, mb, stream);
    case kVariantU2: return launch_stream<2, false, false>(s, d, nbytes, mb, stream);
    case kVariantU8: return launch_stream<8, false, false>(s, d, nbytes, mb, stream);
    case kVariantU1: return launch_stream<1, false, false>(s, d, nbytes, mb, stream);
    case kVariantU4NTChunk: return launch_stream<4, true, true, true>(s, d, nbytes, mb, stream);
    case kVariantU8NTChunk: return launch_stream<8, true, true, true>(s, d, nbytes, mb, stream);
    default: return hipErrorInvalidValue;
  }
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
