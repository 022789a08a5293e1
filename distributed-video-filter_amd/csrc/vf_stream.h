// vf_stream.h — the grid-stride streaming invert kernel and its launcher, as templates over
// the tuning parameters.  The library instantiates the one tools/tune_invert.hip measured
// fastest on MI355X (U = 4 independent 16-B loads per lane, nontemporal loads and stores:
// profiles/r01_tune_sweep{1,2,3_chunk}.txt); the tuning tool instantiates the others.
// Not installed.
#pragma once
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
// CHUNK (tools/tune_invert.hip only): block b takes the contiguous tiles [b * tpb, (b + 1) * tpb)
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

// Bodies above kSplitBytes are cut into equal sub-launches of at most kChunkBytes, issued
// back to back on the stream.  Measured (profiles/r01_large_buffers.txt, tools/tune_invert
// large): ONE grid-stride launch over 1.6-12.7 GB runs at 5.0-5.6 TB/s, the same bytes as
// 192-256 MiB launches at 6.2-6.3 TB/s (64 MiB: 5.7, the grid is then half empty; 1 GiB:
// 6.0).  Each sub-launch is 1.5-2 grid strides, so workgroups re-align at every launch
// boundary instead of drifting apart over tens of strides.
constexpr uint64_t kSplitBytes = 512ull << 20;
constexpr uint64_t kChunkBytes = 256ull << 20;

template <int U, bool NTL, bool NTS, bool CHUNK = false>
inline hipError_t launch_stream(const uint8_t *src, uint8_t *dst, size_t nbytes, int max_blocks,
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

}  // namespace vf
