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

#include <algorithm>
#include <stdint.h>

#include "vf_internal.h"
#include "vf_stream.h"

namespace vf {

// ---- src and dst at different offsets mod 16 ------------------------------------------------
// (caller views at unrelated offsets, or frames packed at odd offsets).  No common 16-B grid
// exists, so the kernel keeps the STORES aligned: dst's head bytes go bytewise, and output
// vector i of the body is the 16 source bytes at delta = 4Q + r bytes into the aligned source
// vectors A_i, A_i+1.  Each lane loads both (two fully coalesced wave-instructions; the second
// overlaps the first by all but one 16-B vector per wave, so HBM sees each byte once) and
// funnel-shifts with v_alignbyte_b32.  Q is a template parameter (uniform register picks), r a
// run-time byte shift.  Reading A_0 and A_n16 touches up to 15 bytes outside the source range,
// always inside the 16-B vectors (hence pages) that hold its first and last bytes.
template <int Q>
__device__ __forceinline__ u32x4 shift16(u32x4 a, u32x4 b, uint32_t r) {
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(w[Q + 1], w[Q + 0], r);
  o.y = __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], r);
  o.z = __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], r);
  o.w = __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], r);
  return o;
}

// body vectors [b0, n16) of one range, U per lane per tile, grid-strided by `stride` vectors
template <int Q, int U>
__device__ __forceinline__ void shift_body(const u32x4 *__restrict__ sa, u32x4 *__restrict__ d, uint64_t n16,
                                           uint32_t r, uint64_t b0, uint64_t stride) {
  constexpr uint64_t TILE = (uint64_t)kBlock * U;
  const uint32_t t = threadIdx.x;
  uint64_t t0 = b0;
  for (; t0 + TILE <= n16; t0 += stride) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      a[j] = ld16<true>(sa + t0 + j * kBlock + t);
      b[j] = ld16<false>(sa + t0 + j * kBlock + t + 1);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) st16<true>(d + t0 + j * kBlock + t, ~shift16<Q>(a[j], b[j], r));
  }
  if (t0 < n16) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t i = t0 + (uint64_t)j * kBlock + t;
      if (i < n16) st16<true>(d + i, ~shift16<Q>(ld16<true>(sa + i), ld16<false>(sa + i + 1), r));
    }
  }
}

template <int Q>
__global__ __launch_bounds__(kBlock) void invert_shift_kernel(
    const u32x4 *__restrict__ sa, u32x4 *__restrict__ d, uint64_t n16, uint32_t r,
    const uint8_t *__restrict__ hsrc, uint8_t *__restrict__ hdst, uint32_t head,
    const uint8_t *__restrict__ tsrc, uint8_t *__restrict__ tdst, uint32_t tail) {
  shift_body<Q, 4>(sa, d, n16, r, (uint64_t)blockIdx.x * kBlock * 4, (uint64_t)gridDim.x * kBlock * 4);
  if (blockIdx.x == 0) {
    const uint32_t t = threadIdx.x;
    if (t < head) hdst[t] = (uint8_t)~hsrc[t];
    if (t < tail) tdst[t] = (uint8_t)~tsrc[t];
  }
}

// aligned body vectors [b0, n16), U per lane per tile (the stream kernel's loop, per frame)
template <int U>
__device__ __forceinline__ void stream_body(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint64_t n16,
                                            uint64_t b0, uint64_t stride) {
  constexpr uint64_t TILE = (uint64_t)kBlock * U;
  const uint32_t t = threadIdx.x;
  uint64_t t0 = b0;
  for (; t0 + TILE <= n16; t0 += stride) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld16<true>(s + t0 + j * kBlock + t);
#pragma unroll
    for (int j = 0; j < U; ++j) st16<true>(d + t0 + j * kBlock + t, ~v[j]);
  }
  if (t0 < n16) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t i = t0 + (uint64_t)j * kBlock + t;
      if (i < n16) st16<true>(d + i, ~ld16<true>(s + i));
    }
  }
}

// One range [s, s + n) of a multi-range launch: blockIdx.x strides within it, U vectors per lane
// per tile; the aligned or the shifting path by the range's own offsets.
template <int U>
__device__ __forceinline__ void invert_range(const uint8_t *s, uint8_t *d, uint64_t n) {
  const uint32_t t = threadIdx.x;
  const uint32_t h = (uint32_t)min((uint64_t)((16 - ((uintptr_t)d & 15)) & 15), n);  // dst head bytes
  const uint64_t n16 = (n - h) >> 4;
  const uint64_t body = n16 << 4;
  if (blockIdx.x == 0) {
    if (t < h) d[t] = (uint8_t)~s[t];
    const uint64_t tail0 = h + body;
    if (tail0 + t < n) d[tail0 + t] = (uint8_t)~s[tail0 + t];
  }
  if (!n16) return;
  const uint64_t b0 = (uint64_t)blockIdx.x * kBlock * U, stride = (uint64_t)gridDim.x * kBlock * U;
  u32x4 *d4 = reinterpret_cast<u32x4 *>(d + h);
  const uintptr_t sb = (uintptr_t)(s + h);
  const uint32_t delta = (uint32_t)(sb & 15);
  const u32x4 *sa = reinterpret_cast<const u32x4 *>(sb - delta);
  switch (delta >> 2) {  // uniform per workgroup
    case 0:
      if (delta == 0) stream_body<U>(sa, d4, n16, b0, stride);
      else shift_body<0, U>(sa, d4, n16, delta & 3, b0, stride);
      break;
    case 1: shift_body<1, U>(sa, d4, n16, delta & 3, b0, stride); break;
    case 2: shift_body<2, U>(sa, d4, n16, delta & 3, b0, stride); break;
    default: shift_body<3, U>(sa, d4, n16, delta & 3, b0, stride); break;
  }
}

// Descriptor-table form (device memory): blockIdx.y = frame, U = 4.
__global__ __launch_bounds__(kBlock) void invert_frames_kernel(const uint8_t *const *srcs,
                                                               uint8_t *const *dsts,
                                                               const size_t *nbytes) {
  const uint32_t f = blockIdx.y;
  invert_range<4>(srcs[f], dsts[f], nbytes[f]);
}

// Page-locked host ranges in place (zero-copy): the kernel reads the caller's source over PCIe
// and writes the caller's destination over PCIe, so each byte crosses the link once each way
// with no HBM staging, no chunk ring and no host step between the two directions.  Measured
// (tools/zerocopy_probe.hip, profiles/r02_zerocopy_probe.jsonl): one launch over 1080p x 32
// moves 48.4-48.5 GB/s each way, equal to two SDMA copies running at once (48.5), with
// 96-128 workgroups and one 16-B vector per lane in flight (more waves only queue behind the
// link: 44-45 GB/s at 384).  The descriptors travel in the kernel arguments (<= kMappedMax
// ranges per launch), so nothing is uploaded first.  Work is split in 4-KiB tiles (256 lanes
// x 16 B) numbered across all ranges, and the grid strides over the tile numbers: ranges of
// different sizes (a 480p / 1080p / 4K batch) get workgroups in proportion to their bytes,
// so the link stays busy until the last byte instead of waiting on the 4K frames' share.
__global__ __launch_bounds__(kBlock) void invert_mapped_kernel(MappedBatch b, uint32_t nranges) {
  const uint32_t total = b.tile0[nranges];
  const uint32_t t = threadIdx.x;
  uint32_t k = 0;
  for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
    while (tile >= b.tile0[k + 1]) ++k;  // uniform: the grid's tiles only move forward
    const uint8_t *s = b.src[k];
    uint8_t *d = b.dst[k];
    const uint64_t n = b.n[k];
    const uint32_t h = (uint32_t)min((uint64_t)((16 - ((uintptr_t)d & 15)) & 15), n);  // dst head bytes
    const uint64_t n16 = (n - h) >> 4;
    const uint32_t lt = tile - b.tile0[k];
    if (lt == 0) {  // the range's first tile also does its head and tail bytes
      if (t < h) d[t] = (uint8_t)~s[t];
      const uint64_t tail0 = h + (n16 << 4);
      if (tail0 + t < n) d[tail0 + t] = (uint8_t)~s[tail0 + t];
    }
    const uint64_t i = (uint64_t)lt * kBlock + t;
    if (i >= n16) continue;
    u32x4 *d4 = reinterpret_cast<u32x4 *>(d + h);
    const uintptr_t sb = (uintptr_t)(s + h);
    const uint32_t delta = (uint32_t)(sb & 15), r = delta & 3;
    const u32x4 *sa = reinterpret_cast<const u32x4 *>(sb - delta);
    switch (delta >> 2) {  // uniform per range
      case 0:
        if (delta == 0) st16<true>(d4 + i, ~ld16<true>(sa + i));
        else st16<true>(d4 + i, ~shift16<0>(ld16<true>(sa + i), ld16<false>(sa + i + 1), r));
        break;
      case 1: st16<true>(d4 + i, ~shift16<1>(ld16<true>(sa + i), ld16<false>(sa + i + 1), r)); break;
      case 2: st16<true>(d4 + i, ~shift16<2>(ld16<true>(sa + i), ld16<false>(sa + i + 1), r)); break;
      default: st16<true>(d4 + i, ~shift16<3>(ld16<true>(sa + i), ld16<false>(sa + i + 1), r)); break;
    }
  }
}

// ---- the drop-in's pageable frame, launched before its bytes have landed ----------------------
// vf_invert_host on an ordinary (pageable) frame (inverter.py:41's call shape): the host pool
// copies the frame into mapped staging in pieces of 2^piece_shift bytes while this kernel
// already runs, so the launch and the PCIe traffic of the first pieces overlap the copy of the
// later ones.  Whole pieces go to whichever host thread asks next, which then sets landed[p]
// (page-locked memory) to nw = 1, so pieces may complete out of order.
// One wave (workgroup 0's first) relays: it reads all the counts in one round trip over PCIe,
// publishes how many leading pieces are complete as (gen << 8) | count in a device-memory word,
// sleeps about a microsecond and reads again until every piece is in.  The other workgroups
// stride over the tiles and, before a tile whose piece is past what they saw complete, read the
// device word (on-chip, not PCIe: polling host memory from every wave flooded the link with
// reads, 0.39 ms for a 480p frame).  A relay or tile wave that waits `budget` wall-clock ticks
// sets *status and leaves (the relay also publishes count 255, which sends every tile wave
// home); the caller then inverts the whole frame again, ungated, from the complete staging
// copy.  The counts are read relaxed: the host writes a piece before its count (x86 stores are
// ordered), a tile reads the staging copy only after the relay saw its count, and no line of a
// piece can sit in a cache before it landed (the launch's acquire dropped the previous frame's
// lines; no earlier tile of this launch touches it).  src is the staging buffer, 16-B aligned
// like dst; the last tile also does the n % 16 tail bytes.  gen tells this launch's word from
// the previous one's (the word is never reset).
__global__ __launch_bounds__(kBlock) void invert_gated_kernel(const u32x4 *__restrict__ s, u32x4 *__restrict__ d,
                                                              uint64_t n, const uint32_t *landed, uint32_t piece_shift,
                                                              uint32_t nw, uint32_t *frontier, uint32_t gen,
                                                              uint32_t *status, uint64_t budget) {
  const uint32_t np = (uint32_t)((n - 1) >> piece_shift) + 1;  // <= 254 (the launcher checks)
  const uint32_t t = threadIdx.x;
  const uint64_t t0 = wall_clock64();
  if (blockIdx.x == 0) {  // the relay
    if (t >= 64) return;
    uint32_t k = 0;
    while (k < np) {
      uint32_t f[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)  // issued together: one PCIe round trip
        f[j] = 64 * j + t < np ? __hip_atomic_load(landed + 64 * j + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : nw;
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t m = __ballot(f[j] >= nw);
        if (c == 64u * j) c += ~m ? (uint32_t)__builtin_ctzll(~m) : 64u;
      }
      const uint32_t kn = min(c, np);
      if (kn != k) {
        k = kn;
        if (t == 0) __hip_atomic_store(frontier, (gen << 8) | k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (k < np) {
        if (wall_clock64() - t0 > budget) {
          if (t == 0) {
            __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(frontier, (gen << 8) | 255u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          return;
        }
        __builtin_amdgcn_s_sleep(32);
      }
    }
    return;
  }
  const uint64_t n16 = n >> 4;
  const uint64_t tiles = (n + kBlock * 16 - 1) / (kBlock * 16);
  uint32_t ready = 0;  // pieces [0, ready) seen complete (wave-uniform)
  for (uint64_t tile = blockIdx.x - 1; tile < tiles; tile += gridDim.x - 1) {
    const uint64_t end = min((tile + 1) * (uint64_t)(kBlock * 16), n);
    const uint32_t need = (uint32_t)((end - 1) >> piece_shift);
    while (ready <= need) {
      const uint32_t v = __hip_atomic_load(frontier, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((v >> 8) == (gen & 0xFFFFFFu)) {
        if ((v & 255u) == 255u) return;  // the relay gave up
        ready = v & 255u;
      }
      if (ready <= need) {
        if (wall_clock64() - t0 > budget) {
          __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    const uint64_t i = tile * kBlock + t;
    if (i < n16) st16<true>(d + i, ~ld16<true>(s + i));
    if (tile == tiles - 1 && t < (uint32_t)(n & 15)) {
      const uint8_t *sb = reinterpret_cast<const uint8_t *>(s) + (n16 << 4);
      reinterpret_cast<uint8_t *>(d)[(n16 << 4) + t] = (uint8_t)~sb[t];
    }
  }
}

// ---- launchers ----------------------------------------------------------------------

hipError_t launch_invert_gated(const uint8_t *src, uint8_t *dst, size_t n, const uint32_t *landed,
                               uint32_t piece_shift, uint32_t nw, uint32_t *frontier, uint32_t gen, uint32_t *status,
                               uint64_t budget_ticks, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) != 0 || ((n - 1) >> piece_shift) >= 254 || (gen & 0xFFFFFFu) == 0)
    return hipErrorInvalidValue;
  const uint64_t tiles = (n + kBlock * 16 - 1) / (kBlock * 16);
  // the relay + tile workgroups, as many as launch_invert_mapped's
  const uint64_t grid = 1 + std::min<uint64_t>(tiles, n < (16ull << 20) ? 256 : 128);
  hipLaunchKernelGGL(invert_gated_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream,
                     reinterpret_cast<const u32x4 *>(src), reinterpret_cast<u32x4 *>(dst), (uint64_t)n, landed,
                     piece_shift, nw, frontier, gen, status, budget_ticks);
  return hipGetLastError();
}

// src and dst at different offsets mod 16: dst's head bytewise, then the shifting body.
static hipError_t launch_shift(const uint8_t *s, uint8_t *d, size_t nbytes, int max_blocks, hipStream_t stream) {
  const uint32_t h = (uint32_t)std::min<size_t>((16 - ((uintptr_t)d & 15)) & 15, nbytes);
  const uint64_t n16 = (nbytes - h) >> 4;
  const uint32_t tail = (uint32_t)((nbytes - h) & 15);
  const uintptr_t sb = (uintptr_t)(s + h);
  const uint32_t delta = (uint32_t)(sb & 15);  // != 0: the offsets differ mod 16
  const u32x4 *sa = reinterpret_cast<const u32x4 *>(sb - delta);
  u32x4 *d4 = reinterpret_cast<u32x4 *>(d + h);
  constexpr uint64_t TILE = (uint64_t)kBlock * 4;
  uint64_t blocks = n16 ? (n16 + TILE - 1) / TILE : 1;
  if (blocks > (uint64_t)max_blocks) blocks = (uint64_t)max_blocks;
  const uint8_t *ts = s + h + (n16 << 4);
  uint8_t *td = d + h + (n16 << 4);
  const dim3 g((unsigned)blocks), b(kBlock);
  switch (delta >> 2) {
    case 0: hipLaunchKernelGGL(invert_shift_kernel<0>, g, b, 0, stream, sa, d4, n16, delta & 3, s, d, h, ts, td, tail); break;
    case 1: hipLaunchKernelGGL(invert_shift_kernel<1>, g, b, 0, stream, sa, d4, n16, delta & 3, s, d, h, ts, td, tail); break;
    case 2: hipLaunchKernelGGL(invert_shift_kernel<2>, g, b, 0, stream, sa, d4, n16, delta & 3, s, d, h, ts, td, tail); break;
    default: hipLaunchKernelGGL(invert_shift_kernel<3>, g, b, 0, stream, sa, d4, n16, delta & 3, s, d, h, ts, td, tail); break;
  }
  return hipGetLastError();
}

hipError_t launch_invert(const void *dsrc, void *ddst, size_t nbytes, const LaunchCfg &cfg,
                         hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  const uint8_t *s = static_cast<const uint8_t *>(dsrc);
  uint8_t *d = static_cast<uint8_t *>(ddst);
  if ((((uintptr_t)s ^ (uintptr_t)d) & 15) != 0) return launch_shift(s, d, nbytes, cfg.max_blocks, stream);
  return launch_stream<4, true, true>(s, d, nbytes, cfg.max_blocks, stream);
}

hipError_t launch_invert_frames(const void *const *dsrcs, void *const *ddsts,
                                const size_t *nbytes, int n, size_t total_bytes,
                                const LaunchCfg &cfg, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  // Spread one frame over enough blocks (one 16-KiB tile each) that the launch fills the chip.
  const uint64_t per_frame = (total_bytes / (uint64_t)n + 64ull * kBlock - 1) / (64ull * kBlock);
  uint64_t gx = per_frame ? per_frame : 1;
  const uint64_t cap = (uint64_t)cfg.max_blocks / (uint64_t)n + 1;
  if (gx > cap) gx = cap;
  hipLaunchKernelGGL(invert_frames_kernel, dim3((unsigned)gx, (unsigned)n), dim3(kBlock), 0,
                     stream, reinterpret_cast<const uint8_t *const *>(dsrcs),
                     reinterpret_cast<uint8_t *const *>(ddsts), nbytes);
  return hipGetLastError();
}

hipError_t launch_invert_mapped(const MappedBatch &b, int n, size_t total_bytes, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (n > kMappedMax) return hipErrorInvalidValue;
  MappedBatch a = b;
  uint64_t tiles = 0;
  for (int k = 0; k < n; ++k) {
    const uint64_t h = std::min<uint64_t>((16 - ((uintptr_t)a.dst[k] & 15)) & 15, a.n[k]);
    const uint64_t n16 = (a.n[k] - h) >> 4;
    a.tile0[k] = (uint32_t)tiles;
    tiles += n16 ? (n16 + kBlock - 1) / kBlock : 1;  // at least one tile: head and tail bytes
    if (tiles > 0xFFFFFFFFull) return hipErrorInvalidValue;  // > 16 TB in one launch
  }
  a.tile0[n] = (uint32_t)tiles;
  // Workgroups: 128 keep the link busy for large launches; below 16 MiB the fixed start-up
  // latency dominates and 256 finish sooner (zerocopy_probe: 6.2 MB at 256 WG 33-34 GB/s,
  // at 128 31-32).
  uint64_t grid = total_bytes < (16ull << 20) ? 256 : 128;
  if (grid > tiles) grid = tiles;
  hipLaunchKernelGGL(invert_mapped_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, a, (uint32_t)n);
  return hipGetLastError();
}

}  // namespace vf
