// vf_jpeg_kernels.hip — gfx950 kernels of the baseline-JPEG path.
//
// The reference's default mode (use_jpeg=True) runs, per frame, PyTurboJPEG decode ->
// cv2.bitwise_not -> PyTurboJPEG encode (inverter.py:32 -> :41 -> :44; the app encodes at
// webcam_app.py:110 and decodes at :140).  The integer arithmetic here is libjpeg-turbo's
// (the codec under PyTurboJPEG), so outputs are bit-exact with it; oracle/vf_jpeg_oracle.c
// restates the same algorithm on the CPU and is pinned against the image's libjpeg-turbo.
//
// Decoder (one batch of frames, grid.y = frame):
//   unstuff      FF00 -> FF over 4 KiB tiles (count, segmented scan, compact)
//   sync         parallel Huffman decoding over fixed 1024-bit subsequences.  A thread
//                decodes its subsequence from a guessed entry state (bit position,
//                coefficient index z, block-in-MCU c); JPEG's prefix codes re-synchronise
//                within a few symbols, so after a pass every thread's exit state is right
//                once its entry state is.  Passes feed each thread its predecessor's exit
//                state until no exit state changes (Weissenberger & Schmidt, "Massively
//                parallel Huffman decoding on GPUs", ICPP 2018 — self-synchronisation).
//   write        the converged entry states + a scan of per-subsequence block counts give
//                every subsequence its first block; coefficients land in zigzag order,
//                DC differences in per-component sequences
//   dc           segmented inclusive scan of the DC differences (jdhuff.c last_dc_val)
//   idct         dequantise + islow IDCT (jidctint.c) into component planes
//   color        fancy upsampling (jdsample.c) + YCbCr -> BGR (jdcolor.c), optionally ~x
// Encoder:
//   fdct         colour conversion (jccolor.c) + edge replication + downsampling
//                (jcsample.c) + islow / ifast forward DCT + reciprocal quantisation
//                (jcdctmgr.c), 8 lanes per block
//   huff         per-block Huffman bit length (jchuff.c encode_one_block, dummy edge blocks
//                of jccoefct.c), segmented exclusive scan, then each block emits its bits
//                at its offset (atomicOr on the two boundary words)
//   stuff        0xFF -> FF 00 with a tile scan; header, EOI
// No MFMA / LDS tiling: the work is integer butterflies and bit manipulation; the entropy
// stages are latency-bound per thread and are parallelised across blocks / subsequences.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <type_traits>

#include "vf_jpeg.h"

namespace vf {
namespace jpeg {

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// ---- workgroup scans (256 threads = 4 waves of 64) -----------------------------------------
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// exclusive scan of v over the workgroup; *total = the sum.  sh: 4 T of LDS.
template <typename T>
__device__ __forceinline__ T wg_excl_scan(T v, T *sh, T *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const T x = wave_incl_scan(v);
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  T base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const T s = sh[i];
    if (i < wid) base += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// ---- segmented scan ----------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void seg_tile_sum(const ScanSeg *segs, const T *in, T *tsum) {
  const ScanSeg sg = segs[blockIdx.y];
  const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
  if (t0 >= sg.len) return;
  __shared__ T sh[4];
  const uint64_t b0 = t0 + (uint64_t)threadIdx.x * kScanPerThread;
  T acc = 0;
#pragma unroll
  for (int j = 0; j < kScanPerThread; ++j)
    if (b0 + j < sg.len) acc += in[sg.base + b0 + j];
  T tot;
  (void)wg_excl_scan(acc, sh, &tot);
  if (threadIdx.x == 0) tsum[sg.tile0 + blockIdx.x] = tot;
}

// Each tile's workgroup adds the sums of the tiles before it in its segment itself (a frame's
// segment has a few hundred tiles at most at 8K, one or two loads per thread, from L2) instead
// of a separate one-workgroup-per-segment kernel scanning them in between: one launch and one
// dependent kernel boundary fewer per scan (five scans per batch).  The segment's last tile
// writes the segment total; a segment with no tiles has its total written as 0 by tile 0.
// PRE_IN: no seg_tile_sum before it -- a tile adds up the inputs of the tiles before it in its
// segment itself (out of place only: another tile may be writing out meanwhile), for segments of
// a few tiles, where the second launch (~4.5 us of a small batch's GPU time) costs more than
// re-reading up to three tiles from L2.  A scan whose segments are all one tile needs neither.
template <typename T, bool INCL, bool PRE_IN = false>
__global__ __launch_bounds__(256) void seg_apply(const ScanSeg *segs, const T *in, const T *tsum, T *out, T *totals) {
  const ScanSeg sg = segs[blockIdx.y];
  const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
  if (t0 >= sg.len) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && totals) totals[blockIdx.y] = T(0);
    return;
  }
  __shared__ T sh[8];
  const uint64_t b0 = t0 + (uint64_t)threadIdx.x * kScanPerThread;
  T v[kScanPerThread];
  T acc = 0;
#pragma unroll
  for (int j = 0; j < kScanPerThread; ++j) {
    v[j] = b0 + j < sg.len ? in[sg.base + b0 + j] : T(0);
    acc += v[j];
  }
  T pre = 0;  // this thread's share of the preceding tiles' sums
  if constexpr (PRE_IN) {
    for (uint64_t i = (uint64_t)threadIdx.x * kScanPerThread; i < t0; i += kScanTile) {
      T w[kScanPerThread];
#pragma unroll
      for (int j = 0; j < kScanPerThread; ++j) w[j] = in[sg.base + i + j];  // i + j < t0 <= len
#pragma unroll
      for (int j = 0; j < kScanPerThread; ++j) pre += w[j];
    }
  } else {
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += 256) pre += tsum[sg.tile0 + i];
  }
  // one barrier for both: the exclusive scan of acc and the sum of pre over the workgroup
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const T x = wave_incl_scan(acc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (lane == 63) sh[wid] = x, sh[4 + wid] = pre;
  __syncthreads();
  T run = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const T t = sh[i];
    if (i < wid) run += t;
    tot += t;
    run += sh[4 + i];  // every wave's preceding-tile share
  }
  const T before = sh[4] + sh[5] + sh[6] + sh[7];
  run += x - acc;
#pragma unroll
  for (int j = 0; j < kScanPerThread; ++j) {
    if (INCL) run += v[j];
    if (b0 + j < sg.len) out[sg.base + b0 + j] = run;
    if (!INCL) run += v[j];
  }
  if (threadIdx.x == 0 && totals && t0 + kScanTile >= sg.len) totals[blockIdx.y] = before + tot;
}

template <typename T>
hipError_t seg_scan(const ScanSeg *segs, int nseg, uint32_t max_tiles, const T *in, T *out, T *tsum,
                    T *totals, bool inclusive, hipStream_t s) {
  if (nseg <= 0 || max_tiles == 0) return hipSuccess;
  const dim3 g(max_tiles, (unsigned)nseg);
  static const uint32_t one_pass_max = [] {  // VF_SCAN_ONE_PASS_TILES (0: always two kernels)
    const char *v = std::getenv("VF_SCAN_ONE_PASS_TILES");
    return v && *v ? (uint32_t)std::atoi(v) : 4u;
  }();
  const bool one = max_tiles == 1 ? one_pass_max > 0 : (in != out && max_tiles <= one_pass_max);
  if (one) {  // tile 0 of a segment reads no tile sums, so one tile per segment is the PRE_IN form too
    if (inclusive) hipLaunchKernelGGL((seg_apply<T, true, true>), g, dim3(256), 0, s, segs, in, tsum, out, totals);
    else hipLaunchKernelGGL((seg_apply<T, false, true>), g, dim3(256), 0, s, segs, in, tsum, out, totals);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(seg_tile_sum<T>, g, dim3(256), 0, s, segs, in, tsum);
  if (inclusive) hipLaunchKernelGGL((seg_apply<T, true>), g, dim3(256), 0, s, segs, in, tsum, out, totals);
  else hipLaunchKernelGGL((seg_apply<T, false>), g, dim3(256), 0, s, segs, in, tsum, out, totals);
  return hipGetLastError();
}

// ---- decoder: unstuffing --------------------------------------------------------------------

// keep-mask of the 16 raw bytes [i0, i0 + 16): a 0x00 right after 0xFF is stuffing
__device__ __forceinline__ uint32_t keep_mask(const uint8_t *s, uint32_t len, uint32_t i0, uint8_t *bytes) {
  uint32_t m = 0;
  uint8_t prev = i0 ? s[i0 - 1] : 0;
  // one 16-B load: i0 is a multiple of 16 and the host stages each segment at a 16-B aligned
  // offset, rounded up to 16 bytes
  const uint4 q = i0 < len ? *reinterpret_cast<const uint4 *>(s + i0) : make_uint4(0, 0, 0, 0);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t i = i0 + j;
    const uint8_t b = i < len ? (uint8_t)(qw[j >> 2] >> (8 * (j & 3))) : 0;
    bytes[j] = b;
    if (i < len && !(b == 0 && prev == 0xFF)) m |= 1u << j;
    prev = b;
  }
  return m;
}

__global__ __launch_bounds__(256) void k_unstuff_count(const DecSeg *__restrict__ sg, const uint8_t *in, uint32_t *cnt) {
  const DecSeg F = sg[blockIdx.y];  // by value: see k_spec
  if (blockIdx.x >= F.ntiles) return;
  __shared__ uint32_t sh[4];
  uint8_t bytes[16];
  const uint32_t i0 = blockIdx.x * kTile + threadIdx.x * 16;
  const uint32_t m = keep_mask(in + F.in_off, F.in_len, i0, bytes);
  uint32_t tot;
  (void)wg_excl_scan((uint32_t)__popc(m), sh, &tot);
  if (threadIdx.x == 0) cnt[F.tile0 + blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_unstuff_write(const DecSeg *__restrict__ sg, const uint8_t *in, const uint32_t *off,
                                                       const uint32_t *us_len, uint8_t *us) {
  const DecSeg F = sg[blockIdx.y];  // by value: see k_spec
  if (blockIdx.x >= F.ntiles) return;
  __shared__ uint32_t sh[4];
  uint8_t bytes[16];
  const uint32_t i0 = blockIdx.x * kTile + threadIdx.x * 16;
  const uint32_t m = keep_mask(in + F.in_off, F.in_len, i0, bytes);
  uint32_t tot;
  // the tile's kept bytes are assembled in LDS, then stored as aligned dwords
  __shared__ uint8_t s_out[kTile];
  uint32_t lp = wg_excl_scan((uint32_t)__popc(m), sh, &tot);
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (m >> j & 1) s_out[lp++] = bytes[j];
  __syncthreads();
  uint8_t *d = us + F.us_off;
  uint8_t *dst = d + off[F.tile0 + blockIdx.x];
  const uint32_t head = min((uint32_t)(-(uintptr_t)dst & 3), tot), nw = (tot - head) >> 2;
  if (threadIdx.x < head) dst[threadIdx.x] = s_out[threadIdx.x];
  for (uint32_t i = threadIdx.x; i < nw; i += 256) {
    const uint32_t a = head + 4 * i;
    reinterpret_cast<uint32_t *>(dst + head)[i] = (uint32_t)s_out[a] | ((uint32_t)s_out[a + 1] << 8) |
                                                  ((uint32_t)s_out[a + 2] << 16) | ((uint32_t)s_out[a + 3] << 24);
  }
  const uint32_t tail = head + 4 * nw;
  if (threadIdx.x < tot - tail) dst[tail + threadIdx.x] = s_out[tail + threadIdx.x];
  // zero tail for the bit reader (libjpeg feeds zeros past the data, jdhuff.c)
  if (blockIdx.x == F.ntiles - 1 && threadIdx.x < 32) d[us_len[blockIdx.y] + threadIdx.x] = 0;
}

// ---- decoder: Huffman ------------------------------------------------------------------------

// The next word is loaded one refill ahead (nxt), so a refill costs no memory wait of its
// own: the load is in flight with the symbol lookups that follow it, and LDS completes in
// order.  A reader therefore reads up to 3 words past its position.
struct BitReader {
  const uint32_t *w;  // words of the stream from word `woff` on (global memory or an LDS copy)
  uint64_t buf;  // next bits, left-aligned
  uint32_t nb;   // valid bits in buf
  uint32_t wi;   // index of nxt (minus woff)
  uint32_t nxt;  // the next word, loaded ahead
  uint32_t pos;  // bit position of the next unread bit
  __device__ __forceinline__ void init(const uint8_t *base, uint32_t p) {
    init_words(reinterpret_cast<const uint32_t *>(base), p, 0);
  }
  __device__ __forceinline__ void init_words(const uint32_t *words, uint32_t p, uint32_t woff) {
    w = words;
    wi = (p >> 5) - woff;
    buf = ((uint64_t)bswap32(w[wi]) << 32) | bswap32(w[wi + 1]);
    wi += 2;
    nxt = w[wi];
    const uint32_t sk = p & 31;
    buf <<= sk;
    nb = 64 - sk;
    pos = p;
  }
  __device__ __forceinline__ void refill() {  // afterwards nb >= 33
    if (nb <= 32) {
      buf |= (uint64_t)bswap32(nxt) << (32 - nb);
      nb += 32;
      nxt = w[++wi];
    }
  }
  __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)(buf >> (64 - n)); }
  __device__ __forceinline__ void skip(uint32_t n) {
    buf <<= n;
    nb -= n;
    pos += n;
  }
};

// Length of a code longer than kLook bits starting the 16 bits c16 (17: none, see HuffDec.lim)
__device__ __forceinline__ uint32_t long_code_len(uint32_t c16, const uint32_t *lim) {
  const uint4 a = *reinterpret_cast<const uint4 *>(lim);
  const uint4 b = *reinterpret_cast<const uint4 *>(lim + 4);
  return kLook + 1 + (c16 >= a.x) + (c16 >= a.y) + (c16 >= a.z) + (c16 >= a.w) + (c16 >= b.x) + (c16 >= b.y) +
         (c16 >= b.z);
}

__device__ __forceinline__ uint64_t pack_state(uint32_t pos, uint32_t z, uint32_t c) {
  return ((uint64_t)pos << 16) | (z << 8) | c;
}

// The frame geometry the Huffman loops need per symbol, in registers.  Geom lives in global
// memory and is indexed by the per-lane block-in-MCU c, so reading g.bcomp[c] inside the loop
// is a dependent vector memory load per symbol; here the component of c is a 2-bit field of
// one register and the per-component values are picked with selects.
struct HuffGeom {
  uint32_t cpack;    // component of block-in-MCU c at bits 2c..2c+1
  uint32_t bpm, nblocks;
  uint32_t pat = 0;  // SpanLaneR: bit j = the table slot of block-in-MCU (j mod bpm)
  uint32_t bpc[3];   // blocks of component k per MCU
  uint32_t cfirst[3];
  __device__ __forceinline__ explicit HuffGeom(const Geom &g) {
    bpm = (uint32_t)g.bpm;
    nblocks = (uint32_t)g.nblocks;
    cpack = 0;
    for (int j = 0; j < g.bpm; ++j) cpack |= (uint32_t)(g.bcomp[j] & 3) << (2 * j);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      bpc[k] = (uint32_t)(g.mh[k] * g.mv[k]);
      cfirst[k] = (uint32_t)g.cfirst[k];
    }
  }
  __device__ __forceinline__ uint32_t comp(uint32_t c) const { return (cpack >> (2 * c)) & 3; }
  template <typename T>
  __device__ __forceinline__ static T sel(const T *a, uint32_t k) { return k == 0 ? a[0] : k == 1 ? a[1] : a[2]; }
};

// The write pass's decoder, on the short per-symbol step of SyncLane: the code and its extra bits are
// consumed together, the bit buffer is refilled with selects, the block end and the table
// switch are selects, so a symbol is one table read, its stores and no branch but the rare
// long code.  Decodes from state X over staged LDS words until `end` (or the segment's last
// block), storing coefficients (dense 64-entry rows, zigzag order) and DC differences
// (jdhuff.c decode_mcu; an unmatched code reads as symbol 0 after 16 bits, a DC size over 16
// as 16).
//
// CHUNKS (the default): no cleared buffer.  A block's AC coefficients are collected in registers
// as 16-B chunks of 8 zigzag positions; each chunk holding a nonzero coefficient is stored whole
// (its zeros included) and the block's byte in nmask records which chunks were stored, so the
// IDCT reads the others as zero.  A block is written by the thread that decoded its DC: past
// `end` that thread decodes on to the block's end, and a thread whose entry state lies inside
// a block skips to that block's end without storing (the block is its predecessor's).  Replaces
// a 134 MB clear per 1080p batch and the 2-byte scatters.
//
// A wave runs this loop in order at ~3 waves per SIMD (k_write's grid is one workgroup per 256
// subsequences), so every instruction of a step is on the lane's chain.  The step is kept to
// selects: the extra bits are one bit-field extract from the buffer's upper word (a code and its
// extra bits are at most 32 bits, and a refilled buffer holds at least 33), the DC goes to a
// per-component running position (each component's DC sequence is in block order) instead of
// an address rebuilt from (MCU, c) -- whose three-way selects over 64-bit bases compiled to
// nested branches -- and the chunk and block-end bookkeeping are selects around the stores.
// k_write's LDS staging of its workgroup's DC values and chunk masks: the blocks a workgroup
// owns are consecutive, so their per-block 4-B and 1-B stores -- scattered over the lanes, a
// sparse store instruction nearly every step -- are collected here by block and written out
// coalesced at the end (blocks past kStageBlocks from the first go straight to memory).
constexpr uint32_t kStageBlocks = 4096;
struct WriteStage {
  int32_t *dc;     // [kStageBlocks] DC differences
  uint16_t *nm;    // [kStageBlocks] 0x100 | chunk mask, 0 while not written
  uint32_t first;  // the workgroup's first block (segment-relative)
};
template <bool CHUNKS, bool STG = false>
__device__ __forceinline__ void write_span(const uint32_t *w, uint32_t woff, uint64_t X, uint32_t end,
                                           const HuffGeom &g, const HuffDec *tabs, uint32_t blk, int16_t *coef,
                                           int32_t *dcseq, const uint64_t *dcbase, uint8_t *nmask,
                                           const WriteStage &stg = WriteStage{nullptr, nullptr, 0}) {
  const uint32_t p = (uint32_t)(X >> 16);
  uint32_t wi = (p >> 5) - woff;
  uint64_t buf = (((uint64_t)bswap32(w[wi]) << 32) | bswap32(w[wi + 1])) << (p & 31);
  uint32_t nb = 64 - (p & 31), pos = p;
  wi += 2;
  uint32_t nxt = w[wi];
  uint32_t z = (X >> 8) & 0xFF, c = X & 0xFF;
  uint32_t k = g.comp(c);
  // DC positions: per component, its base + the blocks of it before this one (the MCUs before,
  // and those of this MCU before c); the host keeps the DC buffer under 2^31 entries
  uint32_t dcp0, dcp1, dcp2;
  {
    const uint32_t mcu = blk / g.bpm;
    const auto at = [&](int q) {
      const int before = min(max((int)c - (int)g.cfirst[q], 0), (int)g.bpc[q]);
      return (uint32_t)dcbase[q] + mcu * g.bpc[q] + (uint32_t)before;
    };
    dcp0 = at(0);
    dcp1 = at(1);
    dcp2 = at(2);
  }
  constexpr uint32_t kTab = (uint32_t)sizeof(HuffDec);
  uint32_t toff = __umul24(k, kTab);  // c's component's DC table (its AC table: 3 tables on)
  bool own = z == 0;            // CHUNKS: the block in progress is this thread's
  uint32_t cq = 0, m8 = 0;      // CHUNKS: the chunk being collected, chunks stored so far
  uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;
  while (blk < g.nblocks && (CHUNKS ? (pos < end ? true : own && z != 0) : pos < end)) {
    const bool f = nb <= 32;
    buf |= f ? (uint64_t)bswap32(nxt) << (32 - nb) : 0ull;
    nb += f ? 32u : 0u;
    wi += f ? 1u : 0u;
    nxt = w[wi];
    const bool dc = z == 0;
    const HuffDec &T = *reinterpret_cast<const HuffDec *>(reinterpret_cast<const char *>(tabs) + toff +
                                                          (dc ? 0u : 3u * kTab));
    const uint32_t hi = (uint32_t)(buf >> 32);
    const uint32_t e = T.fast[hi >> (32 - kLook)];
    uint32_t len = e >> 8, sym = e & 0xFF;
    if (len == 0) {
      const uint32_t c16 = hi >> 16;
      len = long_code_len(c16, T.lim);
      if (len > 16) {
        len = 16;
        sym = 0;
      } else {
        sym = T.vals[(uint32_t)((int32_t)(c16 >> (16 - len)) + T.valoff[len]) & 255];
      }
    }
    const uint32_t r = dc ? 0u : sym >> 4;
    const uint32_t sz = dc ? (sym > 16 ? 16u : sym) : (sym & 15);
    const uint32_t t = len + sz;  // <= 32
    const uint32_t xb = __builtin_amdgcn_ubfe(hi, (32 - t) & 31, sz);  // the extra bits (0 when sz = 0)
    const int v = xb < (1u << sz >> 1) ? (int)xb - (int)((1u << sz) - 1) : (int)xb;  // jdhuff.h HUFF_EXTEND; 0 when sz = 0
    buf <<= t;
    nb -= t;
    pos += t;
    // the zigzag index after the symbol, by selects (ahead of the stores' branches, which the
    // compiler otherwise folds it into)
    const uint32_t zn = dc ? 1u : sz ? z + r + 1 : r == 15 ? z + 16 : 64u;
    if (dc) {
      const uint32_t sb = blk - stg.first;
      if (STG && sb < kStageBlocks) {
        stg.dc[sb] = v;
        stg.nm[sb] = 0x100;
      } else {
        dcseq[k == 0 ? dcp0 : k == 1 ? dcp1 : dcp2] = v;
      }
    } else if (sz) {
      const uint32_t zz = z + r < 63 ? z + r : 63;
      if constexpr (CHUNKS) {
        const uint32_t q = zz >> 3;
        const bool nc = own && q != cq;  // a new chunk: store the one collected (if any)
        if (nc && (m8 >> cq & 1))
          *reinterpret_cast<uint4 *>(coef + (uint64_t)blk * 64 + cq * 8) = make_uint4(q0, q1, q2, q3);
        const uint32_t hv = own ? ((uint32_t)v & 0xFFFFu) << (16 * (zz & 1)) : 0u, wsel = (zz >> 1) & 3;
        q0 = (nc ? 0u : q0) | (wsel == 0 ? hv : 0u);
        q1 = (nc ? 0u : q1) | (wsel == 1 ? hv : 0u);
        q2 = (nc ? 0u : q2) | (wsel == 2 ? hv : 0u);
        q3 = (nc ? 0u : q3) | (wsel == 3 ? hv : 0u);
        cq = nc ? q : cq;
        m8 |= own ? 1u << q : 0u;
      } else {
        coef[(uint64_t)blk * 64 + zz] = (int16_t)v;
      }
    }
    z = zn;
    const bool eob = z >= 64;
    if constexpr (CHUNKS) {
      if (eob && own) {
        if (m8 >> cq & 1)
          *reinterpret_cast<uint4 *>(coef + (uint64_t)blk * 64 + cq * 8) = make_uint4(q0, q1, q2, q3);
        const uint32_t sb = blk - stg.first;
        if (STG && sb < kStageBlocks) stg.nm[sb] = (uint16_t)(0x100 | m8);
        else nmask[blk] = (uint8_t)m8;
      }
      own = own || eob;  // the next block starts here: inside the span (or the loop ends)
      cq = eob ? 0u : cq;
      m8 = eob ? 0u : m8;
      q0 = eob ? 0u : q0;
      q1 = eob ? 0u : q1;
      q2 = eob ? 0u : q2;
      q3 = eob ? 0u : q3;
    }
    dcp0 += eob && k == 0 ? 1u : 0u;
    dcp1 += eob && k == 1 ? 1u : 0u;
    dcp2 += eob && k == 2 ? 1u : 0u;
    const uint32_t c1 = c + 1 == g.bpm ? 0u : c + 1;
    z = eob ? 0u : z;
    blk += eob ? 1u : 0u;
    c = eob ? c1 : c;
    k = g.comp(c);
    toff = __umul24(k, kTab);
  }
  if constexpr (STG) atomicMax(reinterpret_cast<uint32_t *>(stg.dc) + kStageBlocks, blk - stg.first);  // flush bound
}

// frame F's Huffman tables (DecFrame::tabs_off, from the DecFrame array fr)
__device__ __forceinline__ const DecTabs &tabs_of(const DecFrame *fr, const DecFrame &F) {
  return *reinterpret_cast<const DecTabs *>(reinterpret_cast<const char *>(fr) + F.tabs_off);
}

__device__ __forceinline__ void load_tables(const DecTabs &F, HuffDec *tabs) {
  const uint32_t *src = reinterpret_cast<const uint32_t *>(&F.dc[0]);
  uint32_t *dst = reinterpret_cast<uint32_t *>(tabs);
  constexpr uint32_t nw = 6 * sizeof(HuffDec) / 4;
  for (uint32_t j = threadIdx.x; j < nw; j += 256) dst[j] = src[j];
  __syncthreads();
}

// (zigzag advance << 8) | bits of a symbol whose code is longer than kLook bits: jdhuff.c
// jpeg_huff_decode's slow path (an unmatched code reads as symbol 0 after 16 bits)
template <typename BR>
__device__ __forceinline__ uint32_t sync_slow(const BR &br, const HuffSync &t, bool dc) {
  const uint32_t c16 = br.peek(16);
  uint32_t len = long_code_len(c16, t.lim), sym = 0;
  if (len > 16) len = 16;  // corrupt code: symbol 0
  else sym = t.vals[(uint32_t)((int32_t)(c16 >> (16 - len)) + t.valoff[len]) & 255];
  uint32_t extra, adv;
  if (dc) {
    extra = sym > 16 ? 16 : sym;
    adv = 1;
  } else {
    extra = sym & 15;
    adv = extra ? (sym >> 4) + 1 : ((sym >> 4) == 15 ? 16 : 64);
  }
  return (adv << 8) | (len + extra);
}

// One Huffman symbol of the sync decode: the same bits and zigzag / block progression as
// write_span, through one combined lookup (HuffSync) instead of symbol + extra-bits steps.
template <typename BR>
__device__ __forceinline__ void sync_step(BR &br, uint32_t &z, uint32_t &c, uint32_t &blocks,
                                          const HuffGeom &g, const HuffSync *dcT, const HuffSync *acT) {
  br.refill();
  const uint32_t k = g.comp(c);
  const HuffSync &T = z == 0 ? dcT[k] : acT[k];
  uint32_t e = T.sfast[br.peek(kLook)] & 0xFFFF;  // one symbol (SyncLane also takes pairs)
  if (!e) e = sync_slow(br, T, z == 0);
  br.skip(e & 0xFF);
  z += e >> 8;
  if (z >= 64) {
    z = 0;
    c = (c + 1 == g.bpm) ? 0 : c + 1;
    ++blocks;
  }
}

// One lane's sync decoder with a short per-symbol chain, over stream words staged in LDS: the
// bit buffer is refilled with selects (the next word re-read every symbol, off the critical
// path), and the byte offset of c's component tables is kept in a register and recomputed with
// selects, so a symbol is one table read and ~25 VALU with no branch but the rare long code.
// sync_step's branchy form (refill, DC / AC, block end) measured ~530-700 shader cycles per
// symbol for a lone lane on an idle GPU (tools/build_syncg_stats.sh).  Same bits, zigzag and
// block progression as sync_step.
// The span sync's LDS tables: DecFrame's HuffSync entries with, in the AC tables, the pair
// entry (DecFrame::spair) in the upper 16 bits of each word.  The speculative kernels read
// HuffSync itself (single-symbol entries only: with 32-bit entries k_spec's LDS cost it a
// workgroup per CU, 200 -> 218 us at 1080p).
struct SyncTab32 {
  alignas(16) uint32_t lim[8];
  uint32_t sfast[1 << kLook];
  int32_t valoff[18];
  uint8_t vals[256];
};

// F's six sync tables (sdc[3], sac[3]) with the AC pairs into LDS, then a barrier (which also
// publishes whatever the caller staged before the call)
__device__ __forceinline__ void load_sync_tabs32(const DecTabs &F, SyncTab32 *tabs) {
  for (uint32_t j = threadIdx.x; j < 6 * (8 + 18 + 64); j += blockDim.x) {
    const uint32_t t = j / 90, i = j - t * 90;
    const HuffSync &S = t < 3 ? F.sdc[t] : F.sac[t - 3];
    if (i < 8) tabs[t].lim[i] = S.lim[i];
    else if (i < 26) tabs[t].valoff[i - 8] = S.valoff[i - 8];
    else reinterpret_cast<uint32_t *>(tabs[t].vals)[i - 26] = reinterpret_cast<const uint32_t *>(S.vals)[i - 26];
  }
  for (uint32_t j = threadIdx.x; j < 6 * (1 << kLook); j += blockDim.x) {
    const uint32_t t = j >> kLook, i = j & ((1 << kLook) - 1);
    tabs[t].sfast[i] = t < 3 ? (uint32_t)F.sdc[t].sfast[i] : F.sac[t - 3].sfast[i] | ((uint32_t)F.spair[t - 3][i] << 16);
  }
  __syncthreads();
}

// The span sync's 4-table layout (DecFrame::tabs4: at most two distinct (DC, AC) table pairs over
// the components -- every frame whose chroma components share tables): slot s's DC table at
// tabs[s], its AC table with the pairs at tabs[2 + s], from the component tabs4 names for it;
// 9.6 KB of LDS instead of 14.4, so a workgroup stages 25 % more stream (G = 5) at 3 per CU.
// The lanes' cpack then holds slots (tabs4_cpack), not components.  Then a barrier.
template <bool REV = false>  // REV: fast entries at bit-reversed indices (SpanLaneR)
__device__ __forceinline__ void load_sync_tabs4(const DecTabs &F, uint32_t tabs4, SyncTab32 *tabs) {
  const uint32_t rep[2] = {(tabs4 >> 8) & 3u, (tabs4 >> 10) & 3u};
  for (uint32_t j = threadIdx.x; j < 4 * (8 + 18 + 64); j += blockDim.x) {
    const uint32_t t = j / 90, i = j - t * 90;
    const HuffSync &S = t < 2 ? F.sdc[rep[t]] : F.sac[rep[t - 2]];
    if (i < 8) tabs[t].lim[i] = S.lim[i];
    else if (i < 26) tabs[t].valoff[i - 8] = S.valoff[i - 8];
    else reinterpret_cast<uint32_t *>(tabs[t].vals)[i - 26] = reinterpret_cast<const uint32_t *>(S.vals)[i - 26];
  }
  for (uint32_t j = threadIdx.x; j < 4 * (1 << kLook); j += blockDim.x) {
    const uint32_t t = j >> kLook, i = j & ((1 << kLook) - 1);
    uint32_t v = t < 2 ? (uint32_t)F.sdc[rep[t]].sfast[i] : F.sac[rep[t - 2]].sfast[i] | ((uint32_t)F.spair[rep[t - 2]][i] << 16);
    if (REV && (v >> 16) == 0) v |= v << 16;  // SpanLaneR: no pair reads as the first symbol again
    tabs[t].sfast[REV ? __builtin_bitreverse32(i) >> (32 - kLook) : i] = v;
  }
  __syncthreads();
}
__device__ __forceinline__ uint32_t tabs4_cpack(const HuffGeom &hg, uint32_t tabs4) {  // block-in-MCU -> slot
  uint32_t p = 0;
  for (uint32_t c = 0; c < hg.bpm; ++c) p |= ((tabs4 >> (2 * hg.comp(c))) & 3u) << (2 * c);
  return p;
}

// k_spec's lane (six HuffSync tables: three DC, then three AC; no pairs): a 64-bit bit buffer
// refilled with selects, one table read per symbol.  The span sync's lane is SpanLane, below.
template <typename Tab>
struct SyncLane {
  const uint32_t *w;  // staged words, minus woff
  uint64_t buf;       // next bits, left-aligned
  uint32_t nb, wi, nxt, pos;
  uint32_t z, c, n;   // zigzag index, block-in-MCU, blocks completed
  uint32_t toff;      // byte offset of the DC table of c's component (its AC table: 3 tables on)
  uint32_t cpack, bpm;
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t woff, uint64_t X, const HuffGeom &hg) {
    const uint32_t p = (uint32_t)(X >> 16);
    w = words;
    wi = (p >> 5) - woff;
    buf = (((uint64_t)bswap32(w[wi]) << 32) | bswap32(w[wi + 1])) << (p & 31);
    nb = 64 - (p & 31);
    wi += 2;
    nxt = w[wi];
    pos = p;
    z = (X >> 8) & 0xFF;
    c = X & 0xFF;
    n = 0;
    cpack = hg.cpack;
    bpm = hg.bpm;
    toff = __umul24((cpack >> (2 * c)) & 3, (uint32_t)sizeof(Tab));
  }
  // one step: one symbol (`stop` is SpanLane's pair bound; a single symbol never needs it)
  __device__ __forceinline__ void step(const Tab *tabs, uint32_t /*stop*/) {
    const bool f = nb <= 32;
    buf |= f ? (uint64_t)bswap32(nxt) << (32 - nb) : 0ull;
    nb += f ? 32u : 0u;
    wi += f ? 1u : 0u;
    nxt = w[wi];
    const Tab &T = *reinterpret_cast<const Tab *>(reinterpret_cast<const char *>(tabs) + toff +
                                                   (z == 0 ? 0u : 3u * (uint32_t)sizeof(Tab)));
    uint32_t e = T.sfast[(uint32_t)(buf >> (64 - kLook))];
    if (!e) {  // a code longer than kLook bits: jdhuff.c's slow path (rare)
      const uint32_t c16 = (uint32_t)(buf >> 48);
      uint32_t len = long_code_len(c16, T.lim), sym = 0;
      if (len > 16) len = 16;
      else sym = T.vals[(uint32_t)((int32_t)(c16 >> (16 - len)) + T.valoff[len]) & 255];
      uint32_t extra, adv;
      if (z == 0) {
        extra = sym > 16 ? 16 : sym;
        adv = 1;
      } else {
        extra = sym & 15;
        adv = extra ? (sym >> 4) + 1 : ((sym >> 4) == 15 ? 16 : 64);
      }
      e = (adv << 8) | (len + extra);
    }
    const uint32_t len = e & 0xFF;
    buf <<= len;
    nb -= len;
    pos += len;
    z += (e >> 8) & 0xFF;
    const bool eob = z >= 64;
    const uint32_t c1 = c + 1 == bpm ? 0u : c + 1;
    c = eob ? c1 : c;
    z = eob ? 0u : z;
    n += eob ? 1u : 0u;
    toff = __umul24((cpack >> (2 * c)) & 3, (uint32_t)sizeof(Tab));
  }
};

// k_syncg's lane.  One step decodes a symbol, or two (an AC table's pair entry) when the first
// leaves the block open and ends before `stop` -- so a mark's state is still taken at the first
// symbol boundary at or past it, whichever symbol a decoder's pairing started from.  It takes
// about two thirds of the instructions of the buffered step it replaced (SyncLane's reader, 60
// per step; the span sync issues VALU back to back, so its time follows the step's instruction
// count).  There is no bit buffer to refill: a step reads the two staged words
// holding bits pos-1 .. pos+62 with one ds_read2 and aligns them with v_alignbit (a three-word
// window sliding a read ahead, so that the table read is the only LDS read on the chain, was no
// faster).  The words are staged byte-swapped, and the position is kept negated relative to
// the staged words, q = 32 * wbase - pos, so the word index (-(q >> 5) - 1: the word of bit pos-1)
// and the alignment shift (q & 31 = 31 - (pos-1) % 32, v_alignbit reads its low 5 bits) are
// direct functions of q.  Staged word 0 must lie before every position decoded (pos - 32 * wbase
// >= 1).  The block-in-MCU is kept doubled (c2): its table slot is one bit-field extract.
// k_spec runs it on its six HuffSync tables without pairs (PAIRS = false).
template <typename Tab, uint32_t NDC, bool PAIRS = true>  // tabs: NDC DC tables, then NDC AC tables
struct SpanLane {
  const uint32_t *wl;  // staged words, byte-swapped
  uint32_t base;       // 32 * wbase (modular)
  int32_t q;           // base - pos
  uint32_t z, c2, n;   // zigzag index, 2 x block-in-MCU, blocks completed
  uint32_t cpack, bpm2;
  __device__ __forceinline__ void init(const uint32_t *s_w, uint32_t base_, uint64_t X, const HuffGeom &hg) {
    wl = s_w;
    base = base_;
    q = (int32_t)(base - (uint32_t)(X >> 16));
    z = (X >> 8) & 0xFF;
    c2 = (uint32_t)(X & 0xFF) * 2u;
    n = 0;
    cpack = hg.cpack;
    bpm2 = hg.bpm * 2u;
  }
  __device__ __forceinline__ uint32_t pos() const { return base - (uint32_t)q; }
  __device__ __forceinline__ uint32_t c() const { return c2 >> 1; }
  __device__ __forceinline__ uint64_t state() const { return pack_state(pos(), z, c()); }
  // steps while pos < stop
  __device__ __forceinline__ void run(const Tab *tabs, uint32_t stop) {
    const int32_t qs = (int32_t)(base - stop);  // pos < stop <=> q > qs
    while (q > qs) step(tabs, qs);
  }
  __device__ __forceinline__ void step(const Tab *tabs, int32_t qs) {
    const uint32_t *p = wl + (-(q >> 5) - 1);
    const uint32_t r = __builtin_amdgcn_alignbit(p[0], p[1], (uint32_t)q);  // bits pos .. pos+31
    const Tab &T = tabs[((cpack >> c2) & 3u) + min(z, 1u) * NDC];
    uint32_t e = T.sfast[r >> (32 - kLook)];
    if (!e) {  // a code longer than kLook bits (rare): as SyncLane
      const uint32_t c16 = r >> 16;
      uint32_t len = long_code_len(c16, T.lim), sym = 0;
      if (len > 16) len = 16;
      else sym = T.vals[(uint32_t)((int32_t)(c16 >> (16 - len)) + T.valoff[len]) & 255];
      uint32_t extra, adv;
      if (z == 0) {
        extra = sym > 16 ? 16 : sym;
        adv = 1;
      } else {
        extra = sym & 15;
        adv = extra ? (sym >> 4) + 1 : ((sym >> 4) == 15 ? 16 : 64);
      }
      e = (adv << 8) | (len + extra);
    }
    const int32_t q1 = q - (int32_t)(e & 0xFF);
    const uint32_t z1 = z + ((e >> 8) & 0xFF);
    if constexpr (PAIRS) {
      const bool two = (e >> 16) != 0 && z1 < 64 && q1 > qs;  // pair word: (advance << 24) | (length << 16)
      q = two ? q - (int32_t)((e >> 16) & 0xFF) : q1;
      z = two ? z + (e >> 24) : z1;
    } else {
      q = q1;
      z = z1;
    }
    const bool eob = z >= 64;
    const uint32_t c2n = c2 + 2 == bpm2 ? 0u : c2 + 2;
    c2 = eob ? c2n : c2;
    z = eob ? 0u : z;
    n += eob ? 1u : 0u;
  }
};

// k_syncg's lane for frames whose blocks take two table slots in a cycle of a power of two
// (DecFrame::tabs4 with bpm 1, 2, 4, 8 or 16: every TurboJPEG 4:2:2 and grayscale frame), with
// ~22 % fewer instructions per step than SpanLane (35 against 45; the span sync issues a step's
// instructions one after another at 3 waves per SIMD, so its time follows the count):
//  * the staged words are LSB-first (stream bit j of a word at bit j), so the position P itself
//    gives the word's byte address ((P >> 3) & ~3: P counts bits from LDS address 0) and the
//    alignment (v_alignbit reads P's low 5 bits), and the table index is r's low kLook bits --
//    the fast tables are stored at bit-reversed indices;
//  * the table is an LDS address kept per lane: after a step it is the AC table of the block
//    the lane is in, or after a block end the next block's DC table, picked from a per-lane bit
//    pattern (bit k = the table slot of the k-th block from the entry's; the cycle divides 32)
//    by the block count -- no block-in-MCU is carried, it is (c0 + n) & (bpm - 1) at the marks.
// Same symbols, pairs, marks and states as SpanLane (the long-code path reads the code MSB-first
// through a bit reversal).
// Tab: SyncTab32 (32-bit fast entries, pairs in the upper half; k_syncg) or HuffSync (16-bit, one
// symbol; k_spec); NT DC tables then NT AC tables; SB bits per block's table slot in the pattern.
template <typename Tab, uint32_t NT, uint32_t SB, bool PAIRS>
struct SpanLaneRT {
  static constexpr uint32_t kEnt = sizeof(Tab{}.sfast[0]);     // bytes per fast entry: 4 or 2
  static constexpr uint32_t kLead = kEnt == 4 ? 2u : 1u;       // window read from bit pos - kLead
  uint32_t Q;     // bit position - kLead, relative to LDS byte 0 (8 * address + bit)
  uint32_t qofs;  // Q - pos (modular)
  uint32_t z, n, tb, cpl, c0, bpmm, dc0, ac0;
  // s_w: the LSB-first staged words, word i at stream position wb32 + 32 i; pat: bits SB j ..
  // SB j + SB - 1 = table slot of block-in-MCU (j mod bpm); tabs: the NT DC tables, then NT AC
  __device__ __forceinline__ void init(const uint32_t *s_w, uint32_t wb32, uint64_t X, uint32_t pat, uint32_t bpm,
                                       const Tab *tabs) {
    qofs = 8u * (uint32_t)(uintptr_t)s_w - wb32 - kLead;
    Q = (uint32_t)(X >> 16) + qofs;
    z = (X >> 8) & 0xFF;
    c0 = (uint32_t)(X & 0xFF);
    n = 0;
    bpmm = bpm - 1;
    cpl = __builtin_amdgcn_alignbit(pat, pat, SB * c0);  // rotate right: field k = slot of block c0 + k
    dc0 = (uint32_t)(uintptr_t)tabs;
    ac0 = dc0 + NT * (uint32_t)sizeof(Tab);
    tb = (cpl & ((1u << SB) - 1)) * (uint32_t)sizeof(Tab) + (z == 0 ? dc0 : ac0);
  }
  __device__ __forceinline__ uint32_t pos() const { return Q - qofs; }
  __device__ __forceinline__ uint32_t c() const { return (c0 + n) & bpmm; }
  // n = 0 for the next subsequence's count; the slot pattern and c0 move on by the blocks counted
  __device__ __forceinline__ void restart_count() {
    c0 = (c0 + n) & bpmm;
    cpl = __builtin_amdgcn_alignbit(cpl, cpl, SB * n);
    n = 0;
  }
  __device__ __forceinline__ uint64_t state() const { return pack_state(pos(), z, c()); }
  template <typename T>
  __device__ __forceinline__ static T lds(uint32_t a) {
    return *reinterpret_cast<const __attribute__((address_space(3))) T *>((size_t)a);
  }
  // steps while pos < stop
  __device__ __forceinline__ void run(const Tab *, uint32_t stop) {
    const uint32_t Qs = stop + qofs;
    while (Q < Qs) step(Qs);
  }
  // The window is read from bit pos - kLead on, so the fast table's byte offset is r & (kEnt * 511).
  // PAIRS: the fast entries' upper half is the pair entry, or a copy of the lower half where there
  // is none (load_sync_tabs4<true>), so taking "the pair" needs no test of whether there is one.
  __device__ __forceinline__ void step(uint32_t Qs) {
    const uint32_t a = (Q >> 3) & ~3u;
    const uint32_t r = __builtin_amdgcn_alignbit(lds<uint32_t>(a + 4), lds<uint32_t>(a), Q);  // LSB-first
    const uint32_t ea = tb + (uint32_t)offsetof(Tab, sfast) + (r & (((1u << kLook) - 1) * kEnt));
    uint32_t e = kEnt == 4 ? lds<uint32_t>(ea) : (uint32_t)lds<uint16_t>(ea);
    if constexpr (kEnt == 2) asm("" : "+v"(e));  // a 32-bit value from here (else the branch below compiles as an if / else on 16 bits)
    if (!e) {  // a code longer than kLook bits (rare): as SpanLane
      const uint32_t c16 = (__builtin_bitreverse32(r) >> (16 - kLead)) & 0xFFFFu;
      uint32_t len = kLook + 1, sym = 0;
#pragma unroll
      for (int i = 0; i < 7; ++i) len += c16 >= lds<uint32_t>(tb + (uint32_t)offsetof(Tab, lim) + 4u * i) ? 1u : 0u;
      if (len > 16) len = 16;
      else {
        const int32_t vo = lds<int32_t>(tb + (uint32_t)offsetof(Tab, valoff) + 4u * len);
        sym = lds<uint8_t>(tb + (uint32_t)offsetof(Tab, vals) + ((uint32_t)((int32_t)(c16 >> (16 - len)) + vo) & 255u));
      }
      uint32_t extra, adv;
      if (z == 0) {
        extra = sym > 16 ? 16 : sym;
        adv = 1;
      } else {
        extra = sym & 15;
        adv = extra ? (sym >> 4) + 1 : ((sym >> 4) == 15 ? 16 : 64);
      }
      e = (adv << 8) | (len + extra);
      if constexpr (PAIRS) e |= e << 16;  // no pair
    }
    if constexpr (PAIRS) {
      const uint32_t Q1 = Q + (e & 0xFF);
      const uint32_t z1 = z + ((e >> 8) & 0xFF);
      const bool two = z1 < 64 && Q1 < Qs;  // (advance << 24) | (length << 16): both symbols, or the first again
      Q = two ? Q + ((e >> 16) & 0xFF) : Q1;
      z = two ? z + (e >> 24) : z1;
    } else {
      Q += e & 0xFF;
      z += (e >> 8) & 0xFF;
    }
    const bool eob = z >= 64;
    z = eob ? 0u : z;
    n += eob ? 1u : 0u;
    tb = __builtin_amdgcn_ubfe(cpl, SB * n, SB) * (uint32_t)sizeof(Tab) + (eob ? dc0 : ac0);
  }
};
using SpanLaneR = SpanLaneRT<SyncTab32, 2, 1, true>;

template <bool REV = false>  // REV: fast entries at bit-reversed indices (SpanLaneRT)
__device__ __forceinline__ void load_sync_tables(const DecTabs &F, HuffSync *tabs) {
  const uint32_t *src = reinterpret_cast<const uint32_t *>(&F.sdc[0]);
  uint32_t *dst = reinterpret_cast<uint32_t *>(tabs);
  constexpr uint32_t nw = 6 * sizeof(HuffSync) / 4;
  for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) dst[j] = src[j];
  if constexpr (REV) {
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < 6 * (1u << kLook); j += blockDim.x) {
      const uint32_t t = j >> kLook, i = j & ((1u << kLook) - 1);
      tabs[t].sfast[__builtin_bitreverse32(i) >> (32 - kLook)] = (t < 3 ? F.sdc[t] : F.sac[t - 3]).sfast[i];
    }
  }
  __syncthreads();
}

// Checkpoints: kCk marks inside each subsequence, every kCkStep bits.  A decode records its
// state (bit position, zigzag index, block-in-MCU) at the first symbol boundary at or past
// each mark, and the number of blocks that trajectory completes from there to the
// subsequence's end.  A later decode of the same subsequence from another entry that reaches
// a mark in a recorded state has joined the recorded trajectory: its exit is the recorded
// exit and its block count is its count so far plus the recorded remainder, so it stops
// there.  The codes self-synchronise within a few symbols, so a re-decode usually stops at
// the first mark.  Invariant: every valid checkpoint and the exit state describe one
// trajectory (marks a decode did not reach from its entry are invalidated).

constexpr uint64_t kNoCk = ~0ull;
constexpr uint32_t kSpecPadWords = 16;  // staged words past a workgroup's range: overshoot + lookahead
// the write pass's CHUNKS form decodes on to the end of a block begun in its span: one block
// is at most 64 codes of 16 bits + 15 extra bits (and the DC's), 2,000 bits
constexpr uint32_t kBlockPadWords = 64;

// One sync pass.  Every thread decodes its subsequence from its entry state; then, inside
// the workgroup, a thread whose entry differs from its predecessor's current exit takes that
// exit and decodes again (up to the first checkpoint where it rejoins its previous decode),
// until the workgroup is consistent.  Across workgroups the entry of a workgroup's first
// thread is the previous pass's exit of its predecessor; a pass that changes no exit state
// means the whole chain is consistent, and its counts were made from the final entry states.
__global__ __launch_bounds__(256) void k_sync(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, const uint8_t *us, const uint32_t *us_len,
                                              const uint64_t *exit_in, uint64_t *exit_out, const uint32_t *cnt_in,
                                              uint32_t *cnt_out, uint64_t *used, uint64_t *ck, uint32_t *ckrem,
                                              uint32_t *changed, int pass) {
  __shared__ HuffSync tabs[6];
  __shared__ uint64_t s_exit[256];
  __shared__ uint64_t s_ck[kCk][256];
  __shared__ uint32_t s_rem[kCk][256];
  const DecSeg S = sg[blockIdx.y];  // by value: held in scalar registers
  const DecFrame &F = fr[S.frame];
  if (blockIdx.x * 256 >= S.nsub_max) return;
  load_sync_tables(tabs_of(fr, F), tabs);
  const HuffGeom hg(F.g);
  const uint32_t t = threadIdx.x;
  const uint32_t i = blockIdx.x * 256 + t;
  const uint32_t gi = S.sub0 + i;
  const uint32_t nbits = us_len[blockIdx.y] * 8u;
  const uint32_t nsub = (nbits + kSubBits - 1) / kSubBits;
  const bool live = i < nsub;
  const uint32_t base = i * kSubBits;
  const uint32_t end = (i + 1 >= nsub) ? nbits : (i + 1) * kSubBits;
  uint64_t entry = 0, ex = pack_state(nbits, 0, 0);
  uint32_t cnt = 0;
  bool need = false, decoded = false;
  if (live) {
    if (i == 0) entry = 0;
    else if (pass == 0) entry = pack_state(base, 0, 0);
    else entry = exit_in[gi - 1];
#pragma unroll
    for (int m = 0; m < kCk; ++m) {
      s_ck[m][t] = pass > 0 ? ck[(uint64_t)gi * kCk + m] : kNoCk;
      s_rem[m][t] = pass > 0 ? ckrem[(uint64_t)gi * kCk + m] : 0u;
    }
    if (pass > 0) {
      ex = exit_in[gi];
      cnt = cnt_in[gi];
      need = entry != used[gi];  // same entry as last pass: same result
    } else {
      need = true;
    }
  }
  for (;;) {
    if (need) {
      decoded = true;
      BitReader br;
      br.init(us + S.us_off, (uint32_t)(entry >> 16));
      uint32_t z = (entry >> 8) & 0xFF, c = entry & 0xFF, n = 0;
      int m = 0;
      while (m < kCk && base + (uint32_t)(m + 1) * kCkStep <= br.pos) s_ck[m++][t] = kNoCk;
      const int m0 = m;
      int joined = -1;
      while (br.pos < end) {
        sync_step(br, z, c, n, hg, tabs, tabs + 3);
        const uint32_t mk = base + (uint32_t)(m + 1) * kCkStep;
        if (m < kCk && mk < end && br.pos >= mk) {
          const uint64_t st = pack_state(br.pos, z, c);
          if (s_ck[m][t] == st) {
            joined = m;
            break;
          }
          s_ck[m][t] = st;
          s_rem[m][t] = n;  // blocks so far; turned into the remainder below
          ++m;
        }
      }
      if (joined >= 0) {
        cnt = n + s_rem[joined][t];  // ex: the recorded trajectory's exit, unchanged
      } else {
        cnt = n;
        ex = pack_state(br.pos, z, c);
      }
      for (int q = m0; q < m; ++q) s_rem[q][t] = cnt - s_rem[q][t];
    }
    s_exit[t] = ex;
    __syncthreads();
    need = false;
    if (live && t > 0) {
      const uint64_t e = s_exit[t - 1];
      if (e != entry) {
        entry = e;
        need = true;
      }
    }
    if (!__syncthreads_or(need)) break;  // also orders the s_exit reads before the next writes
  }
  if (i < S.nsub_max) {
    exit_out[gi] = ex;
    cnt_out[gi] = cnt;
    if (live) {
      used[gi] = entry;
      if (decoded) {
#pragma unroll
        for (int m = 0; m < kCk; ++m) {
          ck[(uint64_t)gi * kCk + m] = s_ck[m][t];
          ckrem[(uint64_t)gi * kCk + m] = s_rem[m][t];
        }
      }
      if (pass == 0 || ex != exit_in[gi]) atomicOr(changed, 1u);
    }
  }
}

// ---- decoder: pass-based sync over spans of G subsequences ---------------------------------
//
// k_sync's chains re-decode every thread whose entry changed, one subsequence per round: on
// content whose codes resynchronise slowly (noise at q95: the state (pos, z, c) rejoins after
// ~900 bits at the median, 5.5k at p99, tools/sync_distance.py), a workgroup needs ~25 rounds
// and decodes its stream ~5 times per pass (tools/sync_sim.py).  Here a thread decodes G
// consecutive subsequences as one trajectory (the records per subsequence -- checkpoints,
// exit, block count -- are those k_sync writes, so the write pass is unchanged): with G = 4 a
// guessed entry has 4x the bits to resynchronise in, and the simulation gives ~6 rounds and ~2.1
// decodes of the stream per pass.  The records live in global memory and are updated in place;
// a re-decode compares each mark's state with the recorded one (prefetched one mark ahead) and
// stops where it rejoins.  Passes are queued without host round trips: a pass reads the
// previous pass's flag and returns at once when no workgroup's last exit changed (then every
// entry is consistent: within a workgroup by its rounds, across by the unchanged exits).

// Re-decode (or first decode, CHECK = false) of a thread's span from entry state X; returns the
// span's last exit.  `last` is the previous decode's last exit (returned unchanged on a join).
// A re-decode reads each mark's recorded state one mark ahead; that load is issued before the
// current mark's record stores, because vmcnt counts stores too: loaded after them, the wait for
// it at the next mark also waited for the stores' completion, every 64 bits.  The first decode
// (no records yet) has no loads in its loop at all.
template <bool CHECK, uint32_t NDC, bool LSB = false>
__device__ __forceinline__ uint64_t sync_span(const uint32_t *words, uint32_t wb32, uint64_t X, uint32_t i0, uint32_t ng,
                                              uint32_t nsub, uint32_t nbits, uint64_t gi0, uint64_t last,
                                              uint64_t *exits, uint32_t *cnts, uint64_t *ck, uint32_t *ckrem,
                                              const HuffGeom &hg, const SyncTab32 *tabs) {
  std::conditional_t<LSB, SpanLaneR, SpanLane<SyncTab32, NDC>> d;
  if constexpr (LSB) d.init(words, wb32, X, hg.pat, hg.bpm, tabs);
  else d.init(words, wb32, X, hg);
  uint32_t j = 0, bj = i0 * kSubBits;
  uint32_t ej = i0 + 1 >= nsub ? nbits : bj + kSubBits;  // end of subsequence j
  // next mark of subsequence j: checkpoint m < kCk at bj + (m + 1) * kCkStep (if inside it), or
  // m == kCk: its end.  An entry lies less than one symbol (<= 32 bits) past bj, before mark 0.
  uint32_t m = bj + kCkStep < ej ? 0u : (uint32_t)kCk;
  uint32_t mk = m < kCk ? bj + kCkStep : ej;
  uint64_t old = CHECK ? (m < kCk ? ck[gi0 * kCk] : exits[gi0]) : 0;
  uint32_t n0 = 0, n1 = 0, n2 = 0;  // blocks at the checkpoints written in this decode
  static_assert(kCk == 3, "n0..n2");
  for (;;) {
    d.run(tabs, mk);
    const uint64_t st = d.state();
    const uint64_t gj = gi0 + j;
    const bool joined = CHECK && old == st;
    // the mark after this one (j2, m2 at mk2)
    const bool send = m >= kCk;  // this mark ends subsequence j
    const uint32_t j2 = send ? j + 1 : j, bj2 = send ? bj + kSubBits : bj;
    const uint32_t ej2 = send ? (i0 + j2 + 1 >= nsub ? nbits : bj2 + kSubBits) : ej;
    uint32_t m2 = send ? (bj2 + kCkStep >= ej2 ? (uint32_t)kCk : 0u) : m + 1;
    uint32_t mk2 = m2 < kCk ? bj2 + (m2 + 1) * kCkStep : ej2;
    if (m2 < kCk && mk2 >= ej2) {
      m2 = kCk;
      mk2 = ej2;
    }
    if (CHECK && !joined && !(send && j2 == ng))  // prefetch, ahead of this mark's stores
      old = m2 < kCk ? ck[(gi0 + j2) * kCk + m2] : exits[gi0 + j2];
    if (!send) {
      if (joined) {  // rejoined: the rest of the span is the recorded trajectory
        const uint32_t cj = d.n + ckrem[gj * kCk + m];
        cnts[gj] = cj;
        if (m > 0) ckrem[gj * kCk] = cj - n0;
        if (m > 1) ckrem[gj * kCk + 1] = cj - n1;
        return last;
      }
      ck[gj * kCk + m] = st;
      n2 = m == 2 ? d.n : n2;
      n1 = m == 1 ? d.n : n1;
      n0 = m == 0 ? d.n : n0;
    } else {
      const uint32_t nw = bj + kCkStep < ej ? (bj + 2 * kCkStep < ej ? (bj + 3 * kCkStep < ej ? 3u : 2u) : 1u) : 0u;
      cnts[gj] = d.n;
      if (nw > 0) ckrem[gj * kCk] = d.n - n0;
      if (nw > 1) ckrem[gj * kCk + 1] = d.n - n1;
      if (nw > 2) ckrem[gj * kCk + 2] = d.n - n2;
      if (joined) return last;  // the exit, and every later subsequence, unchanged
      exits[gj] = st;
      for (uint32_t q = nw; q < (uint32_t)kCk; ++q) ck[gj * kCk + q] = kNoCk;  // marks past the segment's end
      if (j2 == ng) return st;
      if constexpr (LSB) d.restart_count();
      else d.n = 0;
    }
    j = j2;
    bj = bj2;
    ej = ej2;
    m = m2;
    mk = mk2;
  }
}

// T threads per workgroup, T * G subsequences: the workgroup's stream words (40 KB at most) are
// staged in LDS first, byte-swapped for SpanLane, so a step's words are an LDS read (global
// loads exposed their latency every few symbols: ~500-700 shader cycles per symbol on an idle
// GPU, counted with tools/build_syncg_stats.sh; unstaged, at twice the occupancy, a pass took
// 2.4x as long).
constexpr uint32_t syncg_threads(int G) { return G <= 5 ? 256u : 1024u / (uint32_t)G; }
// Pass 0's guessed entries can be warmed: a thread first decodes the `warm` bits before its span
// from a guessed state (nothing recorded), so its entry is the state at the first symbol boundary
// at or past the span's start, usually the true one already (tools/sync_sim.py --warm).
constexpr uint32_t kSyncWarmMax = 4096;
template <int G, uint32_t NDC, bool LSB = false>  // NDC 3: six tables (one per component); 2: DecFrame::tabs4's four
__global__ __launch_bounds__(256) void k_syncg(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, const uint8_t *us,
                                               const uint32_t *us_len, uint64_t *exits, uint32_t *cnts, uint64_t *used,
                                               uint64_t *ck, uint32_t *ckrem, uint32_t *changed, int pass, uint32_t warm) {
  constexpr uint32_t kWarmWords = kSyncWarmMax / 32;
  constexpr uint32_t T = syncg_threads(G), kWords = 1 + kWarmWords + T * G * (kSubBits / 32) + kSpecPadWords;
  __shared__ SyncTab32 tabs[2 * NDC];
  // exits relative to the workgroup's first bit in 32 bits, (pos - wbit) << 10 | z << 4 | c (as
  // k_spec's): 1 KB less LDS, which with G = 3 makes 4 workgroups per CU fit (40.7 KB)
  __shared__ uint32_t s_exit[T];
  __shared__ uint32_t s_w[kWords];
  const DecSeg S = sg[blockIdx.y];  // by value: held in scalar registers
  const DecFrame &F = fr[S.frame];
  if (blockIdx.x * T * G >= S.nsub_max) return;
  const uint32_t wbit = blockIdx.x * T * G * kSubBits;
  const auto rel = [wbit](uint64_t st) {
    return (((uint32_t)(st >> 16) - wbit) << 10) | (((uint32_t)st >> 4) & 0x3F0u) | ((uint32_t)st & 15u);
  };
  const auto absl = [wbit](uint32_t r) { return pack_state((r >> 10) + wbit, (r >> 4) & 63u, r & 15u); };
  if (pass > 0 && changed[pass - 1] == 0) return;  // converged (workgroup-uniform)
  const uint32_t *gw = reinterpret_cast<const uint32_t *>(us + S.us_off);
  // staged from kWarmWords + 1 before the workgroup's first span (the warm-up of its first
  // thread, and the word before it: SpanLane reads the word of bit pos-1); words before the
  // segment's start read as 0 and are never decoded
  const int32_t wbase = (int32_t)(blockIdx.x * T * G * (kSubBits / 32)) - (int32_t)kWarmWords - 1;
  const uint32_t wb32 = (uint32_t)wbase * 32u;  // modular: s_w[i] holds word wbase + i
  {
    const uint32_t fwords = (((S.in_len + 64) + 15) & ~15u) / 4;
    for (uint32_t i = threadIdx.x; i < kWords; i += T) {
      const int32_t gwi = wbase + (int32_t)i;
      const uint32_t v = gwi >= 0 && (uint32_t)gwi < fwords ? gw[gwi] : 0u;
      s_w[i] = LSB ? bswap32(__builtin_bitreverse32(v)) : bswap32(v);  // LSB-first / byte-swapped
    }
  }
  if constexpr (NDC == 2) load_sync_tabs4<LSB>(tabs_of(fr, F), F.tabs4, tabs);  // its barrier also publishes s_w
  else load_sync_tabs32(tabs_of(fr, F), tabs);
  HuffGeom hg(F.g);
  if constexpr (NDC == 2) hg.cpack = tabs4_cpack(hg, F.tabs4);
  if constexpr (LSB) {
    static_assert(NDC == 2, "SpanLaneR: DecFrame::tabs4's two slots");
    for (uint32_t j = 0, c = 0; j < 32; ++j, c = c + 1 == hg.bpm ? 0u : c + 1) hg.pat |= ((hg.cpack >> (2 * c)) & 1u) << j;
  }
  const uint32_t t = threadIdx.x;
  const uint32_t nbits = us_len[blockIdx.y] * 8u, nsub = (nbits + kSubBits - 1) / kSubBits;
  const uint32_t i0 = (blockIdx.x * T + t) * G;
  const bool live = i0 < nsub;
  const uint32_t ng = live ? min((uint32_t)G, nsub - i0) : 0u;
  const uint64_t gi0 = S.sub0 + i0;
  uint64_t entry = 0, last = 0, last_old = 0;
  bool need = false;
  if (live) {
    if (pass == 0) {
      entry = i0 == 0 ? 0 : pack_state(i0 * kSubBits, 0, 0);  // a guess, except at the segment's start
      if (i0 > 0 && warm > 0) {
        const uint32_t b = i0 * kSubBits, w0 = b > warm ? b - warm : 0u;
        std::conditional_t<LSB, SpanLaneR, SpanLane<SyncTab32, NDC>> d;
        if constexpr (LSB) d.init(s_w, wb32, pack_state(w0, 0, 0), hg.pat, hg.bpm, tabs);
        else d.init(s_w, wb32, pack_state(w0, 0, 0), hg);
        d.run(tabs, b);
        entry = d.state();
      }
      need = true;
    } else {
      entry = t == 0 ? (i0 == 0 ? 0 : exits[gi0 - 1]) : used[gi0];
      last = exits[gi0 + ng - 1];
      need = t == 0 && entry != used[gi0];
    }
  }
  last_old = last;
  bool check = pass > 0;  // records are valid from the first decode on
  for (;;) {
    if (need) {
      last = check ? sync_span<true, NDC, LSB>(s_w, wb32, entry, i0, ng, nsub, nbits, gi0, last, exits, cnts, ck, ckrem, hg, tabs)
                   : sync_span<false, NDC, LSB>(s_w, wb32, entry, i0, ng, nsub, nbits, gi0, last, exits, cnts, ck, ckrem, hg, tabs);
      used[gi0] = entry;
    }
    s_exit[t] = live ? rel(last) : 0u;
    __syncthreads();
    need = false;
    if (live && t > 0) {
      const uint64_t e = absl(s_exit[t - 1]);
      if (e != entry) {
        entry = e;
        need = true;
      }
    }
    check = true;
    if (!__syncthreads_or(need)) break;  // also orders the s_exit reads before the next writes
  }
  if (t == T - 1 && live && i0 + G < nsub && (pass == 0 || last != last_old)) atomicOr(changed + pass, 1u);
}

// ---- decoder: speculative Huffman synchronisation ------------------------------------------
//
// The pass-based k_sync above needs a re-decode chain whenever a guessed entry state has the
// wrong block-in-MCU c: bit positions and zigzag indices resynchronise within a few symbols,
// but a wrong c selects the other component's tables and tends to survive, so corrections
// travel one subsequence per round.  Here:
//   k_spec    every subsequence is decoded from each possible c (bpm trajectories, one lane
//             each: the extra work fills otherwise idle waves), checkpoints recorded; each
//             trajectory of subsequence k-1 is linked to the trajectory of k its exit state
//             rejoins (a short decode to the first matching checkpoint).  Then one lane per
//             entry index e walks the workgroup: trajectory e of the first subsequence, the
//             links after it, and, where a link rejoined nothing, an explicit state decoded
//             on (the walker links it into the next subsequence itself).  Neighbouring
//             workgroups overlap by one subsequence (workgroup w's first is w-1's last, decoded
//             from the same entry states, so its trajectory j IS w-1's last trajectory j): the
//             link across a workgroup boundary is an ordinary in-workgroup link, made in k_spec.
//   k_resolve one workgroup per frame follows the true path across workgroups: walk column
//             e of w-1 ends at trajectory j = wF[e] of the shared subsequence, which is walk
//             column j of w.  Where a walk ended in an explicit state (its last link rejoined
//             nothing), the state is traced on through w first, all such traces of a frame in
//             parallel, until it rejoins a trajectory some walk column passes through (prefix
//             records for the subsequences before that point).
//   k_finalize writes exit state and block count per subsequence for the write pass (a
//             shared subsequence from its first workgroup).
// Only a frame too long for k_resolve's tables, or a stream that never rejoins (corrupt
// data), is reported unresolved; the caller then runs k_sync.

__device__ __forceinline__ uint32_t nib(uint64_t row, uint32_t i) { return (uint32_t)(row >> (4 * i)) & 0xF; }
__device__ __forceinline__ uint32_t spec_lanes(uint32_t bpm) {
  return bpm <= 1 ? 1u : bpm <= 2 ? 2u : bpm <= 4 ? 4u : bpm <= 8 ? 8u : 16u;
}
constexpr uint32_t kSpecWords = 256 * (kSubBits / 32) + kSpecPadWords;  // NS <= 256 subsequences
// maps of <= 16 entries packed as nibbles: (later o earlier)(e); entries >= bpm are absorbing
__device__ __forceinline__ uint64_t map_compose(uint64_t later, uint64_t earlier, uint32_t bpm) {
  uint64_t r = 0;
  for (uint32_t q = 0; q < bpm; ++q) {
    const uint32_t a = nib(earlier, q);
    r |= (uint64_t)(a < bpm ? nib(later, a) : a) << (4 * q);
  }
  return r;
}
constexpr uint8_t kLinkNone = 0xF;  // rejoined no trajectory (explicit state follows)
constexpr uint8_t kLinkLast = 0xE;  // the frame's last subsequence: decoded to the end

// Decode from state X through subsequence [base, end); at each mark compare with the
// checkpoints of trajectories 0..bpm-1 (ck(c, m), rem(c, m)), and at the end with their exit
// states (ex(c)).  Returns the trajectory joined, or kLinkNone with *endst = the state at the
// first symbol boundary at/after `end`, or kLinkLast (the frame's last subsequence, decoded to
// its end).  *count = blocks completed in the subsequence along this path.
// k_spec's lanes: SpanLane, or on LSB-first words the six-table SpanLaneRT (2-bit component slots)
template <bool LSB>
using SpecLane = std::conditional_t<LSB, SpanLaneRT<HuffSync, 3, 2, false>, SpanLane<HuffSync, 3, false>>;
template <bool LSB>
__device__ __forceinline__ void spec_lane_init(SpecLane<LSB> &d, const uint32_t *words, uint32_t wb32, uint64_t X,
                                               const HuffGeom &hg, const HuffSync *tabs) {
  if constexpr (LSB) d.init(words, wb32, X, hg.pat, hg.bpm, tabs);
  else d.init(words, wb32, X, hg);
}

template <bool LSB, typename CK, typename REM, typename EX>
__device__ __forceinline__ uint32_t spec_link(const uint32_t *words, uint32_t wb32, uint64_t X, uint32_t base,
                                              uint32_t end, bool last, const HuffGeom &hg, const HuffSync *tabs, CK ck,
                                              REM rem, EX ex, uint32_t *count, uint64_t *endst) {
  SpecLane<LSB> d;
  spec_lane_init<LSB>(d, words, wb32, X, hg, tabs);
  uint32_t m = 0;
  while (m < kCk && base + (m + 1) * kCkStep <= d.pos()) ++m;
  for (;;) {  // decode to the next mark (a checkpoint inside the subsequence) or to its end
    const uint32_t mk = base + (m + 1) * kCkStep;
    const bool cm = !last && m < kCk && mk < end;
    const uint32_t stop = cm ? mk : end;
    d.run(tabs, stop);
    if (!cm) break;
    const uint64_t st = d.state();
    for (uint32_t c2 = 0; c2 < hg.bpm; ++c2)
      if (ck(c2, m) == st) {
        *count = d.n + rem(c2, m);
        return c2;
      }
    ++m;
  }
  *count = d.n;
  *endst = d.state();
  if (last) return kLinkLast;
#ifndef VF_SPEC_ENDJOIN
#define VF_SPEC_ENDJOIN 1
#endif
  if (!VF_SPEC_ENDJOIN) return kLinkNone;  // A/B builds only
  // past the last mark the path may still have met a trajectory: the same state at the same
  // boundary after `end` is the same path from there on
  for (uint32_t c2 = 0; c2 < hg.bpm; ++c2)
    if (ex(c2) == *endst) return c2;
  return kLinkNone;
}

template <bool LSB>  // LSB: every frame's blocks per MCU divide 16 (SpanLaneRT on LSB-first words)
__global__ __launch_bounds__(256) void k_spec(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, const uint8_t *us, const uint32_t *us_len,
                                              SpecBufs B) {
  // States here are kept relative to the workgroup's first bit in 32 bits (rel / absl below),
  // block counts in 16: 24.6 KB of LDS instead of 31.8, 6 workgroups per CU instead of 5 (the
  // decodes are latency-bound chains: the resident ones are what counts)
  __shared__ HuffSync tabs[6];
  __shared__ uint32_t s_ck[kCk][256];
  __shared__ uint16_t s_rem[kCk][256];
  __shared__ uint32_t s_E[256];
  __shared__ uint32_t s_X[256];
  __shared__ uint16_t s_C[256];
  __shared__ uint8_t s_M[256];
  __shared__ uint32_t s_w[1 + kSpecWords];
  const DecSeg S = sg[blockIdx.y];  // by value: held in scalar registers
  const DecFrame &F = fr[S.frame];
  if (blockIdx.x >= S.nwg) return;
  HuffGeom hg(F.g);
  if constexpr (LSB)  // 2-bit component of block-in-MCU (j mod bpm) at bits 2j, 2j + 1
    for (uint32_t j = 0, c = 0; j < 16; ++j, c = c + 1 == hg.bpm ? 0u : c + 1) hg.pat |= hg.comp(c) << (2 * j);
  const uint32_t L = spec_lanes(hg.bpm), NS = 256 / L, NSS = NS - 1;  // rows, rows not shared with w+1
  const uint32_t t = threadIdx.x, sl = t / L, c0 = t % L;
  const uint32_t s = blockIdx.x * NSS + sl;
  const uint32_t nbits = us_len[blockIdx.y] * 8u, nsub = (nbits + kSubBits - 1) / kSubBits;
  if (blockIdx.x > 0 && blockIdx.x * NSS + 1 >= nsub) return;  // workgroup-uniform: owns no subsequence
  const bool live = c0 < hg.bpm && s < nsub;
  const uint32_t base = s * kSubBits, end = (s + 1 >= nsub) ? nbits : (s + 1) * kSubBits;
  const uint64_t g0 = S.tr0 + (uint64_t)blockIdx.x * 256, ti = g0 + t;
  // the workgroup's stream words (every decode here stays within them, plus overshoot and
  // lookahead), from the frame's padded unstuffed region, byte-swapped for SpanLane from the
  // word before the first (s_w[i] is word woff - 1 + i: SpanLane reads the word of bit pos-1)
  const uint32_t woff = blockIdx.x * NSS * (kSubBits / 32);
  const uint32_t wb32 = (woff - 1u) * 32u;  // modular
  const uint32_t fwords = (((S.in_len + 64) + 15) & ~15u) / 4;
  const uint32_t *gw = reinterpret_cast<const uint32_t *>(us + S.us_off);
  for (uint32_t i = t; i < 1 + NS * (kSubBits / 32) + kSpecPadWords; i += 256) {
    const uint32_t v = woff - 1u + i < fwords ? gw[woff - 1u + i] : 0u;
    s_w[i] = LSB ? bswap32(__builtin_bitreverse32(v)) : bswap32(v);  // LSB-first / byte-swapped
  }
  load_sync_tables<LSB>(tabs_of(fr, F), tabs);  // its barrier also publishes s_w
#ifndef VF_SPEC_PHASES
#define VF_SPEC_PHASES 0
#endif
  // VF_SPEC_PHASES (exp builds; VF_JPEG_SYNC_STATS prints them): wall-clock ticks / 1024 summed
  // over workgroups from here to the end of part A, of part B, and per walker to the end of its
  // serial continuation; with per-row counters, so timing only
  const uint64_t ph0 = VF_SPEC_PHASES ? wall_clock64() : 0;
  // pack_state's (pos << 16 | z << 8 | c) as (pos - the workgroup's first bit) << 10 | z << 4 | c
  // (a workgroup spans at most 256 subsequences, 2^16 bits, plus a symbol's overshoot; z < 64,
  // c < 10), and back; the 32-bit kNoCk (0xFFFFFFFF) reads back with c = 15, which no decode has
  const uint32_t wbit = woff * 32u;
  const auto rel = [wbit](uint64_t st) {
    return (((uint32_t)(st >> 16) - wbit) << 10) | (((uint32_t)st >> 4) & 0x3F0u) | ((uint32_t)st & 15u);
  };
  const auto absl = [wbit](uint32_t r) {
    return pack_state((r >> 10) + wbit, (r >> 4) & 63u, r & 15u);
  };
  // A: the trajectory of subsequence s from (base, z = 0, c = c0), checkpoints recorded
  uint64_t E = 0;
  uint32_t N = 0;
#pragma unroll
  for (int m = 0; m < kCk; ++m) s_ck[m][t] = 0xFFFFFFFFu;
  if (live) {
    SpecLane<LSB> d;
    spec_lane_init<LSB>(d, s_w, wb32, pack_state(base, 0, c0), hg, tabs);
    uint32_t m = 0;
    for (;;) {  // decode to the next checkpoint mark inside the subsequence, or to its end
      const uint32_t mk = base + (m + 1) * kCkStep;
      const bool cm = m < kCk && mk < end;
      const uint32_t stop = cm ? mk : end;
      d.run(tabs, stop);
      if (!cm) break;
      s_ck[m][t] = rel(d.state());
      s_rem[m][t] = (uint16_t)d.n;
      ++m;
    }
    for (uint32_t q = 0; q < m; ++q) s_rem[q][t] = (uint16_t)(d.n - s_rem[q][t]);
    E = d.state();
    N = d.n;
  }
  s_E[t] = live ? rel(E) : 0u;
  __syncthreads();
  if (live) B.tE[ti] = E;
  if (VF_SPEC_PHASES && t == 0) atomicAdd(B.stats + 8, (uint32_t)((wall_clock64() - ph0) >> 10));
  // B: link trajectory c0 of s-1 into s
  uint32_t M = kLinkNone, C = N;
  uint64_t X = 0;
  if (live && sl > 0) {
    const uint32_t row = sl * L;
    M = spec_link<LSB>(s_w, wb32, absl(s_E[(sl - 1) * L + c0]), base, end, s + 1 == nsub, hg, tabs,
                  [&](uint32_t c2, int m) { return absl(s_ck[m][row + c2]); },
                  [&](uint32_t c2, int m) { return (uint32_t)s_rem[m][row + c2]; },
                  [&](uint32_t c2) { return absl(s_E[row + c2]); }, &C, &X);
  }
  s_M[t] = (uint8_t)M;
  s_C[t] = (uint16_t)C;
  s_X[t] = live && sl > 0 && M >= hg.bpm ? rel(X) : 0u;  // an explicit or the frame's last end state
  __syncthreads();
  if (VF_SPEC_PHASES && t == 0) atomicAdd(B.stats + 9, (uint32_t)((wall_clock64() - ph0) >> 10));
  // C: the walks.  Walk e is trajectory e of the first subsequence followed through the links:
  // j_k = f_k(j_{k-1}), f_k(j) = s_M[k * L + j].  While every step is a link (no explicit
  // state), j_k = (f_k o ... o f_1)(e), and map composition is associative, so one lane per
  // subsequence gets every walk's trajectory there from a prefix scan of the link maps (maps
  // of <= 16 entries packed as nibbles; kLinkNone and kLinkLast are absorbing).  A walk that
  // reaches an explicit state (a link that rejoined nothing, rare) continues serially from
  // there, decoding as before.
  const uint32_t nk = blockIdx.x * NSS < nsub ? min(NS, nsub - blockIdx.x * NSS) : 0u;  // subsequences here
  if (nk == 0) return;  // workgroup-uniform
  const uint32_t bpm = hg.bpm;
  auto compose = [bpm](uint64_t later, uint64_t earlier) { return map_compose(later, earlier, bpm); };
  uint64_t ident = 0;
  for (uint32_t q = 0; q < bpm; ++q) ident |= (uint64_t)q << (4 * q);
  uint64_t f = ident;
  if (t > 0 && t < nk) {
    f = 0;
    for (uint32_t q = 0; q < bpm; ++q) f |= (uint64_t)(s_M[t * L + q] & 0xF) << (4 * q);
  }
  const uint32_t lane = t & 63, wv = t >> 6;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(f, d, 64);
    if (lane >= d) f = compose(f, o);
  }
  __shared__ uint64_t s_wt[4];
  __shared__ uint64_t s_fst[kSpecLanesMax];
  __shared__ uint32_t s_first[kSpecLanesMax];
  if (lane == 63) s_wt[wv] = f;
  if (t < kSpecLanesMax) s_first[t] = 0;
  __syncthreads();
  uint64_t pre = ident;  // the maps of the waves before this one
  for (uint32_t q = 0; q < wv; ++q) pre = compose(s_wt[q], pre);
  f = compose(f, pre);
  uint64_t gp = __shfl_up(f, 1, 64);  // G_{t-1}
  if (lane == 0) gp = pre;
  if (t < nk) {
    if (t == 0) {
      for (uint32_t q = 0; q < bpm; ++q) {
        B.tX[g0 + q] = absl(s_E[q]);
        B.tXc[g0 + q] = s_C[q];  // trajectory count (used for the frame's first subsequence)
      }
    } else {
      for (uint32_t q = 0; q < bpm; ++q) {
        const uint32_t p = nib(gp, q);
        if (p >= bpm) continue;  // stopped (last) or explicit (the serial walk below)
        const uint32_t M2 = s_M[t * L + p];
        const uint64_t st = absl(M2 < bpm ? s_E[t * L + M2] : s_X[t * L + p]);
        B.tX[g0 + t * L + q] = st;
        B.tXc[g0 + t * L + q] = s_C[t * L + p];
        if (M2 == kLinkNone) {  // walk q turns explicit here: its serial continuation starts at t + 1
          s_first[q] = t;
          s_fst[q] = st;
        }
      }
    }
    if (t == nk - 1)
      for (uint32_t q = 0; q < bpm; ++q) {
        const uint32_t j = nib(f, q);
        if (j != kLinkNone) B.wF[(uint64_t)(S.wg0 + blockIdx.x) * kSpecLanesMax + q] = (uint8_t)(j < bpm ? j : kLinkNone);
      }
  }
  __syncthreads();
  // serial continuations, walkers 256 / L lanes apart so their divergent decodes run in
  // different waves where possible
  const uint32_t wsp = 256 / L, e = t / wsp;
#ifndef VF_SPEC_NOSERIAL
#define VF_SPEC_NOSERIAL 0  // timing-only builds: skip the serial continuations (outputs wrong)
#endif
  if (!VF_SPEC_NOSERIAL && t % wsp == 0 && e < bpm && s_first[e] != 0) {
    uint32_t j = kLinkNone;  // current trajectory, or kLinkNone while explicit
    uint64_t st = s_fst[e];
    for (uint32_t k = s_first[e] + 1; k < nk; ++k) {
      const uint32_t sk = blockIdx.x * NSS + k;
      uint32_t cnt, M2;
      uint64_t xe = 0;
      if (j < hg.bpm) {
        M2 = s_M[k * L + j];
        cnt = s_C[k * L + j];
        xe = absl(s_X[k * L + j]);
      } else {  // explicit state: link it into subsequence k here
        if (VF_SPEC_PHASES) atomicAdd(B.stats + 2, 1u);  // explicit rows decoded by walkers
        const uint32_t bk = sk * kSubBits, ek = (sk + 1 >= nsub) ? nbits : (sk + 1) * kSubBits;
        const uint32_t row = k * L;
        M2 = spec_link<LSB>(s_w, wb32, st, bk, ek, sk + 1 == nsub, hg, tabs,
                       [&](uint32_t c2, int m) { return absl(s_ck[m][row + c2]); },
                       [&](uint32_t c2, int m) { return (uint32_t)s_rem[m][row + c2]; },
                       [&](uint32_t c2) { return absl(s_E[row + c2]); }, &cnt, &xe);
      }
      if (M2 < hg.bpm) {
        j = M2;
        st = absl(s_E[k * L + j]);
      } else {
        j = M2;  // kLinkNone (explicit) or kLinkLast
        st = xe;
      }
      B.tX[g0 + k * L + e] = st;
      B.tXc[g0 + k * L + e] = cnt;
      if (VF_SPEC_PHASES) atomicAdd(B.stats + 3, 1u);  // rows written by walkers
      if (j == kLinkLast) break;
    }
    if (j == kLinkNone && nk == NS && blockIdx.x * NSS + NS < nsub) {
      // the walk ended explicit: its decode through the next workgroup's row 1 (the subsequence
      // after this workgroup's last, still inside the staged words), for k_resolve's trace of
      // it (records in qX at that row, lane e)
      const uint32_t sk = blockIdx.x * NSS + NS;
      const uint32_t ek = (sk + 1 >= nsub) ? nbits : (sk + 1) * kSubBits;
      const uint32_t lim = min(ek, (woff + NS * (kSubBits / 32) + kSpecPadWords - 4) * 32u);  // binds only on corrupt data
      SpecLane<LSB> d;
      spec_lane_init<LSB>(d, s_w, wb32, st, hg, tabs);
      d.run(tabs, lim);
      B.qX[g0 + 256 + L + e] = d.state();  // slot (w + 1, row 1, lane e)
      B.qC[g0 + 256 + L + e] = d.n;
    }
    B.wF[(uint64_t)(S.wg0 + blockIdx.x) * kSpecLanesMax + e] = (uint8_t)(j < hg.bpm ? j : kLinkNone);
    if (VF_SPEC_PHASES) {
      atomicAdd(B.stats + 10, (uint32_t)((wall_clock64() - ph0) >> 10));
      atomicAdd(B.stats + 1, 1u);  // walkers that ran a serial continuation
    }
  }
}

// Where the speculative path meets an explicit state it must be traced: decoded on until its
// exit equals the exit of some walk column (tX) at a subsequence, after which it IS that
// column.  Which explicit states the true path can meet at workgroup w is known before the
// path is: the end state of a walk column of w-1 whose last link rejoined nothing (tX at
// w-1's last subsequence, wF = kLinkNone).  So k_resolve traces all of a frame's such states
// in parallel, one lane each, before its serial walk across the workgroups only picks the
// result of the one it meets (round 2: ~2 serial traces per 1080p frame were half of
// k_resolve's 68 us per batch).
constexpr uint32_t kResolveLds = 4096;  // workgroups per frame resolved here (else fallback)
constexpr uint32_t kTraceWords = kSubBits / 32 + 6;  // one subsequence + overshoot + lookahead
constexpr uint8_t kRecP = 0x80, kRecQ = 0xC0;  // rL: prefix records in pX / qX, lane = low 4 bits

// Decode from explicit state X through rows k0.. of workgroup w (row k = subsequence
// w * NSS + k; words staged per subsequence into the caller's `tw` row) until the exit equals
// walk column q's exit tX there (returns q, *kend = k), the frame ends (kLinkLast) or the
// workgroup does (kLinkNone, *kend = its last row).  Every row's exit and block count go to rX /
// rC at lane `lane`.
__device__ __forceinline__ uint32_t trace_on(const uint32_t *gw, uint32_t fwords, uint32_t *tw, uint64_t X,
                                             uint32_t w, uint32_t k0, uint32_t NS, uint32_t NSS, uint32_t L,
                                             uint32_t nsub, uint32_t nbits, uint64_t tr0, const HuffGeom &hg,
                                             const HuffSync *tabs, const uint64_t *tX, uint64_t *rX, uint32_t *rC,
                                             uint32_t lane, uint32_t *kend) {
  uint32_t k = k0;
  for (; k < NS && w * NSS + k < nsub; ++k) {
    const uint32_t sk = w * NSS + k;
    const uint32_t ek = (sk + 1 >= nsub) ? nbits : (sk + 1) * kSubBits;
    // the subsequence's words, fetched together (independent loads), then decoded from LDS
    const uint32_t w0 = (uint32_t)(X >> 16) >> 5;
    for (uint32_t q = 0; q < kTraceWords; ++q) tw[q] = w0 + q < fwords ? gw[w0 + q] : 0u;
    SyncLane<HuffSync> d;
    d.init(tw, w0, X, hg);
    const uint32_t lim = min(ek, (w0 + kTraceWords - 4) * 32u);  // stays inside tw (binds only on corrupt data)
    while (d.pos < lim) d.step(tabs, lim);
    X = pack_state(d.pos, d.z, d.c);
    const uint32_t n = d.n;
    const uint64_t at = tr0 + (uint64_t)w * 256 + k * L;
    rX[at + lane] = X;
    rC[at + lane] = n;
    *kend = k;
    if (sk + 1 == nsub) return kLinkLast;
    for (uint32_t c2 = 0; c2 < hg.bpm; ++c2)
      if (tX[at + c2] == X) return c2;  // the path is walk column c2 from here on
  }
  *kend = k ? k - 1 : 0;
  return kLinkNone;
}

// The true path across the workgroups of a frame (one workgroup per frame).  Per workgroup w
// it finds the walk column e* that is the path from row rK on; rows 1..rK-1 take prefix records
// (exit state, count) from pX or qX at lane rL & 15 (row 0 is w-1's last row, resolved there).
// Where the path enters w depends only on the walk column e it followed through w - 1: that
// column ended at trajectory j of the shared subsequence, which is w's walk column j; or it ended
// explicit, and its trace through w (made first, in parallel) says which column it rejoins.  So
// every workgroup's transition e -> (e*, rK, where the records are) is made in parallel (into
// LDS), and the serial walk across the frame is one LDS read per workgroup.  Lane 0 decodes only
// where the path crossed a whole workgroup in a trace without rejoining, into pX lane 0.
constexpr uint32_t kResolveT = 16384;  // transitions staged per frame (workgroups x bpm)
constexpr uint32_t kTrJoined = 1u << 24;  // the path leaves the workgroup as walk column e*
__device__ __forceinline__ uint32_t spec_nwg(uint32_t nsub, uint32_t NS) {  // workgroups owning a subsequence
  return nsub <= NS ? 1u : 1u + (nsub - NS + NS - 2) / (NS - 1);
}
__global__ __launch_bounds__(256) void k_resolve(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, const uint8_t *us, const uint32_t *us_len,
                                                 SpecBufs B, uint32_t *unresolved) {
  __shared__ uint32_t sT[kResolveT];  // [w * bpm + e]: e* | rK << 4 | code << 16 | kTrJoined
  __shared__ uint8_t sE[kResolveLds], sJ[kResolveLds];
  __shared__ uint16_t sK[kResolveLds];
  __shared__ HuffSync tabs[6];
  __shared__ uint32_t s_tw[256][kTraceWords];  // each tracing lane's staged words
  __shared__ uint16_t s_xl[kResolveT];           // (workgroup, walk column) pairs to trace
  __shared__ uint32_t s_nx, s_n1, s_abs;
  __shared__ uint64_t s_wt[4];
  const DecSeg S = sg[blockIdx.x];  // by value: held in scalar registers
  const DecFrame &F = fr[S.frame];
  const HuffGeom hg(F.g);
  const uint32_t bpm = hg.bpm, L = spec_lanes(bpm), NS = 256 / L, NSS = NS - 1;
  const uint32_t nbits = us_len[blockIdx.x] * 8u, nsub = (nbits + kSubBits - 1) / kSubBits;
  const uint32_t nwg = min(S.nwg, spec_nwg(nsub, NS));
  const bool over = nwg > kResolveLds || nwg * bpm > kResolveT;
  if (threadIdx.x == 0)  // every segment's flag, every decode (page-locked host memory)
    __hip_atomic_store(unresolved + blockIdx.x, over ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (over) return;
  const uint32_t lastk = NS - 1;  // every workgroup but the frame's last is full
  {  // the sync tables' copy; the barrier below publishes it
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&tabs_of(fr, F).sdc[0]);
    uint32_t *dst = reinterpret_cast<uint32_t *>(tabs);
    for (uint32_t j = threadIdx.x; j < 6 * sizeof(HuffSync) / 4; j += 256) dst[j] = src[j];
  }
  __syncthreads();
  auto slot = [&](uint32_t w, uint32_t k, uint32_t lane) { return S.tr0 + (uint64_t)w * 256 + k * L + lane; };
  const uint32_t fwords = (((S.in_len + 64) + 15) & ~15u) / 4;
  const uint32_t *gw = reinterpret_cast<const uint32_t *>(us + S.us_off);
  // transitions; every walk column that ended explicit is listed (LDS atomics) and traced,
  // one per lane where there are at most 256 (qX lane e)
  if (threadIdx.x == 0) s_nx = s_n1 = s_abs = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < (nwg - 1) * bpm; i += 256) {
    const uint32_t w = 1 + i / bpm, e = i - (w - 1) * bpm;
    const uint32_t j = B.wF[(uint64_t)(S.wg0 + w - 1) * kSpecLanesMax + e] & 0xF;
    if (j < bpm) {
      sT[w * bpm + e] = j | (1u << 4) | kTrJoined;
    } else {
      const uint32_t q = atomicAdd(&s_nx, 1u);
      s_xl[q] = (uint16_t)i;  // q < kResolveT: one entry per (workgroup, walk column)
    }
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < s_nx; q += 256) {
    const uint32_t i = s_xl[q], w = 1 + i / bpm, e = i - (w - 1) * bpm;
    // row 1 was decoded by k_spec (w - 1's walker, into qX): compare its exit, trace on from row 2
    const uint64_t X1 = B.qX[slot(w, 1, e)];
    uint32_t te = kLinkNone, kf = 1;
    if (w * NSS + 2 == nsub) {
      te = kLinkLast;  // row 1 is the frame's last subsequence
    } else {
      for (uint32_t c2 = 0; c2 < bpm; ++c2)
        if (B.tX[slot(w, 1, c2)] == X1) {
          te = c2;
          break;
        }
      if (te == kLinkNone)
        te = trace_on(gw, fwords, s_tw[threadIdx.x], X1, w, 2, NS, NSS, L, nsub, nbits, S.tr0, hg, tabs, B.tX, B.qX,
                      B.qC, e, &kf);
      else
        atomicAdd(&s_n1, 1u);
    }
    const uint32_t code = (uint32_t)(kRecQ | e) << 16;
    sT[w * bpm + e] = te < bpm ? te | ((kf + 1) << 4) | code | kTrJoined : (NS << 4) | code;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // diagnostics (VF_JPEG_SYNC_STATS): walk columns that ended explicit, traces joined in one row
    atomicAdd(B.stats + 11, s_nx);
    atomicAdd(B.stats + 12, s_n1);
  }
  // The walk across the workgroups: the transition maps e -> e* (a path that leaves a workgroup
  // in records is absorbing) composed by a prefix scan, lanes taking consecutive chunks of
  // workgroups; each lane then follows its chunk from the entry the scan gives it.  A path
  // absorbed before the frame's last workgroup (rare: a trace that rejoined nothing in a
  // whole workgroup) is walked serially below instead.
  {
    const uint32_t n = nwg - 1, C = (n + 255) / 256, t = threadIdx.x;
    const uint32_t wa = min(n, t * C) + 1, wz = min(n, (t + 1) * C) + 1;  // this lane's workgroups [wa, wz)
    uint64_t ident = 0;
    for (uint32_t q = 0; q < bpm; ++q) ident |= (uint64_t)q << (4 * q);
    uint64_t f = ident;
    for (uint32_t w = wa; w < wz; ++w) {
      uint64_t m = 0;
      for (uint32_t q = 0; q < bpm; ++q) {
        const uint32_t tr = sT[w * bpm + q];
        m |= (uint64_t)((tr & kTrJoined) ? tr & 0xF : 0xF) << (4 * q);
      }
      f = map_compose(m, f, bpm);
    }
    const uint32_t lane = t & 63, wv = t >> 6;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint64_t o = __shfl_up(f, d, 64);
      if (lane >= d) f = map_compose(f, o, bpm);
    }
    if (lane == 63) s_wt[wv] = f;
    __syncthreads();
    uint64_t pre = ident;  // the maps of the waves before this one
    for (uint32_t q = 0; q < wv; ++q) pre = map_compose(s_wt[q], pre, bpm);
    uint64_t gp = __shfl_up(f, 1, 64);
    gp = lane == 0 ? pre : map_compose(gp, pre, bpm);  // the maps of every lane before this one
    uint32_t e = nib(gp, 0);  // the frame starts at walk column 0 of workgroup 0
    if (wa < wz) {
      if (e >= bpm) s_abs = 1u;
      for (uint32_t w = wa; w < wz && e < bpm; ++w) {
        const uint32_t tr = sT[w * bpm + e];
        e = tr & 0xF;
        sE[w] = (uint8_t)e;
        sK[w] = (uint16_t)((tr >> 4) & 0x1FF);
        sJ[w] = (uint8_t)(tr >> 16);
        if (!(tr & kTrJoined)) {
          if (w + 1 < wz) s_abs = 1u;
          break;
        }
      }
    }
    if (t == 0) {
      sE[0] = 0;
      sK[0] = 0;
      sJ[0] = 0;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_abs) {
    uint32_t e = 0;
    bool joined = true;
    uint8_t rec = 0;  // where the records of a path that left w - 1 explicit are
    for (uint32_t w = 1; w < nwg; ++w) {
      if (joined) {
        const uint32_t tr = sT[w * bpm + e];
        e = tr & 0xF;
        sE[w] = (uint8_t)e;
        sK[w] = (uint16_t)((tr >> 4) & 0x1FF);
        sJ[w] = rec = (uint8_t)(tr >> 16);
        joined = (tr & kTrJoined) != 0;
        continue;
      }
      // the path crossed w - 1 in a trace that rejoined nothing: decode on (records into pX lane 0)
      const uint64_t X = ((rec & 0x40) ? B.qX : B.pX)[slot(w - 1, lastk, rec & 15)];
      uint32_t kf = 0;
      const uint32_t te = trace_on(gw, fwords, s_tw[0], X, w, 1, NS, NSS, L, nsub, nbits, S.tr0, hg, tabs, B.tX, B.pX,
                                   B.pC, 0, &kf);
      atomicAdd(B.stats + 13, 1u);  // diagnostics: serial traces
      joined = te < bpm;
      e = joined ? te : 0;
      sE[w] = (uint8_t)e;
      sK[w] = (uint16_t)(joined ? kf + 1 : NS);
      sJ[w] = rec = kRecP;
    }
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < nwg; w += 256) {
    B.rE[S.wg0 + w] = sE[w];
    B.rK[S.wg0 + w] = sK[w];
    B.rL[S.wg0 + w] = sJ[w];
  }
}

// Exit state and block count of every subsequence along the resolved path, in the layout
// the write pass and the block-offset scan read (exit_out / cnt_out of k_sync).  A workgroup's
// row 0 is its predecessor's last row, written there.
__global__ __launch_bounds__(256) void k_finalize(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, const uint32_t *us_len, SpecBufs B,
                                                  uint64_t *exit_out, uint32_t *cnt_out) {
  const DecSeg S = sg[blockIdx.y];  // by value: held in scalar registers
  const DecFrame &F = fr[S.frame];
  if (blockIdx.x >= S.nwg) return;
  const uint32_t bpm = (uint32_t)F.g.bpm, L = spec_lanes(bpm), NS = 256 / L;
  const uint32_t nbits = us_len[blockIdx.y] * 8u, nsub = (nbits + kSubBits - 1) / kSubBits;
  const uint32_t sl = threadIdx.x;
  if (sl >= NS || (blockIdx.x > 0 && sl == 0)) return;
  const uint32_t s = blockIdx.x * (NS - 1) + sl;
  if (s >= S.nsub_max) return;
  const uint64_t gi = S.sub0 + s;
  if (s >= nsub) {
    exit_out[gi] = pack_state(nbits, 0, 0);
    cnt_out[gi] = 0;
    return;
  }
  const uint64_t g0 = S.tr0 + (uint64_t)blockIdx.x * 256;
  const uint32_t rk = B.rK[S.wg0 + blockIdx.x], e = B.rE[S.wg0 + blockIdx.x];
  if (sl < rk) {
    const uint8_t rl = B.rL[S.wg0 + blockIdx.x];
    const uint64_t at = g0 + sl * L + (rl & 15);
    exit_out[gi] = (rl & 0x40) ? B.qX[at] : B.pX[at];
    cnt_out[gi] = (rl & 0x40) ? B.qC[at] : B.pC[at];
  } else {
    exit_out[gi] = B.tX[g0 + sl * L + e];
    cnt_out[gi] = B.tXc[g0 + sl * L + e];
  }
}

// The workgroup's stream words are staged in LDS first (as k_spec does): every refill of a
// thread's bit buffer is then an LDS read instead of a dependent global load, the chain a
// subsequence's decode waits on (k_write has only ~3 waves per SIMD to hide it with).
template <bool CHUNKS>
__global__ __launch_bounds__(256) void k_write(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, const uint8_t *us, const uint32_t *us_len,
                                               const uint64_t *exits, const uint32_t *bstart, int16_t *coef,
                                               int32_t *dcseq, uint8_t *nmask) {
  __shared__ HuffDec tabs[6];
  __shared__ uint32_t s_w[kSpecWords + (CHUNKS ? kBlockPadWords : 0)];
  __shared__ int32_t s_dc[kStageBlocks + 1];  // + the flush bound
  __shared__ __attribute__((aligned(16))) uint16_t s_nm[kStageBlocks];
  const DecSeg S = sg[blockIdx.y];  // by value: held in scalar registers
  const DecFrame &F = fr[S.frame];
  if (blockIdx.x * 256 >= S.nsub_max) return;
  // this workgroup's 256 subsequences of stream words, plus overshoot and lookahead, from the
  // frame's padded unstuffed region (an entry state lies at or after its subsequence's start)
  const uint32_t woff = blockIdx.x * 256 * (kSubBits / 32);
  const uint32_t fwords = (((S.in_len + 64) + 15) & ~15u) / 4;
  const uint32_t *gw = reinterpret_cast<const uint32_t *>(us + S.us_off);
  constexpr uint32_t kWords = kSpecWords + (CHUNKS ? kBlockPadWords : 0);
  for (uint32_t k = threadIdx.x; k < kWords; k += 256) s_w[k] = woff + k < fwords ? gw[woff + k] : 0u;
  for (uint32_t k = threadIdx.x; k < kStageBlocks / 8; k += 256) reinterpret_cast<uint4 *>(s_nm)[k] = make_uint4(0, 0, 0, 0);
  if (threadIdx.x == 0) s_dc[kStageBlocks] = 0;
  load_tables(tabs_of(fr, F), tabs);  // its barrier also publishes s_w and the cleared stage
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t nbits = us_len[blockIdx.y] * 8u;
  const uint32_t nsub = (nbits + kSubBits - 1) / kSubBits;
  const uint32_t gi = S.sub0 + i;
  HuffGeom hg(F.g);
  hg.nblocks = S.nblocks;  // the segment's blocks (a restart interval: its whole MCUs)
  const uint32_t i0 = blockIdx.x * 256;  // workgroup-uniform
  const WriteStage stg{s_dc, s_nm, i0 < nsub ? bstart[S.sub0 + i0] : 0u};
  if (i < nsub) {
    const uint64_t st = i == 0 ? 0 : exits[gi - 1];
    const uint32_t end = (i + 1 == nsub) ? nbits : (i + 1) * kSubBits;
    write_span<CHUNKS, true>(s_w, woff, st, end, hg, tabs, bstart[gi], coef + S.blk0 * 64, dcseq, S.dcbase,
                             nmask + S.blk0, stg);
  }
  __syncthreads();
  // the staged blocks, consecutive threads on consecutive blocks: the masks are one coalesced
  // byte run, the DC values a few coalesced runs (one per component)
  const uint32_t nst = min(s_dc[kStageBlocks] + 1, kStageBlocks);
  uint8_t *const nm = nmask + S.blk0;
  for (uint32_t b = threadIdx.x; b < nst; b += 256) {
    const uint32_t f = s_nm[b];
    if (!(f & 0x100)) continue;
    const uint32_t blk = stg.first + b, mcu = blk / hg.bpm, c = blk - mcu * hg.bpm, k = hg.comp(c);
    dcseq[HuffGeom::sel(S.dcbase, k) + (uint64_t)mcu * HuffGeom::sel(hg.bpc, k) + (c - HuffGeom::sel(hg.cfirst, k))] = s_dc[b];
    if (CHUNKS) nm[blk] = (uint8_t)f;
  }
}

// The write pass with 4 lanes per subsequence, for the pass-based sync (k_sync), whose
// converged checkpoints are states of the true path: ck[m] = (pos, z, c) at the first symbol
// boundary at or past mark m, ckrem[m] = blocks completed from there to the subsequence's end
// (kNoCk where the entry state lies past the mark).  Lane q decodes from checkpoint q - 1 (lane
// 0 from the entry state) up to the next lane's start: the decode of a subsequence, a chain of
// dependent table lookups, runs as 4 shorter chains side by side.  A lane whose checkpoint is
// missing idles and the lane before it decodes on.
template <bool CHUNKS>
__global__ __launch_bounds__(256) void k_write4(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, const uint8_t *us,
                                                const uint32_t *us_len, const uint64_t *exits, const uint32_t *cnt,
                                                const uint64_t *ck, const uint32_t *ckrem, const uint32_t *bstart,
                                                int16_t *coef, int32_t *dcseq, uint8_t *nmask) {
  static_assert(kCk + 1 == 4, "one lane per checkpoint-delimited quarter");
  constexpr uint32_t kSubsPerWg = 64,
                     kW4Words = kSubsPerWg * (kSubBits / 32) + kSpecPadWords + (CHUNKS ? kBlockPadWords : 0);
  __shared__ HuffDec tabs[6];
  __shared__ uint32_t s_w[kW4Words];
  const DecSeg S = sg[blockIdx.y];  // by value: held in scalar registers
  const DecFrame &F = fr[S.frame];
  if (blockIdx.x * kSubsPerWg >= S.nsub_max) return;
  const uint32_t woff = blockIdx.x * kSubsPerWg * (kSubBits / 32);
  const uint32_t fwords = (((S.in_len + 64) + 15) & ~15u) / 4;
  const uint32_t *gw = reinterpret_cast<const uint32_t *>(us + S.us_off);
  for (uint32_t k = threadIdx.x; k < kW4Words; k += 256) s_w[k] = woff + k < fwords ? gw[woff + k] : 0u;
  load_tables(tabs_of(fr, F), tabs);  // its barrier also publishes s_w
  const uint32_t i = blockIdx.x * kSubsPerWg + (threadIdx.x >> 2), q = threadIdx.x & 3;
  const uint32_t nbits = us_len[blockIdx.y] * 8u;
  const uint32_t nsub = (nbits + kSubBits - 1) / kSubBits;
  if (i >= nsub) return;
  const uint32_t gi = S.sub0 + i;
  const uint64_t *cki = ck + (uint64_t)gi * kCk;
  uint64_t st;
  uint32_t before = 0;
  if (q == 0) {
    st = i == 0 ? 0 : exits[gi - 1];
  } else {
    st = cki[q - 1];
    if (st == kNoCk) return;
    before = cnt[gi] - ckrem[(uint64_t)gi * kCk + q - 1];
  }
  uint32_t stop = (i + 1 == nsub) ? nbits : (i + 1) * kSubBits;
  for (uint32_t m = q; m < kCk; ++m)
    if (cki[m] != kNoCk) {
      stop = (uint32_t)(cki[m] >> 16);
      break;
    }
  HuffGeom hg(F.g);
  hg.nblocks = S.nblocks;
  write_span<CHUNKS>(s_w, woff, st, stop, hg, tabs, bstart[gi] + before, coef + S.blk0 * 64, dcseq, S.dcbase,
                     nmask + S.blk0);
}

// ---- decoder: IDCT -------------------------------------------------------------------------

#define FIX_0_298631336 2446
#define FIX_0_390180644 3196
#define FIX_0_541196100 4433
#define FIX_0_765366865 6270
#define FIX_0_899976223 7373
#define FIX_1_175875602 9633
#define FIX_1_501321110 12299
#define FIX_1_847759065 15137
#define FIX_1_961570560 16069
#define FIX_2_053119869 16819
#define FIX_2_562915447 20995
#define FIX_3_072711026 25172
#define DESCALE(x, n) (((x) + ((int32_t)1 << ((n)-1))) >> (n))

// jidctint.c jpeg_idct_islow, one 8-point line; `shift` 11 (pass 1) or 18 (pass 2), 32-bit
// products as the C code.  M24: the products by v_mul_i32_i24 / v_mad_i32_i24 (full VALU rate;
// v_mul_lo_u32 issues at a quarter), exact when every multiplicand -- a sum of at most four
// inputs -- lies in [-2^23, 2^23).  The row pass's always do: its inputs are the column pass's
// int32 results shifted right by 11, so |x| <= 2^20 and a sum of four <= 2^22, whatever the
// stream holds.  The column pass's multiplicands are sums of dequantised AC coefficients, only
// bounded by the frame's tables: the host sets kDecIdct24 when they fit (idct_col24_ok) and the
// kernels take the 32-bit column pass for the frames that do not.  (Guarding it per wave with a
// range check and a ballot per line, round 3, made k_idct slower, 129.8 -> 142.5 us.)
template <bool B>
struct BoolTag {
  static constexpr bool value = B;
};
template <bool M24>
__device__ __forceinline__ int32_t imul(int32_t a, int32_t c) {
  if constexpr (M24) return __mul24(a, c);
  else return a * c;
}
// jidctint.c's butterflies; emit(i, v) receives output i before its descale
template <bool M24, typename Emit>
__device__ __forceinline__ void idct_core(const int32_t in[8], Emit emit) {
  int32_t tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13, z1, z2, z3, z4, z5;
  z2 = in[2];
  z3 = in[6];
  z1 = imul<M24>(z2 + z3, FIX_0_541196100);
  tmp2 = z1 + imul<M24>(z3, -FIX_1_847759065);
  tmp3 = z1 + imul<M24>(z2, FIX_0_765366865);
  tmp0 = (in[0] + in[4]) * (1 << 13);
  tmp1 = (in[0] - in[4]) * (1 << 13);
  tmp10 = tmp0 + tmp3;
  tmp13 = tmp0 - tmp3;
  tmp11 = tmp1 + tmp2;
  tmp12 = tmp1 - tmp2;
  tmp0 = in[7];
  tmp1 = in[5];
  tmp2 = in[3];
  tmp3 = in[1];
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  z4 = tmp1 + tmp3;
  z5 = imul<M24>(z3 + z4, FIX_1_175875602);
  tmp0 = imul<M24>(tmp0, FIX_0_298631336);
  tmp1 = imul<M24>(tmp1, FIX_2_053119869);
  tmp2 = imul<M24>(tmp2, FIX_3_072711026);
  tmp3 = imul<M24>(tmp3, FIX_1_501321110);
  z1 = imul<M24>(z1, -FIX_0_899976223);
  z2 = imul<M24>(z2, -FIX_2_562915447);
  z3 = imul<M24>(z3, -FIX_1_961570560);
  z4 = imul<M24>(z4, -FIX_0_390180644);
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  emit(0, tmp10 + tmp3);
  emit(7, tmp10 - tmp3);
  emit(1, tmp11 + tmp2);
  emit(6, tmp11 - tmp2);
  emit(2, tmp12 + tmp1);
  emit(5, tmp12 - tmp1);
  emit(3, tmp13 + tmp0);
  emit(4, tmp13 - tmp0);
}
template <bool M24>
__device__ __forceinline__ void idct_line(const int32_t in[8], int32_t out[8], int shift) {
  const int32_t r = (int32_t)1 << (shift - 1);
  idct_core<M24>(in, [&](int i, int32_t v) { out[i] = (v + r) >> shift; });
}

// The row pass (descale by 18) with jdmaster.c prepare_range_limit_table's post-IDCT limit
// (RANGE_MASK 1023) in three instructions: the table maps
// m = x & 1023 to m + 128 (m < 128), 255 (< 512), 0 (< 896), m - 896, which for every x is
// clamp(((x + 512) & 1023) - 384, 0, 255); with 512 << 18 added to the rounding constant, the
// descale and the mask are one bit-field extract of the 32-bit sum (bits 18..27).
__device__ __forceinline__ void idct_row_limited(const int32_t in[8], uint32_t out[8]) {
  idct_core<true>(in, [&](int i, int32_t v) {
    const int32_t m = (int32_t)__builtin_amdgcn_ubfe((uint32_t)v + ((1u << 17) + (512u << 18)), 18, 10) - 384;
    out[i] = (uint32_t)min(max(m, 0), 255);
  });
}

// Measured (tools/gpu_jpeg_variants.sh, profiles/r01_jpeg_idct_variants.txt; dc + idct ms at
// 1080p / 4K): 1 block per lane group with separate LDS for the two passes 0.200 / 0.73 (the
// earlier kernel); aliased 0.202 / 0.74; 2 blocks not aliased 0.21 / 0.76; 2 blocks aliased
// 0.170 / 0.61; 3 aliased 0.197 / 0.71; 4 aliased 0.205 / 0.74.
constexpr int kIdctNb = 2;                  // blocks per 8-lane group
constexpr int kIdctBlocks = 32 * kIdctNb;   // blocks per workgroup

// LDS placement of a block's coefficients, conflict-free for both accesses of k_idct.  Lane r
// holds zigzag positions 8r..8r+7 (one 16-B load) and stores them; in pass 1 it reads column r.
// A block's row is 72 dwords (8 mod 32), so a 32-lane half (4 blocks x 8 lanes) is free of
// conflicts when, for every store j and every read i, the 8 lanes' dwords differ mod 8.
// Natural position n = 8i + c sits at dword 8i + g(n), where g permutes each natural row and
// also each zigzag class {zigzag 8r + j : r} -- an 8-edge-colouring of the 8-regular bipartite
// graph rows x zigzag-classes (one edge per position; König).  The zigzag store of the
// natural-order scatter it replaces cost 16 extra LDS cycles per block pair and wave, the
// mixed-component dequantisation reads 32 (SQ_LDS_BANK_CONFLICT 3.98e8 per 1080p batch,
// profiles/r01_jpeg_pmc_sq.txt).
__constant__ uint8_t kIdctPos[64] = {  // zigzag index -> dword of the block row (8 * row + g)
    1,  0,  9,  17, 8,  3,  2,  11, 16, 25, 32, 27, 19, 10, 5,  4,  12, 18, 26, 34, 42, 48,
    40, 33, 29, 21, 14, 7,  6,  13, 20, 24, 35, 46, 51, 56, 57, 49, 41, 38, 31, 23, 15, 22,
    28, 36, 43, 50, 58, 59, 52, 44, 37, 30, 39, 45, 54, 60, 61, 53, 47, 55, 62, 63};
__constant__ uint32_t kIdctCol[8] = {  // column c: nibble i = g(8i + c)
    0x00201111u, 0x13023000u, 0x21612333u, 0x32135222u, 0x44360545u, 0x56447464u, 0x65554757u, 0x77776676u};

// 8 lanes per block, kIdctNb blocks per 8-lane group: both blocks' coefficient loads are issued
// before either is transformed, and the column pass's output reuses the block's LDS row (one
// more barrier, half the LDS: 18.4 KB per workgroup for 64 blocks).  Dequantisation happens
// on pass 1's reads, as in jidctint.c (DEQUANTIZE(inptr[DCTSIZE*k], quantptr[DCTSIZE*k])).
// A wave takes block-in-MCU c of 8 * kIdctNb consecutive MCUs (lane group j: MCUs j and
// j + 8), a workgroup 4 such units: the component and its geometry are wave-uniform (scalar),
// no lane divides, and the 8 lanes of a block read the same dequantisation entries.
constexpr uint32_t kIdctGroup = 8 * kIdctNb;  // MCUs per wave
// nmask (the write pass's CHUNKS form): bit r of a block's byte says its coefficient row r (zigzag
// 8r .. 8r + 7, this lane's 16-B load) was stored; the others read as zero.  Null: a cleared buffer.
__global__ __launch_bounds__(256) void k_idct(const DecFrame *__restrict__ fr, const int16_t *coef, const int32_t *dcseq,
                                              const uint8_t *nmask, uint8_t *planes) {
  const DecFrame &F = fr[blockIdx.y];
  const Geom &g = F.g;
  const uint32_t bpm = (uint32_t)g.bpm, nmcu = (uint32_t)g.nmcu;
  const uint32_t ngroups = (nmcu + kIdctGroup - 1) / kIdctGroup;
  if (blockIdx.x * 4 >= ngroups * bpm) return;
  __shared__ int32_t blkv[kIdctBlocks][72];  // coefficients (kIdctPos), then the column pass's [8][9]
  __shared__ int32_t s_q[3][72];     // dequantisation, natural order; rows 8 mod 32 dwords apart
  __shared__ uint8_t s_pos[64];      // kIdctPos
  __shared__ uint32_t s_col[8];      // kIdctCol
  const uint32_t t = threadIdx.x;
  const uint32_t slot = t >> 3, r = t & 7, lm = slot & 7;
  const uint32_t unit = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t grp = unit / bpm, c = unit - grp * bpm;  // scalar
  const bool live = grp < ngroups;
  const uint32_t k = live ? (uint32_t)g.bcomp[c] : 0u;
  const uint32_t mh = (uint32_t)g.mh[k], mv = (uint32_t)g.mv[k], mcux = (uint32_t)g.mcux;
  const uint32_t mx0 = (grp * kIdctGroup) % mcux, my0 = (grp * kIdctGroup) / mcux;
  bool valid[kIdctNb];
  uint32_t bxs[kIdctNb], bys[kIdctNb];
  uint4 raw[kIdctNb];
  int32_t dc[kIdctNb];
  uint32_t nm[kIdctNb];
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {
    const uint32_t mcu = grp * kIdctGroup + h * 8 + lm;
    valid[h] = live && mcu < nmcu;
    uint32_t mx = mx0 + h * 8 + lm, my = my0;
    while (mx >= mcux) mx -= mcux, ++my;  // once at most unless the frame is under 16 MCUs wide
    bxs[h] = mx * mh + (uint32_t)g.bxo[c];
    bys[h] = my * mv + (uint32_t)g.byo[c];
    // unconditional loads (an invalid block reads the frame's first block and DC): loads
    // under a branch made the compiler wait for the first block's before issuing the second's
    const uint64_t bi = valid[h] ? F.blk0 + (uint64_t)mcu * bpm + c : F.blk0;
    const uint64_t di = valid[h] ? F.dcbase[k] + (uint64_t)mcu * (mh * mv) + (c - (uint32_t)g.cfirst[k]) : F.dcbase[k];
    raw[h] = *reinterpret_cast<const uint4 *>(coef + bi * 64 + r * 8);
    dc[h] = dcseq[di];
    nm[h] = nmask ? (uint32_t)nmask[bi] : 0xFFu;
  }
  // the tables after the coefficient loads: their round trips overlap instead of the
  // coefficients waiting behind the tables' barrier
  if (t < 192) s_q[t >> 6][t & 63] = F.q[t >> 6][t & 63];
  if (t < 64) s_pos[t] = kIdctPos[t];
  if (t < 8) s_col[t] = kIdctCol[t];
  __syncthreads();
  // read before the first store (through F after a store, they were re-loaded with a wait)
  uint8_t *const plane = planes + F.plane_off[k];
  const uint32_t pw = (uint32_t)g.pw[k];
  const uint2 pos8 = *reinterpret_cast<const uint2 *>(&s_pos[r * 8]);  // this lane's 8 store dwords
  const uint32_t colg = s_col[r];
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {
    if (!valid[h]) continue;
    const bool st = (nm[h] >> r) & 1;  // a row the write pass did not store is zero
    const uint32_t qw[4] = {st ? raw[h].x : 0u, st ? raw[h].y : 0u, st ? raw[h].z : 0u, st ? raw[h].w : 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int32_t v = (int32_t)(int16_t)(qw[j >> 1] >> (16 * (j & 1)));
      const uint32_t at = ((j < 4 ? pos8.x : pos8.y) >> (8 * (j & 3))) & 0xFF;
      blkv[h * 32 + slot][at] = (r == 0 && j == 0) ? (int32_t)(int16_t)dc[h] : v;
    }
  }
  __syncthreads();
  int32_t col[kIdctNb][8];
  const auto pass1 = [&](auto m24) {  // pass 1: column r, dequantised
#pragma unroll
    for (int h = 0; h < kIdctNb; ++h) {
      if (!valid[h]) continue;
      int32_t in[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        in[i] = __mul24(blkv[h * 32 + slot][i * 8 + ((colg >> (4 * i)) & 7)], s_q[k][i * 8 + r]);  // int16 x u16: exact
      idct_line<decltype(m24)::value>(in, col[h], 11);
    }
  };
  if (F.flags & kDecIdct24) pass1(BoolTag<true>{});  // frame-uniform (scalar) branch
  else pass1(BoolTag<false>{});
  __syncthreads();
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {
    if (!valid[h]) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) blkv[h * 32 + slot][i * 9 + r] = col[h][i];
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {  // pass 2: row r
    if (!valid[h]) continue;
    int32_t in[8];
    uint32_t out[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) in[i] = blkv[h * 32 + slot][r * 9 + i];
    idct_row_limited(in, out);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo |= out[i] << (8 * i);
      hi |= out[i + 4] << (8 * i);
    }
    uint8_t *p = plane + (uint64_t)(bys[h] * 8 + r) * pw + bxs[h] * 8;
    *reinterpret_cast<uint2 *>(p) = make_uint2(lo, hi);
  }
}

// ---- decoder: upsampling + colour ------------------------------------------------------------

__device__ __forceinline__ int up_sample(const uint8_t *p, int pw, int dw, int dh, int he, int ve, bool fancy,
                                         int x, int y) {
  if (he == 1 && ve == 1) return p[(size_t)y * pw + x];
  const int iy = y / ve < dh ? y / ve : dh - 1;
  if (!fancy) return p[(size_t)iy * pw + x / he];
  const uint8_t *r0 = p + (size_t)iy * pw;
  if (he == 2 && ve == 1) {  // h2v1_fancy_upsample
    const int i = x >> 1;
    if (!(x & 1)) return i == 0 ? r0[0] : (3 * r0[i] + r0[i - 1] + 1) >> 2;
    return i == dw - 1 ? r0[i] : (3 * r0[i] + r0[i + 1] + 2) >> 2;
  }
  int ny = (y & 1) ? iy + 1 : iy - 1;  // jdmainct.c context rows: edges replicate
  ny = ny < 0 ? 0 : ny > dh - 1 ? dh - 1 : ny;
  const uint8_t *r1 = p + (size_t)ny * pw;
  if (he == 1) return (3 * r0[x] + r1[x] + ((y & 1) ? 2 : 1)) >> 2;  // h1v2_fancy_upsample
  const int i = x >> 1;  // h2v2_fancy_upsample
  const int t = 3 * r0[i] + r1[i];
  if (!(x & 1)) return i == 0 ? (4 * t + 8) >> 4 : (3 * t + 3 * r0[i - 1] + r1[i - 1] + 8) >> 4;
  return i == dw - 1 ? (4 * t + 7) >> 4 : (3 * t + 3 * r0[i + 1] + r1[i + 1] + 7) >> 4;
}

__device__ __forceinline__ uint32_t clamp255(int v) { return (uint32_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// 8 output samples of a 2x horizontally subsampled row from chroma samples i0-1 .. i0+4
// (cs, edge-clamped column values; for h2v2 already 3 * nearer row + further row)
__device__ __forceinline__ void up2(const int cs[6], int i0, int dw, bool fancy, int ve, int out[8]) {
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int i = i0 + jj, c = cs[jj + 1];
    int a, b;
    if (!fancy) {
      a = b = c;
    } else if (ve == 1) {  // h2v1_fancy_upsample
      a = i == 0 ? c : (3 * c + cs[jj] + 1) >> 2;
      b = i == dw - 1 ? c : (3 * c + cs[jj + 2] + 2) >> 2;
    } else {  // h2v2_fancy_upsample
      a = i == 0 ? (4 * c + 8) >> 4 : (3 * c + cs[jj] + 8) >> 4;
      b = i == dw - 1 ? (4 * c + 7) >> 4 : (3 * c + cs[jj + 2] + 7) >> 4;
    }
    out[2 * jj] = a;
    out[2 * jj + 1] = b;
  }
}

// jdcolor.c ycc_rgb_convert (grayscale: replicated) of 8 pixels, inverted when asked
__device__ __forceinline__ void ycc8(const int v[3][8], int ncomp, int bgr, int invert, uint8_t o[24]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t r, gg, b;
    if (ncomp == 1) {
      r = gg = b = (uint32_t)v[0][j];
    } else {
      const int xcr = v[2][j] - 128, xcb = v[1][j] - 128;  // 24-bit multiplies: |x| <= 128, constants < 2^17
      r = clamp255(v[0][j] + ((__mul24(91881, xcr) + 32768) >> 16));
      gg = clamp255(v[0][j] + ((__mul24(-22554, xcb) + 32768 - __mul24(46802, xcr)) >> 16));
      b = clamp255(v[0][j] + ((__mul24(116130, xcb) + 32768) >> 16));
    }
    if (invert) {
      r ^= 0xFF;
      gg ^= 0xFF;
      b ^= 0xFF;
    }
    o[3 * j] = (uint8_t)(bgr ? b : r);
    o[3 * j + 1] = (uint8_t)gg;
    o[3 * j + 2] = (uint8_t)(bgr ? r : b);
  }
}

__device__ __forceinline__ void unpack8(uint2 q, int v[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (int)(((j < 4 ? q.x : q.y) >> (8 * (j & 3))) & 0xFF);
}

// 8 horizontally adjacent output pixels per thread: one 8-byte load per full-size plane,
// the chroma samples they need (+1 neighbour each side) for 2x horizontal subsampling, and
// three 8-byte stores of interleaved output when the row is 8-byte aligned.
// The 8 output pixels of row y from x0 (24 bytes of interleaved output in o).
__device__ __forceinline__ void color8(const DecFrame &F, const Geom &g, const uint8_t *__restrict__ planes, int y,
                                       int x0, int bgr, int invert, uint8_t o[24]) {
  int v[3][8];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= g.ncomp) break;
    const uint8_t *p = planes + F.plane_off[k];
    const int pw = g.pw[k];
    const int he = g.he[k], ve = g.ve[k], dw = g.dw[k], dh = g.dh[k];
    const bool fancy = (F.flags & 1) && ((he == 2 && dw > 2) || (he == 1 && ve == 2));
    if (he == 1 && ve == 1) {
      const uint2 q = *reinterpret_cast<const uint2 *>(p + (size_t)y * pw + x0);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = (int)(((j < 4 ? q.x : q.y) >> (8 * (j & 3))) & 0xFF);
    } else if (he == 2 && ve <= 2) {
      const int iy = min(y / ve, dh - 1);
      const uint8_t *r0 = p + (size_t)iy * pw;
      const int i0 = x0 >> 1;
      int cs[6];  // column values of chroma samples i0-1 .. i0+4 (edges clamped)
      if (ve == 2 && fancy) {
        int ny = (y & 1) ? iy + 1 : iy - 1;
        ny = ny < 0 ? 0 : ny > dh - 1 ? dh - 1 : ny;
        const uint8_t *r1 = p + (size_t)ny * pw;
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          const int ix = min(max(i0 - 1 + m, 0), dw - 1);
          cs[m] = 3 * r0[ix] + r1[ix];
        }
      } else {
#pragma unroll
        for (int m = 0; m < 6; ++m) cs[m] = r0[min(max(i0 - 1 + m, 0), dw - 1)];
      }
      up2(cs, i0, dw, fancy, ve, v[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[k][j] = up_sample(p, pw, dw, dh, he, ve, fancy && he <= 2 && ve <= 2, min(x0 + j, g.w - 1), y);
    }
  }
  ycc8(v, g.ncomp, bgr, invert, o);
}

// jccolor.c rgb_ycc_convert for one component over a pixel's bytes in memory order:
// (a0 * c0 + a1 * c1 + a2 * c2 + bias) >> 16.  The component and the channel order are
// wave-uniform in k_fdct, so the coefficients sit in scalar registers and a pixel costs three
// multiply-adds with no per-pixel select.  No sum is negative (Cb and Cr carry 128 << 16:
// their smallest sums are 575535 and 65535), so the shift is jccolor.c's.
struct Ycc {
  int a0, a1, a2, bias;
};
__device__ __forceinline__ Ycc ycc_coefs(int k, bool bgr) {
  int r, g, b, bias = (128 << 16) + 32767;
  if (k == 0) {
    r = 19595, g = 38470, b = 7471, bias = 32768;
  } else if (k == 1) {
    r = -11059, g = -21709, b = 32768;
  } else {
    r = 32768, g = -27439, b = -5329;
  }
  return bgr ? Ycc{b, g, r, bias} : Ycc{r, g, b, bias};
}
__device__ __forceinline__ int ycc_apply(const Ycc &q, int c0, int c1, int c2) {  // 8-bit samples, |a| <= 2^16
  return (__mul24(q.a0, c0) + __mul24(q.a1, c1) + __mul24(q.a2, c2) + q.bias) >> 16;
}

// The invert path's encoder input, from the colour pass: the encoder's component samples
// (jccolor.c rgb_ycc_convert of the inverted pixels, then jcsample.c downsampling) of the 8
// pixels x0 .. x0 + 7 of rows y0 and y0 + 1, given as packed R | G << 8 | B << 16 (p1 = p0
// when y0 is the last row: jcprepct.c's bottom expansion to whole row groups).  k_fdct then
// reads one 8-byte sample row per lane instead of converting 8-48 pixels in each component's
// wave, and the 3-byte pixels never reach memory.  Pixels past the right edge take the last
// pixel's values (expand_right_edge); the thread holding it also fills the planes' columns past
// the image, to the components' whole blocks.  Sample rows past rrows[k] are never read
// (k_fdct clamps to the last).  One component at a time, from the packed pixels: the samples
// of all three for both rows held at once cost the kernel two of its six waves per SIMD.
// Two of each sum's three products by one signed v_dot2 over a byte-permuted pair of the
// packed pixel, the third (the coefficient that does not fit int16: 38470 for Y's G, 2^15 for
// Cb's B and Cr's R) a 24-bit multiply-add into the accumulator with the rounding bias:
//   Y  = 19595 R + 7471 B       + (38470 G + ONE_HALF)
//   Cb = -11059 R - 21709 G     + (32768 B + CBCR_OFFSET + ONE_HALF - 1)
//   Cr = -27439 G - 5329 B      + (32768 R + CBCR_OFFSET + ONE_HALF - 1)
// The component's selectors and constants are wave-uniform (scalar): one code path for all.
typedef short vf_i16x2 __attribute__((ext_vector_type(2)));
struct EncCoef {
  uint32_t sel, sh;  // byte permutation of the pair; position of the third channel
  vf_i16x2 c;
  int m, bias;
};
__device__ __forceinline__ EncCoef enc_coef(int k) {
  if (k == 0) return EncCoef{0x0C020C00u, 8u, vf_i16x2{19595, 7471}, 38470, 32768};
  if (k == 1) return EncCoef{0x0C010C00u, 16u, vf_i16x2{-11059, -21709}, 32768, (128 << 16) + 32767};
  return EncCoef{0x0C020C01u, 0u, vf_i16x2{-27439, -5329}, 32768, (128 << 16) + 32767};
}
__device__ __forceinline__ int enc_sample(uint32_t px, const EncCoef &q) {
  const vf_i16x2 pr = __builtin_bit_cast(vf_i16x2, __builtin_amdgcn_perm(px, px, q.sel));
  return __builtin_amdgcn_sdot2(pr, q.c, __mul24((int)((px >> q.sh) & 0xFF), q.m) + q.bias, false) >> 16;
}

// ONE: only row y0 (p1 unused; the encoder's chroma must not be vertically downsampled)
template <bool ONE = false>
__device__ __forceinline__ void enc_store_rows(const EncFrame &E, uint8_t *__restrict__ eplanes, uint32_t (&p0)[8],
                                               uint32_t (&p1)[8], int y0, int x0, int w) {
  const Geom &ge = E.g;
  // The edge thread's fill loops stay one byte per trip: unrolled and vectorised by the
  // compiler, that rare path needed 91 VGPRs and set the whole kernel's occupancy (5 waves per
  // SIMD; 60 VGPRs and 8 waves without it).
  const bool edge = x0 + 8 >= w;  // holds pixel w - 1 (and fills past it, up to the whole blocks)
  uint32_t l0 = 0, l1 = 0;        // the last pixel (edge thread)
  if (edge) {
    const int lp = w - 1 - x0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      l0 = p == lp ? p0[p] : l0;
      l1 = p == lp ? p1[p] : l1;
    }
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      p0[p] = p > lp ? l0 : p0[p];
      p1[p] = p > lp ? l1 : p1[p];
    }
  }
  // a rolled loop: one component's samples live at a time (unrolled, the three components'
  // conversions interleaved and the kernel needed 131 VGPRs, 3 waves per SIMD)
#pragma unroll 1
  for (int k = 0; k < ge.ncomp; ++k) {
    const int he = ge.he[k], ve = ge.ve[k], pitch = ge.wb[k] * 8, rr = ge.rrows[k];
    uint8_t *const pl = eplanes + E.eplane_off[k];
    const EncCoef q = enc_coef(k);
    int c0[8], c1[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) c0[p] = enc_sample(p0[p], q), c1[p] = enc_sample(p1[p], q);
    const int e0 = edge ? enc_sample(l0, q) : 0, e1 = edge ? enc_sample(l1, q) : 0;
    if (ve == 1) {
#pragma unroll
      for (int rw = 0; rw < (ONE ? 1 : 2); ++rw) {
        const int y = y0 + rw;
        if (y >= rr) break;
        uint8_t *row = pl + (size_t)y * pitch;
        if (he == 1) {
          uint32_t lo = 0, hi = 0;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            lo |= (uint32_t)(rw ? c1[p] : c0[p]) << (8 * p);
            hi |= (uint32_t)(rw ? c1[p + 4] : c0[p + 4]) << (8 * p);
          }
#if VF_ABL & 8
          if (lo == 0x12345678u && hi == 0x9ABCDEF0u)
#endif
          *reinterpret_cast<uint2 *>(row + x0) = make_uint2(lo, hi);
        } else {  // h2v1_downsample: bias 0, 1 alternating
          uint32_t v = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            v |= (uint32_t)(((rw ? c1[2 * i] + c1[2 * i + 1] : c0[2 * i] + c0[2 * i + 1]) + (i & 1)) >> 1) << (8 * i);
#if VF_ABL & 8
          if (v == 0x12345678u)
#endif
          *reinterpret_cast<uint32_t *>(row + (x0 >> 1)) = v;
        }
        if (edge) {
          const int ev = rw ? e1 : e0;
          #pragma clang loop unroll(disable) vectorize(disable)
          for (int xs = (x0 + 8) / he; xs < pitch; ++xs) row[xs] = (uint8_t)ev;
        }
      }
    } else {  // two rows into one: int_downsample (1x2: (a + b + 1) >> 1) or h2v2_downsample
      const int y = y0 >> 1;
      if (y < rr) {
        uint8_t *row = pl + (size_t)y * pitch;
        if (he == 1) {
          uint32_t lo = 0, hi = 0;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            lo |= (uint32_t)((c0[p] + c1[p] + 1) >> 1) << (8 * p);
            hi |= (uint32_t)((c0[p + 4] + c1[p + 4] + 1) >> 1) << (8 * p);
          }
          *reinterpret_cast<uint2 *>(row + x0) = make_uint2(lo, hi);
          if (edge)
            #pragma clang loop unroll(disable) vectorize(disable)
            for (int xs = x0 + 8; xs < pitch; ++xs) row[xs] = (uint8_t)((e0 + e1 + 1) >> 1);
        } else {  // bias 1, 2 alternating
          uint32_t v = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            v |= (uint32_t)((c0[2 * i] + c0[2 * i + 1] + c1[2 * i] + c1[2 * i + 1] + 1 + (i & 1)) >> 2) << (8 * i);
          *reinterpret_cast<uint32_t *>(row + (x0 >> 1)) = v;
          if (edge)
            #pragma clang loop unroll(disable) vectorize(disable)
            for (int xs = (x0 + 8) >> 1; xs < pitch; ++xs) row[xs] = (uint8_t)((2 * e0 + 2 * e1 + 1 + (xs & 1)) >> 2);
        }
      }
    }
  }
}

// The same from 8 interleaved output pixels per row (color8's general layouts)
__device__ __forceinline__ void enc_sample_rows(const EncFrame &E, uint8_t *__restrict__ eplanes, const uint8_t o0[24],
                                                const uint8_t o1[24], int y0, int x0, int w, int bgr) {
  uint32_t p0[8], p1[8];
  const int i0 = bgr ? 2 : 0, i2 = bgr ? 0 : 2;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    p0[p] = (uint32_t)o0[3 * p + i0] | (uint32_t)o0[3 * p + 1] << 8 | (uint32_t)o0[3 * p + i2] << 16;
    p1[p] = (uint32_t)o1[3 * p + i0] | (uint32_t)o1[3 * p + 1] << 8 | (uint32_t)o1[3 * p + i2] << 16;
  }
  enc_store_rows(E, eplanes, p0, p1, y0, x0, w);
}

// 8 pixels (24 bytes of o) to dst, of which `left` are inside the row
__device__ __forceinline__ void store24(uint8_t *dst, int left, const uint8_t o[24]) {
  if (left >= 8 && ((uintptr_t)dst & 7) == 0) {
    uint2 *d2 = reinterpret_cast<uint2 *>(dst);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo |= (uint32_t)o[8 * q + j] << (8 * j);
        hi |= (uint32_t)o[8 * q + 4 + j] << (8 * j);
      }
      d2[q] = make_uint2(lo, hi);
    }
  } else {
    const int n = min(8, left) * 3;
    for (int j = 0; j < n; ++j) dst[j] = o[j];
  }
}


// Rows y0 and y0 + 1 (y0 even) for three components with full-size luma and both chroma
// planes 1x1 (MODE 0), 2x1 (MODE 1) or 2x2 (MODE 2) subsampled: the same arithmetic as color8,
// with every plane load of both rows issued before any is used (color8's per-component
// branches leave the compiler waiting on each component's loads in turn: six round trips per
// thread at 4:2:0).  4:2:0 reads chroma rows iy - 1, iy, iy + 1 once for both output rows.
// The decoder's sample planes as color_rows reads them: row(k, y) points at column 0 of
// component k's sample row y.  GlobalPlanes: the planes k_idct wrote (k_color);
// StripPlanes: one MCU row's strip of them in LDS (k_idct_color), indexed by frame columns.
struct GlobalPlanes {
  const uint8_t *__restrict__ planes;
  const DecFrame &F;
  __device__ __forceinline__ const uint8_t *row(int k, int y) const {
    return planes + F.plane_off[k] + (size_t)y * F.g.pw[k];
  }
};

template <int MODE, bool ENC, typename PL, bool ONE = false>
__device__ __forceinline__ void color_rows(const DecFrame &F, const Geom &g, const PL &pl,
                                           uint8_t *__restrict__ pix, const EncFrame *__restrict__ efr, int y0, int x0,
                                           bool two, int bgr, int invert) {
  const int y1 = two ? y0 + 1 : y0;
  int v0[3][8], v1[3][8];
  if constexpr (MODE == 0) {
    uint2 q[3][2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      q[k][0] = *reinterpret_cast<const uint2 *>(pl.row(k, y0) + x0);
      q[k][1] = *reinterpret_cast<const uint2 *>(pl.row(k, y1) + x0);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      unpack8(q[k][0], v0[k]);
      unpack8(q[k][1], v1[k]);
    }
  } else {
    const uint2 qa = *reinterpret_cast<const uint2 *>(pl.row(0, y0) + x0);
    const uint2 qb = *reinterpret_cast<const uint2 *>(pl.row(0, y1) + x0);
    const int dw = g.dw[1], dh = g.dh[1];
    const bool fancy = (F.flags & 1) && dw > 2;
    const int i0 = x0 >> 1;
    int ix[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) ix[m] = min(max(i0 - 1 + m, 0), dw - 1);
    constexpr int NR = MODE == 2 ? 3 : 2;
    int rows[NR];
    if constexpr (MODE == 2) {  // the row above, the row itself, the row below (clamped)
      const int iy = min(y0 >> 1, dh - 1);
      rows[0] = max(iy - 1, 0);
      rows[1] = iy;
      rows[2] = min(iy + 1, dh - 1);
    } else {
      rows[0] = min(y0, dh - 1);
      rows[1] = min(y1, dh - 1);
    }
    int b[2][NR][6];
    // Samples i0 .. i0 + 3 are one aligned dword (i0 is a multiple of 4 and below dw <= pw;
    // rows are pw bytes, a multiple of 8, from 256-B aligned planes) and only the two
    // neighbours are byte loads: 3 loads per chroma row instead of 6.  At the right edge the
    // dword's bytes past dw - 1 are replaced by byte dw - 1 - i0 (the edge clamp), so no lane
    // takes another path.
    const int e = min(dw - 1 - i0, 3);
    int sh[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) sh[m] = 8 * min(m, e);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) {
        const uint8_t *r = pl.row(k + 1, rows[rr]);
        const uint32_t mid = *reinterpret_cast<const uint32_t *>(r + i0);
        b[k][rr][0] = r[ix[0]];
#pragma unroll
        for (int m = 1; m < 5; ++m) b[k][rr][m] = (int)((mid >> sh[m - 1]) & 0xFF);
        b[k][rr][5] = r[ix[5]];
      }
    }
    unpack8(qa, v0[0]);
    unpack8(qb, v1[0]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      int c0[6], c1[6];
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        if constexpr (MODE == 2) {  // y0 even: its further row is above, y0 + 1's below
          c0[m] = fancy ? 3 * b[k][1][m] + b[k][0][m] : b[k][1][m];
          c1[m] = fancy ? 3 * b[k][1][m] + b[k][2][m] : b[k][1][m];
        } else {
          c0[m] = b[k][0][m];
          c1[m] = b[k][1][m];
        }
      }
      up2(c0, i0, dw, fancy, MODE == 2 ? 2 : 1, v0[k + 1]);
      up2(c1, i0, dw, fancy, MODE == 2 ? 2 : 1, v1[k + 1]);
    }
  }
  if constexpr (ENC) {  // decoded YCbCr -> inverted RGB (packed) -> the encoder's samples
    uint32_t p0[8], p1[8];
#pragma unroll
    for (int rw = 0; rw < (ONE ? 1 : 2); ++rw)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int yy = rw ? v1[0][j] : v0[0][j], cb = rw ? v1[1][j] : v0[1][j], cr = rw ? v1[2][j] : v0[2][j];
        const int xcr = cr - 128, xcb = cb - 128;
        const uint32_t r = clamp255(yy + ((__mul24(91881, xcr) + 32768) >> 16));
        const uint32_t gg = clamp255(yy + ((__mul24(-22554, xcb) + 32768 - __mul24(46802, xcr)) >> 16));
        const uint32_t b = clamp255(yy + ((__mul24(116130, xcb) + 32768) >> 16));
        const uint32_t px = (r | gg << 8 | b << 16) ^ (invert ? 0xFFFFFFu : 0u);
        if (rw) p1[j] = two ? px : p0[j];
        else p0[j] = px;
      }
    return enc_store_rows<ONE>(efr[blockIdx.z], pix, p0, p1, y0, x0, g.w);
  }
  uint8_t o0[24], o1[24];
  ycc8(v0, 3, bgr, invert, o0);
  ycc8(v1, 3, bgr, invert, o1);
  // both destinations before the first store (after it, F's fields were re-loaded with a wait)
  const int w = g.w;
  uint8_t *const d0 = pix + F.out_off + ((size_t)y0 * w + x0) * 3, *const d1 = d0 + (size_t)w * 3;
  store24(d0, w - x0, o0);
  if (two) store24(d1, w - x0, o1);
}

// Two rows per workgroup: both rows' plane loads are issued before either row is stored (the
// kernel is bound by load latency per wave; one short row per workgroup left it exposed).
// ENC: the invert path's fused form, pix = the encoder's sample planes (enc_sample_rows).
// CM: the batch's layout when every frame has the same (1..3; 0 general), or -1 for a mixed
// batch (dispatched per frame): a kernel holds only its own path, whose registers alone then
// set its occupancy (with all paths in one kernel, the fused form needed 127 VGPRs).
// (The fused 2x1 form: 96 VGPRs, 5 waves per SIMD; held to 80 for 6 waves it spilled two
// registers and ran no faster, 102.5 vs 103 us at 1080p x 32.)
template <bool ENC, int CM>
__global__ __launch_bounds__(256) void k_color(const DecFrame *__restrict__ fr, const uint8_t *__restrict__ planes,
                                               uint8_t *__restrict__ pix, const EncFrame *__restrict__ efr, int bgr,
                                               int invert) {
  const DecFrame &F = fr[blockIdx.z];
  const Geom &g = F.g;
  const int y0 = blockIdx.y * 2, x0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (y0 >= g.h || x0 >= g.w) return;
  const bool two = y0 + 1 < g.h;
  // the common layouts (classified on the host: one scalar word, where the int8 sampling
  // fields would each be a vector load and a wait) take a path whose plane loads are all
  // issued up front
  const uint32_t cm = CM >= 0 ? (uint32_t)CM : (F.flags >> 1) & 3u;
  const GlobalPlanes gp{planes, F};
  if (cm == 1) return color_rows<0, ENC>(F, g, gp, pix, efr, y0, x0, two, bgr, invert);
  if (cm == 2) return color_rows<1, ENC>(F, g, gp, pix, efr, y0, x0, two, bgr, invert);
  if (cm == 3) return color_rows<2, ENC>(F, g, gp, pix, efr, y0, x0, two, bgr, invert);
  uint8_t o0[24], o1[24];
  color8(F, g, planes, y0, x0, bgr, invert, o0);
  color8(F, g, planes, two ? y0 + 1 : y0, x0, bgr, invert, o1);
  if constexpr (ENC) return enc_sample_rows(efr[blockIdx.z], pix, o0, o1, y0, x0, g.w, bgr);
  const int w = g.w;
  uint8_t *const d0 = pix + F.out_off + ((size_t)y0 * w + x0) * 3;
  store24(d0, w - x0, o0);
  if (two) store24(d0 + (size_t)w * 3, w - x0, o1);
}

// ---- decoder: IDCT + colour in one pass (the invert path, standard 4:2:2) ---------------------
//
// k_idct wrote the decoder's sample planes (133 MB per 1080p batch of 32) and k_color read them
// straight back.  Here a workgroup decodes one MCU row's strip of kStripMcus MCUs into LDS --
// its 30 luma blocks and the 15 + 2 blocks of each chroma component that h2v1 fancy
// upsampling reads (one chroma column each side comes from the neighbouring MCU: its whole
// block is transformed for it) -- 64 blocks, k_idct's workgroup; then converts the strip's
// pixels from LDS with color_rows, the same arithmetic as k_color.  Only standard 4:2:2 frames
// (sampling 2x1, 1x1, 1x1; bpm 4) take it: 4:2:0's vertical context would need the MCU rows
// above and below.
constexpr int kStripMcus = 15;                 // 2 * 15 + 2 * (15 + 2) = 64 blocks
constexpr int kStripY = kStripMcus * 16;       // luma samples per strip row (240)
constexpr int kStripC = (kStripMcus + 2) * 8;  // chroma samples per strip row, one block each side (136)

struct StripPlanes {
  const uint8_t *y, *cb, *cr;  // [8][kStripY], [8][kStripC] x 2 (LDS)
  int y_base, x_base, c_base;  // frame row of strip row 0, frame column of luma / chroma column 0
  __device__ __forceinline__ const uint8_t *row(int k, int yy) const {
    const int r = yy - y_base;
    return k == 0 ? y + r * kStripY - x_base : (k == 1 ? cb : cr) + r * kStripC - c_base;
  }
};

// ONE: the encoder's chroma is not vertically downsampled (its rows are independent), so every
// thread converts one 8-pixel row (240 threads busy); else 8 pixels x 2 rows (120 threads).
template <bool ONE>
__global__ __launch_bounds__(256) void k_idct_color422(const DecFrame *__restrict__ fr, const int16_t *coef,
                                                       const int32_t *dcseq, const uint8_t *nmask,
                                                       uint8_t *__restrict__ eplanes, const EncFrame *__restrict__ efr,
                                                       int invert) {
  const DecFrame &F = fr[blockIdx.z];
  const Geom &g = F.g;
  const int mcux = g.mcux, my = blockIdx.y, m0 = blockIdx.x * kStripMcus;
  if (m0 >= mcux || my >= g.mcuy) return;
  __shared__ int32_t blkv[kIdctBlocks][72];
  // dequantisation in zigzag order: lane r multiplies its 8 coefficients (zigzag 8r .. 8r + 7) as
  // it stores them, so pass 1 reads dequantised values (jidctint.c's DEQUANTIZE, moved earlier)
  __shared__ __attribute__((aligned(16))) uint16_t s_qz[3][64];
  __shared__ uint8_t s_pos[64];
  __shared__ uint32_t s_col[8];
  // the strip's samples reuse the coefficient rows once pass 2 has read them (one barrier more,
  // 4 KB less: 8 workgroups per CU instead of 6)
  uint8_t *const s_y = reinterpret_cast<uint8_t *>(&blkv[0][0]);
  uint8_t *const s_cb = s_y + 8 * kStripY, *const s_cr = s_cb + 8 * kStripC;
  static_assert(8 * (kStripY + 2 * kStripC) <= (int)sizeof(blkv), "strip fits the coefficient rows");
  const uint32_t t = threadIdx.x, slot = t >> 3, r = t & 7;
  // block slot b = h * 32 + slot: 0..29 luma (MCU m0 + b / 2, block b % 2), 30..46 Cb and
  // 47..63 Cr of MCU m0 - 1 + j
  bool valid[kIdctNb];
  uint32_t kk[kIdctNb], lx[kIdctNb];  // component; its strip column block
  uint4 raw[kIdctNb];
  int32_t dc[kIdctNb];
  uint32_t nm[kIdctNb];
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {
    const int b = h * 32 + (int)slot;
    const int k = b < 30 ? 0 : b < 47 ? 1 : 2;
    const int j = k == 0 ? b : k == 1 ? b - 30 : b - 47;
    const int mx = k == 0 ? m0 + (j >> 1) : m0 - 1 + j;
    const int c = k == 0 ? (j & 1) : k + 1;
    kk[h] = (uint32_t)k;
    lx[h] = (uint32_t)j;
    valid[h] = mx >= 0 && mx < mcux;
    const uint64_t mcu = (uint64_t)my * mcux + (valid[h] ? mx : 0);
    const uint64_t bi = valid[h] ? F.blk0 + mcu * 4 + c : F.blk0;
    const uint64_t di = valid[h] ? F.dcbase[k] + mcu * (k == 0 ? 2 : 1) + (k == 0 ? (j & 1) : 0) : F.dcbase[0];
    raw[h] = *reinterpret_cast<const uint4 *>(coef + bi * 64 + r * 8);
    dc[h] = dcseq[di];
    nm[h] = nmask ? (uint32_t)nmask[bi] : 0xFFu;
  }
  if (t < 192) s_qz[t >> 6][kZigOf[t & 63]] = F.q[t >> 6][t & 63];
  if (t < 64) s_pos[t] = kIdctPos[t];
  if (t < 8) s_col[t] = kIdctCol[t];
  __syncthreads();
  const uint2 pos8 = *reinterpret_cast<const uint2 *>(&s_pos[r * 8]);
  const uint32_t colg = s_col[r];
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {
    if (!valid[h]) continue;
    const bool st = (nm[h] >> r) & 1;  // a row the write pass did not store is zero
    const uint32_t qw[4] = {st ? raw[h].x : 0u, st ? raw[h].y : 0u, st ? raw[h].z : 0u, st ? raw[h].w : 0u};
    const uint4 q4 = *reinterpret_cast<const uint4 *>(&s_qz[kk[h]][r * 8]);
    const uint32_t qq[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int32_t v = (r == 0 && j == 0) ? (int32_t)(int16_t)dc[h] : (int32_t)(int16_t)(qw[j >> 1] >> (16 * (j & 1)));
      const uint32_t at = ((j < 4 ? pos8.x : pos8.y) >> (8 * (j & 3))) & 0xFF;
      blkv[h * 32 + slot][at] = __mul24(v, (int32_t)((qq[j >> 1] >> (16 * (j & 1))) & 0xFFFF));
    }
  }
  __syncthreads();
  int32_t col[kIdctNb][8];
  const auto pass1 = [&](auto m24) {  // pass 1: column r, dequantised
#pragma unroll
    for (int h = 0; h < kIdctNb; ++h) {
      if (!valid[h]) continue;
      int32_t in[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) in[i] = blkv[h * 32 + slot][i * 8 + ((colg >> (4 * i)) & 7)];
      idct_line<decltype(m24)::value>(in, col[h], 11);
    }
  };
  if (F.flags & kDecIdct24) pass1(BoolTag<true>{});
  else pass1(BoolTag<false>{});
  __syncthreads();
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {
    if (!valid[h]) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) blkv[h * 32 + slot][i * 9 + r] = col[h][i];
  }
  __syncthreads();
  uint2 row8[kIdctNb];
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {  // pass 2: row r
    int32_t in[8];
    uint32_t out[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) in[i] = blkv[h * 32 + slot][r * 9 + i];
    idct_row_limited(in, out);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo |= out[i] << (8 * i);
      hi |= out[i + 4] << (8 * i);
    }
    row8[h] = make_uint2(lo, hi);
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < kIdctNb; ++h) {  // into the strip
    if (!valid[h]) continue;
    uint8_t *dst = kk[h] == 0 ? s_y + r * kStripY : (kk[h] == 1 ? s_cb : s_cr) + r * kStripC;
    *reinterpret_cast<uint2 *>(dst + lx[h] * 8) = row8[h];
  }
  __syncthreads();
  // colour: 8 pixels x 1 row (ONE: 30 x 8 threads) or x 2 rows (30 x 4 threads)
  constexpr int kRows = ONE ? 1 : 2;
  if (t >= (uint32_t)(2 * kStripMcus * (8 / kRows))) return;
  const int px = (int)t % (2 * kStripMcus), rp = (int)t / (2 * kStripMcus);
  const int y0 = my * 8 + kRows * rp, x0 = m0 * 16 + px * 8;
  if (y0 >= g.h || x0 >= g.w) return;
  const StripPlanes sp{s_y, s_cb, s_cr, my * 8, m0 * 16, (m0 - 1) * 8};
  color_rows<1, true, StripPlanes, ONE>(F, g, sp, eplanes, efr, y0, x0, !ONE && y0 + 1 < g.h, 0, invert);
}

// ---- encoder: colour + downsampling + FDCT + quantisation -----------------------------------

// 24-bit multiplies for the forward DCT.  A 32-bit v_mul_lo_u32 / v_mad_u64_u32 (what `*` on
// int32 compiles to) issues at a quarter of the VALU rate; v_mul_i32_i24 / v_mad_i32_i24 at the
// full rate, and they are exact here: the encoder's samples are 8-bit, so pass 1's multiplicands
// are sums of at most four differences of level-shifted samples (|x| < 2^10) and pass 2's of at
// most four pass-1 outputs (|x| < 2^15), every constant is under 2^15, and each product fits
// the 32-bit result the C code computes.
__device__ __forceinline__ int32_t m24(int32_t a, int32_t b) { return __mul24(a, b); }

// jfdctint.c jpeg_fdct_islow, one line; pass 0 = rows, 1 = columns
__device__ __forceinline__ void fdct_islow_line(int32_t p[8], int pass) {
  int32_t tmp0 = p[0] + p[7], tmp7 = p[0] - p[7];
  int32_t tmp1 = p[1] + p[6], tmp6 = p[1] - p[6];
  int32_t tmp2 = p[2] + p[5], tmp5 = p[2] - p[5];
  int32_t tmp3 = p[3] + p[4], tmp4 = p[3] - p[4];
  const int32_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3;
  const int32_t tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  const int sh = pass ? 15 : 11;
  const int32_t rnd = 1 << (sh - 1);  // DESCALE's rounding, folded into the products' sums
  if (!pass) {
    p[0] = (tmp10 + tmp11) * 4;
    p[4] = (tmp10 - tmp11) * 4;
  } else {
    p[0] = DESCALE(tmp10 + tmp11, 2);
    p[4] = DESCALE(tmp10 - tmp11, 2);
  }
  const int32_t z1 = m24(tmp12 + tmp13, FIX_0_541196100) + rnd;
  p[2] = (z1 + m24(tmp13, FIX_0_765366865)) >> sh;
  p[6] = (z1 + m24(tmp12, -FIX_1_847759065)) >> sh;
  const int32_t z5 = m24(tmp4 + tmp6 + tmp5 + tmp7, FIX_1_175875602) + rnd;
  const int32_t z1o = m24(tmp4 + tmp7, -FIX_0_899976223), z2 = m24(tmp5 + tmp6, -FIX_2_562915447);
  const int32_t z3 = m24(tmp4 + tmp6, -FIX_1_961570560) + z5, z4 = m24(tmp5 + tmp7, -FIX_0_390180644) + z5;
  p[7] = (m24(tmp4, FIX_0_298631336) + z1o + z3) >> sh;
  p[5] = (m24(tmp5, FIX_2_053119869) + z2 + z4) >> sh;
  p[3] = (m24(tmp6, FIX_3_072711026) + z2 + z3) >> sh;
  p[1] = (m24(tmp7, FIX_1_501321110) + z1o + z4) >> sh;
}

// jfdctfst.c jpeg_fdct_ifast, one line (both passes identical)
__device__ __forceinline__ void fdct_ifast_line(int32_t p[8]) {
  int32_t tmp0 = p[0] + p[7], tmp7 = p[0] - p[7];
  int32_t tmp1 = p[1] + p[6], tmp6 = p[1] - p[6];
  int32_t tmp2 = p[2] + p[5], tmp5 = p[2] - p[5];
  int32_t tmp3 = p[3] + p[4], tmp4 = p[3] - p[4];
  int32_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3;
  int32_t tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  p[0] = tmp10 + tmp11;
  p[4] = tmp10 - tmp11;
  const int32_t z1 = m24(tmp12 + tmp13, 181) >> 8;
  p[2] = tmp13 + z1;
  p[6] = tmp13 - z1;
  tmp10 = tmp4 + tmp5;
  tmp11 = tmp5 + tmp6;
  tmp12 = tmp6 + tmp7;
  const int32_t z5 = m24(tmp10 - tmp12, 98) >> 8;
  const int32_t z2 = (m24(tmp10, 139) >> 8) + z5;
  const int32_t z4 = (m24(tmp12, 334) >> 8) + z5;
  const int32_t z3 = m24(tmp11, 181) >> 8;
  const int32_t z11 = tmp7 + z3, z13 = tmp7 - z3;
  p[5] = z13 + z2;
  p[3] = z13 - z2;
  p[1] = z11 + z4;
  p[7] = z11 - z4;
}

// jcdctmgr.c quantize (16-bit DCTELEM reciprocal form), branch-free: the sign is taken off,
// the magnitude scaled by the reciprocal and the sign put back (two's complement), instead of
// a divergent if / else that ran both sides in every wave.  |t| + corr <= 2^16 and recip <
// 2^16, so the unsigned product fits 32 bits as in the C code's UDCTELEM2.
// `sh` carries shift + 16 (0..31) in its low 5 bits; its upper bits are ignored, as the
// hardware's shift does, so the table word that holds it serves other fields too.
__device__ __forceinline__ int16_t quantize(int32_t x, uint32_t recip, uint32_t corr, uint32_t sh) {
  const int32_t t = (int16_t)x;
  const int32_t sg = t >> 31;
  const uint32_t a = (uint32_t)((t ^ sg) - sg);
  const uint32_t p = ((a + corr) * recip) >> (sh & 31);
  return (int16_t)(((int32_t)p ^ sg) - sg);
}

// Zero a block's AC bit image (kAcScratchWords words, a 16-B aligned row) with its 8 lanes: 16-B
// stores, at most two per lane, instead of a loop of 4-B ones
static_assert(kAcScratchWords % 4 == 0 && kAcScratchWords / 4 <= 16, "two 16-B stores per lane");
__device__ __forceinline__ void clear_ac_words(uint32_t *acw_slot, uint32_t r) {
  uint4 *a4 = reinterpret_cast<uint4 *>(acw_slot);
  a4[r] = make_uint4(0, 0, 0, 0);
  if (r + 8 < (uint32_t)kAcScratchWords / 4) a4[r + 8] = make_uint4(0, 0, 0, 0);
}

// The 8 * H pixels of rows py .. py + R - 1 from px that one lane converts, edges replicated
// (jccolor.c on expand_right_edge / expand_bottom_edge input).  Loading and converting are
// split, so a wave issues its pixel loads before it waits on anything else: inside the image
// every row's words are in flight at once; a lane at the right edge (or on an unaligned row)
// reads its pixels one by one while converting.
template <int H, int R>
struct RowPix {
  uint32_t wd[R][6 * H];
  const uint8_t *row[R];
  bool fast;
};
// The loads are unconditional (a lane with no block, or on the slow path, reads `dummy`, any
// 16-B aligned 24 * H readable bytes): with no branch around them the wait for the table load
// issued before them does not have to wait for them too.
template <int H, int R>
__device__ __forceinline__ void rows_load(const uint8_t *img, int w, int h, int px, int py, bool real,
                                          const uint8_t *dummy, RowPix<H, R> &p) {
  p.fast = real && px + 8 * H <= w;
#pragma unroll
  for (int y = 0; y < R; ++y) {
    p.row[y] = img + (size_t)min(py + y, h - 1) * w * 3;
    p.fast = p.fast && ((reinterpret_cast<uintptr_t>(p.row[y]) + (uintptr_t)px * 3) & 3) == 0;
  }
#pragma unroll
  for (int y = 0; y < R; ++y) {
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(p.fast ? p.row[y] + (size_t)px * 3 : dummy);
#pragma unroll
    for (int i = 0; i < 6 * H; ++i) p.wd[y][i] = s32[i];
  }
}

// One component of those pixels, summed over groups of H pixels and over the R rows into v[0..7]
template <int H, int R>
__device__ __forceinline__ void rows_conv(const RowPix<H, R> &p, int w, int px, const Ycc &q, int32_t v[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0;
  if (p.fast) {
#pragma unroll
    for (int y = 0; y < R; ++y)
#pragma unroll
      for (int x = 0; x < 8 * H; ++x) {
        const int c0 = (int)((p.wd[y][(3 * x) / 4] >> (8 * ((3 * x) % 4))) & 0xFF);
        const int c1 = (int)((p.wd[y][(3 * x + 1) / 4] >> (8 * ((3 * x + 1) % 4))) & 0xFF);
        const int c2 = (int)((p.wd[y][(3 * x + 2) / 4] >> (8 * ((3 * x + 2) % 4))) & 0xFF);
        v[x / H] += ycc_apply(q, c0, c1, c2);
      }
  } else {
#pragma unroll
    for (int y = 0; y < R; ++y)
#pragma unroll
      for (int x = 0; x < 8 * H; ++x) {
        const uint8_t *b = p.row[y] + (size_t)min(px + x, w - 1) * 3;
        v[x / H] += ycc_apply(q, b[0], b[1], b[2]);
      }
  }
}

// Pass 1 for one lane: component q of row sy of its block's samples, downsampled by (H, R)
// (jcsample.c): (1, 1) fullsize, (2, 1) h2v1 (bias 0, 1 alternating), (2, 2) h2v2 (bias 1, 2),
// (1, 2) int_downsample over two rows (TJSAMP_440: (sum + 1) / 2), with the level shift
// (jcdctmgr.c: sample - CENTERJSAMPLE) folded into each path's last add, exactly:
// (s + c - 128 * 2^n) >> n == ((s + c) >> n) - 128 for an arithmetic shift; then the FDCT's row
// pass into the block's workspace row.  Between issuing the pixel loads and using them, the
// lane stores its part of the workgroup's table image (tw, loaded before the pixels) and zeroes
// its AC words, so the wave waits on the two memory round trips once, not one after the other.
template <int H, int R, bool FAST>
__device__ __forceinline__ void fdct_pass1(const uint8_t *img, const Geom &g, int bx, int sy, Ycc q, bool real,
                                           const uint4 &tw, const uint8_t *dummy, uint4 *s_tab, uint32_t *acw_slot,
                                           uint32_t r, int32_t *wsrow) {
  RowPix<H, R> p;
  const int px = bx * 8 * H;
  rows_load<H, R>(img, g.w, g.h, px, sy * R, real, dummy, p);
  if (threadIdx.x < 192) s_tab[threadIdx.x] = tw;
  clear_ac_words(acw_slot, r);
  if (!real) return;
  if (H == 1 && R == 1) q.bias -= 128 << 16;
  int32_t v[8];
  rows_conv<H, R>(p, g.w, px, q, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (H == 2 && R == 1) v[j] = (v[j] + (j & 1) - 256) >> 1;
    if (H == 2 && R == 2) v[j] = (v[j] + 1 + (j & 1) - 512) >> 2;
    if (H == 1 && R == 2) v[j] = (v[j] + 1 - 256) >> 1;
  }
  if (FAST) fdct_ifast_line(v);
  else fdct_islow_line(v, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) wsrow[j] = v[j];
}

// Pass 1 from the invert path's sample planes (enc_sample_rows): row sy of the block is one
// 8-byte load; level shift and the FDCT's row pass.  The table image store and the AC-word
// clearing sit between the load and its use, as in fdct_pass1.
// VF_ABL (timing ablations, tools/exp builds only; outputs are wrong): bit 0 no sample-plane
// loads in k_fdct, bit 1 no FDCT arithmetic, bit 2 no AC coding, bit 3 no sample-plane stores in
// k_idct_color422, bit 4 no table image (only with bit 2), bit 5 no quantisation, bit 6 no
// coefficient list (only with bit 2)
#ifndef VF_ABL
#define VF_ABL 0
#endif
template <bool FAST>
__device__ __forceinline__ void fdct_pass1_planes(const uint8_t *plane, int pitch, int bx, int sy, bool real,
                                                  const uint4 &tw, const uint8_t *dummy, uint4 *s_tab,
                                                  uint32_t *acw_slot, uint32_t r, int32_t *wsrow) {
#if VF_ABL & 1
  const uint2 q = make_uint2((uint32_t)(bx * 0x01010101) ^ (uint32_t)sy, (uint32_t)(sy * 0x01030507) ^ r);
#else
  const uint2 q = *reinterpret_cast<const uint2 *>(real ? plane + (size_t)sy * pitch + bx * 8 : dummy);
#endif
  if (threadIdx.x < 192) s_tab[threadIdx.x] = tw;
  clear_ac_words(acw_slot, r);
  if (!real) return;
  int32_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (int32_t)(((j < 4 ? q.x : q.y) >> (8 * (j & 3))) & 0xFF) - 128;
#if !(VF_ABL & 2)
  if (FAST) fdct_ifast_line(v);
  else fdct_islow_line(v, 0);
#endif
#pragma unroll
  for (int j = 0; j < 8; ++j) wsrow[j] = v[j];
}

constexpr uint32_t kAcWords = kAcScratchWords;

// AC scratch layout: blocks in groups of 64, word i of the 64 blocks of a group contiguous,
// so k_pack's one-thread-per-block reads of word i are one 256-B span per wave instead of
// 64 lines 208 B apart (the host rounds the allocation up to whole groups).
__device__ __forceinline__ uint64_t acs_idx(uint64_t gb, uint32_t i) {
  return (gb >> 6) * (64ull * kAcWords) + (uint64_t)i * 64 + (gb & 63);
}

// MSB-first bits of one lane into an LDS word image, from bit `pos` on.  The image is zeroed
// beforehand and every word is OR-ed, so a lane's first and last words, shared with its
// neighbours, need no special case.  put() has no branch: it always ORs the word the bits
// reached -- when that word is complete, its 32 bits; otherwise the prefix of it known so far,
// which the complete word contains (OR is idempotent on it).  acc keeps the pending n < 32
// bits in its low end; bits above them are stale and never read (alignbit takes 32 bits).
struct LdsBits {
  uint32_t *w;
  uint32_t wi, n;
  uint64_t acc;
  __device__ __forceinline__ LdsBits(uint32_t *words, uint32_t pos) : w(words), wi(pos >> 5), n(pos & 31), acc(0) {}
  __device__ __forceinline__ void put(uint32_t bits, uint32_t size) {  // size <= 32
    acc = (acc << size) | bits;
    n += size;
    const bool full = n >= 32;
    const uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32);
    atomicOr(w + wi, __builtin_amdgcn_alignbit(full ? hi : lo, full ? lo : 0u, n & 31));
    wi += full ? 1u : 0u;
    n &= 31;
  }
  __device__ __forceinline__ void finish() {  // the pending bits of a word put() completed last
    atomicOr(w + wi, __builtin_amdgcn_alignbit((uint32_t)acc, 0u, n));
  }
};

// Lane-group (8 lanes) primitives by DPP / swizzle instead of ds_bpermute: OR over the group,
// inclusive prefix sum, and the group's lane 7.
__device__ __forceinline__ uint32_t or8(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return x;
}
__device__ __forceinline__ uint32_t scan8(uint32_t x, uint32_t r) {  // r = lane & 7
  uint32_t y = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += r >= 1 ? y : 0u;
  y = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += r >= 2 ? y : 0u;
  y = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += r >= 4 ? y : 0u;
  return x;
}
__device__ __forceinline__ uint32_t last8(uint32_t x) {  // swizzle: lane (i & 0x18) | 7
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0xF8);
}


// Position of zigzag coefficient zz in a block's row of qo: its 16-B octet (zz / 8, the AC
// coder's one ds_read_b128 per lane) is XOR-ed with (0, 5, 2, 7)[slot % 4].  The row is 32
// dwords (0 mod 32), so unswizzled, the 4 blocks of a 32-lane half store every 16-bit
// coefficient to the same banks: 48 extra LDS cycles per wave over pass 2's eight scattered
// stores; swizzled, 12 (searched exhaustively over per-slot octet XORs that keep the b128
// reads conflict-free; SQ_LDS_BANK_CONFLICT 3.45e8 per 1080p batch before,
// profiles/r01_jpeg_pmc_sq.txt).
__device__ __forceinline__ uint32_t qo_at(uint32_t slot, uint32_t zz) {
  return zz ^ (((0x7250u >> (4 * (slot & 3))) & 7) << 3);  // the octet index's XOR, in place
}

// 8 lanes per block.  A wave codes block-in-MCU c of 8 consecutive MCUs (an MCU group); a
// workgroup takes 4 (group, c) units in group-major order.  The component, its sampling, its
// colour coefficients and its tables are therefore wave-uniform: they live in scalar
// registers, no lane divides, and luma / chroma paths never diverge in a wave.
// After quantisation the 8 lanes Huffman-code the block's AC coefficients (jchuff.c
// encode_one_block, AC part): the quantised block sits in LDS in zigzag order, so lane r
// reads zigzag positions 8r..8r+7 with one 16-B load.  Each lane finds the run before each of
// its nonzero coefficients from a running "previous nonzero" position (seeded from the block's
// 64-bit nonzero mask), lists them by rank, and the 8 lanes code the list 8 nonzeros per round
// (ZRL for each 16 zeros of a run): one code lookup per lane and round, offsets from an 8-lane
// scan of the round's bit counts, bits ORed into an LDS image of the block's AC stream that is
// then copied out.
// Outputs per block: quantised DC, AC bit count, AC bits (MSB-first words).
// Specialised per batch on the chroma downsampling (CH, CV) and the DCT (islow / ifast): luma
// is full size in every TurboJPEG subsampling, so each wave's sample path and butterflies are
// fixed at compile time.
constexpr uint32_t kFdctGroup = 8;  // MCUs per wave
// PL: pix holds the invert path's sample planes (EncFrame::eplane_off; CH, CV unused)
template <int CH, int CV, bool FAST, bool PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_fdct(const EncFrame *__restrict__ fr, const EncTables *tab, const uint8_t *pix,
                                              int16_t *dcq, uint32_t *acbits, uint32_t *acscr, int bgr) {
  const EncFrame &F = fr[blockIdx.y];
  const Geom &g = F.g;
  const uint32_t bpm = (uint32_t)g.bpm, nmcu = (uint32_t)g.nmcu;
  const uint32_t ngroups = (nmcu + kFdctGroup - 1) / kFdctGroup;
  if (blockIdx.x * 4 >= ngroups * bpm) return;
  // Per block slot: the pass-1 workspace ws (8 x 9 words); pass 2 reads its column and writes
  // the quantised block qo over the slot's first 32 words (a wave's LDS reads complete before
  // its later writes, and the slot's 8 lanes are in one wave); the AC coder reads qo into
  // registers and then writes its coefficient list over the slot.  Shared this way, the
  // workgroup's LDS is 18.5 KB: 8 workgroups per CU.
  __shared__ int32_t ws[32][8][9];
  __shared__ __attribute__((aligned(16))) uint32_t acw[32][kAcWords];  // rows of 208 B: 16-B aligned
  // The table image (EncTables::fdct_lds): s_q[t][n] = {recip | corr << 16, (shift + 16) | qo
  // position of zigzag(n) for slot % 4 == j at bits 8 + 6j} (pass 2's lane reads one 8-B entry
  // per coefficient, 8 lanes 64 contiguous bytes, and uses the second word as it is for the
  // shift and through one bit-field extract for its store address), then s_ac[t][256].  Its
  // load is issued first; fdct_pass1 stores it after issuing the pixel loads.
  __shared__ uint4 s_tab[192];
#if VF_ABL & 16
  const uint4 tw = make_uint4(threadIdx.x, 0x3F3F3F3Fu, threadIdx.x, 0x3F3F3F3Fu);
#else
  const uint4 tw = threadIdx.x < 192 ? reinterpret_cast<const uint4 *>(tab->fdct_lds)[threadIdx.x] : make_uint4(0, 0, 0, 0);
#endif
  const uint2 (*const s_q)[64] = reinterpret_cast<const uint2 (*)[64]>(s_tab);
  const uint32_t (*const s_ac)[256] = reinterpret_cast<const uint32_t (*)[256]>(reinterpret_cast<const uint32_t *>(s_tab) + 256);
  const uint32_t slot = threadIdx.x >> 3, r = threadIdx.x & 7, lm = slot & (kFdctGroup - 1);
  int16_t *const qo = reinterpret_cast<int16_t *>(&ws[slot][0][0]);
  const uint32_t unit = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t grp = unit / bpm, c = unit - grp * bpm;  // scalar
  const uint32_t mcu = grp * kFdctGroup + lm;
  const uint32_t b = mcu * bpm + c;
  uint32_t k = 0, bx = 0, by = 0;
  bool real = false;
  if (grp < ngroups) {
    k = (uint32_t)g.bcomp[c];
    const uint32_t mcux = (uint32_t)g.mcux;
    uint32_t mx = (grp * kFdctGroup) % mcux + lm, my = (grp * kFdctGroup) / mcux;
    while (mx >= mcux) mx -= mcux, ++my;  // once at most unless the frame is under 8 MCUs wide
    bx = mx * (uint32_t)g.mh[k] + (uint32_t)g.bxo[c];
    by = my * (uint32_t)g.mv[k] + (uint32_t)g.byo[c];
    real = mcu < nmcu && bx < (uint32_t)g.wb[k] && by < (uint32_t)g.hb[k];  // dummy blocks: k_len / k_pack
  }
  const uint8_t *img = pix + F.img_off;
  const uint8_t *dummy = reinterpret_cast<const uint8_t *>(tab->fdct_lds);  // 3 KB, 16-B aligned
  {  // pass 1: row r of the block's samples (the component is wave-uniform: luma is full size)
    const int sy = min((int)(by * 8 + r), (int)g.rrows[k] - 1);
    if constexpr (PL) {
      fdct_pass1_planes<FAST>(pix + F.eplane_off[k], g.wb[k] * 8, (int)bx, sy, real, tw, dummy, s_tab, acw[slot], r,
                              ws[slot][r]);
    } else {
      const Ycc q = ycc_coefs((int)k, bgr != 0);
      if (k == 0) fdct_pass1<1, 1, FAST>(img, g, (int)bx, sy, q, real, tw, dummy, s_tab, acw[slot], r, ws[slot][r]);
      else fdct_pass1<CH, CV, FAST>(img, g, (int)bx, sy, q, real, tw, dummy, s_tab, acw[slot], r, ws[slot][r]);
    }
  }
  __syncthreads();  // publishes the table image
  const int t = k > 0;
  if (real) {  // pass 2: column r, quantised
    int32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ws[slot][i][r];
#if !(VF_ABL & 2)
    if (FAST) fdct_ifast_line(v);
    else fdct_islow_line(v, 1);
#endif
    const uint32_t qsel = 8 + 6 * (slot & 3);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint2 q = s_q[t][i * 8 + r];
#if VF_ABL & 32
      qo[(q.y >> qsel) & 63] = (int16_t)(v[i] >> 3);
#else
      qo[(q.y >> qsel) & 63] = quantize(v[i], q.x & 0xFFFF, q.x >> 16, q.y);
#endif
    }
  }
  // From here on a block's 8 lanes read only their own slot's LDS (qo, ws, acw), written by
  // lanes of the same wave: LDS operations of a wave complete in order, so a wavefront fence
  // (ordering for the compiler) replaces the workgroup barriers -- the 4 waves of a workgroup
  // code different components (luma waves finish pass 1 sooner than chroma waves) and no
  // longer wait for one another.
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // AC Huffman coding; every lane of the wave takes part in the 8-lane shuffles
  int vz[8];
  {
    const uint4 q4 = real ? *reinterpret_cast<const uint4 *>(&qo[qo_at(slot, r * 8)]) : make_uint4(0, 0, 0, 0);
    const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) vz[j] = (int)(int16_t)(qw[j >> 1] >> (16 * (j & 1)));
  }
  uint32_t m8 = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (vz[j] != 0 && (r | j) != 0) m8 |= 1u << j;
  const uint64_t mask = ((uint64_t)or8(r < 4 ? 0u : m8 << (8 * (r - 4))) << 32) | or8(r < 4 ? m8 << (8 * r) : 0u);
  const uint32_t zrl = s_ac[t][0xF0], eobc = s_ac[t][0x00];
  const uint32_t zlen = zrl & 0xFF;
  const bool eob = mask == 0 || (63 - __clzll(mask)) < 63;
  // the last nonzero position before this lane's first (the DC position starts the first run)
  int prev = r ? 63 - __clzll((mask | 1ull) & ((1ull << (8 * r)) - 1)) : 0;
  // The block's nonzero AC coefficients in zigzag order, as (run << 16) | (uint16) value, in
  // the slot's pass-1 workspace (free since pass 2): lane r writes its own at their ranks.
  // Then rounds of 8: in round i lane r codes nonzero 8i + r, so a block costs ceil(nnz / 8)
  // rounds of one code per lane instead of eight coefficient slots per lane (a 1080p q85 frame
  // averages ~4 nonzero AC coefficients per block).  The list is written without branches: a
  // zero coefficient's entry goes to the lane's own spare word (64 + r; the list uses <= 63).
#if VF_ABL & 64
  if (m8 != 12345u) {
    if (real && r == 0) {
      dcq[F.blk0 + b] = (int16_t)vz[0];
      acbits[F.blk0 + b] = eob ? 2u : 3u;
    }
    return;
  }
#endif
  const uint32_t cnt = __popc(m8);
  const uint32_t rinc = scan8(cnt, r);
  const uint32_t nnz = last8(rinc);
  uint32_t *const lst = reinterpret_cast<uint32_t *>(&ws[slot][0][0]);
  {
    uint32_t *wp = lst + (rinc - cnt);
    uint32_t *const spare = lst + 64 + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = 8 * (int)r + j;
      const bool nz = (m8 >> j) & 1;
      *(nz ? wp : spare) = ((uint32_t)(kk - prev - 1) << 16) | (uint32_t)(uint16_t)vz[j];
      wp += nz ? 1 : 0;
      prev = nz ? kk : prev;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the group's list, read across its lanes
  uint32_t off = 0;  // the block's AC bits so far (the same in its 8 lanes)
#if VF_ABL & 4
  if (nnz != 12345) {
    if (real && r == 0) {
      dcq[F.blk0 + b] = (int16_t)vz[0];
      acbits[F.blk0 + b] = 2u;
    }
    return;
  }
#endif
  for (uint32_t q0 = 0; __ballot(q0 < nnz) != 0; q0 += 8) {
    const uint32_t q = q0 + r;
    const bool act = q < nnz;
    const uint32_t ent = act ? lst[q] : 0u;
    const uint32_t run = ent >> 16;
    const int v = (int)(int16_t)(ent & 0xFFFF);
    const uint32_t av = (uint32_t)(v < 0 ? -v : v);
    const uint32_t nb = 32 - __clz(av);
    const uint32_t e = s_ac[t][((run & 15) << 4) + (nb & 15)];
    const uint32_t code = ((e >> 8) << nb) | ((uint32_t)(v < 0 ? v - 1 : v) & ((1u << nb) - 1));
    const uint32_t clen = (e & 0xFF) + nb;
    const uint32_t nzr = run >> 4;  // ZRL codes before it
    const uint32_t nbits = act ? __umul24(nzr, zlen) + clen : 0u;
    const uint32_t incl = scan8(nbits, r);
    if (act) {
      LdsBits out(acw[slot], off + incl - nbits);
      for (uint32_t z = nzr; z; --z) out.put(zrl >> 8, zlen);
      out.put(code, clen);
      out.finish();
    }
    off += last8(incl);
  }
  if (real && eob && r == 0) {  // jchuff.c: EOB unless the last coefficient is nonzero
    LdsBits out(acw[slot], off);
    out.put(eobc >> 8, eobc & 0xFF);
    out.finish();
  }
  const uint32_t total = off + (eob ? (eobc & 0xFF) : 0u);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the block's AC words, from its own lanes
  if (real) {
    const uint64_t gb = F.blk0 + b;
    const uint32_t nw = (total + 31) >> 5;
    for (uint32_t i = r; i < nw; i += 8) acscr[acs_idx(gb, i)] = acw[slot][i];
    if (r == 0) {
      dcq[gb] = (int16_t)vz[0];  // lane 0 holds zigzag positions 0..7
      acbits[gb] = total;
    }
  }
}

// ---- encoder: DC coding, bit offsets, packing --------------------------------------------------

// Stream positions [a, b) of a word (position 0 = its first bit on the wire) as a mask of the word
// in memory (big-endian bytes).  A word two writers share is merged with an AND of the writer's
// positions cleared and an OR of its bits: the writers' positions are disjoint, so any order of
// the four atomics leaves both writers' bits and nothing stale -- the stream needs no zeroing
// first (it used to take a kernel of its own per batch).
__device__ __forceinline__ uint32_t wire_mask(uint32_t a, uint32_t b) {
  const uint32_t m = (0xFFFFFFFFu >> a) & (b >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> b));
  return bswap32(m);
}
__device__ __forceinline__ void merge_word(uint32_t *w, uint32_t mask, uint32_t v) {
  atomicAnd(w, ~mask);
  atomicOr(w, v);
}

struct BitSink {  // MSB-first bits into big-endian words at a bit offset
  uint32_t *w;
  uint32_t wi;
  uint64_t acc;
  uint32_t n, s;  // s: the first word's first position
  bool first;
  __device__ __forceinline__ BitSink(uint32_t *words, uint32_t off)
      : w(words), wi(off >> 5), acc(0), n(off & 31), s(off & 31), first(true) {}
  __device__ __forceinline__ void put(uint32_t code, uint32_t size) {  // size <= 32
    acc = (acc << size) | code;
    n += size;
    if (n >= 32) {
      n -= 32;
      const uint32_t v = (uint32_t)(acc >> n);
      if (first) merge_word(w + wi, wire_mask(s, 32), bswap32(v));  // shares its leading bits with the previous block
      else w[wi] = bswap32(v);
      first = false;
      ++wi;
      acc &= n ? ((1ull << n) - 1) : 0ull;
    }
  }
  __device__ __forceinline__ void finish() {
    if (n) merge_word(w + wi, wire_mask(first ? s : 0u, n), bswap32((uint32_t)(acc << (32 - n))));
  }
};

__device__ __forceinline__ uint32_t dc_category(int diff) {
  const uint32_t a = (uint32_t)(diff < 0 ? -diff : diff);
  return a ? 32 - __clz(a) : 0;
}

// bits of every block: DC code + extra bits + AC bits (a dummy block's AC is one EOB).  Also
// leaves what k_pack needs without re-deriving the DC prediction: pre = (DC code and extra
// bits << 5) | their length (<= 16 + 11 bits), and for a dummy block acbits = kDummyAc |
// (EOB code << 5) | EOB length (k_fdct never writes a dummy block's acbits).
constexpr uint32_t kDummyAc = 0x80000000u;
// A wave takes block-in-MCU c of 64 consecutive MCUs (as k_fdct groups them): the component,
// its geometry and its tables are wave-uniform (scalar), and each lane locates its MCU with
// one division instead of several per DC lookup.
__device__ __forceinline__ int enc_dc_at(const Geom &g, const int16_t *dcq, int mx, int my, int xi, int yi, int mh,
                                         int mv, int wb, int hb, int cf) {
  for (;;) {  // jccoefct.c dummy blocks: the left neighbour, or the last block of the row above
    const int bx = mx * mh + xi, by = my * mv + yi;
    if (by >= hb) {
      yi -= 1;
      xi = mh - 1;
      continue;
    }
    if (bx >= wb) {
      xi -= 1;
      continue;
    }
    return dcq[((uint64_t)my * (uint32_t)g.mcux + (uint32_t)mx) * (uint32_t)g.bpm + (uint32_t)(cf + yi * mh + xi)];
  }
}

__global__ __launch_bounds__(256) void k_len(const EncFrame *__restrict__ fr, const EncTables *tab, const int16_t *dcq,
                                             uint32_t *acbits, uint32_t *bits, uint32_t *pre) {
  const EncFrame &F = fr[blockIdx.y];
  const Geom &g = F.g;
  const uint32_t bpm = (uint32_t)g.bpm, nmcu = (uint32_t)g.nmcu, mcux = (uint32_t)g.mcux;
  const uint32_t ngroups = (nmcu + 63) / 64;
  const uint32_t unit = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= ngroups * bpm) return;
  const uint32_t grp = unit / bpm, c = unit - grp * bpm;  // scalar
  const uint32_t mcu = grp * 64 + (threadIdx.x & 63);
  if (mcu >= nmcu) return;
  const int k = g.bcomp[c], mh = g.mh[k], mv = g.mv[k], wb = g.wb[k], hb = g.hb[k], cf = g.cfirst[k];
  int mx = (int)((grp * 64) % mcux + (threadIdx.x & 63)), my = (int)((grp * 64) / mcux);
  while (mx >= (int)mcux) mx -= (int)mcux, ++my;  // once at most unless the frame is under 64 MCUs wide
  const int dc = enc_dc_at(g, dcq + F.blk0, mx, my, g.bxo[c], g.byo[c], mh, mv, wb, hb, cf);
  int pred = 0;  // jchuff.c: the previous block of the same component in scan order
  if ((int)c > cf) {
    pred = enc_dc_at(g, dcq + F.blk0, mx, my, g.bxo[c - 1], g.byo[c - 1], mh, mv, wb, hb, cf);
  } else if (mcu > 0) {
    const int pmx = mx > 0 ? mx - 1 : (int)mcux - 1, pmy = mx > 0 ? my : my - 1;
    pred = enc_dc_at(g, dcq + F.blk0, pmx, pmy, mh - 1, mv - 1, mh, mv, wb, hb, cf);
  }
  const bool dummy = mx * mh + g.bxo[c] >= wb || my * mv + g.byo[c] >= hb;
  const int diff = dc - pred;
  const int t = k > 0;
  const uint32_t nb = dc_category(diff);
  const uint32_t e = tab->dc[t][nb];
  const uint32_t extra = nb ? ((uint32_t)(diff < 0 ? diff - 1 : diff) & ((1u << nb) - 1)) : 0u;
  const uint64_t gb = F.blk0 + (uint64_t)mcu * bpm + c;
  pre[gb] = ((((e >> 8) << nb) | extra) << 5) | ((e & 0xFF) + nb);
  uint32_t ac;
  if (dummy) {
    const uint32_t eob = tab->ac[t][0];
    acbits[gb] = kDummyAc | ((eob >> 8) << 5) | (eob & 0xFF);
    ac = eob & 0xFF;
  } else {
    ac = acbits[gb];
  }
  bits[gb] = (e & 0xFF) + nb + ac;
}

// MSB-first bits into big-endian words of an LDS image, every word OR-ed (the image is
// zeroed first, and a lane's first and last words are shared with its neighbours)
struct LdsSink {
  uint32_t *w;
  uint32_t wi;
  uint64_t acc;
  uint32_t n;
  __device__ __forceinline__ LdsSink(uint32_t *words, uint32_t off) : w(words), wi(off >> 5), acc(0), n(off & 31) {}
  __device__ __forceinline__ void put(uint32_t code, uint32_t size) {  // size <= 32
    acc = (acc << size) | code;
    n += size;
    if (n >= 32) {
      n -= 32;
      atomicOr(w + wi, bswap32((uint32_t)(acc >> n)));
      ++wi;
      acc &= n ? ((1ull << n) - 1) : 0ull;
    }
  }
  __device__ __forceinline__ void finish() {
    if (n) atomicOr(w + wi, bswap32((uint32_t)(acc << (32 - n))));
  }
};

// one block's bits: DC code + extra bits (pre), then its AC words (or a dummy block's EOB)
template <typename Sink>
__device__ __forceinline__ void pack_block(Sink &out, uint32_t p, uint32_t n, uint32_t a0, const uint32_t *aw) {
  out.put(p >> 5, p & 31);
  if (n & kDummyAc) {
    out.put((n & ~kDummyAc) >> 5, n & 31);
  } else if (n) {
    if (n >= 32) {
      out.put(a0, 32);
      for (uint32_t i = 1; i < (n >> 5); ++i) out.put(aw[64 * i], 32);
      if (n & 31) out.put(aw[64 * (n >> 5)] >> (32 - (n & 31)), n & 31);
    } else {
      out.put(a0 >> (32 - n), n);
    }
  }
  out.finish();
}

// Every block writes its bits at its offset.  The 64 blocks of a wave are consecutive, so
// their bits are one contiguous span: the wave assembles it in an LDS image (LDS atomics
// where neighbouring blocks share a word) and stores it as whole words, with global atomics
// only on the span's first and last words (shared with the neighbouring waves; merged under
// their masks, wire_mask).  Writing
// each block straight to memory took two global atomics per block, most of them on words a
// neighbouring lane of the same instruction also hit.  A span over kPackWords (very detailed
// content) takes that direct path.
constexpr uint32_t kPackWords = 1024;  // per wave: 64 blocks of 512 bits on average
__global__ __launch_bounds__(256) void k_pack(const EncFrame *__restrict__ fr, const uint32_t *pre, const uint32_t *acbits,
                                              const uint32_t *acscr, const uint32_t *bitoff, uint8_t *stream) {
  __shared__ uint32_t s_img[4][kPackWords];
  const EncFrame &F = fr[blockIdx.y];
  const uint32_t nblocks = (uint32_t)F.g.nblocks, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t bw0 = blockIdx.x * 256 + wv * 64;  // the wave's first block (uniform)
  if (bw0 >= nblocks) return;
  const uint32_t last = min(63u, nblocks - 1 - bw0), b = bw0 + lane;
  const bool valid = lane <= last;
  const uint64_t gb = F.blk0 + (valid ? b : bw0);
  const uint32_t p = pre[gb], n = acbits[gb], off = bitoff[gb];
  const uint32_t *aw = acscr + acs_idx(gb, 0);  // word i at aw[64 * i]
  const uint32_t a0 = aw[0];  // issued with the other loads; unused by a dummy block
  uint32_t *words = reinterpret_cast<uint32_t *>(stream + F.bits_off);
  const uint32_t len = (p & 31) + ((n & kDummyAc) ? (n & 31) : n);
  const uint32_t w0 = __shfl(off, 0) >> 5, w1 = (__shfl(off + len, (int)last) + 31) >> 5;  // words [w0, w1)
  const uint32_t nw = w1 - w0;
  if (nw > kPackWords) {  // wave-uniform
    if (valid) {
      BitSink out(words, off);
      pack_block(out, p, n, a0, aw);
    }
    return;
  }
  uint32_t *img = s_img[wv];
  for (uint32_t i = lane; i < nw; i += 64) img[i] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (valid) {
    LdsSink out(img, off - w0 * 32);
    pack_block(out, p, n, a0, aw);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t s0 = __shfl(off, 0) & 31, e1 = __shfl(off + len, (int)last) - (w1 - 1) * 32;  // 1..32
  for (uint32_t i = lane; i < nw; i += 64) {
    const uint32_t v = img[i];
    if (i == 0 || i == nw - 1) merge_word(words + w0 + i, wire_mask(i == 0 ? s0 : 0u, i == nw - 1 ? e1 : 32u), v);
    else words[w0 + i] = v;
  }
}

// ---- encoder: byte stuffing, header, EOI ------------------------------------------------------

// the 16 bytes of the packed stream at i0, the final partial byte padded with ones
__device__ __forceinline__ uint32_t ff_bytes(const uint8_t *s, uint32_t nbytes, uint32_t tb, uint32_t i0,
                                             uint8_t *bytes) {
  // one 16-B load: i0 is a multiple of 16 below nbytes, and a frame's stream region (256-B
  // aligned) holds at least nbytes + 16 bytes (the host's bits_cap)
  const uint4 q = *reinterpret_cast<const uint4 *>(s + i0);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
  uint32_t n = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t i = i0 + j;
    uint8_t v = i < nbytes ? (uint8_t)(qw[j >> 2] >> (8 * (j & 3))) : 0;
    if (i == nbytes - 1 && (tb & 7)) v |= (uint8_t)(0xFF >> (tb & 7));
    bytes[j] = v;
    n += (i < nbytes && v == 0xFF);
  }
  return n;
}

__global__ __launch_bounds__(256) void k_ff_count(const EncFrame *__restrict__ fr, const uint32_t *total_bits,
                                                  const uint8_t *stream, uint32_t *cnt) {
  // Grid-stride over the frame's worst-case tiles: the stream fills only the first few (a
  // 1080p q85 frame ~45 of ~1,500), so one workgroup per tile launched ~48 k workgroups per
  // batch that mostly wrote a zero.  Tiles past the stream's end get their zero count here.
  // the frame's fields in registers: read through the reference after a store, they were
  // re-loaded from memory (with a wait) on every iteration
  const uint32_t ntiles_max = fr[blockIdx.y].ntiles_max, tile0 = fr[blockIdx.y].tile0;
  const uint8_t *src = stream + fr[blockIdx.y].bits_off;
  __shared__ uint32_t sh[4];
  const uint32_t tb = total_bits[blockIdx.y], nbytes = (tb + 7) >> 3;
  for (uint32_t t = blockIdx.x; t < ntiles_max; t += gridDim.x) {  // t is uniform
    if (t * kTile < nbytes) {
      uint8_t bytes[16];
      const uint32_t i0 = t * kTile + threadIdx.x * 16;
      const uint32_t n = i0 < nbytes ? ff_bytes(src, nbytes, tb, i0, bytes) : 0;
      uint32_t tot;
      (void)wg_excl_scan(n, sh, &tot);
      if (threadIdx.x == 0) cnt[tile0 + t] = tot;
      __syncthreads();  // sh is reused by the next tile's scan
    } else if (threadIdx.x == 0) {
      cnt[tile0 + t] = 0;
    }
  }
}

// Writes the finished JPEGs packed back to back, frame f at the sum over g < f of align64(size
// of g), so the host fetches a batch with one copy (a separate compaction kernel used to move
// them there: 6-8 us per batch and a second pass over the output).  Every size is known here:
// the header, the stream bytes (total_bits) and the stuffed bytes (nff).
__global__ __launch_bounds__(256) void k_ff_write(const EncFrame *__restrict__ fr, const uint32_t *total_bits,
                                                  const uint8_t *stream, const uint32_t *off, const uint32_t *nff,
                                                  const uint8_t *hdr, uint8_t *pack, uint64_t *out_size) {
  const EncFrame &F = fr[blockIdx.y];
  // the frame's fields in registers (k_ff_count)
  const uint32_t hdr_len = F.hdr_len, hdr_off = F.hdr_off, tile0 = F.tile0;
  const uint8_t *src = stream + F.bits_off;
  const uint32_t tb = total_bits[blockIdx.y], nbytes = (tb + 7) >> 3;
  const uint32_t ntiles = (nbytes + kTile - 1) / kTile;
  __shared__ uint32_t sh[4];
  __shared__ uint64_t s_pack;
  if (threadIdx.x < 64) {  // the frame's packed offset (one wave; a batch has <= 65535 frames)
    uint64_t acc = 0;
    for (uint32_t g = threadIdx.x; g < blockIdx.y; g += 64)
      acc += ((uint64_t)fr[g].hdr_len + ((total_bits[g] + 7) >> 3) + nff[g] + 2 + 63) & ~63ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (threadIdx.x == 0) s_pack = acc;
  }
  __syncthreads();
  uint8_t *o = pack + s_pack;
  __shared__ uint8_t s_out[2 * kTile];  // a tile's bytes after stuffing (at most every byte 0xFF)
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {  // grid-stride over the stream's tiles
    if (t == 0)
      for (uint32_t j = threadIdx.x; j < hdr_len; j += 256) o[j] = hdr[hdr_off + j];
    uint8_t bytes[16];
    const uint32_t i0 = t * kTile + threadIdx.x * 16;
    const uint32_t n = i0 < nbytes ? ff_bytes(src, nbytes, tb, i0, bytes) : 0;
    uint32_t tot;
    // the tile's stuffed bytes are assembled in LDS, then stored as aligned dwords (per-lane
    // byte stores at scattered offsets were 16-32 store instructions per lane)
    uint32_t lp = threadIdx.x * 16 + wg_excl_scan(n, sh, &tot);
    for (int j = 0; j < 16; ++j) {
      if (i0 + j >= nbytes) break;
      s_out[lp++] = bytes[j];
      if (bytes[j] == 0xFF) s_out[lp++] = 0;
    }
    __syncthreads();
    const uint32_t len = min((uint32_t)kTile, nbytes - t * kTile) + tot;
    uint8_t *dst = o + (uint64_t)hdr_len + t * kTile + off[tile0 + t];
    const uint32_t head = min((uint32_t)(-(uintptr_t)dst & 3), len), nw = (len - head) >> 2;
    if (threadIdx.x < head) dst[threadIdx.x] = s_out[threadIdx.x];
    for (uint32_t i = threadIdx.x; i < nw; i += 256) {
      const uint32_t a = head + 4 * i;
      reinterpret_cast<uint32_t *>(dst + head)[i] = (uint32_t)s_out[a] | ((uint32_t)s_out[a + 1] << 8) |
                                                    ((uint32_t)s_out[a + 2] << 16) | ((uint32_t)s_out[a + 3] << 24);
    }
    const uint32_t tail = head + 4 * nw;
    if (threadIdx.x < len - tail) dst[tail + threadIdx.x] = s_out[tail + threadIdx.x];
    if (t == ntiles - 1 && threadIdx.x == 0) {
      const uint64_t size = (uint64_t)hdr_len + nbytes + nff[blockIdx.y] + 2;
      o[size - 2] = 0xFF;
      o[size - 1] = 0xD9;
      out_size[blockIdx.y] = size;
    }
    __syncthreads();  // sh is reused by the next tile's scan
  }
}

}  // namespace

// ---- launchers -------------------------------------------------------------------------------

hipError_t scan_u32(const ScanSeg *segs, int nseg, uint32_t max_tiles, const uint32_t *in, uint32_t *out,
                    uint32_t *tsum, uint32_t *totals, bool inclusive, hipStream_t s) {
  return seg_scan<uint32_t>(segs, nseg, max_tiles, in, out, tsum, totals, inclusive, s);
}

hipError_t scan_i32(const ScanSeg *segs, int nseg, uint32_t max_tiles, const int32_t *in, int32_t *out,
                    int32_t *tsum, int32_t *totals, bool inclusive, hipStream_t s) {
  return seg_scan<int32_t>(segs, nseg, max_tiles, in, out, tsum, totals, inclusive, s);
}

hipError_t dec_unstuff_count(const DecSeg *__restrict__ sg, int nseg, uint32_t max_tiles, const uint8_t *in, uint32_t *tile_cnt,
                             hipStream_t s) {
  if (nseg <= 0 || !max_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_unstuff_count, dim3(max_tiles, (unsigned)nseg), dim3(256), 0, s, sg, in, tile_cnt);
  return hipGetLastError();
}

hipError_t dec_unstuff_write(const DecSeg *__restrict__ sg, int nseg, uint32_t max_tiles, const uint8_t *in,
                             const uint32_t *tile_off, const uint32_t *us_len, uint8_t *us, hipStream_t s) {
  if (nseg <= 0 || !max_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_unstuff_write, dim3(max_tiles, (unsigned)nseg), dim3(256), 0, s, sg, in, tile_off, us_len, us);
  return hipGetLastError();
}

hipError_t dec_sync(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, int nseg, uint32_t max_sub, const uint8_t *us,
                    const uint32_t *us_len, const uint64_t *exit_in, uint64_t *exit_out, const uint32_t *cnt_in,
                    uint32_t *cnt_out, uint64_t *used, uint64_t *ck, uint32_t *ckrem, uint32_t *changed, int pass,
                    hipStream_t s) {
  if (nseg <= 0 || !max_sub) return hipSuccess;
  hipLaunchKernelGGL(k_sync, dim3((max_sub + 255) / 256, (unsigned)nseg), dim3(256), 0, s, sg, fr, us, us_len,
                     exit_in, exit_out, cnt_in, cnt_out, used, ck, ckrem, changed, pass);
  return hipGetLastError();
}

hipError_t dec_syncg(int G, const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, int nseg, uint32_t max_sub,
                     const uint8_t *us, const uint32_t *us_len, uint64_t *exits, uint32_t *cnts, uint64_t *used,
                     uint64_t *ck, uint32_t *ckrem, uint32_t *changed, int pass, uint32_t warm, int tabs4,
                     hipStream_t s) {
  if (nseg <= 0 || !max_sub) return hipSuccess;
  warm = std::min<uint32_t>(warm, kSyncWarmMax) & ~31u;
#define VF_SYNCG(GG, ND, LS)                                                                                      \
  if (G == GG && (ND == 2) == (tabs4 != 0) && LS == (tabs4 == 2)) {                                               \
    const uint32_t span = syncg_threads(GG) * GG;                                                                 \
    hipLaunchKernelGGL((k_syncg<GG, ND, LS>), dim3((max_sub + span - 1) / span, (unsigned)nseg),                  \
                       dim3(syncg_threads(GG)), 0, s, sg, fr, us, us_len, exits, cnts, used, ck, ckrem, changed,  \
                       pass, warm);                                                                               \
    return hipGetLastError();                                                                                     \
  }
  VF_SYNCG(1, 3, false)
  VF_SYNCG(2, 3, false)
  VF_SYNCG(3, 3, false)
  VF_SYNCG(4, 3, false)
  VF_SYNCG(8, 3, false)
  VF_SYNCG(4, 2, false)
  VF_SYNCG(5, 2, false)
  VF_SYNCG(4, 2, true)
  VF_SYNCG(5, 2, true)
#undef VF_SYNCG
  return hipErrorInvalidValue;
}

hipError_t dec_sync_spec(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, int nseg, uint32_t max_wg, const uint8_t *us,
                         const uint32_t *us_len, const SpecBufs &b, uint64_t *exit_out, uint32_t *cnt_out,
                         uint32_t *unresolved, int lsb, hipStream_t s) {
  if (nseg <= 0 || !max_wg) return hipSuccess;
  if (lsb) hipLaunchKernelGGL(k_spec<true>, dim3(max_wg, (unsigned)nseg), dim3(256), 0, s, sg, fr, us, us_len, b);
  else hipLaunchKernelGGL(k_spec<false>, dim3(max_wg, (unsigned)nseg), dim3(256), 0, s, sg, fr, us, us_len, b);
  hipLaunchKernelGGL(k_resolve, dim3((unsigned)nseg), dim3(256), 0, s, sg, fr, us, us_len, b, unresolved);
  hipLaunchKernelGGL(k_finalize, dim3(max_wg, (unsigned)nseg), dim3(256), 0, s, sg, fr, us_len, b, exit_out, cnt_out);
  return hipGetLastError();
}

hipError_t dec_write(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, int nseg, uint32_t max_sub, const uint8_t *us,
                     const uint32_t *us_len, const uint64_t *exits, const uint32_t *bstart, int16_t *coef,
                     int32_t *dcseq, uint8_t *nmask, hipStream_t s) {
  if (nseg <= 0 || !max_sub) return hipSuccess;
  const dim3 grid((max_sub + 255) / 256, (unsigned)nseg);
  if (nmask)
    hipLaunchKernelGGL(k_write<true>, grid, dim3(256), 0, s, sg, fr, us, us_len, exits, bstart, coef, dcseq, nmask);
  else
    hipLaunchKernelGGL(k_write<false>, grid, dim3(256), 0, s, sg, fr, us, us_len, exits, bstart, coef, dcseq, nmask);
  return hipGetLastError();
}

hipError_t dec_write4(const DecSeg *__restrict__ sg, const DecFrame *__restrict__ fr, int nseg, uint32_t max_sub, const uint8_t *us,
                      const uint32_t *us_len, const uint64_t *exits, const uint32_t *cnt, const uint64_t *ck,
                      const uint32_t *ckrem, const uint32_t *bstart, int16_t *coef, int32_t *dcseq, uint8_t *nmask,
                      hipStream_t s) {
  if (nseg <= 0 || !max_sub) return hipSuccess;
  const dim3 grid((max_sub + 63) / 64, (unsigned)nseg);
  if (nmask)
    hipLaunchKernelGGL(k_write4<true>, grid, dim3(256), 0, s, sg, fr, us, us_len, exits, cnt, ck, ckrem, bstart, coef,
                       dcseq, nmask);
  else
    hipLaunchKernelGGL(k_write4<false>, grid, dim3(256), 0, s, sg, fr, us, us_len, exits, cnt, ck, ckrem, bstart, coef,
                       dcseq, nmask);
  return hipGetLastError();
}

hipError_t dec_idct(const DecFrame *__restrict__ fr, int n, uint32_t max_blocks, const int16_t *coef, const int32_t *dcseq,
                    const uint8_t *nmask, uint8_t *planes, hipStream_t s) {
  if (n <= 0 || !max_blocks) return hipSuccess;
  // 4 units of 16 blocks per workgroup; a frame has ceil(nmcu / 16) * bpm <= (nblocks + 150) / 16 units
  hipLaunchKernelGGL(k_idct, dim3((max_blocks + 150 + 63) / 64, (unsigned)n), dim3(256), 0, s, fr,
                     coef, dcseq, nmask, planes);
  return hipGetLastError();
}

hipError_t dec_color(const DecFrame *__restrict__ fr, int n, int max_w, int max_h, const uint8_t *planes, uint8_t *pix, int bgr,
                     int invert, const EncFrame *efr, int cm, hipStream_t s) {
  if (n <= 0 || max_w <= 0 || max_h <= 0) return hipSuccess;
  const dim3 grid((unsigned)((max_w + 2047) / 2048), (unsigned)((max_h + 1) / 2), (unsigned)n);
#define VF_COLOR(E, C) hipLaunchKernelGGL((k_color<E, C>), grid, dim3(256), 0, s, fr, planes, pix, efr, bgr, invert)
  if (efr) {
    if (cm == 0) VF_COLOR(true, 0);
    else if (cm == 1) VF_COLOR(true, 1);
    else if (cm == 2) VF_COLOR(true, 2);
    else if (cm == 3) VF_COLOR(true, 3);
    else VF_COLOR(true, -1);
  } else {
    if (cm == 0) VF_COLOR(false, 0);
    else if (cm == 1) VF_COLOR(false, 1);
    else if (cm == 2) VF_COLOR(false, 2);
    else if (cm == 3) VF_COLOR(false, 3);
    else VF_COLOR(false, -1);
  }
#undef VF_COLOR
  return hipGetLastError();
}

hipError_t dec_idct_color422(const DecFrame *__restrict__ fr, int n, int max_w, int max_h, const int16_t *coef,
                             const int32_t *dcseq, const uint8_t *nmask, uint8_t *eplanes, const EncFrame *efr,
                             int invert, int one_row, hipStream_t s) {
  if (n <= 0 || max_w <= 0 || max_h <= 0) return hipSuccess;
  const unsigned mcux = (unsigned)((max_w + 15) / 16), mcuy = (unsigned)((max_h + 7) / 8);
  const dim3 grid((mcux + kStripMcus - 1) / kStripMcus, mcuy, (unsigned)n);
  if (one_row)
    hipLaunchKernelGGL(k_idct_color422<true>, grid, dim3(256), 0, s, fr, coef, dcseq, nmask, eplanes, efr, invert);
  else
    hipLaunchKernelGGL(k_idct_color422<false>, grid, dim3(256), 0, s, fr, coef, dcseq, nmask, eplanes, efr, invert);
  return hipGetLastError();
}

hipError_t enc_fdct(const EncFrame *__restrict__ fr, int n, uint32_t max_blocks, const EncTables *tab, const uint8_t *pix,
                    int16_t *dcq, uint32_t *acbits, uint32_t *acscr, int bgr, int fastdct, int ch, int cv, int planes,
                    hipStream_t s) {
  if (n <= 0 || !max_blocks) return hipSuccess;
  // a workgroup takes 4 units of 8 blocks; a frame has ceil(nmcu / 8) * bpm <= (nblocks + 70) / 8 units
  const dim3 grid((max_blocks + 70 + 31) / 32, (unsigned)n);
  if (planes) {  // pix: the invert path's sample planes
    if (fastdct) hipLaunchKernelGGL((k_fdct<1, 1, true, true>), grid, dim3(256), 0, s, fr, tab, pix, dcq, acbits, acscr, bgr);
    else hipLaunchKernelGGL((k_fdct<1, 1, false, true>), grid, dim3(256), 0, s, fr, tab, pix, dcq, acbits, acscr, bgr);
    return hipGetLastError();
  }
#define VF_FDCT(CH, CV)                                                                                              \
  if (ch == CH && cv == CV) {                                                                                        \
    if (fastdct)                                                                                                     \
      hipLaunchKernelGGL((k_fdct<CH, CV, true, false>), grid, dim3(256), 0, s, fr, tab, pix, dcq, acbits, acscr, bgr); \
    else                                                                                                             \
      hipLaunchKernelGGL((k_fdct<CH, CV, false, false>), grid, dim3(256), 0, s, fr, tab, pix, dcq, acbits, acscr, bgr); \
    return hipGetLastError();                                                                                        \
  }
  VF_FDCT(1, 1)
  VF_FDCT(2, 1)
  VF_FDCT(2, 2)
  VF_FDCT(1, 2)
#undef VF_FDCT
  return hipErrorInvalidValue;  // no TurboJPEG subsampling downsamples chroma otherwise
}

hipError_t enc_len(const EncFrame *__restrict__ fr, int n, uint32_t max_blocks, const EncTables *tab, const int16_t *dcq,
                   uint32_t *acbits, uint32_t *bits, uint32_t *pre, hipStream_t s) {
  if (n <= 0 || !max_blocks) return hipSuccess;
  // 4 units of 64 MCUs per workgroup; a frame has ceil(nmcu / 64) * bpm <= nblocks / 64 + 10 units
  hipLaunchKernelGGL(k_len, dim3((max_blocks / 64 + 10 + 3) / 4, (unsigned)n), dim3(256), 0, s, fr, tab, dcq, acbits,
                     bits, pre);
  return hipGetLastError();
}

hipError_t enc_pack(const EncFrame *__restrict__ fr, int n, uint32_t max_blocks, const uint32_t *pre, const uint32_t *acbits,
                    const uint32_t *acscr, const uint32_t *bitoff, const uint32_t *total_bits, uint8_t *stream,
                    hipStream_t s) {
  if (n <= 0 || !max_blocks) return hipSuccess;
  hipLaunchKernelGGL(k_pack, dim3((max_blocks + 255) / 256, (unsigned)n), dim3(256), 0, s, fr, pre, acbits, acscr,
                     bitoff, stream);
  return hipGetLastError();
}

constexpr uint32_t kFFGrid = 64;  // stuffing workgroups per frame (grid-stride over tiles)

hipError_t enc_ff_count(const EncFrame *__restrict__ fr, int n, uint32_t max_tiles, const uint32_t *total_bits,
                        const uint8_t *stream, uint32_t *tile_cnt, hipStream_t s) {
  if (n <= 0 || !max_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_ff_count, dim3(max_tiles < kFFGrid ? max_tiles : kFFGrid, (unsigned)n), dim3(256), 0, s, fr,
                     total_bits, stream, tile_cnt);
  return hipGetLastError();
}

hipError_t enc_ff_write(const EncFrame *__restrict__ fr, int n, uint32_t max_tiles, const uint32_t *total_bits,
                        const uint8_t *stream, const uint32_t *tile_off, const uint32_t *nff, const uint8_t *hdr,
                        uint8_t *pack, uint64_t *out_size, hipStream_t s) {
  if (n <= 0 || !max_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_ff_write, dim3(max_tiles < kFFGrid ? max_tiles : kFFGrid, (unsigned)n), dim3(256), 0, s, fr,
                     total_bits, stream, tile_off, nff, hdr, pack, out_size);
  return hipGetLastError();
}

}  // namespace jpeg
}  // namespace vf
