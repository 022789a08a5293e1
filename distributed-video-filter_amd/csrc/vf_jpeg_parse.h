// vf_jpeg_parse.h — the JPEG host parse on untrusted bytes: marker segments, Huffman tables,
// MCU geometry and the restart-interval (DRI) segment layout.  Host-only C++ (no HIP), so the
// same code is built by hipcc into libvfilter_hip.so and by g++ with ASan / UBSan into the CPU
// fuzzer (tests/fuzz/jpeg_parse_fuzz.cc, tests/test_jpeg_fuzz.py).
//
// The frames a worker decodes arrive from the network (inverter.py:31-32; the reference
// catches whatever the decoder raises at worker.py:74-76): every routine here either accepts
// its input or returns an error, and a frame whose SOF asks for more than the context's pixel
// limit is refused before anything is sized from it.  Marker syntax and table construction
// follow libjpeg-turbo (jdmarker.c, jdhuff.c, jcparam.c, jchuff.c), restated.  Not installed.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "vf_jpeg_types.h"

namespace vf {
namespace jpeg {

inline constexpr uint8_t kNatH[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                           12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                           35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                           58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ITU T.81 Annex K (jcparam.c std tables)
inline constexpr unsigned kLumaQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                             14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                             18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                             49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
inline constexpr unsigned kChromaQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                               24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                               99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                               99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
inline constexpr uint8_t kDcLBits[17] = {0, 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
inline constexpr uint8_t kDcCBits[17] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
inline constexpr uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
inline constexpr uint8_t kAcLBits[17] = {0, 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
inline constexpr uint8_t kAcLVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22,
    0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33,
    0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34,
    0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55,
    0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76,
    0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96,
    0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5,
    0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4,
    0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1,
    0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
inline constexpr uint8_t kAcCBits[17] = {0, 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
inline constexpr uint8_t kAcCVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13,
    0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62,
    0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29,
    0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54,
    0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75,
    0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94,
    0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3,
    0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2,
    0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea,
    0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
inline constexpr int16_t kAanScales[64] = {
    16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  22725, 31521, 29692, 26722, 22725,
    17855, 12299, 6270,  21407, 29692, 27969, 25172, 21407, 16819, 11585, 5906,  19266, 26722,
    25172, 22654, 19266, 15137, 10426, 5315,  16384, 22725, 21407, 19266, 16384, 12873, 8867,
    4520,  12873, 17855, 16819, 15137, 12873, 10114, 6967,  3552,  8867,  12299, 11585, 10426,
    8867,  6967,  4799,  2446,  4520,  6270,  5906,  5315,  4520,  3552,  2446,  1247};
inline constexpr int kSampH[5] = {1, 2, 2, 1, 1};  // TJSAMP_444, 422, 420, GRAY, 440 (turbojpeg.h tjMCUWidth/8)
inline constexpr int kSampV[5] = {1, 1, 2, 1, 2};

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// jcparam.c jpeg_quality_scaling + jpeg_add_quant_table(force_baseline = TRUE)
inline void quality_table(int quality, bool chroma, uint16_t out[64]) {
  quality = std::min(100, std::max(1, quality));
  const int scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  for (int i = 0; i < 64; ++i) {
    long t = ((long)(chroma ? kChromaQ : kLumaQ)[i] * scale + 50L) / 100L;
    out[i] = (uint16_t)std::min(255L, std::max(1L, t));
  }
}

// jchuff.c jpeg_make_c_derived_tbl -> (code << 8) | size by symbol
inline void code_table(const uint8_t bits[17], const uint8_t *vals, uint32_t *out, int nslots) {
  std::memset(out, 0, sizeof(uint32_t) * (size_t)nslots);
  uint32_t code = 0;
  int p = 0;
  for (int l = 1; l <= 16; ++l) {
    for (int i = 0; i < bits[l]; ++i, ++p, ++code)
      if (vals[p] < nslots) out[vals[p]] = (code << 8) | (uint32_t)l;
    code <<= 1;
  }
}

// jdhuff.c jpeg_make_d_derived_tbl + a kLook-bit lookahead.  Rejects what jdhuff.c rejects
// with JERR_BAD_HUFF_TABLE: more than 256 symbols, a code that does not fit its length or is
// all ones (code + 1 >= 2^l; checked per code, BEFORE the lookahead write it would overrun),
// and DC symbols above 15.
inline bool decode_table(const uint8_t bits[17], const uint8_t *vals, bool dc, HuffDec *t) {
  std::memset(t, 0, sizeof *t);
  int p = 0;
  uint32_t code = 0;
  for (int l = 1; l <= 16; ++l) {
    if (bits[l]) {
      t->valoff[l] = p - (int32_t)code;
      for (int i = 0; i < bits[l]; ++i, ++p, ++code) {
        if (p >= 256) return false;
        if (code + 1 >= (1u << l)) return false;  // over-subscribed, or the all-ones code
        if (dc && vals[p] > 15) return false;
        t->vals[p] = vals[p];
        if (l <= kLook) {
          const uint32_t base = code << (kLook - l);
          for (uint32_t s = 0; s < (1u << (kLook - l)); ++s) t->fast[base + s] = (uint16_t)((l << 8) | vals[p]);
        }
      }
      t->maxcode[l] = (int32_t)code - 1;
    } else {
      t->maxcode[l] = -1;
    }
    code <<= 1;
  }
  t->maxcode[17] = 0xFFFFF;
  uint32_t run = 0;
  for (int i = 0; i < 8; ++i) {
    const int l = kLook + 1 + i;
    if (l > 16) {  // no such length: never counted
      t->lim[i] = 0xFFFFFFFFu;
      continue;
    }
    const uint32_t v = t->maxcode[l] < 0 ? 0u : (uint32_t)(t->maxcode[l] + 1) << (16 - l);
    run = v > run ? v : run;
    t->lim[i] = run;
  }
  return true;
}

// jdhuff.c decode semantics folded into one lookup for the sync decoders (see HuffSync)
inline void sync_entry(uint32_t f, bool dc, uint32_t *len, uint32_t *adv) {  // code + extra bits, zigzag advance
  const uint32_t sym = f & 0xFF;
  uint32_t extra;
  if (dc) {
    extra = sym > 16 ? 16 : sym;
    *adv = 1;
  } else {
    extra = sym & 15;
    *adv = extra ? (sym >> 4) + 1 : ((sym >> 4) == 15 ? 16 : 64);
  }
  *len = (f >> 8) + extra;
}

inline void sync_table(const HuffDec &t, bool dc, HuffSync *s) {
  std::memcpy(s->lim, t.lim, sizeof s->lim);
  std::memcpy(s->maxcode, t.maxcode, sizeof s->maxcode);
  std::memcpy(s->valoff, t.valoff, sizeof s->valoff);
  std::memcpy(s->vals, t.vals, sizeof s->vals);
  for (int i = 0; i < (1 << kLook); ++i) {
    const uint32_t f = t.fast[i];
    uint32_t len = 0, adv = 0;
    if (f) sync_entry(f, dc, &len, &adv);
    s->sfast[i] = f ? (uint16_t)((adv << 8) | len) : 0;
  }
}

// DecFrame::spair for one AC table: the next code must be whole inside the kLook - len bits
// known after the first symbol, and its extra bits too
inline void pair_table(const HuffDec &t, uint16_t *pair) {
  for (int i = 0; i < (1 << kLook); ++i) {
    pair[i] = 0;
    const uint32_t f = t.fast[i];
    if (!f) continue;
    uint32_t len, adv;
    sync_entry(f, false, &len, &adv);
    if (len >= (uint32_t)kLook || adv >= 64) continue;
    const uint32_t f2 = t.fast[((uint32_t)i << len) & ((1u << kLook) - 1)];
    if (!f2 || (f2 >> 8) > (uint32_t)kLook - len) continue;
    uint32_t len2, adv2;
    sync_entry(f2, false, &len2, &adv2);
    if (len + len2 <= (uint32_t)kLook) pair[i] = (uint16_t)(((adv + adv2) << 8) | (len + len2));
  }
}

// decode_table + sync_table through a small per-thread cache keyed by the DHT content: the
// frames of a stream share their tables (one encoder, one set of settings), so a batch builds
// each distinct table once per parsing thread instead of 6 times per frame (2 x 2^kLook
// entries each; the table build was most of the host-side parse of a 480p batch).
inline bool build_tables(const uint8_t bits[17], const uint8_t *vals, bool dc, HuffDec *t, HuffSync *s,
                         uint16_t *pair = nullptr) {
  struct Entry {
    bool valid = false, dc = false;
    uint8_t bits[17];
    uint8_t vals[256];
    HuffDec t;
    HuffSync s;
    uint16_t pair[1 << kLook];  // AC tables
  };
  static thread_local Entry cache[4];
  static thread_local int next = 0;
  int nvals = 0;
  for (int l = 1; l <= 16; ++l) nvals += bits[l];
  if (nvals > 256) return false;
  for (Entry &e : cache)
    if (e.valid && e.dc == dc && std::memcmp(e.bits, bits, 17) == 0 && std::memcmp(e.vals, vals, (size_t)nvals) == 0) {
      std::memcpy(t, &e.t, sizeof *t);
      std::memcpy(s, &e.s, sizeof *s);
      if (pair) std::memcpy(pair, e.pair, sizeof e.pair);
      return true;
    }
  if (!decode_table(bits, vals, dc, t)) return false;
  sync_table(*t, dc, s);
  Entry &e = cache[next];
  next = (next + 1) & 3;
  e.valid = true;
  e.dc = dc;
  std::memcpy(e.bits, bits, 17);
  std::memset(e.vals, 0, sizeof e.vals);
  std::memcpy(e.vals, vals, (size_t)nvals);
  std::memcpy(&e.t, t, sizeof *t);
  std::memcpy(&e.s, s, sizeof *s);
  if (dc) std::memset(e.pair, 0, sizeof e.pair);
  else pair_table(*t, e.pair);
  if (pair) std::memcpy(pair, e.pair, sizeof e.pair);
  return true;
}

struct Parsed {
  int w = 0, h = 0, ncomp = 0, restart = 0;
  int id[3] = {}, hs[3] = {}, vs[3] = {}, tq[3] = {}, td[3] = {}, ta[3] = {};
  uint16_t qt[4][64] = {};
  uint8_t dcbits[4][17] = {}, acbits[4][17] = {};
  uint8_t dcvals[4][256] = {}, acvals[4][256] = {};
  int qdef = 0, dcdef = 0, acdef = 0;
  size_t scan_off = 0, scan_end = 0;
  // with DRI: each RSTn marker in the scan as (end of the interval's data before it, marker
  // number); the next interval starts 2 bytes after the data end plus any fill bytes
  std::vector<std::pair<size_t, size_t>> rst;  // (data end, position of the marker's 0xFF)
};

// jdmarker.c restated for baseline / extended sequential Huffman, one interleaved scan
// Markers up to SOS.  With find_scan_end the entropy-coded segment's end is located too (the
// first marker other than RSTn after SOS); memchr skips to each 0xFF (1 in ~256 bytes of
// entropy data), so this costs a fraction of a byte-by-byte scan.  header_info does not need it.
inline int parse(const uint8_t *b, size_t n, Parsed *P, std::string *err, bool find_scan_end = true) {
  auto fail = [&](const char *m) {
    *err = m;
    return -1;
  };
  if (n < 4 || b[0] != 0xFF || b[1] != 0xD8) return fail("not a JPEG (no SOI)");
  size_t p = 2;
  bool sof = false;
  for (;;) {
    while (p < n && b[p] != 0xFF) p++;
    while (p < n && b[p] == 0xFF) p++;
    if (p >= n) return fail("truncated JPEG (no SOS)");
    const int m = b[p++];
    if (m == 0xD9) return fail("EOI before SOS");
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (p + 2 > n) return fail("truncated marker");
    const size_t len = ((size_t)b[p] << 8) | b[p + 1];
    if (len < 2 || p + len > n) return fail("truncated marker segment");
    const uint8_t *s = b + p + 2, *e = b + p + len;
    if (m == 0xDB) {
      while (s < e) {
        const int pq = s[0] >> 4, tq = s[0] & 15;
        ++s;
        if (tq > 3 || s + (pq ? 128 : 64) > e) return fail("bad DQT");
        for (int i = 0; i < 64; ++i) P->qt[tq][kNatH[i]] = pq ? (uint16_t)((s[2 * i] << 8) | s[2 * i + 1]) : s[i];
        P->qdef |= 1 << tq;
        s += pq ? 128 : 64;
      }
    } else if (m == 0xC4) {
      while (s < e) {
        if (s + 17 > e) return fail("bad DHT");
        const int tc = s[0] >> 4, th = s[0] & 15;
        if (tc > 1 || th > 3) return fail("bad DHT class/id");
        int cnt = 0;
        for (int l = 1; l <= 16; ++l) cnt += s[l];
        if (cnt > 256 || s + 17 + cnt > e) return fail("bad DHT counts");
        uint8_t *bits = tc ? P->acbits[th] : P->dcbits[th];
        uint8_t *vals = tc ? P->acvals[th] : P->dcvals[th];
        bits[0] = 0;
        std::memcpy(bits + 1, s + 1, 16);
        std::memcpy(vals, s + 17, (size_t)cnt);
        (tc ? P->acdef : P->dcdef) |= 1 << th;
        s += 17 + cnt;
      }
    } else if (m == 0xC0 || m == 0xC1) {
      if (len < 8 || s[0] != 8) return fail("only 8-bit sequential JPEG is supported");
      P->h = (s[1] << 8) | s[2];
      P->w = (s[3] << 8) | s[4];
      P->ncomp = s[5];
      if (P->ncomp != 1 && P->ncomp != 3) return fail("only 1- or 3-component JPEG is supported");
      if ((int)len != 8 + 3 * P->ncomp || !P->w || !P->h) return fail("bad SOF");
      for (int c = 0; c < P->ncomp; ++c) {
        P->id[c] = s[6 + 3 * c];
        P->hs[c] = s[7 + 3 * c] >> 4;
        P->vs[c] = s[7 + 3 * c] & 15;
        P->tq[c] = s[8 + 3 * c];
        if (P->hs[c] < 1 || P->hs[c] > 4 || P->vs[c] < 1 || P->vs[c] > 4 || P->tq[c] > 3) return fail("bad SOF");
      }
      sof = true;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return fail("progressive / lossless / arithmetic JPEG is not supported");
    } else if (m == 0xDD) {
      if (len != 4) return fail("bad DRI");
      P->restart = (s[0] << 8) | s[1];
    } else if (m == 0xDA) {
      if (!sof) return fail("SOS before SOF");
      if (len < 3) return fail("bad SOS");  // s[0] must lie inside the segment
      const int ns = s[0];
      if (ns != P->ncomp || (int)len != 6 + 2 * ns) return fail("only single-scan interleaved JPEG is supported");
      for (int i = 0; i < ns; ++i) {
        if (s[1 + 2 * i] != P->id[i]) return fail("scan component order differs from the frame");
        P->td[i] = s[2 + 2 * i] >> 4;
        P->ta[i] = s[2 + 2 * i] & 15;
        if (P->td[i] > 3 || P->ta[i] > 3) return fail("bad SOS table id");
      }
      if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0) return fail("not a baseline scan");
      P->scan_off = p + len;
      size_t q = P->scan_off;
      if (!find_scan_end) q = n;
      P->rst.clear();
      while (q + 1 < n) {
        const void *f = std::memchr(b + q, 0xFF, n - q);
        if (!f) {
          q = n;
          break;
        }
        q = (size_t)(static_cast<const uint8_t *>(f) - b);
        if (q + 1 >= n) break;
        const uint8_t nx = b[q + 1];
        if (nx != 0x00 && !(nx >= 0xD0 && nx <= 0xD7) && nx != 0xFF) break;
        if (nx >= 0xD0 && nx <= 0xD7) {  // RSTn: fill bytes (0xFF runs) before it are not data
          size_t e = q;
          const size_t lo = P->rst.empty() ? P->scan_off : P->rst.back().second + 2;
          while (e > lo && b[e - 1] == 0xFF) --e;
          P->rst.emplace_back(e, q);
        }
        ++q;
      }
      P->scan_end = q + 1 < n ? q : n;
      for (int c = 0; c < P->ncomp; ++c)
        if (!(P->qdef >> P->tq[c] & 1) || !(P->dcdef >> P->td[c] & 1) || !(P->acdef >> P->ta[c] & 1))
          return fail("scan refers to an undefined table");
      return 0;
    }
    p += len;
  }
}

inline int subsamp_of(const Parsed &P) {
  if (P.ncomp == 1) return 3;  // TJSAMP_GRAY
  if (P.hs[1] != 1 || P.vs[1] != 1 || P.hs[2] != 1 || P.vs[2] != 1) return -1;
  for (int s = 0; s < 5; ++s)
    if (s != 3 && P.hs[0] == kSampH[s] && P.vs[0] == kSampV[s]) return s;
  if (P.hs[0] == 4 && P.vs[0] == 1) return 5;  // TJSAMP_411
  return -1;
}

inline bool make_geom(int w, int h, int ncomp, const int *hs, const int *vs, Geom *g) {
  std::memset(g, 0, sizeof *g);
  if (w <= 0 || h <= 0 || w > 65535 || h > 65535 || (ncomp != 1 && ncomp != 3)) return false;
  int maxh = 1, maxv = 1;
  for (int k = 0; k < ncomp; ++k) {
    if (hs[k] < 1 || hs[k] > 4 || vs[k] < 1 || vs[k] > 4) return false;
    maxh = std::max(maxh, hs[k]);
    maxv = std::max(maxv, vs[k]);
  }
  for (int k = 0; k < ncomp; ++k)
    if (maxh % hs[k] || maxv % vs[k]) return false;
  g->w = w;
  g->h = h;
  g->ncomp = ncomp;
  g->maxh = maxh;
  g->maxv = maxv;
  if (ncomp == 1) {  // non-interleaved scan: one block per MCU
    g->hs[0] = hs[0];
    g->vs[0] = vs[0];
    g->mh[0] = g->mv[0] = 1;
    g->wb[0] = ceil_div(w * hs[0], 8 * maxh);
    g->hb[0] = ceil_div(h * vs[0], 8 * maxv);
    g->mcux = g->wb[0];
    g->mcuy = g->hb[0];
    g->pw[0] = g->wb[0] * 8;
    g->ph[0] = g->hb[0] * 8;
    g->bpm = 1;
  } else {
    g->mcux = ceil_div(w, 8 * maxh);
    g->mcuy = ceil_div(h, 8 * maxv);
    int b = 0;
    for (int k = 0; k < 3; ++k) {
      g->hs[k] = hs[k];
      g->vs[k] = vs[k];
      g->mh[k] = hs[k];
      g->mv[k] = vs[k];
      g->wb[k] = ceil_div(w * hs[k], 8 * maxh);
      g->hb[k] = ceil_div(h * vs[k], 8 * maxv);
      g->pw[k] = g->mcux * hs[k] * 8;
      g->ph[k] = g->mcuy * vs[k] * 8;
      g->cfirst[k] = b;
      for (int yi = 0; yi < vs[k]; ++yi)
        for (int xi = 0; xi < hs[k]; ++xi) {
          if (b >= kMaxBpm) return false;
          g->bcomp[b] = k;
          g->bxo[b] = xi;
          g->byo[b] = yi;
          ++b;
        }
    }
    g->bpm = b;
  }
  for (int k = 0; k < ncomp; ++k) {  // per-component quotients the kernels would otherwise divide for
    g->he[k] = maxh / g->hs[k];
    g->ve[k] = maxv / g->vs[k];
    g->dw[k] = ceil_div(w * g->hs[k], maxh);
    g->dh[k] = ceil_div(h * g->vs[k], maxv);
    g->rrows[k] = ceil_div(h, maxv) * g->vs[k];
  }
  const long long nm = (long long)g->mcux * g->mcuy;
  if (nm * g->bpm > (1ll << 30)) return false;
  g->nmcu = (int32_t)nm;
  g->nblocks = (int32_t)(nm * g->bpm);
  return true;
}

// The context's size limits on a parsed frame, before anything is sized from it: libjpeg's
// per-side limit and the pixel limit (a 300-byte header may otherwise claim 65535 x 65535).
inline bool check_frame_size(const Parsed &P, uint64_t max_pixels, std::string *err) {
  if (P.w > kMaxDimension || P.h > kMaxDimension) {
    *err = "frame dimensions above 65500 (JPEG_MAX_DIMENSION)";
    return false;
  }
  if ((uint64_t)P.w * (uint64_t)P.h > max_pixels) {
    *err = "frame of " + std::to_string(P.w) + " x " + std::to_string(P.h) + " pixels is above the context's limit of " +
           std::to_string(max_pixels) + " pixels";
    return false;
  }
  return true;
}

// Restart markers of a parsed scan against its geometry: one per interval boundary, numbered
// 0..7 cyclically (jdhuff.c process_restart / jdmarker.c read_restart_marker; libjpeg-turbo
// resynchronises on a missing or misnumbered one with a corrupt-data warning -- refused here),
// and every entropy-coded segment non-empty and under 2^28 bytes.  A marker after the last
// interval with nothing behind it (some encoders end the scan with one) closes an empty
// interval: dropped, as libjpeg-turbo skips it.
inline bool check_segments(const uint8_t *jpeg, Parsed *P, const Geom &g, std::string *err) {
  const size_t nint = P->restart ? ((size_t)g.nmcu + P->restart - 1) / P->restart : 1;
  while (P->rst.size() + 1 > nint && P->rst.back().second + 2 >= P->scan_end) P->rst.pop_back();
  if (P->rst.size() + 1 != nint) {
    *err = P->restart ? "restart markers missing or extra (corrupt JPEG)" : "RSTn marker in a scan without DRI";
    return false;
  }
  for (size_t i = 0; i < P->rst.size(); ++i)
    if (jpeg[P->rst[i].second + 1] != 0xD0 + (i & 7)) {
      *err = "restart marker out of sequence (corrupt JPEG)";
      return false;
    }
  size_t start = P->scan_off;
  for (size_t i = 0; i <= P->rst.size(); ++i) {
    const size_t end = i < P->rst.size() ? P->rst[i].first : P->scan_end;
    if (end <= start || end - start > (1u << 28)) {
      *err = "empty or oversized entropy-coded segment";
      return false;
    }
    if (i < P->rst.size()) start = P->rst[i].second + 2;
  }
  return true;
}

// Everything the decoder's host side derives from one frame's bytes, in order: markers, the
// size limits, geometry, restart layout, and the six Huffman tables (DecFrame's tables).
// The bytes that determine a frame's Huffman tables (per component: its DC and AC tables' code
// counts and symbols), and their FNV-1a hash: frames with equal keys share a DecTabs.
inline uint64_t table_key(const Parsed &P, std::vector<uint8_t> *key) {
  key->clear();
  key->push_back((uint8_t)P.ncomp);
  auto put = [&](const uint8_t bits[17], const uint8_t *vals) {
    int nv = 0;
    for (int l = 1; l <= 16; ++l) nv += bits[l];
    key->insert(key->end(), bits, bits + 17);
    key->insert(key->end(), vals, vals + std::min(nv, 256));
  };
  for (int c = 0; c < P.ncomp; ++c) {
    put(P.dcbits[P.td[c]], P.dcvals[P.td[c]]);
    put(P.acbits[P.ta[c]], P.acvals[P.ta[c]]);
  }
  uint64_t h = 1469598103934665603ull;
  for (uint8_t b : *key) h = (h ^ b) * 1099511628211ull;
  return h;
}

// tables null: markers, geometry and segments only (the Huffman tables are the caller's to build)
inline bool parse_frame(const uint8_t *jpeg, size_t size, uint64_t max_pixels, Parsed *P, Geom *g,
                        HuffDec dc[3], HuffDec ac[3], HuffSync sdc[3], HuffSync sac[3], uint16_t spair[3][1 << kLook],
                        std::string *err) {
  if (!jpeg) {
    *err = "NULL JPEG buffer";
    return false;
  }
  if (parse(jpeg, size, P, err) != 0) return false;
  if (!check_frame_size(*P, max_pixels, err)) return false;
  if (!make_geom(P->w, P->h, P->ncomp, P->hs, P->vs, g)) {
    *err = "unsupported sampling geometry";
    return false;
  }
  if (!check_segments(jpeg, P, *g, err)) return false;
  if (!dc) return true;  // tables built by the caller (Codec::prepare_decode: one set per distinct DHT)
  for (int c = 0; c < P->ncomp; ++c)
    if (!build_tables(P->dcbits[P->td[c]], P->dcvals[P->td[c]], true, &dc[c], &sdc[c]) ||
        !build_tables(P->acbits[P->ta[c]], P->acvals[P->ta[c]], false, &ac[c], &sac[c], spair[c])) {
      *err = "bad Huffman table";
      return false;
    }
  return true;
}

}  // namespace jpeg
}  // namespace vf
