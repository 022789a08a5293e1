/*
 * vf_jpeg_oracle.c — CPU ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the baseline JPEG codec the reference runs in its default mode
 * (use_jpeg=True): every frame is decoded, inverted and re-encoded by PyTurboJPEG
 *     frame = self.jpeg.decode(frame_bytes)        # inverter.py:32
 *     return self.jpeg.encode(inverted)            # inverter.py:44
 * and produced / consumed the same way by the app (webcam_app.py:110,140).  PyTurboJPEG
 * (git HEAD, unpinned, requirements.txt:4) wraps libturbojpeg from libjpeg-turbo; neither is
 * vendored in the reference or installed here.  What is restated is libjpeg-turbo's
 * published algorithm for the calls the reference makes, with PyTurboJPEG's defaults
 * (quality 85, TJSAMP_422, TJPF_BGR, flags 0):
 *
 *   encode: BGR -> YCbCr (jccolor.c rgb_ycc_convert tables), edge replication to whole
 *           MCUs (jcprepct.c / jcsample.c expand_*_edge), h2v1 / h2v2 / generic
 *           downsampling (jcsample.c), forward DCT — accurate integer "islow" (jfdctint.c)
 *           or "ifast" AA&N (jfdctfst.c) — reciprocal quantisation (jcdctmgr.c
 *           compute_reciprocal / quantize), dummy edge blocks (jccoefct.c), sequential
 *           Huffman coding with the Annex K tables (jchuff.c, jcparam.c), JFIF markers
 *           (jcmarker.c), quality scaling (jcparam.c jpeg_quality_scaling);
 *   decode: marker parsing (jdmarker.c), Huffman decoding (jdhuff.c), accurate integer
 *           IDCT with its range-limit table (jidctint.c, jdmaster.c), fancy (triangle)
 *           or replicating upsampling (jdsample.c, with jdmainct.c's edge context rows),
 *           YCbCr -> BGR (jdcolor.c ycc_rgb_convert tables).
 *
 * Which forward DCT libturbojpeg picks at quality < 96 depends on its version (2.x: "fast"
 * unless TJFLAG_ACCURATEDCT; 3.x: accurate unless TJFLAG_FASTDCT), so both are restated and
 * the caller chooses.  Pinning: oracle/jpeg_xcheck.c cross-checks this file against the
 * image's own libjpeg-turbo 2.1.2 (libjpeg.so.8, the codec libturbojpeg wraps), and
 * tests/golden/jpeg/ holds vectors made from it — see DESIGN.md "JPEG".  Never linked into
 * the product (libvfilter_hip.so).
 *
 * Scope: 8-bit baseline / extended-sequential Huffman JPEG (SOF0/SOF1), 1 or 3 components,
 * integer sampling ratios, restart intervals.  Progressive / arithmetic / 12-bit -> error.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "vf_jpeg_oracle.h"

/* ---- shared tables ------------------------------------------------------------------- */

/* zigzag index -> natural index, with 16 guard entries for corrupt run lengths (jutils.c) */
static const int kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

/* ITU T.81 Annex K.1 (natural order), as jcparam.c std_luminance/chrominance_quant_tbl */
static const unsigned kStdLumaQ[64] = {
    16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
    14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
    18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const unsigned kStdChromaQ[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

/* ITU T.81 Annex K.3 Huffman tables (jcparam.c / jstdhuff.c std_huff_tables) */
static const uint8_t kDcLumaBits[17] = {0, 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t kDcLumaVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t kDcChromaBits[17] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t kDcChromaVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t kAcLumaBits[17] = {0, 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t kAcLumaVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
static const uint8_t kAcChromaBits[17] = {0, 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t kAcChromaVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

/* TurboJPEG MCU geometry per TJSAMP_* (turbojpeg.h tjMCUWidth / tjMCUHeight), luma factors */
static const int kSampH[5] = {1, 2, 2, 1, 1};
static const int kSampV[5] = {1, 1, 2, 1, 2};

static int ceil_div(int a, int b) { return (a + b - 1) / b; }

/* ---- encoder --------------------------------------------------------------------------- */

/* jcparam.c jpeg_quality_scaling + jpeg_add_quant_table(force_baseline=TRUE) */
int vfo_jpeg_quality_table(int quality, int chroma, uint16_t out[64]) {
  if (quality <= 0) quality = 1;
  if (quality > 100) quality = 100;
  const int scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  const unsigned *basic = chroma ? kStdChromaQ : kStdLumaQ;
  for (int i = 0; i < 64; ++i) {
    long t = ((long)basic[i] * scale + 50L) / 100L;
    if (t <= 0) t = 1;
    if (t > 32767) t = 32767;
    if (t > 255) t = 255;
    out[i] = (uint16_t)t;
  }
  return 0;
}

/* jccolor.c rgb_ycc_start tables (SCALEBITS 16); Y alone for grayscale (rgb_gray_convert) */
#define SCALEBITS 16
#define ONE_HALF ((int32_t)1 << (SCALEBITS - 1))
#define FIX16(x) ((int32_t)((x) * (1L << SCALEBITS) + 0.5))
#define CBCR_OFFSET ((int32_t)128 << SCALEBITS)

static void rgb_to_ycc(int r, int g, int b, uint8_t *y, uint8_t *cb, uint8_t *cr) {
  *y = (uint8_t)((FIX16(0.29900) * r + FIX16(0.58700) * g + FIX16(0.11400) * b + ONE_HALF) >> SCALEBITS);
  *cb = (uint8_t)((-FIX16(0.16874) * r - FIX16(0.33126) * g + FIX16(0.50000) * b + CBCR_OFFSET +
                   ONE_HALF - 1) >> SCALEBITS);
  *cr = (uint8_t)((FIX16(0.50000) * r - FIX16(0.41869) * g - FIX16(0.08131) * b + CBCR_OFFSET +
                   ONE_HALF - 1) >> SCALEBITS);
}

/* jfdctint.c jpeg_fdct_islow (CONST_BITS 13, PASS1_BITS 2); output scaled by 8 */
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

void vfo_fdct_islow(int32_t d[64]) {
  for (int pass = 0; pass < 2; ++pass) {
    const int st = pass ? 8 : 1; /* element stride inside a line */
    const int ls = pass ? 1 : 8; /* stride between lines */
    const int sh = pass ? 13 + 2 : 13 - 2;
    for (int l = 0; l < 8; ++l) {
      int32_t *p = d + l * ls;
      int32_t tmp0 = p[0 * st] + p[7 * st], tmp7 = p[0 * st] - p[7 * st];
      int32_t tmp1 = p[1 * st] + p[6 * st], tmp6 = p[1 * st] - p[6 * st];
      int32_t tmp2 = p[2 * st] + p[5 * st], tmp5 = p[2 * st] - p[5 * st];
      int32_t tmp3 = p[3 * st] + p[4 * st], tmp4 = p[3 * st] - p[4 * st];
      int32_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3;
      int32_t tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
      int32_t z1, z2, z3, z4, z5;
      if (!pass) {
        p[0 * st] = (tmp10 + tmp11) * 4; /* LEFT_SHIFT(.., PASS1_BITS) */
        p[4 * st] = (tmp10 - tmp11) * 4;
      } else {
        p[0 * st] = DESCALE(tmp10 + tmp11, 2);
        p[4 * st] = DESCALE(tmp10 - tmp11, 2);
      }
      z1 = (tmp12 + tmp13) * FIX_0_541196100;
      p[2 * st] = DESCALE(z1 + tmp13 * FIX_0_765366865, sh);
      p[6 * st] = DESCALE(z1 + tmp12 * -FIX_1_847759065, sh);
      z1 = tmp4 + tmp7;
      z2 = tmp5 + tmp6;
      z3 = tmp4 + tmp6;
      z4 = tmp5 + tmp7;
      z5 = (z3 + z4) * FIX_1_175875602;
      tmp4 *= FIX_0_298631336;
      tmp5 *= FIX_2_053119869;
      tmp6 *= FIX_3_072711026;
      tmp7 *= FIX_1_501321110;
      z1 *= -FIX_0_899976223;
      z2 *= -FIX_2_562915447;
      z3 *= -FIX_1_961570560;
      z4 *= -FIX_0_390180644;
      z3 += z5;
      z4 += z5;
      p[7 * st] = DESCALE(tmp4 + z1 + z3, sh);
      p[5 * st] = DESCALE(tmp5 + z2 + z4, sh);
      p[3 * st] = DESCALE(tmp6 + z2 + z3, sh);
      p[1 * st] = DESCALE(tmp7 + z1 + z4, sh);
    }
  }
}

/* jfdctfst.c jpeg_fdct_ifast (CONST_BITS 8, truncating MULTIPLY); output scaled by aanscales */
#define IFAST_MUL(v, c) (((v) * (c)) >> 8)
void vfo_fdct_ifast(int32_t d[64]) {
  for (int pass = 0; pass < 2; ++pass) {
    const int st = pass ? 8 : 1;
    const int ls = pass ? 1 : 8;
    for (int l = 0; l < 8; ++l) {
      int32_t *p = d + l * ls;
      int32_t tmp0 = p[0 * st] + p[7 * st], tmp7 = p[0 * st] - p[7 * st];
      int32_t tmp1 = p[1 * st] + p[6 * st], tmp6 = p[1 * st] - p[6 * st];
      int32_t tmp2 = p[2 * st] + p[5 * st], tmp5 = p[2 * st] - p[5 * st];
      int32_t tmp3 = p[3 * st] + p[4 * st], tmp4 = p[3 * st] - p[4 * st];
      int32_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3;
      int32_t tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
      p[0 * st] = tmp10 + tmp11;
      p[4 * st] = tmp10 - tmp11;
      int32_t z1 = IFAST_MUL(tmp12 + tmp13, 181);
      p[2 * st] = tmp13 + z1;
      p[6 * st] = tmp13 - z1;
      tmp10 = tmp4 + tmp5;
      tmp11 = tmp5 + tmp6;
      tmp12 = tmp6 + tmp7;
      int32_t z5 = IFAST_MUL(tmp10 - tmp12, 98);
      int32_t z2 = IFAST_MUL(tmp10, 139) + z5;
      int32_t z4 = IFAST_MUL(tmp12, 334) + z5;
      int32_t z3 = IFAST_MUL(tmp11, 181);
      int32_t z11 = tmp7 + z3, z13 = tmp7 - z3;
      p[5 * st] = z13 + z2;
      p[3 * st] = z13 - z2;
      p[1 * st] = z11 + z4;
      p[7 * st] = z11 - z4;
    }
  }
}

/* jcdctmgr.c aanscales (14-bit) */
static const int16_t kAanScales[64] = {
    16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  22725, 31521, 29692, 26722, 22725,
    17855, 12299, 6270,  21407, 29692, 27969, 25172, 21407, 16819, 11585, 5906,  19266, 26722,
    25172, 22654, 19266, 15137, 10426, 5315,  16384, 22725, 21407, 19266, 16384, 12873, 8867,
    4520,  12873, 17855, 16819, 15137, 12873, 10114, 6967,  3552,  8867,  12299, 11585, 10426,
    8867,  6967,  4799,  2446,  4520,  6270,  5906,  5315,  4520,  3552,  2446,  1247};

/* jcdctmgr.c compute_reciprocal with 16-bit DCTELEM (the SIMD build) */
void vfo_jpeg_divisors(const uint16_t q[64], int fastdct, uint16_t recip[64], uint16_t corr[64],
                       int16_t shift[64]) {
  for (int i = 0; i < 64; ++i) {
    uint32_t divisor = fastdct ? (uint32_t)(((int32_t)q[i] * kAanScales[i] + (1 << 10)) >> 11)
                               : (uint32_t)q[i] << 3;
    if (divisor == 1) {
      recip[i] = 1;
      corr[i] = 0;
      shift[i] = -16;
      continue;
    }
    int b = 31 - __builtin_clz(divisor); /* flss(divisor) - 1 */
    int r = 16 + b;
    uint32_t fq = ((uint32_t)1 << r) / divisor;
    uint32_t fr = ((uint32_t)1 << r) % divisor;
    uint32_t c = divisor / 2;
    if (fr == 0) {
      fq >>= 1;
      r--;
    } else if (fr <= divisor / 2U) {
      c++;
    } else {
      fq++;
    }
    recip[i] = (uint16_t)fq;
    corr[i] = (uint16_t)c;
    shift[i] = (int16_t)(r - 16);
  }
}

/* jcdctmgr.c quantize (natural order in, natural order out) */
static void quantize(const int32_t ws[64], const uint16_t recip[64], const uint16_t corr[64],
                     const int16_t shift[64], int16_t out[64]) {
  for (int i = 0; i < 64; ++i) {
    int32_t t = (int16_t)ws[i];
    uint32_t product;
    if (t < 0) {
      product = (uint32_t)(-t + corr[i]) * recip[i];
      product >>= shift[i] + 16;
      out[i] = (int16_t)(-(int16_t)product);
    } else {
      product = (uint32_t)(t + corr[i]) * recip[i];
      product >>= shift[i] + 16;
      out[i] = (int16_t)product;
    }
  }
}

typedef struct {
  uint8_t *buf;
  size_t cap, len;
  uint64_t acc;
  int nbits;
  int overflow;
} bitw_t;

static void put_byte(bitw_t *w, uint8_t b) {
  if (w->len < w->cap) w->buf[w->len] = b;
  else w->overflow = 1;
  w->len++;
}

static void put_bits(bitw_t *w, uint32_t code, int size) {
  if (!size) return;
  w->acc = (w->acc << size) | (code & ((1u << size) - 1));
  w->nbits += size;
  while (w->nbits >= 8) {
    w->nbits -= 8;
    uint8_t b = (uint8_t)(w->acc >> w->nbits);
    put_byte(w, b);
    if (b == 0xFF) put_byte(w, 0); /* byte stuffing */
  }
}

static void flush_bits(bitw_t *w) {
  if (w->nbits) put_bits(w, 0x7F, 8 - w->nbits); /* pad the partial byte with ones */
  w->acc = 0;
  w->nbits = 0;
}

static void put_u16(bitw_t *w, int v) {
  put_byte(w, (uint8_t)(v >> 8));
  put_byte(w, (uint8_t)v);
}

/* jchuff.c jpeg_make_c_derived_tbl */
void vfo_huff_encode_table(const uint8_t bits[17], const uint8_t *vals, uint16_t code[256],
                           uint8_t size[256]) {
  uint8_t huffsize[257];
  uint16_t huffcode[257];
  int p = 0;
  for (int l = 1; l <= 16; ++l)
    for (int i = 0; i < bits[l]; ++i) huffsize[p++] = (uint8_t)l;
  huffsize[p] = 0;
  const int lastp = p;
  uint32_t c = 0;
  int si = huffsize[0];
  p = 0;
  while (huffsize[p]) {
    while (huffsize[p] == si) huffcode[p++] = (uint16_t)c++;
    c <<= 1;
    si++;
  }
  memset(code, 0, 256 * sizeof(uint16_t));
  memset(size, 0, 256);
  for (p = 0; p < lastp; ++p) {
    code[vals[p]] = huffcode[p];
    size[vals[p]] = huffsize[p];
  }
}

typedef struct {
  uint16_t dc_code[256], ac_code[256];
  uint8_t dc_size[256], ac_size[256];
} enc_huff_t;

/* jchuff.c encode_one_block */
static void encode_block(bitw_t *w, const int16_t blk[64], int last_dc, const enc_huff_t *t) {
  int temp = blk[0] - last_dc, temp2 = temp;
  if (temp < 0) {
    temp = -temp;
    temp2--;
  }
  int nbits = 0;
  while (temp) {
    nbits++;
    temp >>= 1;
  }
  put_bits(w, t->dc_code[nbits], t->dc_size[nbits]);
  if (nbits) put_bits(w, (uint32_t)temp2, nbits);
  int r = 0;
  for (int k = 1; k < 64; ++k) {
    temp = blk[kNatural[k]];
    if (temp == 0) {
      r++;
      continue;
    }
    while (r > 15) {
      put_bits(w, t->ac_code[0xF0], t->ac_size[0xF0]);
      r -= 16;
    }
    temp2 = temp;
    if (temp < 0) {
      temp = -temp;
      temp2--;
    }
    nbits = 1;
    while ((temp >>= 1)) nbits++;
    const int i = (r << 4) + nbits;
    put_bits(w, t->ac_code[i], t->ac_size[i]);
    put_bits(w, (uint32_t)temp2, nbits);
    r = 0;
  }
  if (r > 0) put_bits(w, t->ac_code[0], t->ac_size[0]);
}

static void emit_dqt(bitw_t *w, int idx, const uint16_t q[64]) {
  put_byte(w, 0xFF);
  put_byte(w, 0xDB);
  put_u16(w, 64 + 1 + 2);
  put_byte(w, (uint8_t)idx);
  for (int i = 0; i < 64; ++i) put_byte(w, (uint8_t)q[kNatural[i]]);
}

static void emit_dht(bitw_t *w, int idx, const uint8_t bits[17], const uint8_t *vals) {
  int n = 0;
  for (int l = 1; l <= 16; ++l) n += bits[l];
  put_byte(w, 0xFF);
  put_byte(w, 0xC4);
  put_u16(w, 2 + 1 + 16 + n);
  put_byte(w, (uint8_t)idx);
  for (int l = 1; l <= 16; ++l) put_byte(w, bits[l]);
  for (int i = 0; i < n; ++i) put_byte(w, vals[i]);
}

/* Markers before the entropy-coded segment, exactly as jcmarker.c writes them for
 * jpeg_set_defaults + jpeg_set_quality(q, TRUE) + jpeg_set_colorspace(YCbCr | GRAYSCALE). */
size_t vfo_jpeg_write_headers(int w, int h, int quality, int subsamp, uint8_t *out, size_t cap) {
  bitw_t bw = {out, cap, 0, 0, 0, 0};
  const int nc = subsamp == VFO_SAMP_GRAY ? 1 : 3;
  uint16_t q0[64], q1[64];
  vfo_jpeg_quality_table(quality, 0, q0);
  vfo_jpeg_quality_table(quality, 1, q1);
  put_byte(&bw, 0xFF);
  put_byte(&bw, 0xD8);
  /* JFIF APP0: version 1.01, density_unit 0, density 1:1, no thumbnail */
  static const uint8_t app0[18] = {0xFF, 0xE0, 0, 16, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
  for (int i = 0; i < 18; ++i) put_byte(&bw, app0[i]);
  emit_dqt(&bw, 0, q0);
  if (nc == 3) emit_dqt(&bw, 1, q1);
  put_byte(&bw, 0xFF);
  put_byte(&bw, 0xC0);
  put_u16(&bw, 8 + 3 * nc);
  put_byte(&bw, 8);
  put_u16(&bw, h);
  put_u16(&bw, w);
  put_byte(&bw, (uint8_t)nc);
  for (int c = 0; c < nc; ++c) {
    put_byte(&bw, (uint8_t)(c + 1));
    const int hs = c == 0 ? kSampH[subsamp] : 1, vs = c == 0 ? kSampV[subsamp] : 1;
    put_byte(&bw, (uint8_t)((hs << 4) + vs));
    put_byte(&bw, c == 0 ? 0 : 1);
  }
  emit_dht(&bw, 0x00, kDcLumaBits, kDcLumaVals);
  emit_dht(&bw, 0x10, kAcLumaBits, kAcLumaVals);
  if (nc == 3) {
    emit_dht(&bw, 0x01, kDcChromaBits, kDcChromaVals);
    emit_dht(&bw, 0x11, kAcChromaBits, kAcChromaVals);
  }
  put_byte(&bw, 0xFF);
  put_byte(&bw, 0xDA);
  put_u16(&bw, 2 * nc + 6);
  put_byte(&bw, (uint8_t)nc);
  for (int c = 0; c < nc; ++c) {
    put_byte(&bw, (uint8_t)(c + 1));
    put_byte(&bw, c == 0 ? 0x00 : 0x11);
  }
  put_byte(&bw, 0);
  put_byte(&bw, 63);
  put_byte(&bw, 0);
  return bw.overflow ? 0 : bw.len;
}

/* Encode an interleaved 8-bit image (pixel_format VFO_PF_RGB / VFO_PF_BGR, 3 bytes per
 * pixel).  Returns the JPEG size, or 0 on error / when `cap` is too small. */
size_t vfo_jpeg_encode(const uint8_t *img, int w, int h, int pixel_format, int quality,
                       int subsamp, int fastdct, uint8_t *out, size_t cap) {
  if (!img || w <= 0 || h <= 0 || w > 65535 || h > 65535 || subsamp < 0 ||
      subsamp > VFO_SAMP_440 || (pixel_format != VFO_PF_RGB && pixel_format != VFO_PF_BGR))
    return 0;
  const int ro = pixel_format == VFO_PF_RGB ? 0 : 2, bo = 2 - ro;
  const int nc = subsamp == VFO_SAMP_GRAY ? 1 : 3;
  const int maxh = kSampH[subsamp], maxv = kSampV[subsamp];
  const int mcux = ceil_div(w, 8 * maxh), mcuy = ceil_div(h, 8 * maxv);
  /* full-resolution Y/Cb/Cr, edge-replicated to whole MCUs */
  const int fw = mcux * 8 * maxh, fh = mcuy * 8 * maxv;
  uint8_t *full[3] = {0, 0, 0};
  uint8_t *plane[3] = {0, 0, 0};
  int16_t *coef[3] = {0, 0, 0};
  size_t result = 0;
  for (int c = 0; c < nc; ++c)
    if (!(full[c] = (uint8_t *)malloc((size_t)fw * fh))) goto done;
  for (int y = 0; y < fh; ++y) {
    const int sy = y < h ? y : h - 1;
    for (int x = 0; x < fw; ++x) {
      const int sx = x < w ? x : w - 1;
      const uint8_t *p = img + ((size_t)sy * w + sx) * 3;
      uint8_t Y, Cb, Cr;
      rgb_to_ycc(p[ro], p[1], p[bo], &Y, &Cb, &Cr);
      full[0][(size_t)y * fw + x] = Y;
      if (nc == 3) {
        full[1][(size_t)y * fw + x] = Cb;
        full[2][(size_t)y * fw + x] = Cr;
      }
    }
  }
  /* Downsampled planes (jcsample.c).  The row-group edge replication of jcprepct.c is what
   * the full-resolution replication above already gives, because whole MCUs are covered.
   * Rows past ceil(h / maxv) * v of a component repeat its last downsampled row
   * (expand_bottom_edge to a whole iMCU row). */
  int hs[3], vs[3], wb[3], hb[3];
  for (int c = 0; c < nc; ++c) {
    hs[c] = c == 0 ? maxh : 1;
    vs[c] = c == 0 ? maxv : 1;
    const int he = maxh / hs[c], ve = maxv / vs[c];
    wb[c] = ceil_div(w * hs[c], 8 * maxh);
    hb[c] = ceil_div(h * vs[c], 8 * maxv);
    const int pw = mcux * hs[c] * 8, ph = mcuy * vs[c] * 8;
    const int real_rows = ceil_div(h, maxv) * vs[c];
    if (!(plane[c] = (uint8_t *)malloc((size_t)pw * ph))) goto done;
    for (int y = 0; y < ph; ++y) {
      const int yy = y < real_rows ? y : real_rows - 1;
      for (int x = 0; x < pw; ++x) {
        const int xx = x < wb[c] * 8 ? x : wb[c] * 8 - 1; /* columns past output_cols unused */
        int v;
        if (he == 1 && ve == 1) {
          v = full[c][(size_t)yy * fw + xx];
        } else if (he == 2 && ve == 1) {
          const uint8_t *s = full[c] + (size_t)yy * fw + 2 * xx;
          v = (s[0] + s[1] + (xx & 1)) >> 1;
        } else if (he == 2 && ve == 2) {
          const uint8_t *s0 = full[c] + (size_t)(2 * yy) * fw + 2 * xx, *s1 = s0 + fw;
          v = (s0[0] + s0[1] + s1[0] + s1[1] + 1 + (xx & 1)) >> 2;
        } else { /* int_downsample */
          int sum = 0;
          for (int a = 0; a < ve; ++a)
            for (int b = 0; b < he; ++b) sum += full[c][(size_t)(yy * ve + a) * fw + xx * he + b];
          v = (sum + he * ve / 2) / (he * ve);
        }
        plane[c][(size_t)y * pw + x] = (uint8_t)v;
      }
    }
  }
  /* DCT + quantisation of every block inside width/height_in_blocks */
  {
    uint16_t q[2][64], recip[2][64], corr[2][64];
    int16_t shift[2][64];
    for (int t = 0; t < 2; ++t) {
      vfo_jpeg_quality_table(quality, t, q[t]);
      vfo_jpeg_divisors(q[t], fastdct, recip[t], corr[t], shift[t]);
    }
    for (int c = 0; c < nc; ++c) {
      const int pw = mcux * hs[c] * 8;
      const int bw = mcux * hs[c], bh = mcuy * vs[c];
      if (!(coef[c] = (int16_t *)calloc((size_t)bw * bh * 64, sizeof(int16_t)))) goto done;
      for (int by = 0; by < hb[c]; ++by)
        for (int bx = 0; bx < wb[c]; ++bx) {
          int32_t ws[64];
          for (int i = 0; i < 64; ++i)
            ws[i] = (int32_t)plane[c][(size_t)(by * 8 + i / 8) * pw + bx * 8 + i % 8] - 128;
          if (fastdct) vfo_fdct_ifast(ws);
          else vfo_fdct_islow(ws);
          quantize(ws, recip[c > 0], corr[c > 0], shift[c > 0], coef[c] + ((size_t)by * bw + bx) * 64);
        }
    }
  }
  /* headers + entropy-coded MCUs */
  {
    size_t hl = vfo_jpeg_write_headers(w, h, quality, subsamp, out, cap);
    if (!hl) goto done;
    bitw_t bw = {out, cap, hl, 0, 0, 0};
    enc_huff_t tab[2];
    vfo_huff_encode_table(kDcLumaBits, kDcLumaVals, tab[0].dc_code, tab[0].dc_size);
    vfo_huff_encode_table(kAcLumaBits, kAcLumaVals, tab[0].ac_code, tab[0].ac_size);
    vfo_huff_encode_table(kDcChromaBits, kDcChromaVals, tab[1].dc_code, tab[1].dc_size);
    vfo_huff_encode_table(kAcChromaBits, kAcChromaVals, tab[1].ac_code, tab[1].ac_size);
    int last_dc[3] = {0, 0, 0};
    const int nmcux = nc == 1 ? wb[0] : mcux, nmcuy = nc == 1 ? hb[0] : mcuy;
    for (int my = 0; my < nmcuy; ++my)
      for (int mx = 0; mx < nmcux; ++mx)
        for (int c = 0; c < nc; ++c) {
          const int mh = nc == 1 ? 1 : hs[c], mv = nc == 1 ? 1 : vs[c];
          const int bwc = mcux * hs[c];
          int16_t prev_dc = 0;
          for (int yi = 0; yi < mv; ++yi)
            for (int xi = 0; xi < mh; ++xi) {
              const int bx = mx * mh + xi, by = my * mv + yi;
              int16_t blk[64];
              if (by < hb[c] && bx < wb[c]) {
                memcpy(blk, coef[c] + ((size_t)by * bwc + bx) * 64, sizeof blk);
              } else {
                /* dummy block (jccoefct.c): zero AC; DC of the previous block of this
                 * component in the MCU (its left neighbour at the right edge, the last block
                 * of the row above in a dummy bottom row) */
                memset(blk, 0, sizeof blk);
                blk[0] = prev_dc;
              }
              prev_dc = blk[0];
              encode_block(&bw, blk, last_dc[c], &tab[c > 0]);
              last_dc[c] = blk[0];
            }
        }
    flush_bits(&bw);
    put_byte(&bw, 0xFF);
    put_byte(&bw, 0xD9);
    result = bw.overflow ? 0 : bw.len;
  }
done:
  for (int c = 0; c < 3; ++c) {
    free(full[c]);
    free(plane[c]);
    free(coef[c]);
  }
  return result;
}

/* Worst-case output size for vfo_jpeg_encode (every coefficient coded at 16+11 bits plus
 * full byte stuffing, plus headers). */
size_t vfo_jpeg_encode_bound(int w, int h, int subsamp) {
  const int maxh = kSampH[subsamp], maxv = kSampV[subsamp];
  const size_t mcus = (size_t)ceil_div(w, 8 * maxh) * ceil_div(h, 8 * maxv);
  const size_t blocks = mcus * (size_t)(subsamp == VFO_SAMP_GRAY ? 1 : maxh * maxv + 2);
  return blocks * 64 * 27 / 8 * 2 + 2048;
}

/* ---- decoder --------------------------------------------------------------------------- */

typedef struct {
  int32_t maxcode[18];
  int32_t valoffset[18];
  uint8_t vals[256];
  int defined;
} dec_huff_t;

/* jdhuff.c jpeg_make_d_derived_tbl (canonical decode part; a DC table's symbols must be
 * 0..15, as jdhuff.c's isDC check requires) */
static int make_dec_table(const uint8_t bits[17], const uint8_t *vals, int nvals, int dc, dec_huff_t *t) {
  uint8_t huffsize[257];
  uint32_t huffcode[257];
  int p = 0;
  for (int l = 1; l <= 16; ++l)
    for (int i = 0; i < bits[l]; ++i) {
      if (p >= 256) return -1;
      huffsize[p++] = (uint8_t)l;
    }
  if (p != nvals) return -1;
  if (dc)
    for (int i = 0; i < nvals; ++i)
      if (vals[i] > 15) return -1;
  huffsize[p] = 0;
  uint32_t code = 0;
  int si = huffsize[0];
  p = 0;
  while (huffsize[p]) {
    while (huffsize[p] == si) huffcode[p++] = code++;
    if (code >= ((uint32_t)1 << si)) return -1; /* bad table */
    code <<= 1;
    si++;
  }
  p = 0;
  for (int l = 1; l <= 16; ++l) {
    if (bits[l]) {
      t->valoffset[l] = p - (int32_t)huffcode[p];
      p += bits[l];
      t->maxcode[l] = (int32_t)huffcode[p - 1];
    } else {
      t->maxcode[l] = -1;
    }
  }
  t->valoffset[17] = 0;
  t->maxcode[17] = 0xFFFFF;
  memcpy(t->vals, vals, (size_t)nvals);
  t->defined = 1;
  return 0;
}

typedef struct {
  const uint8_t *d;
  size_t n, pos;
  uint32_t acc;
  int nbits;
  int hit_marker;
} bitr_t;

/* jdhuff.c jpeg_fill_bit_buffer: unstuff FF00; a marker stops the data and zeros are fed */
static int get_bit(bitr_t *r) {
  if (!r->nbits) {
    uint8_t b = 0;
    if (!r->hit_marker && r->pos < r->n) {
      b = r->d[r->pos];
      if (b == 0xFF) {
        if (r->pos + 1 < r->n && r->d[r->pos + 1] == 0x00) {
          r->pos += 2;
        } else {
          r->hit_marker = 1;
          b = 0;
        }
      } else {
        r->pos++;
      }
    }
    r->acc = b;
    r->nbits = 8;
  }
  r->nbits--;
  return (int)((r->acc >> r->nbits) & 1);
}

static int get_bits(bitr_t *r, int n) {
  int v = 0;
  for (int i = 0; i < n; ++i) v = (v << 1) | get_bit(r);
  return v;
}

static int huff_decode(bitr_t *r, const dec_huff_t *t) {
  int32_t code = get_bit(r);
  int l = 1;
  while (l <= 16 && code > t->maxcode[l]) {
    code = (code << 1) | get_bit(r);
    l++;
  }
  if (l > 16) return 0; /* corrupt data: jdhuff.c warns and returns symbol 0 */
  return t->vals[(int)(code + t->valoffset[l]) & 255];
}

#define HUFF_EXTEND(x, s) ((x) < (1 << ((s)-1)) ? (x) + (int)(((unsigned)-1 << (s)) + 1) : (x))

/* jidctint.c jpeg_idct_islow + the jdmaster.c post-IDCT range-limit table (RANGE_MASK 1023) */
static uint8_t idct_limit(int32_t x) {
  const int m = (int)(x & 1023);
  if (m < 128) return (uint8_t)(m + 128);
  if (m < 512) return 255;
  if (m < 896) return 0;
  return (uint8_t)(m - 896);
}

void vfo_idct_islow(const int16_t coef[64], const uint16_t q[64], uint8_t *out, int stride) {
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) { /* pass 1: columns */
    const int16_t *in = coef + c;
    const uint16_t *qq = q + c;
    int32_t tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13, z1, z2, z3, z4, z5;
    z2 = in[16] * (int32_t)qq[16];
    z3 = in[48] * (int32_t)qq[48];
    z1 = (z2 + z3) * FIX_0_541196100;
    tmp2 = z1 + z3 * -FIX_1_847759065;
    tmp3 = z1 + z2 * FIX_0_765366865;
    z2 = in[0] * (int32_t)qq[0];
    z3 = in[32] * (int32_t)qq[32];
    tmp0 = (z2 + z3) * (1 << 13);
    tmp1 = (z2 - z3) * (1 << 13);
    tmp10 = tmp0 + tmp3;
    tmp13 = tmp0 - tmp3;
    tmp11 = tmp1 + tmp2;
    tmp12 = tmp1 - tmp2;
    tmp0 = in[56] * (int32_t)qq[56];
    tmp1 = in[40] * (int32_t)qq[40];
    tmp2 = in[24] * (int32_t)qq[24];
    tmp3 = in[8] * (int32_t)qq[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    z4 = tmp1 + tmp3;
    z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    ws[c + 0] = DESCALE(tmp10 + tmp3, 11);
    ws[c + 56] = DESCALE(tmp10 - tmp3, 11);
    ws[c + 8] = DESCALE(tmp11 + tmp2, 11);
    ws[c + 48] = DESCALE(tmp11 - tmp2, 11);
    ws[c + 16] = DESCALE(tmp12 + tmp1, 11);
    ws[c + 40] = DESCALE(tmp12 - tmp1, 11);
    ws[c + 24] = DESCALE(tmp13 + tmp0, 11);
    ws[c + 32] = DESCALE(tmp13 - tmp0, 11);
  }
  for (int rr = 0; rr < 8; ++rr) { /* pass 2: rows */
    const int32_t *w = ws + rr * 8;
    uint8_t *o = out + (size_t)rr * stride;
    int32_t tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13, z1, z2, z3, z4, z5;
    z2 = w[2];
    z3 = w[6];
    z1 = (z2 + z3) * FIX_0_541196100;
    tmp2 = z1 + z3 * -FIX_1_847759065;
    tmp3 = z1 + z2 * FIX_0_765366865;
    tmp0 = (w[0] + w[4]) * (1 << 13);
    tmp1 = (w[0] - w[4]) * (1 << 13);
    tmp10 = tmp0 + tmp3;
    tmp13 = tmp0 - tmp3;
    tmp11 = tmp1 + tmp2;
    tmp12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    z4 = tmp1 + tmp3;
    z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    o[0] = idct_limit(DESCALE(tmp10 + tmp3, 18));
    o[7] = idct_limit(DESCALE(tmp10 - tmp3, 18));
    o[1] = idct_limit(DESCALE(tmp11 + tmp2, 18));
    o[6] = idct_limit(DESCALE(tmp11 - tmp2, 18));
    o[2] = idct_limit(DESCALE(tmp12 + tmp1, 18));
    o[5] = idct_limit(DESCALE(tmp12 - tmp1, 18));
    o[3] = idct_limit(DESCALE(tmp13 + tmp0, 18));
    o[4] = idct_limit(DESCALE(tmp13 - tmp0, 18));
  }
}

/* jdcolor.c build_ycc_rgb_table + ycc_rgb_convert (range_limit = clamp to [0,255]) */
static uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

static void ycc_to_rgb(int y, int cb, int cr, uint8_t *r, uint8_t *g, uint8_t *b) {
  const int x_cr = cr - 128, x_cb = cb - 128;
  const int cr_r = (FIX16(1.40200) * x_cr + ONE_HALF) >> SCALEBITS;
  const int cb_b = (FIX16(1.77200) * x_cb + ONE_HALF) >> SCALEBITS;
  const int32_t cr_g = -FIX16(0.71414) * x_cr;
  const int32_t cb_g = -FIX16(0.34414) * x_cb + ONE_HALF;
  *r = clamp255(y + cr_r);
  *g = clamp255(y + ((cb_g + cr_g) >> SCALEBITS));
  *b = clamp255(y + cb_b);
}

int vfo_jpeg_parse(const uint8_t *jpg, size_t n, vfo_jpeg_info *info) {
  memset(info, 0, sizeof *info);
  if (n < 4 || jpg[0] != 0xFF || jpg[1] != 0xD8) return VFO_JE_NOT_JPEG;
  size_t p = 2;
  int have_sof = 0;
  for (;;) {
    while (p < n && jpg[p] != 0xFF) p++; /* tolerate garbage between markers */
    while (p < n && jpg[p] == 0xFF) p++;
    if (p >= n) return VFO_JE_TRUNCATED;
    const int m = jpg[p++];
    if (m == 0xD9) return VFO_JE_TRUNCATED; /* EOI before SOS */
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (p + 2 > n) return VFO_JE_TRUNCATED;
    const int len = (jpg[p] << 8) | jpg[p + 1];
    if (len < 2 || p + (size_t)len > n) return VFO_JE_TRUNCATED;
    const uint8_t *s = jpg + p + 2, *e = jpg + p + len;
    if (m == 0xDB) { /* DQT */
      while (s < e) {
        const int pq = s[0] >> 4, tq = s[0] & 15;
        s++;
        if (tq > 3 || s + (pq ? 128 : 64) > e) return VFO_JE_BAD;
        for (int i = 0; i < 64; ++i)
          info->qt[tq][kNatural[i]] = pq ? (uint16_t)((s[2 * i] << 8) | s[2 * i + 1]) : s[i];
        info->qt_defined |= 1 << tq;
        s += pq ? 128 : 64;
      }
    } else if (m == 0xC4) { /* DHT */
      while (s < e) {
        if (s + 17 > e) return VFO_JE_BAD;
        const int tc = s[0] >> 4, th = s[0] & 15;
        if (tc > 1 || th > 3) return VFO_JE_BAD;
        int cnt = 0;
        for (int l = 1; l <= 16; ++l) cnt += s[l];
        if (cnt > 256 || s + 17 + cnt > e) return VFO_JE_BAD;
        uint8_t *bits = tc ? info->ac_bits[th] : info->dc_bits[th];
        uint8_t *vals = tc ? info->ac_vals[th] : info->dc_vals[th];
        bits[0] = 0;
        memcpy(bits + 1, s + 1, 16);
        memcpy(vals, s + 17, (size_t)cnt);
        if (tc) info->ac_defined |= 1 << th;
        else info->dc_defined |= 1 << th;
        s += 17 + cnt;
      }
    } else if (m == 0xC0 || m == 0xC1) { /* SOF0 / SOF1: sequential Huffman */
      if (len < 8 || s[0] != 8) return VFO_JE_UNSUPPORTED;
      info->height = (s[1] << 8) | s[2];
      info->width = (s[3] << 8) | s[4];
      info->ncomp = s[5];
      if (info->ncomp != 1 && info->ncomp != 3) return VFO_JE_UNSUPPORTED;
      if (len != 8 + 3 * info->ncomp || info->width == 0 || info->height == 0) return VFO_JE_BAD;
      for (int c = 0; c < info->ncomp; ++c) {
        info->comp_id[c] = s[6 + 3 * c];
        info->h[c] = s[7 + 3 * c] >> 4;
        info->v[c] = s[7 + 3 * c] & 15;
        info->tq[c] = s[8 + 3 * c];
        if (info->h[c] < 1 || info->h[c] > 4 || info->v[c] < 1 || info->v[c] > 4 || info->tq[c] > 3)
          return VFO_JE_BAD;
      }
      have_sof = 1;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return VFO_JE_UNSUPPORTED; /* progressive, lossless, arithmetic, hierarchical */
    } else if (m == 0xDD) {
      if (len != 4) return VFO_JE_BAD;
      info->restart_interval = (s[0] << 8) | s[1];
    } else if (m == 0xDA) { /* SOS */
      if (!have_sof) return VFO_JE_BAD;
      const int ns = s[0];
      if (ns != info->ncomp || len != 6 + 2 * ns) return VFO_JE_UNSUPPORTED; /* one interleaved scan */
      for (int i = 0; i < ns; ++i) {
        if (s[1 + 2 * i] != info->comp_id[i]) return VFO_JE_UNSUPPORTED;
        info->td[i] = s[2 + 2 * i] >> 4;
        info->ta[i] = s[2 + 2 * i] & 15;
        if (info->td[i] > 3 || info->ta[i] > 3) return VFO_JE_BAD;
      }
      if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0) return VFO_JE_UNSUPPORTED;
      info->scan_offset = p + (size_t)len;
      /* the entropy-coded data ends at a marker other than RSTn (FF00 is a stuffed FF) */
      size_t q = info->scan_offset;
      while (q + 1 < n) {
        if (jpg[q] == 0xFF && jpg[q + 1] != 0x00 && !(jpg[q + 1] >= 0xD0 && jpg[q + 1] <= 0xD7) &&
            jpg[q + 1] != 0xFF)
          break;
        q++;
      }
      info->scan_end = q < n ? q : n;
      int maxh = 1, maxv = 1;
      for (int c = 0; c < info->ncomp; ++c) {
        if (info->h[c] > maxh) maxh = info->h[c];
        if (info->v[c] > maxv) maxv = info->v[c];
      }
      for (int c = 0; c < info->ncomp; ++c)
        if (maxh % info->h[c] || maxv % info->v[c]) return VFO_JE_UNSUPPORTED;
      info->max_h = maxh;
      info->max_v = maxv;
      for (int c = 0; c < info->ncomp; ++c) {
        if (!(info->qt_defined >> info->tq[c] & 1) || !(info->dc_defined >> info->td[c] & 1) ||
            !(info->ac_defined >> info->ta[c] & 1))
          return VFO_JE_BAD;
      }
      return VFO_JE_OK;
    }
    p += (size_t)len;
  }
}

/* Decode to interleaved 8-bit pixels in `pixel_format` (RGB or BGR).  fast_upsample = the
 * TJFLAG_FASTUPSAMPLE behaviour (replicating upsampling).  `out` holds w*h*3 bytes. */
int vfo_jpeg_decode(const uint8_t *jpg, size_t n, int pixel_format, int fast_upsample, uint8_t *out,
                    size_t cap) {
  vfo_jpeg_info info;
  int rc = vfo_jpeg_parse(jpg, n, &info);
  if (rc) return rc;
  if (pixel_format != VFO_PF_RGB && pixel_format != VFO_PF_BGR) return VFO_JE_ARG;
  const int w = info.width, h = info.height, nc = info.ncomp;
  if (cap < (size_t)w * h * 3) return VFO_JE_ARG;
  const int maxh = info.max_h, maxv = info.max_v;
  const int mcux = ceil_div(w, 8 * maxh), mcuy = ceil_div(h, 8 * maxv);
  dec_huff_t dct[4], act[4];
  memset(dct, 0, sizeof dct);
  memset(act, 0, sizeof act);
  for (int c = 0; c < nc; ++c) {
    int cnt = 0;
    for (int l = 1; l <= 16; ++l) cnt += info.dc_bits[info.td[c]][l];
    if (!dct[info.td[c]].defined &&
        make_dec_table(info.dc_bits[info.td[c]], info.dc_vals[info.td[c]], cnt, 1, &dct[info.td[c]]))
      return VFO_JE_BAD;
    cnt = 0;
    for (int l = 1; l <= 16; ++l) cnt += info.ac_bits[info.ta[c]][l];
    if (!act[info.ta[c]].defined &&
        make_dec_table(info.ac_bits[info.ta[c]], info.ac_vals[info.ta[c]], cnt, 0, &act[info.ta[c]]))
      return VFO_JE_BAD;
  }
  /* component planes (whole blocks of the interleaved MCU grid) */
  uint8_t *plane[3] = {0, 0, 0};
  int pw[3], ph[3], wb[3], hb[3];
  rc = VFO_JE_NOMEM;
  for (int c = 0; c < nc; ++c) {
    wb[c] = ceil_div(w * info.h[c], 8 * maxh);
    hb[c] = ceil_div(h * info.v[c], 8 * maxv);
    pw[c] = (nc == 1 ? wb[c] : mcux * info.h[c]) * 8;
    ph[c] = (nc == 1 ? hb[c] : mcuy * info.v[c]) * 8;
    if (!(plane[c] = (uint8_t *)malloc((size_t)pw[c] * ph[c]))) goto done;
  }
  {
    bitr_t br = {jpg + info.scan_offset, info.scan_end - info.scan_offset, 0, 0, 0, 0};
    int last_dc[3] = {0, 0, 0};
    const int nmcux = nc == 1 ? wb[0] : mcux, nmcuy = nc == 1 ? hb[0] : mcuy;
    const long total = (long)nmcux * nmcuy;
    int next_rst = 0;
    for (long mcu = 0; mcu < total; ++mcu) {
      if (info.restart_interval && mcu > 0 && mcu % info.restart_interval == 0) {
        /* jdhuff.c process_restart: discard the partial byte, expect RSTn, reset DC */
        br.nbits = 0;
        const size_t q = br.pos;
        if (!(q + 1 < br.n && br.d[q] == 0xFF && br.d[q + 1] == (0xD0 + next_rst))) {
          rc = VFO_JE_BAD;
          goto done;
        }
        br.pos = q + 2;
        br.hit_marker = 0;
        next_rst = (next_rst + 1) & 7;
        last_dc[0] = last_dc[1] = last_dc[2] = 0;
      }
      const int mx = (int)(mcu % nmcux), my = (int)(mcu / nmcux);
      for (int c = 0; c < nc; ++c) {
        const int mh = nc == 1 ? 1 : info.h[c], mv = nc == 1 ? 1 : info.v[c];
        for (int yi = 0; yi < mv; ++yi)
          for (int xi = 0; xi < mh; ++xi) {
            int16_t blk[64];
            memset(blk, 0, sizeof blk);
            int s = huff_decode(&br, &dct[info.td[c]]);
            if (s > 16) s = 16;
            if (s) {
              const int r = get_bits(&br, s);
              s = HUFF_EXTEND(r, s);
            }
            last_dc[c] += s;
            blk[0] = (int16_t)last_dc[c];
            for (int k = 1; k < 64; ++k) {
              s = huff_decode(&br, &act[info.ta[c]]);
              int r = s >> 4;
              s &= 15;
              if (s) {
                k += r;
                r = get_bits(&br, s);
                s = HUFF_EXTEND(r, s);
                blk[kNatural[k]] = (int16_t)s;
              } else {
                if (r != 15) break;
                k += 15;
              }
            }
            const int bx = mx * mh + xi, by = my * mv + yi;
            if (bx * 8 < pw[c] && by * 8 < ph[c])
              vfo_idct_islow(blk, info.qt[info.tq[c]], plane[c] + (size_t)by * 8 * pw[c] + bx * 8, pw[c]);
          }
      }
    }
  }
  {
    /* upsample to full resolution (jdsample.c) and convert (jdcolor.c) */
    const int ro = pixel_format == VFO_PF_RGB ? 0 : 2, bo = 2 - ro;
    uint8_t *row[3] = {0, 0, 0};
    for (int c = 0; c < nc; ++c)
      if (!(row[c] = (uint8_t *)malloc((size_t)w + 16))) {
        for (int k = 0; k < c; ++k) free(row[k]);
        goto done;
      }
    for (int y = 0; y < h; ++y) {
      for (int c = 0; c < nc; ++c) {
        const int he = maxh / info.h[c], ve = maxv / info.v[c];
        const int dw = ceil_div(w * info.h[c], maxh); /* downsampled_width */
        const int dh = ceil_div(h * info.v[c], maxv); /* downsampled_height */
        const int fancy = !fast_upsample && ((he == 2 && ve == 1 && dw > 2) ||
                                             (he == 2 && ve == 2 && dw > 2) || (he == 1 && ve == 2));
        const int iy = y / ve;
        const uint8_t *in0 = plane[c] + (size_t)(iy < dh ? iy : dh - 1) * pw[c];
        uint8_t *o = row[c];
        if (he == 1 && ve == 1) {
          memcpy(o, in0, (size_t)w);
        } else if (!fancy) {
          for (int x = 0; x < w; ++x) o[x] = in0[x / he];
        } else if (he == 2 && ve == 1) { /* h2v1_fancy_upsample */
          for (int i = 0; i < dw; ++i) {
            const int v3 = in0[i] * 3;
            const int a = i == 0 ? in0[0] : (v3 + in0[i - 1] + 1) >> 2;
            const int b = i == dw - 1 ? in0[i] : (v3 + in0[i + 1] + 2) >> 2;
            if (2 * i < w) o[2 * i] = (uint8_t)a;
            if (2 * i + 1 < w) o[2 * i + 1] = (uint8_t)b;
          }
        } else {
          /* the other input row: above for the upper output row of a pair, below for the
           * lower; jdmainct.c replicates the first / last real row at the image edges */
          int ny = (y % 2 == 0) ? iy - 1 : iy + 1;
          if (ny < 0) ny = 0;
          if (ny > dh - 1) ny = dh - 1;
          const uint8_t *in1 = plane[c] + (size_t)ny * pw[c];
          if (he == 2) { /* h2v2_fancy_upsample */
            for (int i = 0; i < dw; ++i) {
              const int t = in0[i] * 3 + in1[i];
              const int l = i > 0 ? in0[i - 1] * 3 + in1[i - 1] : 0;
              const int r = i < dw - 1 ? in0[i + 1] * 3 + in1[i + 1] : 0;
              const int a = i == 0 ? (t * 4 + 8) >> 4 : (t * 3 + l + 8) >> 4;
              const int b = i == dw - 1 ? (t * 4 + 7) >> 4 : (t * 3 + r + 7) >> 4;
              if (2 * i < w) o[2 * i] = (uint8_t)a;
              if (2 * i + 1 < w) o[2 * i + 1] = (uint8_t)b;
            }
          } else { /* h1v2_fancy_upsample */
            const int bias = (y % 2 == 0) ? 1 : 2;
            for (int x = 0; x < w; ++x) o[x] = (uint8_t)((in0[x] * 3 + in1[x] + bias) >> 2);
          }
        }
      }
      uint8_t *op = out + (size_t)y * w * 3;
      for (int x = 0; x < w; ++x) {
        if (nc == 1) {
          op[3 * x] = op[3 * x + 1] = op[3 * x + 2] = row[0][x];
        } else {
          uint8_t r, g, b;
          ycc_to_rgb(row[0][x], row[1][x], row[2][x], &r, &g, &b);
          op[3 * x + ro] = r;
          op[3 * x + 1] = g;
          op[3 * x + bo] = b;
        }
      }
    }
    for (int c = 0; c < nc; ++c) free(row[c]);
  }
  rc = VFO_JE_OK;
done:
  for (int c = 0; c < 3; ++c) free(plane[c]);
  return rc;
}
