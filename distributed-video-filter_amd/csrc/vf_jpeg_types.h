// vf_jpeg_types.h — the JPEG batch descriptors and table layouts shared by the kernels
// (vf_jpeg_kernels.hip), their host side (vf_jpeg_host.hip) and the host parse
// (vf_jpeg_parse.h).  Plain C++ (no HIP), so the parse builds under g++ with sanitizers.
// Not installed.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace vf {
namespace jpeg {

// libjpeg's JPEG_MAX_DIMENSION (jmorecfg.h): jdinput.c initial_setup refuses larger frames
// with JERR_IMAGE_TOO_BIG
constexpr int kMaxDimension = 65500;
// default per-frame pixel limit of a context's decoder (vf_jpeg_set_max_pixels): 8192 x 8192
constexpr uint64_t kDefaultMaxPixels = 8192ull * 8192ull;

constexpr int kMaxBpm = 10;     // blocks per MCU (T.81 B.2.3)
constexpr int kSubBits = 256;  // bits per Huffman-decoding subsequence
constexpr int kTile = 4096;     // bytes per (un)stuffing tile
constexpr int kMaxPasses = 64;  // sync-pass flags kept on the device
constexpr int kQueuedPasses = 4;  // span sync passes queued per batch (k_syncg)
#ifndef VF_KLOOK
#define VF_KLOOK 9
#endif
constexpr int kLook = VF_KLOOK;        // Huffman lookahead bits
constexpr int kAcScratchWords = 52;  // per-block AC bit scratch (63 codes of <= 26 bits + EOB)
constexpr int kCkStep = kSubBits / 8 < 64 ? 64 : kSubBits / 8;  // Huffman-sync checkpoint spacing (bits)
constexpr int kCk = kSubBits / kCkStep - 1;                       // checkpoints per subsequence
// DecFrame.flags bit: every multiplicand of the IDCT's column pass fits a signed 24-bit multiply
// (idct_col24_ok); the row pass's always do (idct_line)
constexpr uint32_t kDecIdct24 = 8u;

// The column pass of jpeg_idct_islow multiplies sums of at most four dequantised AC coefficients
// of one column by constants (the DC only enters through a shift).  An AC coefficient is an
// extend() of at most `ac_size` bits (the largest size nibble among the AC tables' symbols), so
// its magnitude is under 2^ac_size; times the largest AC quantiser entry and four terms, the
// multiplicands stay within v_mul_i32_i24's exact range when this holds.  Annex K tables (sizes
// <= 10) with 8-bit quantisers are far inside it.
inline bool idct_col24_ok(int ac_size, uint32_t q_ac_max) {
  return ac_size <= 16 && 4ull * (uint64_t)q_ac_max * ((1ull << ac_size) - 1) < (1ull << 23);
}

// MCU geometry of one frame (libjpeg jdinput.c / jcmaster.c per-scan setup, restated)
struct Geom {
  int32_t w, h, ncomp, bpm;
  int32_t maxh, maxv, mcux, mcuy, nmcu, nblocks;
  int32_t hs[3], vs[3];  // sampling factors
  int32_t mh[3], mv[3];  // blocks of the component per MCU (1x1 in a single-component scan)
  int32_t wb[3], hb[3];  // width/height_in_blocks (real blocks)
  int32_t pw[3], ph[3];  // component plane in samples (whole MCUs)
  int32_t cfirst[3];     // first block-in-MCU of the component
  int32_t dw[3], dh[3];  // downsampled size in samples: ceil(w * hs / maxh), ceil(h * vs / maxv)
  int32_t rrows[3];      // encoder: sample rows from real pixel rows, ceil(h / maxv) * vs
  // 32-bit, as every field here: a kernel reads a wave-uniform entry with one scalar load,
  // where an 8-bit field would be a vector load and a wait
  int32_t bcomp[kMaxBpm], bxo[kMaxBpm], byo[kMaxBpm];  // block-in-MCU -> component, x/y (blocks)
  int32_t he[3], ve[3];  // expansion factors maxh / hs, maxv / vs
};


// natural (row-major) index -> zigzag position (inverse of jutils.c jpeg_natural_order)
inline constexpr uint8_t kZigOf[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                       3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                       10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                       21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// Position of zigzag coefficient zz in the row of k_fdct's quantised-block image for the
// block in workgroup slot `slot`: its 16-B octet (zz / 8, the AC coder's one ds_read_b128 per
// lane) XOR-ed with (0, 5, 2, 7)[slot % 4], which keeps the 4 blocks of a 32-lane half from
// storing to the same LDS banks (searched exhaustively with the b128 reads kept conflict-free).
constexpr uint32_t qo_pos(uint32_t slot, uint32_t zz) { return zz ^ (((0x7250u >> (4 * (slot & 3))) & 7) << 3); }

// Encoder tables: jcdctmgr.c reciprocal divisors, jchuff.c derived code tables
struct EncTables {
  uint16_t recip[2][64];  // natural order; [0] luma, [1] chroma
  uint16_t corr[2][64];
  int16_t shift[2][64];
  uint32_t dc[2][16];   // (code << 8) | size by magnitude category
  uint32_t ac[2][256];  // (code << 8) | size by run/size symbol
  // k_fdct's LDS table image, copied in with one 16-B load per thread: per table t and natural
  // position n the quantiser entry {recip | corr << 16, (shift + 16) | qo_pos(j, zigzag(n)) <<
  // (8 + 6j) for j = 0..3} (words [0, 256)), then ac[2][256] (words [256, 768))
  alignas(16) uint32_t fdct_lds[768];
};

// Codes longer than kLook bits: lim[i] = (maxcode[l] + 1) << (16 - l) for l = kLook + 1 + i,
// running maximum over i (lim[7] unused).  The length of the code starting the next 16 bits
// c16 is kLook + 1 + #{i : c16 >= lim[i]} (17 = no code: jdhuff.c's corrupt-data case), the
// same as jdhuff.c jpeg_huff_decode's length-by-length maxcode walk, in one 32-B LDS read.
static_assert(kLook >= 9 && kLook <= 15, "lim[] holds code lengths kLook + 1 .. 16 (at most 7)");

// Huffman decoding table: jdhuff.c derived table plus a kLook-bit lookahead
struct HuffDec {
  alignas(16) uint32_t lim[8];
  uint16_t fast[1 << kLook];  // (length << 8) | symbol for codes of <= kLook bits, else 0
  int32_t maxcode[18];
  int32_t valoff[18];
  uint8_t vals[256];
};

// The same table for the synchronisation decoders, which only need how far each symbol moves:
// sfast[next kLook bits] = (zigzag advance << 8) | (code length + extra bits) for codes of
// <= kLook bits (advance 1 for a DC symbol, run + 1 for an AC coefficient, 16 for ZRL, 64 for
// EOB), 0 for longer codes (decoded through maxcode / valoff / vals).
struct HuffSync {
  alignas(16) uint32_t lim[8];
  uint16_t sfast[1 << kLook];
  int32_t maxcode[18];
  int32_t valoff[18];
  uint8_t vals[256];
};

// A frame's Huffman tables, 20.5 KB.  The frames of a batch that share their tables (one encoder,
// one set of settings: a stream's every frame) share one DecTabs; the batch's distinct ones follow
// its DecFrame array in the same buffer, and DecFrame::tabs_off locates a frame's.
struct DecTabs {
  HuffDec dc[3], ac[3];    // per component (kept adjacent: loaded into LDS as one block)
  HuffSync sdc[3], sac[3];  // the same, for the synchronisation decoders (adjacent too)
  // AC pairs for the span sync: spair[k][next kLook bits] = (advance << 8) | length of an AC
  // symbol of component k together with the one after it, when both codes and their extra bits
  // lie inside the kLook bits (0: no pair); a step then moves over two symbols with one table
  // read, unless the first ends the block or reaches a mark
  uint16_t spair[3][1 << kLook];
};

struct DecFrame {
  Geom g;
  uint16_t q[3][64];       // dequantisation per component, natural order
  uint64_t tabs_off;       // its DecTabs, in bytes from the start of the DecFrame array
  uint32_t flags;          // bit 0: fancy upsampling allowed; bits 1-2: k_color layout (0 other,
                           // 1 4:4:4, 2 chroma 2x1, 3 chroma 2x2; three components, full-size luma);
                           // kDecIdct24: the IDCT's column pass may use 24-bit multiplies
  // The span sync's 4-table layout (vf_jpeg_kernels.hip load_sync_tabs4): bits 0-5 the table
  // slot (0 / 1) of each component, 2 bits each; bits 8-9 / 10-11 the component whose tables
  // fill slot 0 / 1; bit 31: the frame has at most two distinct (DC, AC) table pairs
  uint32_t tabs4;
  uint64_t blk0;           // first block in the batch coefficient buffer
  uint64_t dcbase[3];      // per-component DC sequences in the DC buffer
  uint64_t plane_off[3];   // component planes in the plane buffer
  uint64_t out_off;        // interleaved pixels in the pixel buffer
};

// One entropy-coded segment, the unit of the unstuff / sync / write stages: a frame's whole
// scan, or one restart interval of it.  With DRI every interval starts byte-aligned after an
// RSTn marker with the DC predictions reset (T.81 F.1.2.3, jdhuff.c process_restart), so the
// intervals decode as independent segments whose blocks and DC sequences tile the frame's.
struct DecSeg {
  uint32_t frame;          // its frame in the DecFrame array (tables, geometry)
  uint32_t nblocks;        // blocks coded in the segment (whole MCUs)
  uint64_t in_off;         // raw entropy-coded bytes in the batch input buffer (16-aligned)
  uint32_t in_len;
  uint32_t ntiles;         // kTile tiles over the raw bytes
  uint32_t tile0;          // first tile slot
  uint32_t sub0;           // first subsequence slot
  uint32_t nsub_max;       // subsequence slots (ceil(in_len * 8 / kSubBits))
  uint32_t wg0, nwg;       // speculative sync: first workgroup slot, workgroups (spec_lanes)
  uint64_t tr0;            // speculative sync: first trajectory slot (nwg * 256 per segment)
  uint64_t us_off;         // unstuffed stream in the unstuffed buffer (16-aligned)
  uint64_t blk0;           // its first block in the batch coefficient buffer
  uint64_t dcbase[3];      // its first entries of the frame's per-component DC sequences
};

struct EncFrame {
  Geom g;
  uint64_t img_off;     // interleaved input pixels in the pixel buffer
  uint64_t blk0;        // first block in the batch coefficient buffer
  uint64_t bits_off;    // packed bitstream (bytes, 16-aligned) in the bit buffer
  uint64_t out_off;     // finished JPEG in the output buffer
  uint32_t hdr_off, hdr_len;  // header bytes in the header buffer
  uint32_t tile0, ntiles_max;  // stuffing tiles
  // invert path: the encoder's component samples, written by the decoder's colour pass
  // (k_color<true>) in place of pixels; plane k is wb[k] * 8 samples wide, rrows[k] rows
  uint64_t eplane_off[3];
};

// Segmented scans over per-frame arrays (Huffman bit offsets, block counts, DC prediction,
// tile counts): segment s covers elements [base, base + len) and owns tile-sum slots
// [tile0, tile0 + ceil(len / kScanTile)).
constexpr int kScanPerThread = 8;
constexpr int kScanTile = 256 * kScanPerThread;
struct ScanSeg {
  uint64_t base;
  uint32_t len;
  uint32_t tile0;
};

}  // namespace jpeg
}  // namespace vf
