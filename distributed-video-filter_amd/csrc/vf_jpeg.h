// vf_jpeg.h — shared between the JPEG kernels (vf_jpeg_kernels.hip) and their host side
// (vf_jpeg_host.hip).  Not installed.
//
// The reference's default mode (use_jpeg=True) decodes, inverts and re-encodes every frame
// with PyTurboJPEG (inverter.py:32 -> :41 -> :44).  These structures describe one batch of
// frames laid out in HBM for the gfx950 baseline-JPEG codec; see DESIGN.md "JPEG".
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace vf {
namespace jpeg {

constexpr int kMaxBpm = 10;     // blocks per MCU (T.81 B.2.3)
constexpr int kSubBits = 256;  // bits per Huffman-decoding subsequence
constexpr int kTile = 4096;     // bytes per (un)stuffing tile
constexpr int kMaxPasses = 64;  // sync-pass flags kept on the device
#ifndef VF_KLOOK
#define VF_KLOOK 9
#endif
constexpr int kLook = VF_KLOOK;        // Huffman lookahead bits
constexpr int kAcScratchWords = 52;  // per-block AC bit scratch (63 codes of <= 26 bits + EOB)
constexpr int kCkStep = kSubBits / 8 < 64 ? 64 : kSubBits / 8;  // Huffman-sync checkpoint spacing (bits)
constexpr int kCk = kSubBits / kCkStep - 1;                       // checkpoints per subsequence

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

bool make_geom(int w, int h, int ncomp, const int *hs, const int *vs, Geom *g);

// Encoder tables: jcdctmgr.c reciprocal divisors, jchuff.c derived code tables
struct EncTables {
  uint16_t recip[2][64];  // natural order; [0] luma, [1] chroma
  uint16_t corr[2][64];
  int16_t shift[2][64];
  uint32_t dc[2][16];   // (code << 8) | size by magnitude category
  uint32_t ac[2][256];  // (code << 8) | size by run/size symbol
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

struct DecFrame {
  Geom g;
  uint16_t q[3][64];       // dequantisation per component, natural order
  HuffDec dc[3], ac[3];    // per component (kept adjacent: loaded into LDS as one block)
  HuffSync sdc[3], sac[3];  // the same, for the synchronisation decoders (adjacent too)
  uint32_t flags;          // bit 0: fancy upsampling allowed; bits 1-2: k_color layout (0 other,
                           // 1 4:4:4, 2 chroma 2x1, 3 chroma 2x2; three components, full-size luma)
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

// ---- launchers (vf_jpeg_kernels.hip) ----------------------------------------------------
hipError_t scan_u32(const ScanSeg *segs, int nseg, uint32_t max_tiles, const uint32_t *in, uint32_t *out,
                    uint32_t *tsum, uint32_t *totals, bool inclusive, hipStream_t s);
hipError_t scan_i32(const ScanSeg *segs, int nseg, uint32_t max_tiles, const int32_t *in, int32_t *out,
                    int32_t *tsum, int32_t *totals, bool inclusive, hipStream_t s);

hipError_t dec_unstuff_count(const DecSeg *sg, int nseg, uint32_t max_tiles, const uint8_t *in,
                             uint32_t *tile_cnt, hipStream_t s);
hipError_t dec_unstuff_write(const DecSeg *sg, int nseg, uint32_t max_tiles, const uint8_t *in,
                             const uint32_t *tile_off, const uint32_t *us_len, uint8_t *us, hipStream_t s);
hipError_t dec_sync(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_sub, const uint8_t *us, const uint32_t *us_len,
                    const uint64_t *exit_in, uint64_t *exit_out, const uint32_t *cnt_in, uint32_t *cnt_out,
                    uint64_t *used, uint64_t *ck, uint32_t *ckrem, uint32_t *changed, int pass, hipStream_t s);
// Speculative sync (one pass, no host round trip): k_spec decodes every subsequence from
// each possible block-in-MCU and links neighbouring subsequences, k_wglink links workgroups,
// k_resolve / k_finalize pick each subsequence's true trajectory.  *unresolved != 0 after
// the call means some link did not rejoin a trajectory: run the pass-based dec_sync instead.
struct SpecBufs {
  // per lane slot [tr0 + workgroup * 256 + subsequence-in-workgroup * lanes + lane]
  uint64_t *tE;    // trajectory exit states
  uint8_t *tG;     // walk with entry `lane`: trajectory at the subsequence (or kLinkNone)
  uint64_t *tX;    //   its exit state
  uint32_t *tXc;   //   its block count in the subsequence
  uint64_t *pX;    // resolved prefix records (lane 0 slots)
  uint32_t *pC;
  // per workgroup [wg0 + workgroup] (x kSpecLanesMax where indexed by a lane)
  uint8_t *wF;     // walk e: trajectory at the last subsequence (kLinkNone if explicit)
  uint64_t *wck;   // checkpoints of each workgroup's first subsequence [(wg * 16 + c) * kCk + m]
  uint32_t *wrem;  // blocks from each of them to that subsequence's end
  uint8_t *wB;     // boundary link from the predecessor's last trajectory j
  uint32_t *wBC;
  uint64_t *wBX;
  uint8_t *rE;     // resolved walk column
  uint32_t *rK;    // resolved: prefix covers subsequences 0..rK
  uint32_t *stats;  // diagnostics (VF_SYNC_STATS builds): [1] walker decodes [2] traced workgroups
                    // [3] traced subsequences [4] link misses
};
constexpr int kSpecLanesMax = 16;
inline uint32_t spec_lanes_host(int bpm) { return bpm <= 1 ? 1u : bpm <= 2 ? 2u : bpm <= 4 ? 4u : bpm <= 8 ? 8u : 16u; }
hipError_t dec_sync_spec(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_wg, const uint8_t *us, const uint32_t *us_len,
                         const SpecBufs &b, uint64_t *exit_out, uint32_t *cnt_out, uint32_t *unresolved,
                         hipStream_t s);
hipError_t dec_write(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_sub, const uint8_t *us, const uint32_t *us_len,
                     const uint64_t *exits, const uint32_t *bstart, int16_t *coef, int32_t *dcseq,
                     hipStream_t s);
// the write pass with 4 lanes per subsequence from the pass-based sync's converged checkpoints
hipError_t dec_write4(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_sub, const uint8_t *us,
                      const uint32_t *us_len, const uint64_t *exits, const uint32_t *cnt, const uint64_t *ck,
                      const uint32_t *ckrem, const uint32_t *bstart, int16_t *coef, int32_t *dcseq, hipStream_t s);
hipError_t dec_idct(const DecFrame *fr, int n, uint32_t max_blocks, const int16_t *coef, const int32_t *dcseq,
                    uint8_t *planes, hipStream_t s);
hipError_t dec_color(const DecFrame *fr, int n, int max_w, int max_h, const uint8_t *planes, uint8_t *pix,
                     int bgr, int invert, hipStream_t s);

hipError_t enc_fdct(const EncFrame *fr, int n, uint32_t max_blocks, const EncTables *tab, const uint8_t *pix,
                    int16_t *dcq, uint32_t *acbits, uint32_t *acscr, int bgr, int fastdct, hipStream_t s);
hipError_t enc_len(const EncFrame *fr, int n, uint32_t max_blocks, const EncTables *tab, const int16_t *dcq,
                   uint32_t *acbits, uint32_t *bits, uint32_t *pre, hipStream_t s);
hipError_t enc_pack(const EncFrame *fr, int n, uint32_t max_blocks, const uint32_t *pre, const uint32_t *acbits,
                    const uint32_t *acscr, const uint32_t *bitoff, const uint32_t *total_bits, uint8_t *stream,
                    hipStream_t s);
hipError_t enc_ff_count(const EncFrame *fr, int n, uint32_t max_tiles, const uint32_t *total_bits,
                        const uint8_t *stream, uint32_t *tile_cnt, hipStream_t s);
hipError_t enc_ff_write(const EncFrame *fr, int n, uint32_t max_tiles, const uint32_t *total_bits,
                        const uint8_t *stream, const uint32_t *tile_off, const uint32_t *nff,
                        const uint8_t *hdr, uint8_t *out, uint64_t *out_size, hipStream_t s);
// the batch's finished JPEGs packed back to back (each at a 64-B aligned offset) for one D2H
hipError_t enc_compact(const EncFrame *fr, int n, const uint64_t *out_size, const uint8_t *out, uint8_t *pack,
                       hipStream_t s);

}  // namespace jpeg
}  // namespace vf
