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

#include "vf_jpeg_types.h"

namespace vf {
namespace jpeg {


// ---- launchers (vf_jpeg_kernels.hip) ----------------------------------------------------
hipError_t scan_u32(const ScanSeg *segs, int nseg, uint32_t max_tiles, const uint32_t *in, uint32_t *out,
                    uint32_t *tsum, uint32_t *totals, bool inclusive, hipStream_t s);
hipError_t scan_i32(const ScanSeg *segs, int nseg, uint32_t max_tiles, const int32_t *in, int32_t *out,
                    int32_t *tsum, int32_t *totals, bool inclusive, hipStream_t s);

hipError_t dec_unstuff_count(const DecSeg *sg, int nseg, uint32_t max_tiles, const uint8_t *in,
                             uint32_t *tile_cnt, hipStream_t s);
hipError_t dec_unstuff_write(const DecSeg *sg, int nseg, uint32_t max_tiles, const uint8_t *in,
                             const uint32_t *tile_off, const uint32_t *us_len, uint8_t *us, hipStream_t s);
// pass-based sync, G (1, 2, 4, 8) subsequences per thread, records updated in place; pass p
// returns at once when changed[p - 1] == 0, so passes are queued without host round trips
hipError_t dec_syncg(int G, const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_sub, const uint8_t *us,
                     const uint32_t *us_len, uint64_t *exits, uint32_t *cnts, uint64_t *used, uint64_t *ck,
                     uint32_t *ckrem, uint32_t *changed, int pass, uint32_t warm, int tabs4, hipStream_t s);
// tabs4: every frame's DecFrame::tabs4 is set (G = 4 or 5 then; else G = 1, 2, 3, 4 or 8); 2: and every
// frame's bpm divides 32 (the LSB-first lane)
hipError_t dec_sync(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_sub, const uint8_t *us, const uint32_t *us_len,
                    const uint64_t *exit_in, uint64_t *exit_out, const uint32_t *cnt_in, uint32_t *cnt_out,
                    uint64_t *used, uint64_t *ck, uint32_t *ckrem, uint32_t *changed, int pass, hipStream_t s);
// Speculative sync (one pass, no host round trip): k_spec decodes every subsequence from
// each possible block-in-MCU and links neighbouring subsequences (workgroups overlap by one
// subsequence, so the links across workgroup boundaries are made there too), k_resolve /
// k_finalize pick each subsequence's true trajectory.  *unresolved != 0 after the call means a
// frame had more workgroups than k_resolve stages: run the pass-based dec_sync instead.
struct SpecBufs {
  // per lane slot [tr0 + workgroup * 256 + row * lanes + lane]; row k of workgroup w is
  // subsequence w * (256 / lanes - 1) + k
  uint64_t *tE;    // trajectory exit states
  uint64_t *tX;    // walk with entry `lane`: its exit state at the subsequence
  uint32_t *tXc;   //   its block count in the subsequence
  uint64_t *pX;    // prefix records of k_resolve's serial traces (lane 0 slots)
  uint32_t *pC;
  // per workgroup [wg0 + workgroup] (x kSpecLanesMax where indexed by a lane)
  uint8_t *wF;     // walk e: trajectory at the last row (kLinkNone if explicit)
  uint8_t *rE;     // resolved walk column
  uint32_t *rK;    // resolved: the walk column from row rK on, prefix records before it
  uint64_t *qX;    // prefix records of the traces of walk columns that ended explicit (lane = e)
  uint32_t *qC;
  uint8_t *rL;     // resolved: where the prefix records are (0x80 | lane: pX, 0xC0 | lane: qX)
  uint32_t *stats;  // diagnostics (VF_JPEG_SYNC_STATS; k_spec's phases in VF_SPEC_PHASES builds)
};
constexpr int kSpecLanesMax = 16;
inline uint32_t spec_lanes_host(int bpm) { return bpm <= 1 ? 1u : bpm <= 2 ? 2u : bpm <= 4 ? 4u : bpm <= 8 ? 8u : 16u; }
hipError_t dec_sync_spec(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_wg, const uint8_t *us, const uint32_t *us_len,
                         const SpecBufs &b, uint64_t *exit_out, uint32_t *cnt_out, uint32_t *unresolved,
                         int lsb, hipStream_t s);  // lsb: every frame's blocks per MCU divide 16
hipError_t dec_write(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_sub, const uint8_t *us, const uint32_t *us_len,
                     const uint64_t *exits, const uint32_t *bstart, int16_t *coef, int32_t *dcseq,
                     uint8_t *nmask, hipStream_t s);  // nmask: chunked coefficient rows (else a cleared buffer)
// the write pass with 4 lanes per subsequence from the pass-based sync's converged checkpoints
hipError_t dec_write4(const DecSeg *sg, const DecFrame *fr, int nseg, uint32_t max_sub, const uint8_t *us,
                      const uint32_t *us_len, const uint64_t *exits, const uint32_t *cnt, const uint64_t *ck,
                      const uint32_t *ckrem, const uint32_t *bstart, int16_t *coef, int32_t *dcseq, uint8_t *nmask,
                      hipStream_t s);
// nmask: per-block stored-row masks from the write pass's chunked form (null: a cleared buffer)
hipError_t dec_idct(const DecFrame *fr, int n, uint32_t max_blocks, const int16_t *coef, const int32_t *dcseq,
                    const uint8_t *nmask, uint8_t *planes, hipStream_t s);
hipError_t dec_color(const DecFrame *fr, int n, int max_w, int max_h, const uint8_t *planes, uint8_t *pix,
                     int bgr, int invert, const EncFrame *efr, int cm, hipStream_t s);
// the invert path's IDCT + colour in one pass for a batch of standard 4:2:2 frames (sampling 2x1,
// 1x1, 1x1): the decoder planes stay in LDS, the encoder's sample planes come out
hipError_t dec_idct_color422(const DecFrame *fr, int n, int max_w, int max_h, const int16_t *coef,
                             const int32_t *dcseq, const uint8_t *nmask, uint8_t *eplanes, const EncFrame *efr,
                             int invert, int one_row,
                             hipStream_t s);  // one_row: the encoder's chroma is not vertically downsampled

hipError_t enc_fdct(const EncFrame *fr, int n, uint32_t max_blocks, const EncTables *tab, const uint8_t *pix,
                    int16_t *dcq, uint32_t *acbits, uint32_t *acscr, int bgr, int fastdct, int ch, int cv, int planes,
                    hipStream_t s);  // (ch, cv): chroma downsampling factors
hipError_t enc_len(const EncFrame *fr, int n, uint32_t max_blocks, const EncTables *tab, const int16_t *dcq,
                   uint32_t *acbits, uint32_t *bits, uint32_t *pre, hipStream_t s);
hipError_t enc_pack(const EncFrame *fr, int n, uint32_t max_blocks, const uint32_t *pre, const uint32_t *acbits,
                    const uint32_t *acscr, const uint32_t *bitoff, const uint32_t *total_bits, uint8_t *stream,
                    hipStream_t s);
hipError_t enc_ff_count(const EncFrame *fr, int n, uint32_t max_tiles, const uint32_t *total_bits,
                        const uint8_t *stream, uint32_t *tile_cnt, hipStream_t s);
hipError_t enc_ff_write(const EncFrame *fr, int n, uint32_t max_tiles, const uint32_t *total_bits,
                        const uint8_t *stream, const uint32_t *tile_off, const uint32_t *nff,
                        const uint8_t *hdr, uint8_t *pack, uint64_t *out_size, hipStream_t s);

}  // namespace jpeg
}  // namespace vf
