// vf_jpeg_codec.h — the per-context JPEG codec object behind the vf_jpeg_* entry points.
// Not installed.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "vf_jpeg.h"

namespace vf {
namespace jpeg {

// status codes (match VF_* in include/vfilter.h)
constexpr int kOk = 0;
constexpr int kInvalid = -1;
constexpr int kHip = -2;
constexpr int kNoMem = -3;
constexpr int kJpeg = -5;
constexpr int kResync = -100;  // internal: check_decode found the queued sync passes unconverged

// TurboJPEG flag bits honoured (turbojpeg.h)
constexpr int kFlagFastUpsample = 256;
constexpr int kFlagFastDct = 2048;

// grow-only device / pinned buffers
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n);
  template <typename T>
  T *as() const {
    return static_cast<T *>(p);
  }
  ~DevBuf();
};

struct HostBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n);
  template <typename T>
  T *as() const {
    return static_cast<T *>(p);
  }
  ~HostBuf();
};

// A few persistent host threads for the per-frame host work of a batch (parsing, staging and
// output copies): fn(i) for i in [0, n), indices handed out by an atomic counter; the caller
// takes part and returns when every index is done.
class TaskPool {
 public:
  explicit TaskPool(int nthreads);
  ~TaskPool();
  TaskPool(const TaskPool &) = delete;
  TaskPool &operator=(const TaskPool &) = delete;
  void run(int n, const std::function<void(int)> &fn);

 private:
  void loop();
  void drain();
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  bool stop_ = false;
  int active_ = 0;
  int n_ = 0;
  std::atomic<int> next_{0};
  const std::function<void(int)> *fn_ = nullptr;
};

// Orders the GPU compute of the codecs of one context (VF_JPEG_GATE=1; off by default): a
// codec holds `mu` while it queues its kernels, its stream first waits for `last` (the
// previous holder's kernels-done event) and then publishes its own, so kernels of two batches
// never share the GPU.  Round 1 measured two concurrent 4K batches at 12 ms each instead of 6,
// but the codecs' streams then shared one hardware queue with the engine's idle streams; with
// the engine's streams created on first use, two batches in flight run faster ungated
// (worker form, 1080p 22.6 k vs 20.0 k fps, 480p 64.2 k vs 50.9 k, 4K 6.88 k vs 6.36 k:
// profiles/r02_jpeg_hwq2.jsonl).
struct ComputeGate {
  std::mutex mu;
  hipEvent_t last = nullptr;
};

int header_info(const uint8_t *jpeg, size_t size, int *w, int *h, int *subsamp, int *colorspace, std::string *err);
size_t buffer_size(int w, int h, int subsamp);

class Codec {
 public:
  explicit Codec(int device, ComputeGate *gate = nullptr);
  ~Codec();
  Codec(const Codec &) = delete;
  Codec &operator=(const Codec &) = delete;

  // host -> host; every call returns after its outputs are in the caller's buffers
  int encode(const uint8_t *const *imgs, const int *ws, const int *hs, int n, int pixel_format, int quality,
             int subsamp, int flags, uint8_t *const *outs, const size_t *caps, size_t *sizes, std::string *err);
  int decode(const uint8_t *const *jpegs, const size_t *sizes, int n, int pixel_format, int flags,
             uint8_t *const *outs, const size_t *caps, std::string *err);
  int invert(const uint8_t *const *jpegs, const size_t *sizes, int n, int quality, int subsamp, int flags,
             uint8_t *const *outs, const size_t *caps, size_t *out_sizes, std::string *err);
  // invert() in three steps, so one host thread can keep batches of two codecs in flight:
  // submit_invert returns once everything is queued (inputs staged: the caller's buffers may go);
  // done_invert never blocks; wait_invert blocks and gives the packed output size; fetch_invert
  // copies the packed outputs (frame f at offs[f], sizes[f] bytes; out may be NULL).
  int submit_invert(const uint8_t *const *jpegs, const size_t *sizes, int n, int quality, int subsamp, int flags,
                    std::string *err);
  bool done_invert();
  int wait_invert(size_t *total, std::string *err);
  int fetch_invert(uint8_t *out, size_t cap, size_t *sizes, size_t *offs, std::string *err);
  // after wait_invert: frame f's JPEG into outs[f] when it is not NULL and fits caps[f];
  // sizes[f] = its size either way, *placed = how many were copied; the batch stays fetchable
  int scatter_invert(uint8_t *const *outs, const size_t *caps, size_t *sizes, int *placed);
  uint64_t fetch_refills() const { return fetch_refills_; }
  // frames whose SOF claims more pixels are refused before anything is sized from them
  void set_max_pixels(uint64_t v) { max_pixels_ = v ? v : kDefaultMaxPixels; }
  bool waited() const { return waited_; }
  // wait for anything still queued on the codec's stream (after a failed call, before the codec
  // and its pinned buffers go to the next caller)
  void quiesce();
  // the device part of invert() `iters` times on resident inputs; mean wall ms per iteration,
  // stage_ms[0..6] = unstuff, sync, write, dc+idct, colour, fdct+huffman, stuffing; [7] = passes
  int bench_invert(const uint8_t *const *jpegs, const size_t *sizes, int n, int quality, int subsamp, int flags,
                   int iters, float *ms, float *stage_ms, std::string *err);

 private:
  int init(std::string *err);
  int prepare_decode(const uint8_t *const *jpegs, const size_t *sizes, int n, int flags, std::string *err);
  int run_decode(int bgr, bool invert, std::string *err);
  int run_decode_post(int bgr, bool invert, std::string *err);  // write, DC, IDCT, colour
  int finish_sync(std::string *err);  // host-looped span passes after the queued ones
  int check_decode(std::string *err);
  int prepare_encode(const int *ws, const int *hs, const uint64_t *img_offs, int n, int quality, int subsamp,
                     bool fastdct, std::string *err);
  int run_encode(int bgr, bool fastdct, std::string *err);
  int queue_fetch(uint64_t guess, std::string *err);
  int finish_fetch(std::string *err);
  int copy_out(uint8_t *const *outs, const size_t *caps, size_t *sizes, std::string *err);

  int device_;
  ComputeGate *gate_;
  uint64_t max_pixels_ = kDefaultMaxPixels;
  hipStream_t s_ = nullptr;
  hipEvent_t ev_[10] = {};
  bool stage_events_ = false;  // record ev_[0..8] between the stages (bench_invert's breakdown only)
  hipError_t stage_event(int i) { return stage_events_ ? hipEventRecord(ev_[i], s_) : hipSuccess; }
  hipEvent_t done_ = nullptr;  // the last call's downloads have landed

  // decode layout
  // the batch's frames (21 KB each, mostly tables), built by the parse tasks straight into
  // page-locked memory and uploaded from there: no 21 KB-per-frame zero fill and copy on the
  // submitting thread
  HostBuf h_dfr_;
  DecFrame *dfr_ = nullptr;
  int ntabs_ = 0;  // distinct Huffman table sets (DecTabs) of the batch, after its DecFrames
  std::vector<DecSeg> dsg_;    // entropy-coded segments: one per frame, or one per restart interval
  std::vector<const uint8_t *> seg_src_;  // each segment's raw bytes in the caller's JPEG
  int dn_ = 0, dnseg_ = 0, ndcseg_ = 0;
  uint32_t dmax_tiles_ = 0, dmax_sub_ = 0, dmax_blocks_ = 0, dc_max_tiles_ = 0;
  int dmax_w_ = 0, dmax_h_ = 0;
  uint64_t dblocks_ = 0, dpix_bytes_ = 0;
  uint32_t dmax_wg_ = 0;       // speculative sync: workgroups of the largest segment
  bool spec_ok_ = true;        // every frame fits the speculative resolver
  bool tabs4_ = true;          // every frame fits the span sync's 4-table layout (DecFrame::tabs4)
  bool pow2bpm_ = true;        // every frame's blocks per MCU divide 16 (the syncs' LSB-first lanes)
  uint64_t spec_calls_ = 0, spec_fallbacks_ = 0;
  DevBuf d_tE_, d_tX_, d_tXc_, d_pX_, d_pC_, d_wF_, d_rE_, d_rK_, d_qX_, d_qC_, d_rL_,
      d_unres_;
  int sync_passes_ = 0;
  DevBuf d_in_, d_dfr_, d_dsg_, d_segs_, d_tile_, d_tsum_, d_totals_, d_us_, d_exit_[2], d_cnt_[2], d_used_, d_ck_, d_ckrem_, d_bstart_,
      d_changed_, d_coef_, d_nmask_, d_dcseq_, d_dcpred_, d_planes_, d_pix_;

  // encode layout
  std::vector<EncFrame> efr_;
  int en_ = 0;
  int esub_ = 1;  // TJSAMP_* of the prepared encode
  uint32_t emax_blocks_ = 0, emax_tiles_ = 0;
  uint64_t eblocks_ = 0, ebits_bytes_ = 0;
  DevBuf d_eplanes_;  // the invert path's encoder sample planes (fuse_)
  bool fuse_ = false;
  int dcm_ = -1;  // k_color layout shared by the batch's frames (1..3, 0 general), -1 mixed
  bool d422_ = false;  // every frame of the batch is standard 4:2:2 (the fused IDCT + colour pass)
  uint64_t dbits_per_block_ = 0;  // the batch's entropy-coded bits per block (span-sync warm-up)
  uint32_t sync_warm() const;
  DevBuf d_efr_, d_etab_, d_hdr_, d_esegs_, d_etsum_, d_etotals_, d_dcq_, d_acbits_, d_acscr_, d_bits_, d_pre_, d_bitoff_, d_stream_, d_ffcnt_,
      d_outsize_, d_pack_;

  HostBuf h_unres_;            // k_resolve's per-segment unresolved flags (stored through the mapping)
  void *unres_dev_ = nullptr, *dtot_dev_ = nullptr;  // device addresses of h_unres_ / h_dtot_
  HostBuf h_stage_, h_out_, h_flag_;  // h_flag_: the speculative sync's unresolved flag
  HostBuf h_ddesc_, h_edesc_, h_meta_, h_dtot_;  // pinned descriptor uploads; output sizes; block totals
  uint64_t guess_ = 0, out_total_ = 0, fetch_refills_ = 0;
  bool waited_ = false;
  std::vector<uint64_t> out_sizes_, out_offs_;
  bool spec_check_ = false;           // run_decode queued that flag's read; check_decode tests it
  bool pass_check_ = false;           // the same for the last queued sync pass's change flag
  int sync_g_ = 4;                    // span width of the queued passes (finish_sync continues them)
  int sync_t4_ = 0;                   // and their table layout (DecFrame::tabs4)
  int queued_ = kQueuedPasses;        // span passes queued by run_decode
  bool sync_spec_ = false;            // run_decode took the speculative sync (the write pass's form)
  int sync_last_ = 0;                 // exit / count slot of the pass-based sync's result
  bool enc_fast_ = false;             // submit_invert's DCT (wait_invert re-encodes after finish_sync)
  // output bytes per input byte of the codec's last invert batch (0: none yet): the next batch's
  // first D2H copy is sized from it instead of from the input sizes alone (VF_JPEG_FETCH_LEARN=0:
  // the fixed rule), so content that shrinks when re-encoded does not drag twice its output over PCIe
  double out_ratio_ = 0;
  uint64_t in_bytes_ = 0;
  TaskPool pool_{4};
  double prep_ms_[3] = {0, 0, 0};  // VF_JPEG_TRACE: prepare_decode's parse / descriptor loop / staging
  std::vector<uint64_t> ekey_;     // prepare_encode's last batch shape (n, settings, sizes, offsets)
  bool ekey_valid_ = false;        // ... and its device-side descriptors are current
  uint64_t enc_prep_reused_ = 0;
};

}  // namespace jpeg
}  // namespace vf
