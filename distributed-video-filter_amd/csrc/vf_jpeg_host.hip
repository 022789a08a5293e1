// vf_jpeg_host.hip — host side of the gfx950 baseline-JPEG path: marker parsing, tables,
// batch layout in HBM and the launch sequence of vf_jpeg_kernels.hip.
//
// What it replaces (reference default mode, use_jpeg=True):
//   frame = self.jpeg.decode(frame_bytes)     inverter.py:32   -> Codec::decode
//   inverted = cv2.bitwise_not(frame)         inverter.py:41   -> fused into the decode's colour stage
//   return self.jpeg.encode(inverted)         inverter.py:44   -> Codec::encode
// PyTurboJPEG defaults: quality 85, TJSAMP_422, TJPF_BGR, flags 0.  Marker syntax and table
// construction follow libjpeg-turbo (jdmarker.c, jdhuff.c, jcparam.c, jcmarker.c, jchuff.c,
// jcdctmgr.c), restated here for the product; oracle/vf_jpeg_oracle.c is the checker.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "vf_host_mem.h"
#include "vf_jpeg.h"
#include "vf_jpeg_codec.h"
#include "vf_jpeg_parse.h"

namespace vf {
namespace jpeg {

namespace {


// jcmarker.c: SOI, JFIF APP0, DQT(s), SOF0, DHT(s), SOS for the TurboJPEG defaults
size_t write_header(int w, int h, int quality, int subsamp, uint8_t *o) {
  size_t n = 0;
  auto b = [&](int v) { o[n++] = (uint8_t)v; };
  auto u16 = [&](int v) {
    b(v >> 8);
    b(v & 0xFF);
  };
  const int nc = subsamp == 3 ? 1 : 3;
  uint16_t q[2][64];
  quality_table(quality, false, q[0]);
  quality_table(quality, true, q[1]);
  b(0xFF);
  b(0xD8);
  const uint8_t app0[18] = {0xFF, 0xE0, 0, 16, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
  for (uint8_t v : app0) b(v);
  for (int t = 0; t < (nc == 3 ? 2 : 1); ++t) {
    b(0xFF);
    b(0xDB);
    u16(67);
    b(t);
    for (int i = 0; i < 64; ++i) b(q[t][kNatH[i]]);
  }
  b(0xFF);
  b(0xC0);
  u16(8 + 3 * nc);
  b(8);
  u16(h);
  u16(w);
  b(nc);
  for (int c = 0; c < nc; ++c) {
    b(c + 1);
    b(c == 0 ? (kSampH[subsamp] << 4) | kSampV[subsamp] : 0x11);
    b(c == 0 ? 0 : 1);
  }
  auto dht = [&](int idx, const uint8_t *bits, const uint8_t *vals) {
    int cnt = 0;
    for (int l = 1; l <= 16; ++l) cnt += bits[l];
    b(0xFF);
    b(0xC4);
    u16(19 + cnt);
    b(idx);
    for (int l = 1; l <= 16; ++l) b(bits[l]);
    for (int i = 0; i < cnt; ++i) b(vals[i]);
  };
  dht(0x00, kDcLBits, kDcVals);
  dht(0x10, kAcLBits, kAcLVals);
  if (nc == 3) {
    dht(0x01, kDcCBits, kDcVals);
    dht(0x11, kAcCBits, kAcCVals);
  }
  b(0xFF);
  b(0xDA);
  u16(6 + 2 * nc);
  b(nc);
  for (int c = 0; c < nc; ++c) {
    b(c + 1);
    b(c == 0 ? 0x00 : 0x11);
  }
  b(0);
  b(63);
  b(0);
  return n;
}

// jcdctmgr.c start_pass_fdctmgr + compute_reciprocal (16-bit DCTELEM, the SIMD build)
void build_enc_tables(int quality, bool fastdct, EncTables *t) {
  std::memset(t, 0, sizeof *t);
  for (int tb = 0; tb < 2; ++tb) {
    uint16_t q[64];
    quality_table(quality, tb == 1, q);
    for (int i = 0; i < 64; ++i) {
      const uint32_t divisor = fastdct ? (uint32_t)(((int32_t)q[i] * kAanScales[i] + (1 << 10)) >> 11)
                                       : (uint32_t)q[i] << 3;
      if (divisor == 1) {
        t->recip[tb][i] = 1;
        t->corr[tb][i] = 0;
        t->shift[tb][i] = -16;
        continue;
      }
      const int b = 31 - __builtin_clz(divisor);
      int r = 16 + b;
      uint32_t fq = (1u << r) / divisor, fr = (1u << r) % divisor, c = divisor / 2;
      if (fr == 0) {
        fq >>= 1;
        --r;
      } else if (fr <= divisor / 2u) {
        ++c;
      } else {
        ++fq;
      }
      t->recip[tb][i] = (uint16_t)fq;
      t->corr[tb][i] = (uint16_t)c;
      t->shift[tb][i] = (int16_t)(r - 16);
    }
  }
  for (int tb = 0; tb < 2; ++tb)
    for (int i = 0; i < 64; ++i) {
      uint32_t y = (uint32_t)(t->shift[tb][i] + 16);
      for (uint32_t j = 0; j < 4; ++j) y |= qo_pos(j, kZigOf[i]) << (8 + 6 * j);
      t->fdct_lds[2 * (64 * tb + i)] = (uint32_t)t->recip[tb][i] | ((uint32_t)t->corr[tb][i] << 16);
      t->fdct_lds[2 * (64 * tb + i) + 1] = y;
    }
  code_table(kDcLBits, kDcVals, t->dc[0], 16);
  code_table(kDcCBits, kDcVals, t->dc[1], 16);
  code_table(kAcLBits, kAcLVals, t->ac[0], 256);
  code_table(kAcCBits, kAcCVals, t->ac[1], 256);
  std::memcpy(t->fdct_lds + 256, t->ac, sizeof t->ac);
}

// worst case per block: DC 16 + 11 bits, 63 AC codes of 16 + 10 bits
constexpr size_t kMaxBlockBytes = (27 + 63 * 26 + 7) / 8 + 1;

}  // namespace


// ---- device / pinned buffers ---------------------------------------------------------------

hipError_t DevBuf::ensure(size_t n) {
  if (n <= cap) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  n = align_up(std::max<size_t>(n, 256), 1 << 20);
  hipError_t e = hipMalloc(&p, n);
  if (e == hipSuccess) cap = n;
  return e;
}

DevBuf::~DevBuf() {
  if (p) (void)hipFree(p);
}

hipError_t HostBuf::ensure(size_t n) {
  if (n <= cap) return hipSuccess;
  (void)numa_pinned_free(p);
  p = nullptr;
  cap = 0;
  n = align_up(std::max<size_t>(n, 256), 1 << 20);
  int dev = 0;
  (void)hipGetDevice(&dev);  // the codec's device (Codec::init set it on this thread)
  hipError_t e = numa_pinned_alloc(&p, n, device_numa_node(dev));
  if (e == hipSuccess) cap = n;
  return e;
}

HostBuf::~HostBuf() { (void)numa_pinned_free(p); }

// ---- codec -------------------------------------------------------------------------------------

TaskPool::TaskPool(int nthreads) {
  for (int i = 1; i < nthreads; ++i) threads_.emplace_back([this] { loop(); });
}

TaskPool::~TaskPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
    ++gen_;
  }
  cv_.notify_all();
  for (auto &t : threads_) t.join();
}

void TaskPool::drain() {
  for (int i = next_.fetch_add(1); i < n_; i = next_.fetch_add(1)) (*fn_)(i);
}

void TaskPool::run(int n, const std::function<void(int)> &fn) {
  if (n <= 1 || threads_.empty()) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    fn_ = &fn;
    n_ = n;
    next_.store(0);
    active_ = (int)threads_.size();
    ++gen_;
  }
  cv_.notify_all();
  drain();
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [this] { return active_ == 0; });
  fn_ = nullptr;
}

void TaskPool::loop() {
  uint64_t seen = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (stop_) return;
    }
    drain();
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (--active_ == 0) done_cv_.notify_one();
    }
  }
}

Codec::Codec(int device, ComputeGate *gate) : device_(device), gate_(gate) {}

Codec::~Codec() {
  (void)hipSetDevice(device_);
  if (s_) {
    (void)hipStreamSynchronize(s_);
    (void)hipStreamDestroy(s_);
  }
  for (hipEvent_t e : ev_)
    if (e) (void)hipEventDestroy(e);
  if (done_) (void)hipEventDestroy(done_);
}

#define CK(call)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) {                                                               \
      *err = std::string(#call) + ": " + hipGetErrorString(e_);                           \
      return e_ == hipErrorOutOfMemory || e_ == hipErrorMemoryAllocation ? kNoMem : kHip; \
    }                                                                                     \
  } while (0)

int Codec::init(std::string *err) {
  if (s_) return kOk;
  CK(hipSetDevice(device_));
  CK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  for (hipEvent_t &e : ev_) CK(hipEventCreate(&e));
  CK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  return kOk;
}

// Host parse of every frame + batch layout + upload of inputs and descriptors.
// The invert path's fused colour pass (k_color writes the encoder's sample planes, k_fdct reads
// them); VF_JPEG_FUSE=0 keeps the pixel round trip (read per call: tests switch it).
// Bits a span-sync thread decodes before its span in pass 0, so that its entry is (usually)
// synchronised already: 12 blocks' worth of the batch's bits per block -- the full state (bit
// position, zigzag index, block-in-MCU) resynchronises at block boundaries (hard 1080p: ~250
// bits per block, 3,008 bits of warm-up; 4K scenes: ~20, 240).  12 rather than 8 blocks: hard
// 1080p sync 4-9 % shorter on each of four content seeds, 4K scenes unchanged
// (profiles/r05_jpeg_sync_warm_ab.txt).  VF_JPEG_SYNC_WARM=<bits> overrides (0: guessed
// entries), read per call: tests and A/Bs switch it inside one process.
uint32_t Codec::sync_warm() const {
  const char *v = std::getenv("VF_JPEG_SYNC_WARM");
  if (v && *v && std::strcmp(v, "auto") != 0) return (uint32_t)std::strtoul(v, nullptr, 10);
  return (uint32_t)std::min<uint64_t>(4096, 12 * dbits_per_block_) & ~31u;
}

static bool fuse_enabled() {
  const char *v = std::getenv("VF_JPEG_FUSE");
  return !(v && std::strcmp(v, "0") == 0);
}

int Codec::prepare_decode(const uint8_t *const *jpegs, const size_t *sizes, int n, int flags, std::string *err) {
  fuse_ = false;
  if (n <= 0) {
    *err = "empty batch";
    return kInvalid;
  }
  // [n DecFrames][the batch's distinct DecTabs], one pinned buffer and one upload
  const size_t toff = align_up(sizeof(DecFrame) * (size_t)n, 256);
  CK(h_dfr_.ensure(toff + sizeof(DecTabs) * (size_t)n));
  dfr_ = h_dfr_.as<DecFrame>();
  seg_src_.clear();
  std::vector<Parsed> parsed((size_t)n);
  uint64_t in_off = 0, us_off = 0, blk = 0, dcoff = 0, plane = 0, pix = 0;
  uint32_t tiles = 0, subs = 0, wgs = 0;
  uint64_t trs = 0;
  dmax_tiles_ = dmax_sub_ = dmax_blocks_ = dmax_wg_ = 0;
  spec_ok_ = true;
  dmax_w_ = dmax_h_ = 0;
  // per frame, in parallel: markers, scan end, geometry and decode tables
  std::vector<std::string> ferr((size_t)n);
  using clk = std::chrono::steady_clock;
  const auto tp0 = clk::now();
  // per frame on its parse task: markers, geometry, quantisers, the largest AC quantiser (the
  // bound k_idct's column pass needs for 24-bit multiplies, vf_jpeg_types.h) and the key of its
  // Huffman tables; the tables themselves are built once per distinct key below
  std::vector<uint32_t> qmax((size_t)n);
  std::vector<uint64_t> khash((size_t)n);
  std::vector<std::vector<uint8_t>> keys((size_t)n);
  pool_.run(n, [&](int f) {
    Parsed &P = parsed[(size_t)f];
    std::string &e = ferr[(size_t)f];
    DecFrame &F = *new (&dfr_[(size_t)f]) DecFrame();  // value-initialised, by the frame's own task
    parse_frame(jpegs[f], sizes[f], max_pixels_, &P, &F.g, nullptr, nullptr, nullptr, nullptr, nullptr, &e);  // vf_jpeg_parse.h
    if (!e.empty()) return;
    uint32_t q_ac = 0;
    for (int c = 0; c < P.ncomp; ++c) {
      std::memcpy(F.q[c], P.qt[P.tq[c]], sizeof F.q[c]);
      for (int i = 1; i < 64; ++i) q_ac = std::max(q_ac, (uint32_t)F.q[c][i]);
    }
    qmax[(size_t)f] = q_ac;
    khash[(size_t)f] = table_key(P, &keys[(size_t)f]);
  });
  const auto tp1 = clk::now();
  for (int f = 0; f < n; ++f)
    if (!ferr[(size_t)f].empty()) {
      *err = "frame " + std::to_string(f) + ": " + ferr[(size_t)f];
      return kJpeg;
    }
  // the distinct table sets (a batch of one stream has one): built into the buffer after the frames
  std::vector<int> uniq;      // first frame of each distinct set
  std::vector<int> acmax;     // its largest AC size (unused symbol slots are zero)
  std::vector<uint8_t> m24ok((size_t)n);  // the frame's tables and quantisers fit kDecIdct24
  for (int f = 0; f < n; ++f) {
    int u = 0;
    for (; u < (int)uniq.size(); ++u)
      if (khash[(size_t)uniq[(size_t)u]] == khash[(size_t)f] && keys[(size_t)uniq[(size_t)u]] == keys[(size_t)f]) break;
    if (u == (int)uniq.size()) {
      const Parsed &P = parsed[(size_t)f];
      DecTabs &T = *new (h_dfr_.as<uint8_t>() + toff + sizeof(DecTabs) * uniq.size()) DecTabs();
      for (int c = 0; c < P.ncomp; ++c)
        if (!build_tables(P.dcbits[P.td[c]], P.dcvals[P.td[c]], true, &T.dc[c], &T.sdc[c]) ||
            !build_tables(P.acbits[P.ta[c]], P.acvals[P.ta[c]], false, &T.ac[c], &T.sac[c], T.spair[c])) {
          *err = "frame " + std::to_string(f) + ": bad Huffman table";
          return kJpeg;
        }
      int a = 0;
      for (int c = 0; c < P.ncomp; ++c)
        for (int i = 0; i < 256; ++i) a = std::max(a, (int)(T.ac[c].vals[i] & 15));
      uniq.push_back(f);
      acmax.push_back(a);
    }
    dfr_[(size_t)f].tabs_off = toff + sizeof(DecTabs) * (size_t)u;
    m24ok[(size_t)f] = idct_col24_ok(acmax[(size_t)u], qmax[(size_t)f]) ? 1 : 0;
  }
  ntabs_ = (int)uniq.size();
  dsg_.clear();
  dcm_ = -2;  // the batch's common k_color layout, or -1 (mixed)
  // VF_JPEG_IDCT24=0: every frame on the 32-bit column pass (an A/B and test selector)
  const char *i24 = std::getenv("VF_JPEG_IDCT24");
  const bool idct24 = !(i24 && std::strcmp(i24, "0") == 0);
  d422_ = true;  // every frame standard 4:2:2 (k_idct_color422)
  tabs4_ = true;  // every frame fits the span sync's 4-table layout (DecFrame::tabs4)
  pow2bpm_ = true;  // every frame's blocks per MCU divide 16 (the span and speculative syncs' LSB-first lanes)
  for (int f = 0; f < n; ++f) {
    const Parsed &P = parsed[(size_t)f];
    DecFrame &F = dfr_[(size_t)f];
    F.flags = (flags & kFlagFastUpsample) ? 0u : 1u;
    {  // k_color's layout (vf_jpeg.h DecFrame.flags), read as one scalar word on the device
      const Geom &g = F.g;
      uint32_t cm = 0;
      if (g.ncomp == 3 && g.he[0] == 1 && g.ve[0] == 1 && g.he[1] == g.he[2] && g.ve[1] == g.ve[2])
        cm = g.he[1] == 1 && g.ve[1] == 1 ? 1u : g.he[1] == 2 && g.ve[1] == 1 ? 2u : g.he[1] == 2 && g.ve[1] == 2 ? 3u : 0u;
      F.flags |= cm << 1;
      if (idct24 && m24ok[(size_t)f]) F.flags |= kDecIdct24;
      dcm_ = dcm_ == -2 || dcm_ == (int)cm ? (int)cm : -1;
      d422_ = d422_ && g.ncomp == 3 && g.hs[0] == 2 && g.vs[0] == 1 && g.hs[1] == 1 && g.vs[1] == 1 &&
              g.hs[2] == 1 && g.vs[2] == 1 && g.bpm == 4;
    }
    {  // the span sync's 4-table layout: components with the same (DC, AC) table ids share a
       // slot; a frame with three distinct pairs keeps the batch on the 6-table form
      uint32_t s4 = 0, rep = 0;
      int key[2] = {-1, -1}, nsl = 0;
      bool ok = true;
      for (int c = 0; c < P.ncomp && ok; ++c) {
        const int k = P.td[c] * 16 + P.ta[c];
        int sl = k == key[0] ? 0 : k == key[1] ? 1 : -1;
        if (sl < 0 && nsl == 2) ok = false;
        if (sl < 0 && ok) {
          key[nsl] = k;
          rep |= (uint32_t)c << (8 + 2 * nsl);
          sl = nsl++;
        }
        if (ok) s4 |= (uint32_t)sl << (2 * c);
      }
      if (ok && nsl == 1) rep |= (rep & 0x300u) << 2;  // slot 1 unused: a copy of slot 0
      F.tabs4 = ok ? (s4 | rep | 0x80000000u) : 0u;
      tabs4_ = tabs4_ && ok;
      pow2bpm_ = pow2bpm_ && F.g.bpm >= 1 && F.g.bpm <= 16 && (F.g.bpm & (F.g.bpm - 1)) == 0;
    }
    F.blk0 = blk;
    for (int c = 0; c < P.ncomp; ++c) {
      F.dcbase[c] = dcoff;
      dcoff += (uint64_t)F.g.nmcu * F.g.mh[c] * F.g.mv[c];
      F.plane_off[c] = plane;
      plane += align_up((size_t)F.g.pw[c] * F.g.ph[c], 256);
    }
    F.out_off = pix;
    pix += align_up((size_t)P.w * P.h * 3, 256);
    blk += (uint64_t)F.g.nblocks;
    // entropy-coded segments: the scan, or its restart intervals (whole MCUs each, the last
    // one the remainder), with their blocks and DC sequence entries inside the frame's
    const uint32_t nmcu = (uint32_t)F.g.nmcu, per = P.restart ? (uint32_t)P.restart : nmcu;
    size_t start = P.scan_off;
    for (size_t i = 0; i <= P.rst.size(); ++i) {
      const size_t end = i < P.rst.size() ? P.rst[i].first : P.scan_end;
      const size_t len = end - start;
      const uint32_t m0 = (uint32_t)i * per, mc = std::min(per, nmcu - m0);
      DecSeg S{};
      S.frame = (uint32_t)f;
      S.nblocks = mc * (uint32_t)F.g.bpm;
      S.blk0 = F.blk0 + (uint64_t)m0 * F.g.bpm;
      for (int c = 0; c < P.ncomp; ++c) S.dcbase[c] = F.dcbase[c] + (uint64_t)m0 * F.g.mh[c] * F.g.mv[c];
      S.in_off = in_off;
      S.in_len = (uint32_t)len;
      S.ntiles = (uint32_t)((len + kTile - 1) / kTile);
      S.tile0 = tiles;
      S.sub0 = subs;
      S.nsub_max = (uint32_t)((len * 8 + kSubBits - 1) / kSubBits);
      {  // speculative sync layout: spec_lanes(bpm) lanes per subsequence, 256 lanes per workgroup,
         // ns rows per workgroup of which the last is the next workgroup's first
        const uint32_t ns = 256 / spec_lanes_host(F.g.bpm);
        S.nwg = S.nsub_max <= ns ? 1u : 1u + (S.nsub_max - ns + ns - 2) / (ns - 1);
        S.wg0 = wgs;
        S.tr0 = trs;
        wgs += S.nwg;
        trs += (uint64_t)S.nwg * 256;
        dmax_wg_ = std::max(dmax_wg_, S.nwg);
        // k_resolve stages at most 4096 workgroups and 16384 (workgroup, entry) transitions per segment
        if (S.nwg > 4096 || (uint64_t)S.nwg * (uint64_t)F.g.bpm > 16384) spec_ok_ = false;
      }
      S.us_off = us_off;
      in_off += align_up(len, 16);
      us_off += align_up(len + 64, 16);
      tiles += S.ntiles;
      subs += S.nsub_max;
      dmax_tiles_ = std::max(dmax_tiles_, S.ntiles);
      dmax_sub_ = std::max(dmax_sub_, S.nsub_max);
      seg_src_.push_back(jpegs[f] + start);
      dsg_.push_back(S);
      if (i < P.rst.size()) start = P.rst[i].second + 2;
    }
    dmax_blocks_ = std::max(dmax_blocks_, (uint32_t)F.g.nblocks);
    dmax_w_ = std::max(dmax_w_, P.w);
    dmax_h_ = std::max(dmax_h_, P.h);
  }
  dn_ = n;
  dnseg_ = (int)dsg_.size();
  if (dnseg_ > 65535) {
    *err = "more than 65535 restart intervals in one batch (split the batch)";
    return kInvalid;
  }
  if (dcoff >= (1ull << 31)) {  // the write pass keeps DC sequence positions in 32 bits
    *err = "more than 2^31 blocks in one batch (split the batch)";
    return kInvalid;
  }
  dblocks_ = blk;
  dpix_bytes_ = pix;
  {
    uint64_t bits = 0;
    for (const DecSeg &S : dsg_) bits += (uint64_t)S.in_len * 8;
    dbits_per_block_ = blk ? bits / blk : 0;
  }
  // scan segments: [0, nseg) unstuff tiles, [nseg, 2 nseg) subsequence counts, then DC sequences
  // (per entropy-coded segment and component: restart intervals reset the DC prediction)
  std::vector<ScanSeg> segs;
  uint32_t t0 = 0;
  auto add = [&](uint64_t base, uint32_t len) {
    segs.push_back(ScanSeg{base, len, t0});
    t0 += (len + kScanTile - 1) / kScanTile;
  };
  for (auto &S : dsg_) add(S.tile0, S.ntiles);
  for (auto &S : dsg_) add(S.sub0, S.nsub_max);
  ndcseg_ = 0;
  dc_max_tiles_ = 0;
  for (auto &S : dsg_) {
    const Geom &g = dfr_[S.frame].g;
    for (int c = 0; c < g.ncomp; ++c) {
      const uint32_t len = S.nblocks / (uint32_t)g.bpm * (uint32_t)(g.mh[c] * g.mv[c]);
      add(S.dcbase[c], len);
      dc_max_tiles_ = std::max(dc_max_tiles_, (len + kScanTile - 1) / kScanTile);
      ++ndcseg_;
    }
  }
  const auto tp2 = clk::now();
  // staging: inputs packed, then uploaded in one copy
  CK(h_stage_.ensure(in_off));
  pool_.run(dnseg_, [&](int i) {
    const DecSeg &S = dsg_[(size_t)i];
    std::memcpy(h_stage_.as<uint8_t>() + S.in_off, seg_src_[(size_t)i], S.in_len);
  });
  CK(hipSetDevice(device_));
  CK(d_in_.ensure(in_off));
  CK(d_dfr_.ensure(toff + sizeof(DecTabs) * (size_t)ntabs_));
  CK(d_dsg_.ensure(sizeof(DecSeg) * (size_t)dnseg_));
  CK(d_segs_.ensure(sizeof(ScanSeg) * segs.size()));
  CK(d_tile_.ensure(sizeof(uint32_t) * tiles));
  CK(d_tsum_.ensure(sizeof(int32_t) * (t0 + 1)));
  CK(d_totals_.ensure(sizeof(int32_t) * segs.size()));
  // page-locked per-segment results the kernels store through the mapping (check_decode)
  CK(h_dtot_.ensure(sizeof(uint32_t) * (size_t)dnseg_ + 64));
  CK(h_unres_.ensure(sizeof(uint32_t) * (size_t)dnseg_ + 64));
  CK(hipHostGetDevicePointer(&dtot_dev_, h_dtot_.p, 0));
  CK(hipHostGetDevicePointer(&unres_dev_, h_unres_.p, 0));
  CK(d_us_.ensure(us_off));
  CK(d_exit_[0].ensure(sizeof(uint64_t) * subs));
  CK(d_exit_[1].ensure(sizeof(uint64_t) * subs));
  CK(d_cnt_[0].ensure(sizeof(uint32_t) * subs));
  CK(d_cnt_[1].ensure(sizeof(uint32_t) * subs));
  CK(d_used_.ensure(sizeof(uint64_t) * subs));
  CK(d_ck_.ensure(sizeof(uint64_t) * subs * kCk));
  CK(d_ckrem_.ensure(sizeof(uint32_t) * subs * kCk));
  CK(d_bstart_.ensure(sizeof(uint32_t) * subs));
  {  // speculative sync (see SpecBufs)
    const size_t sl = (size_t)trs, wl = (size_t)wgs * kSpecLanesMax;
    CK(d_tE_.ensure(sizeof(uint64_t) * sl));
    CK(d_tX_.ensure(sizeof(uint64_t) * sl));
    CK(d_tXc_.ensure(sizeof(uint32_t) * sl));
    CK(d_pX_.ensure(sizeof(uint64_t) * sl));
    CK(d_pC_.ensure(sizeof(uint32_t) * sl));
    CK(d_wF_.ensure(wl));
    CK(d_rE_.ensure(wgs));
    CK(d_rK_.ensure(sizeof(uint32_t) * wgs));
    CK(d_qX_.ensure(sizeof(uint64_t) * sl));
    CK(d_qC_.ensure(sizeof(uint32_t) * sl));
    CK(d_rL_.ensure(wgs));
    CK(d_unres_.ensure(sizeof(uint32_t) * 16));
  }
  CK(d_changed_.ensure(sizeof(uint32_t) * kMaxPasses));
  CK(d_coef_.ensure(blk * 128));
  CK(d_nmask_.ensure(blk + 16));
  CK(d_dcseq_.ensure(sizeof(int32_t) * (dcoff + 1)));
  CK(d_dcpred_.ensure(sizeof(int32_t) * (dcoff + 1)));  // the scan's output: out of place, so short sequences scan in one pass
  CK(d_planes_.ensure(plane));
  CK(d_pix_.ensure(pix));
  // descriptors go through pinned memory too, so every upload stays asynchronous and nothing
  // waits for the GPU before the kernels are queued (the pinned buffers are reused only by the
  // codec's next call, which starts after this one has synchronised)
  const size_t dsz = toff + sizeof(DecTabs) * (size_t)ntabs_, gsz = sizeof(DecSeg) * (size_t)dnseg_,
               ssz = sizeof(ScanSeg) * segs.size();
  CK(h_ddesc_.ensure(gsz + ssz));
  std::memcpy(h_ddesc_.as<uint8_t>(), dsg_.data(), gsz);
  std::memcpy(h_ddesc_.as<uint8_t>() + gsz, segs.data(), ssz);
  CK(hipMemcpyAsync(d_in_.p, h_stage_.p, in_off, hipMemcpyHostToDevice, s_));
  CK(hipMemcpyAsync(d_dfr_.p, h_dfr_.p, dsz, hipMemcpyHostToDevice, s_));
  CK(hipMemcpyAsync(d_dsg_.p, h_ddesc_.p, gsz, hipMemcpyHostToDevice, s_));
  CK(hipMemcpyAsync(d_segs_.p, h_ddesc_.as<uint8_t>() + gsz, ssz, hipMemcpyHostToDevice, s_));
  {  // VF_JPEG_TRACE's split of prep_dec: parse tasks | descriptor loop | staging, buffers, uploads
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    prep_ms_[0] = ms(tp0, tp1);
    prep_ms_[1] = ms(tp1, tp2);
    prep_ms_[2] = ms(tp2, clk::now());
  }
  return kOk;
}

// Device part of the decode: unstuff -> sync passes -> write -> DC -> IDCT -> colour.
int Codec::run_decode(int bgr, bool invert, std::string *err) {
  const DecFrame *fr = d_dfr_.as<DecFrame>();
  const DecSeg *sg = d_dsg_.as<DecSeg>();
  const ScanSeg *segs = d_segs_.as<ScanSeg>();
  const int ns = dnseg_;
  CK(stage_event(0));
  // 1. unstuff
  CK(dec_unstuff_count(sg, ns, dmax_tiles_, d_in_.as<uint8_t>(), d_tile_.as<uint32_t>(), s_));
  uint32_t *us_len = d_totals_.as<uint32_t>();  // totals of scan segments [0, ns)
  CK(scan_u32(segs, ns, (dmax_tiles_ + kScanTile - 1) / kScanTile, d_tile_.as<uint32_t>(), d_tile_.as<uint32_t>(),
              d_tsum_.as<uint32_t>(), us_len, false, s_));
  CK(dec_unstuff_write(sg, ns, dmax_tiles_, d_in_.as<uint8_t>(), d_tile_.as<uint32_t>(), us_len,
                       d_us_.as<uint8_t>(), s_));
  CK(stage_event(1));
  // 2. synchronise the subsequence entry states: speculative (one pass, one flag read), with
  // the pass-based sync as the fallback when a link did not rejoin (VF_JPEG_SYNC=pass forces it)
  // VF_JPEG_SYNC = spec | pass | auto (default).  auto: speculative for frames of up to
  // kSpecAutoSubs subsequences (measured, MI355X, q85 4:2:2 batches of 32: 480p 50.4k vs 37.6k
  // fps, 1080p 18.0k vs 17.2k; 4K 5.48k vs 5.65k, where the bpm-fold trajectory decode costs
  // more than the pass chains it removes).
  const int mode = [] {  // read per call: tests switch it inside one process
    const char *v = std::getenv("VF_JPEG_SYNC");
    if (v && std::strcmp(v, "pass") == 0) return 1;
    if (v && std::strcmp(v, "spec") == 0) return 2;
    return 0;
  }();
  // the LSB-first lanes (SpanLaneRT) when every frame's block cycle divides 16 (k_spec's
  // 2-bit component slots; k_syncg's 1-bit table slots need it to divide 32); VF_JPEG_SYNC_LSB=0: off
  const bool lsb = pow2bpm_ && [] {  // read per call: tests switch it inside one process
    const char *v = std::getenv("VF_JPEG_SYNC_LSB");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  constexpr uint32_t kSpecAutoSubs = 12288;
  const bool use_spec = spec_ok_ && (mode == 2 || (mode == 0 && dmax_sub_ <= kSpecAutoSubs));
  int pass = 0, last = 0;
  uint32_t flag = 1;
  if (use_spec) {
    SpecBufs sb{d_tE_.as<uint64_t>(),  d_tX_.as<uint64_t>(), d_tXc_.as<uint32_t>(),
                d_pX_.as<uint64_t>(),  d_pC_.as<uint32_t>(), d_wF_.as<uint8_t>(),  d_rE_.as<uint8_t>(),
                d_rK_.as<uint32_t>(),  d_qX_.as<uint64_t>(), d_qC_.as<uint32_t>(), d_rL_.as<uint8_t>(),
                d_unres_.as<uint32_t>()};
    // k_resolve reports a frame unresolved only when it has more workgroups than it stages,
    // which prepare_decode already excludes (spec_ok_), so the rest is queued without a host
    // round trip; check_decode reads the flags after its synchronisation and turns one into an
    // error.  Each segment's k_resolve workgroup stores its flag (0 or 1) straight into the
    // codec's page-locked h_unres_ through the mapping: no fill and no download on the stream.
    const bool stats = std::getenv("VF_JPEG_SYNC_STATS") != nullptr;
    if (stats) CK(hipMemsetAsync(d_unres_.p, 0, sizeof(uint32_t) * 16, s_));  // SpecBufs::stats
    CK(dec_sync_spec(sg, fr, ns, dmax_wg_, d_us_.as<uint8_t>(), us_len, sb, d_exit_[0].as<uint64_t>(),
                     d_cnt_[0].as<uint32_t>(), static_cast<uint32_t *>(unres_dev_), lsb ? 1 : 0, s_));
    spec_check_ = true;
    flag = 0;  // exits / counts are in slot 0
    ++spec_calls_;
    if (stats) {
      uint32_t st[16];
      CK(hipStreamSynchronize(s_));  // the codec's stream is non-blocking: the copy below would not wait
      CK(hipMemcpy(st, d_unres_.p, sizeof st, hipMemcpyDeviceToHost));
      st[0] = 0;
      for (int i = 0; i < ns; ++i) st[0] += h_unres_.as<uint32_t>()[i];
      // VF_SPEC_PHASES builds only: [8] [9] [10] wall-clock ticks / 1024 summed over workgroups from
      // after the table load to the end of part A, of part B, and (per walker) of the serial
      // continuations; [1] walkers, [2] their explicit rows, [3] rows they wrote
      std::fprintf(stderr, "[vf_jpeg] k_spec phases (VF_SPEC_PHASES, 1024 wall ticks summed): part A %u, part B %u, "
                   "walkers end %u; walkers %u explicit rows %u rows written %u (workgroups %u)\n", st[8], st[9], st[10],
                   st[1], st[2], st[3], dmax_wg_ * (uint32_t)ns);
      std::fprintf(stderr, "[vf_jpeg] spec: unresolved %u; walk columns ended explicit %u, their traces joined in one "
                   "subsequence %u, serial traces %u (segments %d)\n", st[0], st[11], st[12], st[13], ns);
    }
  }
  // pass-based: spans of G subsequences per thread (VF_JPEG_SYNC_G = 1, 2, 4, 8; 0 = the
  // host-looped one-subsequence k_sync), kQueuedPasses passes queued without a host round trip
  // (a pass after convergence returns at once); the last pass's flag is read at check_decode
  // With every frame on 4 table slots (DecFrame::tabs4; VF_JPEG_SYNC_TABS4=0 turns it off) the
  // span sync's LDS leaves room for G = 5 at 3 workgroups per CU: 25 % more stream resident.
  const bool t4 = tabs4_ && [] {
    const char *v = std::getenv("VF_JPEG_SYNC_TABS4");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  const int sync_g = [t4] {  // read per call: tests switch it inside one process
    const char *v = std::getenv("VF_JPEG_SYNC_G");
    const int g = v ? std::atoi(v) : t4 ? 5 : 4;
    if (g == 5) return t4 ? 5 : 4;
    return g >= 0 && g <= 4 ? g : g == 8 ? 8 : 4;
  }();

  const int g_t4 = t4 && (sync_g == 4 || sync_g == 5) ? (lsb ? 2 : 1) : 0;
  if (flag && sync_g > 0) {
    // VF_JPEG_SYNC_QUEUED = 1..kQueuedPasses (tests): fewer queued passes, so check_decode
    // reports them unconverged and finish_sync runs the rest
    const char *qv = std::getenv("VF_JPEG_SYNC_QUEUED");
    queued_ = qv ? std::min(std::max(std::atoi(qv), 1), kQueuedPasses) : kQueuedPasses;
    CK(hipMemsetAsync(d_changed_.p, 0, sizeof(uint32_t) * kMaxPasses, s_));
    for (int p = 0; p < queued_; ++p)
      CK(dec_syncg(sync_g, sg, fr, ns, dmax_sub_, d_us_.as<uint8_t>(), us_len, d_exit_[0].as<uint64_t>(),
                   d_cnt_[0].as<uint32_t>(), d_used_.as<uint64_t>(), d_ck_.as<uint64_t>(), d_ckrem_.as<uint32_t>(),
                   d_changed_.as<uint32_t>(), p, sync_warm(), g_t4, s_));
    CK(h_flag_.ensure(64));
    CK(hipMemcpyAsync(h_flag_.p, d_changed_.as<uint32_t>() + queued_ - 1, sizeof(uint32_t),
                      hipMemcpyDeviceToHost, s_));
    pass_check_ = true;
    flag = 0;
    last = 0;
    pass = queued_;
  }
  if (flag) CK(hipMemsetAsync(d_changed_.p, 0, sizeof(uint32_t) * kMaxPasses, s_));
  for (; flag;) {
    const int a = pass & 1;
    CK(dec_sync(sg, fr, ns, dmax_sub_, d_us_.as<uint8_t>(), us_len, d_exit_[a ^ 1].as<uint64_t>(),
                d_exit_[a].as<uint64_t>(), d_cnt_[a ^ 1].as<uint32_t>(), d_cnt_[a].as<uint32_t>(),
                d_used_.as<uint64_t>(), d_ck_.as<uint64_t>(), d_ckrem_.as<uint32_t>(),
                d_changed_.as<uint32_t>() + (pass % kMaxPasses), pass > 0 ? 1 : 0, s_));
    last = a;
    ++pass;
    if (pass < 2) continue;  // passes 0 and 1 are queued without a host round trip
    CK(hipMemcpyAsync(&flag, d_changed_.as<uint32_t>() + ((pass - 1) % kMaxPasses), sizeof flag,
                      hipMemcpyDeviceToHost, s_));
    CK(hipStreamSynchronize(s_));
    if (!flag) break;
    CK(hipMemsetAsync(d_changed_.as<uint32_t>() + (pass % kMaxPasses), 0, sizeof(uint32_t), s_));
    if (pass > (int)dmax_sub_ + 2) {
      *err = "Huffman synchronisation did not converge (corrupt stream?)";
      return kJpeg;
    }
  }
  sync_passes_ = pass;
  if (std::getenv("VF_JPEG_SYNC_STATS")) {
    uint32_t st[4];
    CK(hipMemcpy(st, d_changed_.as<uint32_t>() + kMaxPasses - 4, sizeof st, hipMemcpyDeviceToHost));
    std::fprintf(stderr,
                 "[vf_jpeg] sync: spec calls %llu fallbacks %llu; passes %d; rounds pass0 max %u sum %u, pass1 max %u "
                 "sum %u (WGs %u)\n",
                 (unsigned long long)spec_calls_, (unsigned long long)spec_fallbacks_, pass, st[3], st[1], st[2], st[0],
                 (dmax_sub_ + 255) / 256 * (uint32_t)ns);
  }
  CK(stage_event(2));
  sync_spec_ = use_spec;
  sync_last_ = last;
  sync_g_ = sync_g;
  sync_t4_ = g_t4;
  return run_decode_post(bgr, invert, err);
}

// The queued span passes left a workgroup's last exit changing (a stream that takes more than
// kQueuedPasses - 1 workgroups of 1024 subsequences to resynchronise: corrupt or adversarial
// data in practice): more passes, each followed by a flag read, until none changes.  The caller
// then queues the stages after the sync again.
int Codec::finish_sync(std::string *err) {
  const DecFrame *fr = d_dfr_.as<DecFrame>();
  const DecSeg *sg = d_dsg_.as<DecSeg>();
  const uint32_t *us_len = d_totals_.as<uint32_t>();
  for (int p = queued_;; ++p) {
    if (p >= kMaxPasses) {
      *err = "Huffman synchronisation did not converge (corrupt stream?)";
      return kJpeg;
    }
    CK(dec_syncg(sync_g_, sg, fr, dnseg_, dmax_sub_, d_us_.as<uint8_t>(), us_len, d_exit_[0].as<uint64_t>(),
                 d_cnt_[0].as<uint32_t>(), d_used_.as<uint64_t>(), d_ck_.as<uint64_t>(), d_ckrem_.as<uint32_t>(),
                 d_changed_.as<uint32_t>(), p, sync_warm(), sync_t4_, s_));
    uint32_t flag = 0;
    CK(hipMemcpyAsync(&flag, d_changed_.as<uint32_t>() + p, sizeof flag, hipMemcpyDeviceToHost, s_));
    CK(hipStreamSynchronize(s_));
    if (!flag) break;
  }
  return kOk;
}

// Decode stages after the sync: block offsets, write pass, DC prediction, IDCT, colour.
int Codec::run_decode_post(int bgr, bool invert, std::string *err) {
  const DecFrame *fr = d_dfr_.as<DecFrame>();
  const DecSeg *sg = d_dsg_.as<DecSeg>();
  const ScanSeg *segs = d_segs_.as<ScanSeg>();
  const int n = dn_, ns = dnseg_;
  const uint32_t *us_len = d_totals_.as<uint32_t>();
  const bool use_spec = sync_spec_;
  const int last = sync_last_;
  // 3. block offsets of the subsequences, then the write pass
  // the segments' decoded block counts go straight to the page-locked h_dtot_ (check_decode)
  uint32_t *blocks_total = static_cast<uint32_t *>(dtot_dev_);
  CK(scan_u32(segs + ns, ns, (dmax_sub_ + kScanTile - 1) / kScanTile, d_cnt_[last].as<uint32_t>(),
              d_bstart_.as<uint32_t>(), d_tsum_.as<uint32_t>(), blocks_total, false, s_));
  // The write pass stores whole 16-B coefficient rows with a per-block mask of the rows stored,
  // which the IDCT reads: no clear of the coefficient buffer (134 MB per 1080p batch, 1.06 GB
  // per 4K one).  After the speculative sync always (k_write + clear 118 -> 105 us at 1080p).
  // After the pass-based sync only when blocks are short: its write pass runs 4 lanes per
  // subsequence, each of which decodes on to its last block's end and skips its first, which
  // costs a block per lane -- on hard content (~500 bits per block) k_write4 342 -> 1227 us,
  // on 4K scenes (~22 bits per block) huffman_write 0.50 -> 0.29 ms, resident 11.1 -> 12.0 k fps
  // (profiles/r04_jpeg_fuse_chunks_warm_ab.txt, r04_jpeg_chunks_4k_ab.txt).  VF_JPEG_CHUNKS=0 / 1
  // forces either form.
  constexpr uint64_t kChunkBitsPerBlock = 128;
  const bool chunks = [use_spec, this] {  // read per call: tests switch it inside one process
    const char *v = std::getenv("VF_JPEG_CHUNKS");
    return v && *v ? std::strcmp(v, "0") != 0 : use_spec || dbits_per_block_ <= kChunkBitsPerBlock;
  }();
  uint8_t *const nmask = chunks ? d_nmask_.as<uint8_t>() : nullptr;
  if (!chunks) CK(hipMemsetAsync(d_coef_.p, 0, dblocks_ * 128, s_));
  // after the pass-based sync, every subsequence's checkpoints are states of the true path: the
  // write pass runs 4 lanes per subsequence from them (VF_JPEG_WRITE4=0: one lane)
  const bool write4 = [] {  // read per call: tests switch it inside one process
    const char *v = std::getenv("VF_JPEG_WRITE4");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  if (!use_spec && write4)
    CK(dec_write4(sg, fr, ns, dmax_sub_, d_us_.as<uint8_t>(), us_len, d_exit_[last].as<uint64_t>(),
                  d_cnt_[last].as<uint32_t>(), d_ck_.as<uint64_t>(), d_ckrem_.as<uint32_t>(),
                  d_bstart_.as<uint32_t>(), d_coef_.as<int16_t>(), d_dcseq_.as<int32_t>(), nmask, s_));
  else
    CK(dec_write(sg, fr, ns, dmax_sub_, d_us_.as<uint8_t>(), us_len, d_exit_[last].as<uint64_t>(),
                 d_bstart_.as<uint32_t>(), d_coef_.as<int16_t>(), d_dcseq_.as<int32_t>(), nmask, s_));
  CK(stage_event(3));
  // 4. DC prediction (inclusive scan per component sequence)
  CK(scan_i32(segs + 2 * ns, ndcseg_, dc_max_tiles_, d_dcseq_.as<int32_t>(), d_dcpred_.as<int32_t>(),
              d_tsum_.as<int32_t>(), nullptr, true, s_));
  // 5. IDCT, 6. upsample + colour (+ invert).  The invert path on standard 4:2:2 frames does both
  // in one pass with the decoder planes in LDS (k_idct_color422; VF_JPEG_FUSE_IDCT=0: two passes)
  const bool fuse_idct = fuse_ && d422_ && [] {  // read per call: tests switch it inside one process
    const char *v = std::getenv("VF_JPEG_FUSE_IDCT");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  if (fuse_idct) {
    CK(stage_event(4));  // the DC scan above is the dc_idct stage; the fused pass the colour stage
    CK(dec_idct_color422(fr, n, dmax_w_, dmax_h_, d_coef_.as<int16_t>(), d_dcpred_.as<int32_t>(), nmask,
                         d_eplanes_.as<uint8_t>(), d_efr_.as<EncFrame>(), invert ? 1 : 0, kSampV[esub_] == 1 ? 1 : 0,
                         s_));
    CK(stage_event(5));
    return kOk;
  }
  CK(dec_idct(fr, n, dmax_blocks_, d_coef_.as<int16_t>(), d_dcpred_.as<int32_t>(), nmask, d_planes_.as<uint8_t>(), s_));
  CK(stage_event(4));
  // the invert path (fuse_): the encoder's sample planes instead of pixels (enc_sample_rows)
  CK(dec_color(fr, n, dmax_w_, dmax_h_, d_planes_.as<uint8_t>(), fuse_ ? d_eplanes_.as<uint8_t>() : d_pix_.as<uint8_t>(),
               bgr, invert ? 1 : 0, fuse_ ? d_efr_.as<EncFrame>() : nullptr, dcm_, s_));
  CK(stage_event(5));
  return kOk;
}

// Check that every frame decoded all its blocks (after a synchronisation: run_decode_post's
// block-offset scan stores each segment's count into h_dtot_ through the mapping).
int Codec::check_decode(std::string *err) {
  const uint32_t *tot = h_dtot_.as<uint32_t>();
  if (pass_check_) {
    pass_check_ = false;
    if (*h_flag_.as<uint32_t>()) return kResync;  // the caller runs finish_sync and its stages again
  }
  if (spec_check_) {
    spec_check_ = false;
    bool unresolved = false;
    for (int i = 0; i < dnseg_; ++i) unresolved = unresolved || h_unres_.as<uint32_t>()[i] != 0;
    if (unresolved) {
      ++spec_fallbacks_;
      *err = "speculative Huffman synchronisation left a frame unresolved";
      return kJpeg;
    }
  }
  for (int i = 0; i < dnseg_; ++i) {
    const DecSeg &S = dsg_[(size_t)i];
    if (tot[(size_t)i] < S.nblocks) {
      const bool whole = S.nblocks == (uint32_t)dfr_[S.frame].g.nblocks;
      *err = "frame " + std::to_string(S.frame) + (whole ? std::string() : " (restart interval at block " +
             std::to_string(S.blk0 - dfr_[S.frame].blk0) + ")") + ": entropy-coded data ends after " +
             std::to_string(tot[(size_t)i]) + " of " + std::to_string(S.nblocks) + " blocks (truncated or corrupt JPEG)";
      return kJpeg;
    }
  }
  return kOk;
}

// Layout + tables + headers for encoding n frames whose pixels sit in d_pix_ at img_offs.
int Codec::prepare_encode(const int *ws, const int *hs, const uint64_t *img_offs, int n, int quality, int subsamp,
                          bool fastdct, std::string *err) {
  if (subsamp < 0 || subsamp > 4) {
    *err = "unsupported subsampling (TJSAMP_444, 422, 420, GRAY, 440)";
    return kInvalid;
  }
  fuse_ = false;  // the invert paths turn it on after both prepares
  // Everything below depends only on the frames' sizes and layout and the settings: a batch shaped
  // like this codec's previous one (a worker's steady state) reuses its descriptors, tables,
  // headers and buffers, already on the device (nothing else writes them).
  {
    std::vector<uint64_t> key;
    key.reserve(3 * (size_t)n + 4);
    key.push_back((uint64_t)n);
    key.push_back((uint64_t)quality);
    key.push_back((uint64_t)subsamp);
    key.push_back(fastdct ? 1u : 0u);
    for (int f = 0; f < n; ++f) {
      key.push_back((uint64_t)(uint32_t)ws[f] << 32 | (uint32_t)hs[f]);
      key.push_back(img_offs[f]);
    }
    if (ekey_valid_ && key == ekey_) {
      ++enc_prep_reused_;
      return kOk;
    }
    ekey_valid_ = false;  // until this prepare completes
    ekey_.swap(key);
  }
  efr_.assign((size_t)n, EncFrame());
  std::vector<uint8_t> hdr;
  uint64_t blk = 0, bits = 0, out = 0, epl = 0;
  uint32_t tiles = 0;
  emax_blocks_ = emax_tiles_ = 0;
  const int nc = subsamp == 3 ? 1 : 3;
  const int hsamp[3] = {kSampH[subsamp], 1, 1}, vsamp[3] = {kSampV[subsamp], 1, 1};
  for (int f = 0; f < n; ++f) {
    EncFrame &F = efr_[(size_t)f];
    if (!make_geom(ws[f], hs[f], nc, hsamp, vsamp, &F.g)) {
      *err = "frame " + std::to_string(f) + ": bad image size";
      return kInvalid;
    }
    F.img_off = img_offs[f];
    for (int k = 0; k < 3; ++k) {  // the invert path's sample planes: wb * 8 x rrows each
      F.eplane_off[k] = epl;
      if (k < nc) epl += align_up((size_t)F.g.wb[k] * 8 * (size_t)F.g.rrows[k], 256);
    }
    F.blk0 = blk;
    F.bits_off = bits;
    const uint64_t bits_cap = align_up((size_t)F.g.nblocks * kMaxBlockBytes + 16, 256);
    F.out_off = out;
    F.hdr_off = (uint32_t)hdr.size();
    uint8_t h[1024];
    F.hdr_len = (uint32_t)write_header(ws[f], hs[f], quality, subsamp, h);
    hdr.insert(hdr.end(), h, h + F.hdr_len);
    F.tile0 = tiles;
    F.ntiles_max = (uint32_t)((bits_cap + kTile - 1) / kTile);
    blk += (uint64_t)F.g.nblocks;
    bits += bits_cap;
    out += align_up(F.hdr_len + 2 * bits_cap + 2, 256);
    tiles += F.ntiles_max;
    emax_blocks_ = std::max(emax_blocks_, (uint32_t)F.g.nblocks);
    emax_tiles_ = std::max(emax_tiles_, F.ntiles_max);
  }
  en_ = n;
  esub_ = subsamp;
  eblocks_ = blk;
  ebits_bytes_ = bits;
  std::vector<ScanSeg> segs;
  uint32_t t0 = 0;
  auto add = [&](uint64_t base, uint32_t len) {
    segs.push_back(ScanSeg{base, len, t0});
    t0 += (len + kScanTile - 1) / kScanTile;
  };
  for (auto &F : efr_) add(F.blk0, (uint32_t)F.g.nblocks);
  for (auto &F : efr_) add(F.tile0, F.ntiles_max);
  EncTables tab;
  build_enc_tables(quality, fastdct, &tab);
  CK(hipSetDevice(device_));
  CK(d_efr_.ensure(sizeof(EncFrame) * (size_t)n));
  CK(d_etab_.ensure(sizeof(EncTables)));
  CK(d_hdr_.ensure(hdr.size()));
  CK(d_esegs_.ensure(sizeof(ScanSeg) * segs.size()));
  CK(d_etsum_.ensure(sizeof(uint32_t) * (t0 + 1)));
  CK(d_etotals_.ensure(sizeof(uint32_t) * segs.size()));
  CK(d_dcq_.ensure(sizeof(int16_t) * blk));
  CK(d_acbits_.ensure(sizeof(uint32_t) * blk));
  CK(d_acscr_.ensure(sizeof(uint32_t) * kAcScratchWords * ((blk + 63) & ~(size_t)63)));  // whole 64-block groups
  CK(d_bits_.ensure(sizeof(uint32_t) * blk));
  CK(d_pre_.ensure(sizeof(uint32_t) * blk));
  CK(d_bitoff_.ensure(sizeof(uint32_t) * blk));
  CK(d_stream_.ensure(bits));
  CK(d_ffcnt_.ensure(sizeof(uint32_t) * tiles));
  CK(d_pack_.ensure(out));
  CK(d_outsize_.ensure(sizeof(uint64_t) * (size_t)n));
  CK(d_eplanes_.ensure(epl));
  // frame descriptors, tables, headers and scan segments: one pinned blob, asynchronous uploads
  const size_t fsz = sizeof(EncFrame) * (size_t)n, ssz = sizeof(ScanSeg) * segs.size();
  const size_t o_tab = align_up(fsz, 256), o_hdr = o_tab + align_up(sizeof tab, 256),
               o_seg = o_hdr + align_up(hdr.size(), 256);
  CK(h_edesc_.ensure(o_seg + ssz));
  uint8_t *hb = h_edesc_.as<uint8_t>();
  std::memcpy(hb, efr_.data(), fsz);
  std::memcpy(hb + o_tab, &tab, sizeof tab);
  std::memcpy(hb + o_hdr, hdr.data(), hdr.size());
  std::memcpy(hb + o_seg, segs.data(), ssz);
  CK(hipMemcpyAsync(d_efr_.p, hb, fsz, hipMemcpyHostToDevice, s_));
  CK(hipMemcpyAsync(d_etab_.p, hb + o_tab, sizeof tab, hipMemcpyHostToDevice, s_));
  CK(hipMemcpyAsync(d_hdr_.p, hb + o_hdr, hdr.size(), hipMemcpyHostToDevice, s_));
  CK(hipMemcpyAsync(d_esegs_.p, hb + o_seg, ssz, hipMemcpyHostToDevice, s_));
  ekey_valid_ = true;
  return kOk;
}

int Codec::run_encode(int bgr, bool fastdct, std::string *err) {
  const EncFrame *fr = d_efr_.as<EncFrame>();
  const EncTables *tab = d_etab_.as<EncTables>();
  const ScanSeg *segs = d_esegs_.as<ScanSeg>();
  const int n = en_;
  CK(stage_event(6));
  CK(enc_fdct(fr, n, emax_blocks_, tab, fuse_ ? d_eplanes_.as<uint8_t>() : d_pix_.as<uint8_t>(), d_dcq_.as<int16_t>(),
              d_acbits_.as<uint32_t>(), d_acscr_.as<uint32_t>(), bgr, fastdct ? 1 : 0, kSampH[esub_], kSampV[esub_],
              fuse_ ? 1 : 0, s_));
  CK(enc_len(fr, n, emax_blocks_, tab, d_dcq_.as<int16_t>(), d_acbits_.as<uint32_t>(), d_bits_.as<uint32_t>(),
             d_pre_.as<uint32_t>(), s_));
  uint32_t *total_bits = d_etotals_.as<uint32_t>();
  CK(scan_u32(segs, n, (emax_blocks_ + kScanTile - 1) / kScanTile, d_bits_.as<uint32_t>(), d_bitoff_.as<uint32_t>(),
              d_etsum_.as<uint32_t>(), total_bits, false, s_));
  CK(enc_pack(fr, n, emax_blocks_, d_pre_.as<uint32_t>(), d_acbits_.as<uint32_t>(), d_acscr_.as<uint32_t>(),
              d_bitoff_.as<uint32_t>(), total_bits, d_stream_.as<uint8_t>(), s_));
  CK(stage_event(7));
  CK(enc_ff_count(fr, n, emax_tiles_, total_bits, d_stream_.as<uint8_t>(), d_ffcnt_.as<uint32_t>(), s_));
  uint32_t *nff = d_etotals_.as<uint32_t>() + n;
  CK(scan_u32(segs + n, n, (emax_tiles_ + kScanTile - 1) / kScanTile, d_ffcnt_.as<uint32_t>(),
              d_ffcnt_.as<uint32_t>(), d_etsum_.as<uint32_t>(), nff, false, s_));
  CK(enc_ff_write(fr, n, emax_tiles_, total_bits, d_stream_.as<uint8_t>(), d_ffcnt_.as<uint32_t>(), nff,
                  d_hdr_.as<uint8_t>(), d_pack_.as<uint8_t>(), d_outsize_.as<uint64_t>(), s_));  // packed in place
  CK(stage_event(8));
  return kOk;
}

// Queue, behind the encode kernels: the D2H of every output size, and of the first `guess`
// bytes of the packed outputs (k_compact's layout: frames 64-B aligned, back to back), guessed
// from the inputs' sizes, so the common case needs no second round trip; then the done event.
int Codec::queue_fetch(uint64_t guess, std::string *err) {
  const int n = en_;
  CK(h_meta_.ensure(sizeof(uint64_t) * (size_t)n * 2 + 64));
  uint64_t *sz = h_meta_.as<uint64_t>() + n;  // the sizes (h_dtot_ holds the decode's block totals)
  CK(hipMemcpyAsync(sz, d_outsize_.p, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost, s_));
  guess = std::min<uint64_t>(guess, d_pack_.cap);
  CK(h_out_.ensure(guess));
  guess_ = guess;
  if (guess) CK(hipMemcpyAsync(h_out_.p, d_pack_.p, guess, hipMemcpyDeviceToHost, s_));
  CK(hipEventRecord(done_, s_));
  return kOk;
}

// After done_: the packed layout (sizes, offsets, total) and, when the guess fell short, the
// rest of the outputs (one more round trip).
int Codec::finish_fetch(std::string *err) {
  const int n = en_;
  const uint64_t *sz = h_meta_.as<uint64_t>() + n;
  out_sizes_.resize((size_t)n);
  out_offs_.resize((size_t)n);
  uint64_t total = 0;
  for (int f = 0; f < n; ++f) {
    out_sizes_[(size_t)f] = sz[f];
    out_offs_[(size_t)f] = total;
    total += align_up(sz[f], 64);
  }
  out_total_ = total;
  if (total > guess_) {
    ++fetch_refills_;
    if (total > h_out_.cap) {  // grow, keeping what already arrived
      HostBuf bigger;
      CK(bigger.ensure(total));
      std::memcpy(bigger.p, h_out_.p, guess_);
      std::swap(bigger.p, h_out_.p);
      std::swap(bigger.cap, h_out_.cap);
    }
    CK(hipMemcpyAsync(h_out_.as<uint8_t>() + guess_, d_pack_.as<uint8_t>() + guess_, total - guess_,
                      hipMemcpyDeviceToHost, s_));
    CK(hipStreamSynchronize(s_));
  }
  return kOk;
}

// ---- public operations ---------------------------------------------------------------------------

int Codec::encode(const uint8_t *const *imgs, const int *ws, const int *hs, int n, int pixel_format, int quality,
                  int subsamp, int flags, uint8_t *const *outs, const size_t *caps, size_t *sizes, std::string *err) {
  int rc = init(err);
  if (rc) return rc;
  if (n <= 0) return kOk;
  if (pixel_format != 0 && pixel_format != 1) {
    *err = "pixel_format must be TJPF_RGB (0) or TJPF_BGR (1)";
    return kInvalid;
  }
  std::vector<uint64_t> offs((size_t)n);
  uint64_t pix = 0;
  for (int f = 0; f < n; ++f) {
    if (!imgs[f] || ws[f] <= 0 || hs[f] <= 0 || ws[f] > 65535 || hs[f] > 65535) {
      *err = "frame " + std::to_string(f) + ": bad image";
      return kInvalid;
    }
    offs[(size_t)f] = pix;
    pix += align_up((size_t)ws[f] * hs[f] * 3, 256);
  }
  const bool fast = (flags & kFlagFastDct) != 0;
  if ((rc = prepare_encode(ws, hs, offs.data(), n, quality, subsamp, fast, err))) return rc;
  CK(h_stage_.ensure(pix));
  CK(d_pix_.ensure(pix));
  pool_.run(n, [&](int f) {
    std::memcpy(h_stage_.as<uint8_t>() + offs[(size_t)f], imgs[f], (size_t)ws[f] * hs[f] * 3);
  });
  CK(hipMemcpyAsync(d_pix_.p, h_stage_.p, pix, hipMemcpyHostToDevice, s_));
  if ((rc = run_encode(pixel_format, fast, err))) return rc;
  uint64_t guess = 0;
  for (int f = 0; f < n; ++f) guess += align_up((size_t)ws[f] * hs[f] / 4 + 8192, 64);
  if ((rc = queue_fetch(guess, err))) return rc;
  CK(hipEventSynchronize(done_));
  if ((rc = finish_fetch(err))) return rc;
  return copy_out(outs, caps, sizes, err);
}

// Per-frame copies of the fetched packed outputs into the caller's buffers (caps checked).
int Codec::copy_out(uint8_t *const *outs, const size_t *caps, size_t *sizes, std::string *err) {
  const int n = en_;
  for (int f = 0; f < n; ++f) {
    sizes[f] = (size_t)out_sizes_[(size_t)f];
    if (out_sizes_[(size_t)f] > caps[f] || !outs[f]) {
      *err = "frame " + std::to_string(f) + ": output buffer of " + std::to_string(caps[f]) +
             " bytes is too small for the " + std::to_string(out_sizes_[(size_t)f]) + "-byte JPEG";
      return kInvalid;
    }
  }
  pool_.run(n, [&](int f) {
    std::memcpy(outs[f], h_out_.as<uint8_t>() + out_offs_[(size_t)f], out_sizes_[(size_t)f]);
  });
  return kOk;
}

int Codec::decode(const uint8_t *const *jpegs, const size_t *jsizes, int n, int pixel_format, int flags,
                  uint8_t *const *outs, const size_t *caps, std::string *err) {
  int rc = init(err);
  if (rc) return rc;
  if (n <= 0) return kOk;
  if (pixel_format != 0 && pixel_format != 1) {
    *err = "pixel_format must be TJPF_RGB (0) or TJPF_BGR (1)";
    return kInvalid;
  }
  if ((rc = prepare_decode(jpegs, jsizes, n, flags, err))) return rc;
  for (int f = 0; f < n; ++f) {
    const size_t need = (size_t)dfr_[(size_t)f].g.w * dfr_[(size_t)f].g.h * 3;
    if (!outs[f] || caps[f] < need) {
      *err = "frame " + std::to_string(f) + ": output buffer smaller than " + std::to_string(need) + " bytes";
      return kInvalid;
    }
  }
  if ((rc = run_decode(pixel_format, false, err))) return rc;
  for (bool again = false;; again = true) {
    if (again && ((rc = finish_sync(err)) || (rc = run_decode_post(pixel_format, false, err)))) return rc;
    CK(h_out_.ensure(dpix_bytes_));
    CK(hipMemcpyAsync(h_out_.p, d_pix_.p, dpix_bytes_, hipMemcpyDeviceToHost, s_));
    CK(hipStreamSynchronize(s_));
    rc = check_decode(err);
    if (rc != kResync) break;
  }
  if (rc) return rc;
  pool_.run(n, [&](int f) {
    std::memcpy(outs[f], h_out_.as<uint8_t>() + dfr_[(size_t)f].out_off,
                (size_t)dfr_[(size_t)f].g.w * dfr_[(size_t)f].g.h * 3);
  });
  return kOk;
}

// The fused default-mode filter, split so one host thread can keep two batches in flight:
// submit_invert (parse, stage, queue every upload, kernel and download; returns without
// waiting for the GPU), wait_invert (the done event, the decode checks, the packed layout),
// fetch_invert (copy-out).  invert() is the three in a row.
int Codec::submit_invert(const uint8_t *const *jpegs, const size_t *jsizes, int n, int quality, int subsamp,
                         int flags, std::string *err) {
  int rc = init(err);
  if (rc) return rc;
  waited_ = false;
  if (n <= 0) {
    *err = "empty batch";
    return kInvalid;
  }
  static const bool trace = std::getenv("VF_JPEG_TRACE") != nullptr;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  if ((rc = prepare_decode(jpegs, jsizes, n, flags, err))) return rc;
  const auto t1 = clk::now();
  std::vector<int> ws((size_t)n), hs((size_t)n);
  std::vector<uint64_t> offs((size_t)n);
  // the first D2H copy's size: an inverted frame re-encoded at the input's quality codes to about
  // the input's size (+25 % + 8 KB per frame, the rule before any batch); after the codec's first
  // batch, its measured output/input ratio + 6 % + 1 KB per frame (q95 input re-encoded at q85
  // halves: the fixed rule then copied 2.4x the output).  Short guesses take finish_fetch's
  // second copy.
  static const bool learn = [] {
    const char *v = std::getenv("VF_JPEG_FETCH_LEARN");
    return !(v && v[0] == '0');
  }();
  const double ratio = learn ? out_ratio_ : 0.0;
  uint64_t guess = 0;
  in_bytes_ = 0;
  for (int f = 0; f < n; ++f) {
    ws[(size_t)f] = dfr_[(size_t)f].g.w;
    hs[(size_t)f] = dfr_[(size_t)f].g.h;
    offs[(size_t)f] = dfr_[(size_t)f].out_off;
    in_bytes_ += jsizes[f];
    guess += ratio > 0 ? align_up((uint64_t)((double)jsizes[f] * ratio * 1.06) + 1024, 64)
                       : align_up(jsizes[f] + jsizes[f] / 4 + 8192, 64);
  }
  const bool fast = (flags & kFlagFastDct) != 0;
  if ((rc = prepare_encode(ws.data(), hs.data(), offs.data(), n, quality, subsamp, fast, err))) return rc;
  fuse_ = fuse_enabled();
  const auto t2 = clk::now();
  {
    std::unique_lock<std::mutex> gl;
    if (gate_) {
      gl = std::unique_lock<std::mutex>(gate_->mu);
      if (gate_->last) CK(hipStreamWaitEvent(s_, gate_->last, 0));
    }
    // decode (BGR, inverted: cv2.bitwise_not, inverter.py:41) straight into the encoder's input
    enc_fast_ = fast;
    if ((rc = run_decode(1, true, err))) return rc;
    if ((rc = run_encode(1, fast, err))) return rc;
    if (gate_) {
      CK(hipEventRecord(ev_[9], s_));
      gate_->last = ev_[9];
    }
  }
  if ((rc = queue_fetch(guess, err))) return rc;
  if (trace) {
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    static const clk::time_point origin = t0;
    std::fprintf(stderr, "[vf_jpeg] submit codec %p n=%d at %.3f: prep_dec %.3f (parse %.3f loop %.3f stage %.3f) "
                 "prep_enc %.3f queue %.3f ms\n", (void *)this, n, ms(origin, t0), ms(t0, t1), prep_ms_[0], prep_ms_[1],
                 prep_ms_[2], ms(t1, t2), ms(t2, clk::now()));
  }
  return kOk;
}

void Codec::quiesce() {
  if (!s_) return;
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(s_);
  (void)hipGetLastError();
}

bool Codec::done_invert() {
  const hipError_t q = hipEventQuery(done_);
  if (q == hipSuccess) return true;
  (void)hipGetLastError();
  return q != hipErrorNotReady;  // an error counts as done: wait_invert reports it
}

int Codec::wait_invert(size_t *total, std::string *err) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  CK(hipEventSynchronize(done_));
  int rc = check_decode(err);
  while (rc == kResync) {  // more sync passes, then every stage after the sync again
    if ((rc = finish_sync(err)) || (rc = run_decode_post(1, true, err)) || (rc = run_encode(1, enc_fast_, err)) ||
        (rc = queue_fetch(guess_, err)))
      return rc;
    CK(hipEventSynchronize(done_));
    rc = check_decode(err);
  }
  if (rc) return rc;
  if ((rc = finish_fetch(err))) return rc;
  if (in_bytes_) out_ratio_ = (double)out_total_ / (double)in_bytes_;
  waited_ = true;
  *total = (size_t)out_total_;
  if (std::getenv("VF_JPEG_TRACE"))
    std::fprintf(stderr, "[vf_jpeg] wait codec %p: %.3f ms, %llu B fetched (%s)\n", (void *)this,
                 std::chrono::duration<double, std::milli>(clk::now() - t0).count(),
                 (unsigned long long)out_total_, out_total_ > guess_ ? "second copy" : "one copy");
  return kOk;
}

int Codec::scatter_invert(uint8_t *const *outs, const size_t *caps, size_t *sizes, int *placed) {
  const int n = en_;
  int count = 0;
  for (int f = 0; f < n; ++f) {
    sizes[f] = (size_t)out_sizes_[(size_t)f];
    count += outs[f] && out_sizes_[(size_t)f] <= caps[f];
  }
  pool_.run(n, [&](int f) {
    if (outs[f] && out_sizes_[(size_t)f] <= caps[f])
      std::memcpy(outs[f], h_out_.as<uint8_t>() + out_offs_[(size_t)f], out_sizes_[(size_t)f]);
  });
  *placed = count;
  return kOk;
}

int Codec::fetch_invert(uint8_t *out, size_t cap, size_t *sizes, size_t *offs, std::string *err) {
  const int n = en_;
  if (out && cap < out_total_) {
    *err = "output buffer of " + std::to_string(cap) + " bytes is smaller than the " +
           std::to_string(out_total_) + " packed bytes";
    return kInvalid;
  }
  for (int f = 0; f < n; ++f) {
    if (sizes) sizes[f] = (size_t)out_sizes_[(size_t)f];
    if (offs) offs[f] = (size_t)out_offs_[(size_t)f];
  }
  if (out && out_total_) {  // one packed copy, split over the pool
    constexpr int kParts = 8;
    const uint64_t per = align_up((out_total_ + kParts - 1) / kParts, 4096);
    pool_.run(kParts, [&](int i) {
      const uint64_t b = std::min<uint64_t>(out_total_, per * (uint64_t)i);
      const uint64_t e = std::min<uint64_t>(out_total_, b + per);
      if (e > b) std::memcpy(out + b, h_out_.as<uint8_t>() + b, e - b);
    });
  }
  return kOk;
}

int Codec::invert(const uint8_t *const *jpegs, const size_t *jsizes, int n, int quality, int subsamp, int flags,
                  uint8_t *const *outs, const size_t *caps, size_t *sizes, std::string *err) {
  if (n <= 0) return init(err);
  int rc = submit_invert(jpegs, jsizes, n, quality, subsamp, flags, err);
  size_t total = 0;
  if (!rc) rc = wait_invert(&total, err);
  if (!rc) rc = copy_out(outs, caps, sizes, err);
  return rc;
}

int Codec::bench_invert(const uint8_t *const *jpegs, const size_t *jsizes, int n, int quality, int subsamp,
                        int flags, int iters, float *ms, float *stage_ms, std::string *err) {
  int rc = init(err);
  if (rc) return rc;
  if (n <= 0 || iters <= 0) {
    *err = "bench_invert: empty batch or iters <= 0";
    return kInvalid;
  }
  if ((rc = prepare_decode(jpegs, jsizes, n, flags, err))) return rc;
  std::vector<int> ws((size_t)n), hs((size_t)n);
  std::vector<uint64_t> offs((size_t)n);
  for (int f = 0; f < n; ++f) {
    ws[(size_t)f] = dfr_[(size_t)f].g.w;
    hs[(size_t)f] = dfr_[(size_t)f].g.h;
    offs[(size_t)f] = dfr_[(size_t)f].out_off;
  }
  const bool fast = (flags & kFlagFastDct) != 0;
  if ((rc = prepare_encode(ws.data(), hs.data(), offs.data(), n, quality, subsamp, fast, err))) return rc;
  fuse_ = fuse_enabled();
  float acc[8] = {0};
  double total_ms = 0;
  int passes = 0;
  // the timed iterations run as the product does (no stage events: each costs ~5 us of GPU
  // time between kernels, ~45 us per batch); then, for the stage breakdown, as many again with
  // the events recorded
  for (int pass = 0; pass < (stage_ms ? 2 : 1); ++pass) {
    stage_events_ = pass == 1;
    for (int it = 0; it < iters; ++it) {
      CK(hipStreamSynchronize(s_));
      const auto t0 = std::chrono::steady_clock::now();
      if ((rc = run_decode(1, true, err)) || (rc = run_encode(1, fast, err))) {
        stage_events_ = false;
        return rc;
      }
      CK(hipStreamSynchronize(s_));
      if (pass == 0) {
        total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        passes += sync_passes_;
        continue;
      }
      // stage times: unstuff, sync, write, dc+idct, colour, fdct+huff, stuff
      const int pairs[7][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {6, 7}, {7, 8}};
      for (int i = 0; i < 7; ++i) {
        float t = 0.f;
        if (hipEventElapsedTime(&t, ev_[pairs[i][0]], ev_[pairs[i][1]]) == hipSuccess) acc[i] += t;
      }
    }
  }
  stage_events_ = false;
  CK(hipStreamSynchronize(s_));
  rc = check_decode(err);
  while (rc == kResync) {
    if ((rc = finish_sync(err)) || (rc = run_decode_post(1, true, err)) || (rc = run_encode(1, fast, err)))
      return rc;
    CK(hipStreamSynchronize(s_));
    rc = check_decode(err);
  }
  if (rc) return rc;
  *ms = (float)(total_ms / iters);
  if (stage_ms) {
    for (int i = 0; i < 7; ++i) stage_ms[i] = acc[i] / iters;
    stage_ms[7] = (float)passes / iters;  // mean sync passes
  }
  return kOk;
}

int header_info(const uint8_t *jpeg, size_t size, int *w, int *h, int *subsamp, int *colorspace, std::string *err) {
  Parsed P;
  if (!jpeg || parse(jpeg, size, &P, err, false) != 0) {
    if (!jpeg) *err = "NULL JPEG buffer";
    return kJpeg;
  }
  *w = P.w;
  *h = P.h;
  *subsamp = subsamp_of(P);
  *colorspace = P.ncomp == 1 ? 2 : 1;  // TJCS_GRAY = 2, TJCS_YCbCr = 1
  return kOk;
}

size_t buffer_size(int w, int h, int subsamp) {
  if (w <= 0 || h <= 0 || subsamp < 0 || subsamp > 4) return 0;
  const int nc = subsamp == 3 ? 1 : 3;
  const int hsamp[3] = {kSampH[subsamp], 1, 1}, vsamp[3] = {kSampV[subsamp], 1, 1};
  Geom g;
  if (!make_geom(w, h, nc, hsamp, vsamp, &g)) return 0;
  return 1024 + 2 * (size_t)g.nblocks * kMaxBlockBytes + 2;
}

}  // namespace jpeg
}  // namespace vf
