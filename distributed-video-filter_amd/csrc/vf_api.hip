// vf_api.hip — C ABI of libvfilter_hip.so (declared in include/vfilter.h).
//
// Host side of the MI355X frame filter.  What it replaces in the reference:
//   * InverterWorker per-process state          inverter.py:10-20   -> vf_create / vf_destroy
//   * cv2.bitwise_not(frame) on one frame       inverter.py:41      -> vf_invert_host
//   * the one-frame-per-iteration worker loop   worker.py:35-57     -> vf_invert_batch_host,
//                                                                      vf_invert_frames_host
// Host->host calls run a slot pipeline: the byte stream (one range, a packed batch, or a
// gather list of frames) is cut into slot-sized chunks; chunk i uses slot i % S.  Two HIP
// streams carry the work: the IN stream runs H2D(i) -> kernel(i), the OUT stream waits on
// kernel(i)'s event and runs D2H(i).  Keeping the two directions on separate streams puts
// them on separate SDMA engines, so DMA in, the kernel and DMA out of different chunks all
// overlap (one stream per slot serialises both directions on one engine: measured 28 GB/s
// each way vs 46 GB/s with split streams, profiles/r01_pcie_probe.txt).
// Pageable caller memory is staged through pinned slot buffers by a small host copy pool;
// caller memory that is already page-locked (vf_alloc_host / vf_host_register, e.g. a
// shared-memory frame ring) is DMA'd directly with no host copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/vfilter.h"
#include "vf_internal.h"

#define VF_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kMaxSlots = 8;

struct ErrState {
  int hip = 0;
  char msg[512] = "no error";
};
thread_local ErrState g_thread_err;

// ---- host copy pool -------------------------------------------------------------------
// memcpy of large staging chunks split over a few persistent threads: one core moves
// ~10 GB/s, well under one PCIe Gen5 x16 direction, so a single-threaded stage would cap
// the end-to-end rate (1080p x 32 pageable: 30.5 GB/s each way with 4 threads, 40.5 with 8;
// pinned, i.e. no staging: 42.9).
class CopyPool {
 public:
  explicit CopyPool(int nthreads) : n_(std::max(1, nthreads)) {
    for (int i = 1; i < n_; ++i) threads_.emplace_back([this, i] { run(i); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto &t : threads_) t.join();
  }
  // Copies each (dst, src, len) job; big jobs are split across the pool.
  void copy(uint8_t *dst, const uint8_t *src, size_t len) {
    if (len < kSplitMin || n_ == 1) {
      std::memcpy(dst, src, len);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      dst_ = dst;
      src_ = src;
      len_ = len;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    do_part(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
  }

 private:
  static constexpr size_t kSplitMin = 1 << 20;
  void do_part(int i) {
    size_t per = (len_ / n_ + 63) & ~size_t(63);
    size_t b = std::min(len_, per * (size_t)i);
    size_t e = std::min(len_, b + per);
    if (i == n_ - 1) e = len_;
    if (e > b) std::memcpy(dst_ + b, src_ + b, e - b);
  }
  void run(int i) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      do_part(i);
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }
  int n_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  bool stop_ = false;
  int pending_ = 0;
  uint8_t *dst_ = nullptr;
  const uint8_t *src_ = nullptr;
  size_t len_ = 0;
};

struct OutPiece {
  uint8_t *dst;
  size_t off;  // offset in the slot
  size_t len;
};

struct Slot {
  hipEvent_t h0 = nullptr;                // H2D start (IN stream)
  hipEvent_t k0 = nullptr, k1 = nullptr;  // kernel start / end (IN stream)
  hipEvent_t done = nullptr;              // D2H complete (OUT stream)
  size_t bytes = 0;
  uint8_t *pin_in = nullptr, *pin_out = nullptr;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  bool busy = false;
  bool staged_out = false;
  std::vector<OutPiece> out;
};

// A contiguous run of the logical byte stream: src[0..len) -> dst[0..len).
struct Seg {
  const uint8_t *src;
  uint8_t *dst;
  size_t len;
};

size_t env_size(const char *name, size_t dflt) {
  const char *v = std::getenv(name);
  if (!v || !*v) return dflt;
  char *end = nullptr;
  unsigned long long x = std::strtoull(v, &end, 0);
  return (end && *end == 0) ? (size_t)x : dflt;
}

}  // namespace

struct vf_ctx {
  int device = -1;
  int num_cus = 256;
  int nslots = 4;
  size_t slot_bytes = 0;
  hipStream_t s_in = nullptr, s_out = nullptr;
  Slot slots[kMaxSlots];
  vf::LaunchCfg cfg;
  CopyPool *pool = nullptr;
  int hip = 0;
  char msg[512] = "no error";
  float last_kernel_ms = 0.f;
  hipEvent_t t0 = nullptr;  // start of the last host->host call (IN stream)
  // per chunk of the last host->host call: {H2D start, kernel start, kernel end, D2H end}
  // in ms after t0, and the chunk's bytes (vf_last_timeline)
  std::vector<std::array<float, 4>> timeline;
  std::vector<size_t> timeline_bytes;
  // asynchronous submissions (page-locked memory only; vf_invert_frames_async)
  static constexpr int kTickets = 32;
  hipEvent_t tk_start[kTickets] = {};
  hipEvent_t tk_end[kTickets] = {};
  uint64_t tk_next = 1;       // id of the next submission
  uint64_t tk_done_upto = 0;  // every submission with id <= this has completed
  int async_slot = 0;         // next device slot for an asynchronous chunk
  bool slot_used[kMaxSlots] = {};
  // host ranges page-locked through this context (vf_alloc_host / vf_host_register)
  std::vector<std::pair<uintptr_t, size_t>> pinned;
};

namespace {

int set_err(vf_ctx *ctx, int status, int hip, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  ErrState &t = g_thread_err;
  t.hip = hip;
  std::snprintf(t.msg, sizeof t.msg, "%s", buf);
  if (ctx) {
    ctx->hip = hip;
    std::snprintf(ctx->msg, sizeof ctx->msg, "%s", buf);
  }
  return status;
}

int fail_hip(vf_ctx *ctx, hipError_t e, const char *what, int line) {
  return set_err(ctx, VF_E_HIP, (int)e, "%s failed: %s (%s, vf_api.hip:%d)", what,
                 hipGetErrorString(e), hipGetErrorName(e), line);
}

#define VF_HIP(ctx, call)                                         \
  do {                                                            \
    hipError_t e_ = (call);                                       \
    if (e_ != hipSuccess) return fail_hip((ctx), e_, #call, __LINE__); \
  } while (0)

#define VF_CHECK_CTX(ctx)                                                        \
  do {                                                                           \
    if (!(ctx)) return set_err(nullptr, VF_E_INVALID, 0, "%s: ctx is NULL", __func__); \
  } while (0)

bool is_pinned(const void *p);

// [p, p+len) inside a range this context page-locked?  Avoids a runtime query per frame.
bool in_pinned_cache(const vf_ctx *ctx, const void *p, size_t len) {
  const uintptr_t a = (uintptr_t)p;
  for (const auto &r : ctx->pinned)
    if (a >= r.first && a + len <= r.first + r.second) return true;
  return false;
}

bool is_pinned_range(const vf_ctx *ctx, const void *p, size_t len) {
  return in_pinned_cache(ctx, p, len) || is_pinned(p);
}

bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof a);
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // pageable pointers report an error on some runtimes
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

int release_slots(vf_ctx *ctx) {
  if (ctx->s_in) (void)hipStreamSynchronize(ctx->s_in);
  if (ctx->s_out) (void)hipStreamSynchronize(ctx->s_out);
  for (int i = 0; i < kMaxSlots; ++i) {
    Slot &s = ctx->slots[i];
    if (s.h0) (void)hipEventDestroy(s.h0);
    if (s.k0) (void)hipEventDestroy(s.k0);
    if (s.k1) (void)hipEventDestroy(s.k1);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.pin_in) (void)hipHostFree(s.pin_in);
    if (s.pin_out) (void)hipHostFree(s.pin_out);
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_out) (void)hipFree(s.d_out);
    s = Slot();
  }
  if (ctx->t0) (void)hipEventDestroy(ctx->t0);
  ctx->t0 = nullptr;
  for (int i = 0; i < vf_ctx::kTickets; ++i) {
    if (ctx->tk_start[i]) (void)hipEventDestroy(ctx->tk_start[i]);
    if (ctx->tk_end[i]) (void)hipEventDestroy(ctx->tk_end[i]);
    ctx->tk_start[i] = ctx->tk_end[i] = nullptr;
  }
  if (ctx->s_in) (void)hipStreamDestroy(ctx->s_in);
  if (ctx->s_out) (void)hipStreamDestroy(ctx->s_out);
  ctx->s_in = ctx->s_out = nullptr;
  return VF_OK;
}

// Wait for slot `s`, scatter its staged output, add its kernel time.
int complete_slot(vf_ctx *ctx, Slot &s) {
  if (!s.busy) return VF_OK;
  VF_HIP(ctx, hipEventSynchronize(s.done));
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, s.k0, s.k1) == hipSuccess) ctx->last_kernel_ms += ms;
  std::array<float, 4> tl{};
  hipEvent_t evs[4] = {s.h0, s.k0, s.k1, s.done};
  for (int i = 0; i < 4; ++i)
    if (hipEventElapsedTime(&tl[i], ctx->t0, evs[i]) != hipSuccess) tl[i] = -1.f;
  ctx->timeline.push_back(tl);
  ctx->timeline_bytes.push_back(s.bytes);
  if (s.staged_out)
    for (const OutPiece &p : s.out) ctx->pool->copy(p.dst, s.pin_out + p.off, p.len);
  s.out.clear();
  s.busy = false;
  return VF_OK;
}

// The slot pipeline over a list of segments (see file header).
// Chunk size: the slot size for big calls; for small calls at least 2 chunks per slot so
// the pipeline fills (480p x 32 = 29 MB in 16 MiB chunks was 2 chunks: no overlap).
size_t chunk_size(const vf_ctx *ctx, size_t total) {
  const size_t kMinChunk = (size_t)1 << 20;
  size_t chunk = (total / (2 * (size_t)ctx->nslots) + 65535) & ~(size_t)65535;
  return std::min(ctx->slot_bytes, std::max(kMinChunk, chunk));
}

bool all_pinned(const vf_ctx *ctx, const Seg *segs, size_t nseg, size_t *total) {
  bool direct = true;
  *total = 0;
  for (size_t i = 0; i < nseg; ++i) {
    *total += segs[i].len;
    if (segs[i].len && direct &&
        !(is_pinned_range(ctx, segs[i].src, segs[i].len) && is_pinned_range(ctx, segs[i].dst, segs[i].len)))
      direct = false;
  }
  return direct;
}

// Wait for every asynchronous submission (before the synchronous path reuses the slots).
int drain_async(vf_ctx *ctx) {
  if (ctx->tk_done_upto + 1 < ctx->tk_next) {
    VF_HIP(ctx, hipStreamSynchronize(ctx->s_out));
    ctx->tk_done_upto = ctx->tk_next - 1;
  }
  return VF_OK;
}

int run_pipeline(vf_ctx *ctx, const Seg *segs, size_t nseg) {
  VF_HIP(ctx, hipSetDevice(ctx->device));
  int rc0 = drain_async(ctx);
  if (rc0 != VF_OK) return rc0;
  ctx->last_kernel_ms = 0.f;
  ctx->timeline.clear();
  ctx->timeline_bytes.clear();
  size_t total = 0;
  const bool direct = all_pinned(ctx, segs, nseg, &total);  // every byte page-locked?
  if (total == 0) return VF_OK;
  const size_t chunk = chunk_size(ctx, total);
  size_t seg = 0, seg_off = 0;
  int next = 0;
  int rc = VF_OK;
  VF_HIP(ctx, hipEventRecord(ctx->t0, ctx->s_in));
  while (seg < nseg && rc == VF_OK) {
    Slot &s = ctx->slots[next];
    next = (next + 1) % ctx->nslots;
    if ((rc = complete_slot(ctx, s)) != VF_OK) break;
    s.out.clear();
    if (direct) {  // direct H2D copies are issued while filling
      hipError_t e = hipEventRecord(s.h0, ctx->s_in);
      if (e != hipSuccess) { rc = fail_hip(ctx, e, "hipEventRecord", __LINE__); break; }
    }
    // Fill the slot from the segment cursor.
    size_t filled = 0;
    while (seg < nseg && filled < chunk) {
      const Seg &g = segs[seg];
      size_t take = std::min(g.len - seg_off, chunk - filled);
      if (take) {
        if (direct) {
          hipError_t e = hipMemcpyAsync(s.d_in + filled, g.src + seg_off, take,
                                        hipMemcpyHostToDevice, ctx->s_in);
          if (e != hipSuccess) { rc = fail_hip(ctx, e, "hipMemcpyAsync(H2D)", __LINE__); break; }
        } else {
          ctx->pool->copy(s.pin_in + filled, g.src + seg_off, take);
        }
        s.out.push_back(OutPiece{g.dst + seg_off, filled, take});
        filled += take;
        seg_off += take;
      }
      if (seg_off == g.len) { ++seg; seg_off = 0; }
    }
    if (rc != VF_OK) break;
    if (filled == 0) break;
    hipError_t e = hipSuccess;
    if (!direct) e = hipEventRecord(s.h0, ctx->s_in);
    if (!direct && e == hipSuccess)
      e = hipMemcpyAsync(s.d_in, s.pin_in, filled, hipMemcpyHostToDevice, ctx->s_in);
    if (e == hipSuccess) e = hipEventRecord(s.k0, ctx->s_in);
    if (e == hipSuccess) e = vf::launch_invert(s.d_in, s.d_out, filled, ctx->cfg, ctx->s_in);
    if (e == hipSuccess) e = hipEventRecord(s.k1, ctx->s_in);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx->s_out, s.k1, 0);
    if (e == hipSuccess) {
      if (direct) {
        for (const OutPiece &p : s.out) {
          e = hipMemcpyAsync(p.dst, s.d_out + p.off, p.len, hipMemcpyDeviceToHost, ctx->s_out);
          if (e != hipSuccess) break;
        }
      } else {
        e = hipMemcpyAsync(s.pin_out, s.d_out, filled, hipMemcpyDeviceToHost, ctx->s_out);
      }
    }
    if (e == hipSuccess) e = hipEventRecord(s.done, ctx->s_out);
    if (e != hipSuccess) { rc = fail_hip(ctx, e, "slot submit", __LINE__); break; }
    s.staged_out = !direct;
    s.bytes = filled;
    s.busy = true;
  }
  // Drain in submission order (oldest first).
  for (int k = 0; k < ctx->nslots; ++k) {
    Slot &s = ctx->slots[(next + k) % ctx->nslots];
    int r = complete_slot(ctx, s);
    if (rc == VF_OK) rc = r;
  }
  return rc;
}

// Asynchronous form for page-locked memory: the whole chain is enqueued and the call
// returns.  Slot reuse is ordered on the device (the IN stream waits for the slot's last D2H
// before overwriting its device output), so the host never blocks; a worker can receive
// and enqueue batch i+1 while batch i is still moving.
int submit_async(vf_ctx *ctx, const Seg *segs, size_t nseg, uint64_t *ticket) {
  VF_HIP(ctx, hipSetDevice(ctx->device));
  size_t total = 0;
  if (!all_pinned(ctx, segs, nseg, &total))
    return set_err(ctx, VF_E_INVALID, 0,
                   "vf_invert_frames_async: every buffer must be page-locked "
                   "(vf_alloc_host / vf_host_register); use vf_invert_frames_host otherwise");
  const uint64_t t = ctx->tk_next;
  const int k = (int)(t % vf_ctx::kTickets);
  if (t > (uint64_t)vf_ctx::kTickets && ctx->tk_done_upto < t - vf_ctx::kTickets) {
    VF_HIP(ctx, hipEventSynchronize(ctx->tk_end[k]));  // bound the submissions in flight
    ctx->tk_done_upto = t - vf_ctx::kTickets;
  }
  VF_HIP(ctx, hipEventRecord(ctx->tk_start[k], ctx->s_in));
  const size_t chunk = chunk_size(ctx, total);
  size_t seg = 0, seg_off = 0;
  hipError_t e = hipSuccess;
  while (seg < nseg && e == hipSuccess) {
    const int si = ctx->async_slot;
    ctx->async_slot = (si + 1) % ctx->nslots;
    Slot &s = ctx->slots[si];
    if (ctx->slot_used[si]) e = hipStreamWaitEvent(ctx->s_in, s.done, 0);
    s.out.clear();
    size_t filled = 0;
    while (e == hipSuccess && seg < nseg && filled < chunk) {
      const Seg &g = segs[seg];
      size_t take = std::min(g.len - seg_off, chunk - filled);
      if (take) {
        e = hipMemcpyAsync(s.d_in + filled, g.src + seg_off, take, hipMemcpyHostToDevice, ctx->s_in);
        s.out.push_back(OutPiece{g.dst + seg_off, filled, take});
        filled += take;
        seg_off += take;
      }
      if (seg_off == g.len) { ++seg; seg_off = 0; }
    }
    if (filled == 0) break;
    if (e == hipSuccess) e = vf::launch_invert(s.d_in, s.d_out, filled, ctx->cfg, ctx->s_in);
    if (e == hipSuccess) e = hipEventRecord(s.k1, ctx->s_in);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx->s_out, s.k1, 0);
    for (size_t i = 0; i < s.out.size() && e == hipSuccess; ++i)
      e = hipMemcpyAsync(s.out[i].dst, s.d_out + s.out[i].off, s.out[i].len, hipMemcpyDeviceToHost,
                         ctx->s_out);
    if (e == hipSuccess) e = hipEventRecord(s.done, ctx->s_out);
    ctx->slot_used[si] = true;
  }
  if (e == hipSuccess) e = hipEventRecord(ctx->tk_end[k], ctx->s_out);
  if (e != hipSuccess) return fail_hip(ctx, e, "vf_invert_frames_async", __LINE__);
  ctx->tk_next = t + 1;
  *ticket = t;
  return VF_OK;
}

}  // namespace

// ---- library / context ---------------------------------------------------------------

VF_EXPORT int vf_get_abi_version(void) { return VF_ABI_VERSION; }

VF_EXPORT const char *vf_status_string(int status) {
  switch (status) {
    case VF_OK: return "VF_OK";
    case VF_E_INVALID: return "VF_E_INVALID: invalid argument";
    case VF_E_HIP: return "VF_E_HIP: HIP runtime error";
    case VF_E_NOMEM: return "VF_E_NOMEM: out of memory";
    case VF_E_NODEVICE: return "VF_E_NODEVICE: no usable gfx950 device";
    default: return "unknown vfilter status";
  }
}

VF_EXPORT int vf_device_count(int *out_count) {
  if (!out_count) return set_err(nullptr, VF_E_INVALID, 0, "vf_device_count: out_count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  *out_count = n;
  return VF_OK;
}

VF_EXPORT int vf_create(int device, size_t max_frame_bytes, int max_batch, vf_ctx **out) {
  if (!out) return set_err(nullptr, VF_E_INVALID, 0, "vf_create: out is NULL");
  *out = nullptr;
  if (max_batch < 1) max_batch = 1;
  int ndev = 0;
  vf_device_count(&ndev);
  if (device < 0 || device >= ndev)
    return set_err(nullptr, VF_E_NODEVICE, 0, "vf_create: device %d not available (%d visible)",
                   device, ndev);
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return fail_hip(nullptr, e, "hipGetDeviceProperties", __LINE__);
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(nullptr, VF_E_NODEVICE, 0,
                   "vf_create: device %d is %s; libvfilter_hip.so is built for gfx950 only",
                   device, prop.gcnArchName);
  vf_ctx *ctx = new (std::nothrow) vf_ctx();
  if (!ctx) return set_err(nullptr, VF_E_NOMEM, 0, "vf_create: out of host memory");
  ctx->device = device;
  ctx->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  ctx->cfg.variant = (int)env_size("VF_VARIANT", (size_t)vf::kVariantU4NT);
  if (ctx->cfg.variant < 0 || ctx->cfg.variant >= vf::kVariantCount) ctx->cfg.variant = vf::kVariantU4NT;
  ctx->cfg.max_blocks = (int)env_size("VF_MAX_BLOCKS", (size_t)ctx->num_cus * 32);
  if (ctx->cfg.max_blocks < 1) ctx->cfg.max_blocks = ctx->num_cus * 32;
  ctx->nslots = (int)std::min<size_t>(kMaxSlots, std::max<size_t>(2, env_size("VF_SLOTS", 4)));
  size_t want = max_frame_bytes ? max_frame_bytes * (size_t)max_batch : (size_t)8 << 20;
  size_t slot = env_size("VF_SLOT_BYTES", std::min(want, (size_t)16 << 20));
  slot = std::max<size_t>(slot, (size_t)1 << 20);
  slot = std::min<size_t>(slot, (size_t)64 << 20);
  slot = (slot + 4095) & ~(size_t)4095;
  ctx->slot_bytes = slot;
  int rc = VF_OK;
  e = hipSetDevice(device);
  if (e != hipSuccess) rc = fail_hip(ctx, e, "hipSetDevice", __LINE__);
  if (rc == VF_OK &&
      ((e = hipStreamCreateWithFlags(&ctx->s_in, hipStreamNonBlocking)) != hipSuccess ||
       (e = hipStreamCreateWithFlags(&ctx->s_out, hipStreamNonBlocking)) != hipSuccess))
    rc = fail_hip(ctx, e, "hipStreamCreateWithFlags", __LINE__);
  if (rc == VF_OK && (e = hipEventCreate(&ctx->t0)) != hipSuccess)
    rc = fail_hip(ctx, e, "hipEventCreate", __LINE__);
  for (int i = 0; i < vf_ctx::kTickets && rc == VF_OK; ++i)
    if ((e = hipEventCreate(&ctx->tk_start[i])) != hipSuccess ||
        (e = hipEventCreate(&ctx->tk_end[i])) != hipSuccess)
      rc = fail_hip(ctx, e, "hipEventCreate", __LINE__);
  for (int i = 0; i < ctx->nslots && rc == VF_OK; ++i) {
    Slot &s = ctx->slots[i];
    if ((e = hipEventCreate(&s.h0)) != hipSuccess || (e = hipEventCreate(&s.k0)) != hipSuccess ||
        (e = hipEventCreate(&s.k1)) != hipSuccess || (e = hipEventCreate(&s.done)) != hipSuccess) {
      rc = fail_hip(ctx, e, "event create", __LINE__);
      break;
    }
    if ((e = hipHostMalloc((void **)&s.pin_in, slot, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc((void **)&s.pin_out, slot, hipHostMallocDefault)) != hipSuccess ||
        (e = hipMalloc((void **)&s.d_in, slot)) != hipSuccess ||
        (e = hipMalloc((void **)&s.d_out, slot)) != hipSuccess) {
      rc = set_err(ctx, VF_E_NOMEM, (int)e, "vf_create: slot allocation of %zu bytes failed: %s",
                   slot, hipGetErrorString(e));
      break;
    }
  }
  if (rc != VF_OK) {
    g_thread_err.hip = ctx->hip;
    std::snprintf(g_thread_err.msg, sizeof g_thread_err.msg, "%s", ctx->msg);
    release_slots(ctx);
    delete ctx;
    return rc;
  }
  ctx->pool = new CopyPool((int)env_size("VF_HOST_THREADS", 8));
  *out = ctx;
  return VF_OK;
}

VF_EXPORT int vf_destroy(vf_ctx *ctx) {
  if (!ctx) return VF_OK;
  (void)hipSetDevice(ctx->device);
  release_slots(ctx);
  delete ctx->pool;
  delete ctx;
  return VF_OK;
}

VF_EXPORT const char *vf_last_error(const vf_ctx *ctx) {
  return ctx ? ctx->msg : g_thread_err.msg;
}

VF_EXPORT int vf_last_hip_error(const vf_ctx *ctx) { return ctx ? ctx->hip : g_thread_err.hip; }

VF_EXPORT int vf_ctx_device(const vf_ctx *ctx, int *out_device) {
  if (!ctx || !out_device) return set_err(nullptr, VF_E_INVALID, 0, "vf_ctx_device: NULL argument");
  *out_device = ctx->device;
  return VF_OK;
}

// ---- host -> host ----------------------------------------------------------------------

static bool overlaps_partially(const uint8_t *a, const uint8_t *b, size_t n) {
  if (a == b || n == 0) return false;
  return (a < b + n) && (b < a + n);
}

VF_EXPORT int vf_invert_host(vf_ctx *ctx, const uint8_t *src, uint8_t *dst, size_t nbytes) {
  VF_CHECK_CTX(ctx);
  if (nbytes == 0) { ctx->last_kernel_ms = 0.f; return VF_OK; }
  if (!src || !dst) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_host: NULL buffer");
  if (overlaps_partially(src, dst, nbytes))
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_host: src and dst partially overlap");
  Seg s{src, dst, nbytes};
  return run_pipeline(ctx, &s, 1);
}

VF_EXPORT int vf_invert_batch_host(vf_ctx *ctx, const uint8_t *src, uint8_t *dst,
                                   size_t frame_bytes, int n) {
  VF_CHECK_CTX(ctx);
  if (n < 0) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_batch_host: n < 0");
  if (n == 0 || frame_bytes == 0) { ctx->last_kernel_ms = 0.f; return VF_OK; }
  if (frame_bytes > SIZE_MAX / (size_t)n)
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_batch_host: size overflow");
  return vf_invert_host(ctx, src, dst, frame_bytes * (size_t)n);
}

VF_EXPORT int vf_invert_frames_host(vf_ctx *ctx, const uint8_t *const *srcs, uint8_t *const *dsts,
                                    const size_t *nbytes, int n) {
  VF_CHECK_CTX(ctx);
  if (n < 0) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_host: n < 0");
  if (n == 0) { ctx->last_kernel_ms = 0.f; return VF_OK; }
  if (!srcs || !dsts || !nbytes)
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_host: NULL array");
  std::vector<Seg> segs;
  segs.reserve((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (nbytes[i] == 0) continue;
    if (!srcs[i] || !dsts[i])
      return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_host: frame %d has a NULL buffer", i);
    if (overlaps_partially(srcs[i], dsts[i], nbytes[i]))
      return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_host: frame %d src/dst partially overlap", i);
    segs.push_back(Seg{srcs[i], dsts[i], nbytes[i]});
  }
  if (segs.empty()) { ctx->last_kernel_ms = 0.f; return VF_OK; }
  return run_pipeline(ctx, segs.data(), segs.size());
}

// ---- asynchronous host -> host (page-locked memory) ----------------------------------------

VF_EXPORT int vf_invert_frames_async(vf_ctx *ctx, const uint8_t *const *srcs, uint8_t *const *dsts,
                                     const size_t *nbytes, int n, uint64_t *ticket) {
  VF_CHECK_CTX(ctx);
  if (!ticket) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_async: ticket is NULL");
  *ticket = 0;
  if (n < 0) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_async: n < 0");
  if (n > 0 && (!srcs || !dsts || !nbytes))
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_async: NULL array");
  std::vector<Seg> segs;
  segs.reserve((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (nbytes[i] == 0) continue;
    if (!srcs[i] || !dsts[i])
      return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_async: frame %d has a NULL buffer", i);
    if (overlaps_partially(srcs[i], dsts[i], nbytes[i]))
      return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_async: frame %d src/dst partially overlap", i);
    segs.push_back(Seg{srcs[i], dsts[i], nbytes[i]});
  }
  return submit_async(ctx, segs.data(), segs.size(), ticket);
}

VF_EXPORT int vf_wait(vf_ctx *ctx, uint64_t ticket, float *gpu_ms) {
  VF_CHECK_CTX(ctx);
  if (gpu_ms) *gpu_ms = -1.f;
  if (ticket == 0 || ticket >= ctx->tk_next)
    return set_err(ctx, VF_E_INVALID, 0, "vf_wait: unknown ticket %llu", (unsigned long long)ticket);
  const int k = (int)(ticket % vf_ctx::kTickets);
  const bool recycled = ticket + vf_ctx::kTickets < ctx->tk_next;  // events reused since
  if (ticket > ctx->tk_done_upto) {
    // If the event was re-recorded for a later submission, waiting for it still covers this
    // one: the OUT stream completes submissions in order.
    VF_HIP(ctx, hipSetDevice(ctx->device));
    VF_HIP(ctx, hipEventSynchronize(ctx->tk_end[k]));
    ctx->tk_done_upto = ticket;
  }
  if (gpu_ms && !recycled) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->tk_start[k], ctx->tk_end[k]) == hipSuccess) *gpu_ms = ms;
  }
  return VF_OK;
}

VF_EXPORT int vf_query(vf_ctx *ctx, uint64_t ticket, int *done) {
  VF_CHECK_CTX(ctx);
  if (!done) return set_err(ctx, VF_E_INVALID, 0, "vf_query: done is NULL");
  if (ticket == 0 || ticket >= ctx->tk_next)
    return set_err(ctx, VF_E_INVALID, 0, "vf_query: unknown ticket %llu", (unsigned long long)ticket);
  if (ticket <= ctx->tk_done_upto || ticket + vf_ctx::kTickets < ctx->tk_next) {
    *done = 1;
    return VF_OK;
  }
  hipError_t e = hipEventQuery(ctx->tk_end[ticket % vf_ctx::kTickets]);
  if (e == hipSuccess) {
    *done = 1;
    ctx->tk_done_upto = std::max(ctx->tk_done_upto, ticket);
  } else if (e == hipErrorNotReady) {
    (void)hipGetLastError();
    *done = 0;
  } else {
    return fail_hip(ctx, e, "hipEventQuery", __LINE__);
  }
  return VF_OK;
}

// ---- device-resident ---------------------------------------------------------------------

VF_EXPORT int vf_invert_device(vf_ctx *ctx, const void *dsrc, void *ddst, size_t nbytes,
                               void *stream) {
  VF_CHECK_CTX(ctx);
  if (nbytes == 0) return VF_OK;
  if (!dsrc || !ddst) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_device: NULL buffer");
  if (overlaps_partially((const uint8_t *)dsrc, (const uint8_t *)ddst, nbytes))
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_device: src and dst partially overlap");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, vf::launch_invert(dsrc, ddst, nbytes, ctx->cfg, (hipStream_t)stream));
  return VF_OK;
}

VF_EXPORT int vf_invert_device_frames(vf_ctx *ctx, const void *const *dsrcs, void *const *ddsts,
                                      const size_t *nbytes, int n, size_t total_bytes,
                                      void *stream) {
  VF_CHECK_CTX(ctx);
  if (n < 0 || n > 65535)
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_device_frames: n=%d outside [0, 65535]", n);
  if (n == 0) return VF_OK;
  if (!dsrcs || !ddsts || !nbytes)
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_device_frames: NULL descriptor array");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, vf::launch_invert_frames(dsrcs, ddsts, nbytes, n, total_bytes, ctx->cfg,
                                       (hipStream_t)stream));
  return VF_OK;
}

// ---- memory helpers ------------------------------------------------------------------------

VF_EXPORT int vf_alloc_device(vf_ctx *ctx, size_t nbytes, void **out) {
  VF_CHECK_CTX(ctx);
  if (!out) return set_err(ctx, VF_E_INVALID, 0, "vf_alloc_device: out is NULL");
  *out = nullptr;
  VF_HIP(ctx, hipSetDevice(ctx->device));
  hipError_t e = hipMalloc(out, nbytes ? nbytes : 1);
  if (e != hipSuccess)
    return set_err(ctx, VF_E_NOMEM, (int)e, "hipMalloc(%zu) failed: %s", nbytes, hipGetErrorString(e));
  return VF_OK;
}

VF_EXPORT int vf_free_device(vf_ctx *ctx, void *p) {
  VF_CHECK_CTX(ctx);
  if (!p) return VF_OK;
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, hipFree(p));
  return VF_OK;
}

VF_EXPORT int vf_alloc_host(vf_ctx *ctx, size_t nbytes, void **out) {
  VF_CHECK_CTX(ctx);
  if (!out) return set_err(ctx, VF_E_INVALID, 0, "vf_alloc_host: out is NULL");
  *out = nullptr;
  VF_HIP(ctx, hipSetDevice(ctx->device));
  hipError_t e = hipHostMalloc(out, nbytes ? nbytes : 1, hipHostMallocDefault);
  if (e != hipSuccess)
    return set_err(ctx, VF_E_NOMEM, (int)e, "hipHostMalloc(%zu) failed: %s", nbytes, hipGetErrorString(e));
  ctx->pinned.emplace_back((uintptr_t)*out, nbytes ? nbytes : 1);
  return VF_OK;
}

static void forget_pinned(vf_ctx *ctx, void *p) {
  auto &v = ctx->pinned;
  v.erase(std::remove_if(v.begin(), v.end(), [p](const std::pair<uintptr_t, size_t> &r) {
            return r.first == (uintptr_t)p;
          }), v.end());
}

VF_EXPORT int vf_free_host(vf_ctx *ctx, void *p) {
  VF_CHECK_CTX(ctx);
  if (!p) return VF_OK;
  int rc = drain_async(ctx);
  if (rc != VF_OK) return rc;
  forget_pinned(ctx, p);
  VF_HIP(ctx, hipHostFree(p));
  return VF_OK;
}

VF_EXPORT int vf_host_register(vf_ctx *ctx, void *p, size_t nbytes) {
  VF_CHECK_CTX(ctx);
  if (!p || !nbytes) return set_err(ctx, VF_E_INVALID, 0, "vf_host_register: empty range");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, hipHostRegister(p, nbytes, hipHostRegisterDefault));
  ctx->pinned.emplace_back((uintptr_t)p, nbytes);
  return VF_OK;
}

VF_EXPORT int vf_host_unregister(vf_ctx *ctx, void *p) {
  VF_CHECK_CTX(ctx);
  if (!p) return VF_OK;
  int rc = drain_async(ctx);
  if (rc != VF_OK) return rc;
  forget_pinned(ctx, p);
  VF_HIP(ctx, hipHostUnregister(p));
  return VF_OK;
}

VF_EXPORT int vf_upload(vf_ctx *ctx, void *ddst, const void *hsrc, size_t nbytes, void *stream) {
  VF_CHECK_CTX(ctx);
  if (!nbytes) return VF_OK;
  if (!ddst || !hsrc) return set_err(ctx, VF_E_INVALID, 0, "vf_upload: NULL buffer");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, hipMemcpyAsync(ddst, hsrc, nbytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return VF_OK;
}

VF_EXPORT int vf_download(vf_ctx *ctx, void *hdst, const void *dsrc, size_t nbytes, void *stream) {
  VF_CHECK_CTX(ctx);
  if (!nbytes) return VF_OK;
  if (!hdst || !dsrc) return set_err(ctx, VF_E_INVALID, 0, "vf_download: NULL buffer");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, hipMemcpyAsync(hdst, dsrc, nbytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  return VF_OK;
}

VF_EXPORT int vf_memset_device(vf_ctx *ctx, void *d, int value, size_t nbytes, void *stream) {
  VF_CHECK_CTX(ctx);
  if (!nbytes) return VF_OK;
  if (!d) return set_err(ctx, VF_E_INVALID, 0, "vf_memset_device: NULL buffer");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, hipMemsetAsync(d, value, nbytes, (hipStream_t)stream));
  return VF_OK;
}

VF_EXPORT int vf_sync(vf_ctx *ctx, void *stream) {
  VF_CHECK_CTX(ctx);
  VF_HIP(ctx, hipSetDevice(ctx->device));
  if (stream) {
    VF_HIP(ctx, hipStreamSynchronize((hipStream_t)stream));
  } else {
    VF_HIP(ctx, hipDeviceSynchronize());
  }
  return VF_OK;
}

// ---- timing ----------------------------------------------------------------------------

VF_EXPORT int vf_elapsed_ms(const vf_ctx *ctx, float *out_ms) {
  if (!ctx || !out_ms) return set_err(nullptr, VF_E_INVALID, 0, "vf_elapsed_ms: NULL argument");
  *out_ms = ctx->last_kernel_ms;
  return VF_OK;
}

VF_EXPORT int vf_last_timeline(const vf_ctx *ctx, float *out4, size_t *chunk_bytes, int max_chunks,
                               int *n_chunks) {
  if (!ctx || !n_chunks) return set_err(nullptr, VF_E_INVALID, 0, "vf_last_timeline: NULL argument");
  const int n = (int)ctx->timeline.size();
  *n_chunks = n;
  for (int i = 0; i < n && i < max_chunks; ++i) {
    if (out4)
      for (int j = 0; j < 4; ++j) out4[4 * i + j] = ctx->timeline[i][j];
    if (chunk_bytes) chunk_bytes[i] = ctx->timeline_bytes[i];
  }
  return VF_OK;
}

VF_EXPORT int vf_bench_device_ring(vf_ctx *ctx, void *const *srcs, void *const *dsts, int nbuf,
                                   size_t nbytes, int steps, void *stream, float *per_launch_ms,
                                   float *region_ms) {
  VF_CHECK_CTX(ctx);
  if (!srcs || !dsts || nbuf < 1 || steps < 0)
    return set_err(ctx, VF_E_INVALID, 0, "vf_bench_device_ring: bad arguments");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const bool each = per_launch_ms != nullptr;
  std::vector<hipEvent_t> ev((each ? 2 * (size_t)steps : 0) + 2, nullptr);
  int rc = VF_OK;
  for (auto &e : ev) {
    hipError_t h = hipEventCreate(&e);
    if (h != hipSuccess) { rc = fail_hip(ctx, h, "hipEventCreate", __LINE__); break; }
  }
  hipEvent_t r0 = ev[ev.size() - 2], r1 = ev[ev.size() - 1];
  if (rc == VF_OK) {
    hipError_t h = hipEventRecord(r0, st);
    if (h != hipSuccess) rc = fail_hip(ctx, h, "hipEventRecord", __LINE__);
  }
  for (int s = 0; s < steps && rc == VF_OK; ++s) {
    hipError_t h = each ? hipEventRecord(ev[2 * s], st) : hipSuccess;
    if (h == hipSuccess) h = vf::launch_invert(srcs[s % nbuf], dsts[s % nbuf], nbytes, ctx->cfg, st);
    if (h == hipSuccess && each) h = hipEventRecord(ev[2 * s + 1], st);
    if (h != hipSuccess) rc = fail_hip(ctx, h, "bench launch", __LINE__);
  }
  if (rc == VF_OK) {
    hipError_t h = hipEventRecord(r1, st);
    if (h == hipSuccess) h = hipStreamSynchronize(st);
    if (h != hipSuccess) rc = fail_hip(ctx, h, "hipStreamSynchronize", __LINE__);
  }
  for (int s = 0; s < steps && rc == VF_OK && each; ++s) {
    float ms = 0.f;
    hipError_t h = hipEventElapsedTime(&ms, ev[2 * s], ev[2 * s + 1]);
    if (h != hipSuccess) { rc = fail_hip(ctx, h, "hipEventElapsedTime", __LINE__); break; }
    per_launch_ms[s] = ms;
  }
  if (rc == VF_OK && region_ms) {
    float ms = 0.f;
    hipError_t h = hipEventElapsedTime(&ms, r0, r1);
    if (h != hipSuccess) rc = fail_hip(ctx, h, "hipEventElapsedTime", __LINE__);
    *region_ms = ms;
  }
  for (auto &e : ev)
    if (e) (void)hipEventDestroy(e);
  return rc;
}
