// vf_engine.hip — the host->host pipeline engine of a vf_ctx.
//
// What it replaces: the reference filters one frame per loop iteration, synchronously, in
// the worker process (worker.py:35-57 -> inverter.py:41).  Here every host->host request
// (one frame, a packed batch, a gather list of frames; synchronous or asynchronous) becomes
// a JOB queued to one engine thread per context, which streams the jobs' bytes through a
// ring of device slots without draining between jobs:
//
//   fill    slot i: (pageable: copy the chunk into the slot's pinned staging buffer)
//           H2D -> invert kernel on the IN stream, event k1
//   d2h     once k1 has fired: D2H on the OUT stream, event done
//   retire  once done has fired: (pageable: scatter the staged result) -> slot free
//
// The engine reacts to event completion on the host instead of chaining the two streams
// with hipStreamWaitEvent.  Measured on MI355X (tools/pcie_probe.hip): device-side
// cross-stream waits enqueued while earlier batches are still executing drop the pipeline
// from 45 to 26 GB/s per direction; the host-driven form holds 45-46 GB/s with work queued
// concurrently (profiles/r01_pcie_probe_pipelines.txt).  IN and OUT are separate streams, so
// the two directions run on separate SDMA engines at once.
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "vf_host_mem.h"
#include "vf_internal.h"

namespace vf {

namespace {
constexpr int kStatusHip = -2;  // VF_E_HIP
// run_gated: pieces of at least 32 KiB, at most 254 of them (32 MiB of staging = 128 x 256 KiB),
// their landed marks and the status word in one page-locked page
constexpr uint32_t kGateMinShift = 15;
constexpr size_t kGateFlagBytes = 4096;
constexpr size_t kGateStatus = 1023;  // index of the status word in the flag page

size_t env_or(const char *name, size_t dflt) {
  const char *v = std::getenv(name);
  if (!v || !*v) return dflt;
  char *end = nullptr;
  unsigned long long x = std::strtoull(v, &end, 0);
  return (end && *end == 0) ? (size_t)x : dflt;
}

bool fired(hipEvent_t e, hipError_t *err) {
  hipError_t q = hipEventQuery(e);
  if (q == hipSuccess) return true;
  (void)hipGetLastError();  // clear hipErrorNotReady so it cannot leak into a later check
  if (q != hipErrorNotReady) *err = q;
  return false;
}
}  // namespace

// ---- host copy pool -----------------------------------------------------------------------
// Workers sleep on a futex over the task generation, not on a condition variable: a condition
// variable's waiters re-take its mutex one after another when woken, so the ninth worker of a
// drop-in frame's copy started tens of microseconds after the first.  Each worker now wakes
// straight into the task, and the caller waits for the last one on the pending count.
namespace {
long futex_wait(std::atomic<uint32_t> *a, uint32_t v) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t *>(a), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
long futex_wake(std::atomic<uint32_t> *a, int n) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t *>(a), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}
}  // namespace

CopyPool::CopyPool(int nthreads, size_t split_min) : split_min_(split_min), n_(std::max(1, nthreads)) {
  for (int i = 1; i < n_; ++i) threads_.emplace_back([this, i] { run(i); });
}

CopyPool::~CopyPool() {
  stop_.store(true, std::memory_order_relaxed);
  gen_.fetch_add(1, std::memory_order_release);
  futex_wake(&gen_, INT32_MAX);
  for (auto &t : threads_) t.join();
}

void CopyPool::post() {  // the task fields are set: publish a new generation and wake every worker
  pending_.store((uint32_t)(n_ - 1), std::memory_order_relaxed);
  gen_.fetch_add(1, std::memory_order_release);
  futex_wake(&gen_, INT32_MAX);
}

void CopyPool::wait_all() {
  for (int spin = 0; spin < 4096; ++spin) {  // the workers usually finish within microseconds of the caller
    if (pending_.load(std::memory_order_acquire) == 0) return;
    __builtin_ia32_pause();
  }
  for (uint32_t p; (p = pending_.load(std::memory_order_acquire)) != 0;) futex_wait(&pending_, p);
}

void CopyPool::copy(uint8_t *dst, const uint8_t *src, size_t len) {
  if (len < split_min_ || n_ == 1) {
    std::memcpy(dst, src, len);
    return;
  }
  fn_ = nullptr;
  dst_ = dst;
  src_ = src;
  len_ = len;
  post();
  part(0);
  wait_all();
}

void CopyPool::start(std::function<void(int, int)> fn) {
  if (n_ == 1) {  // no worker threads (VF_HOST_THREADS=0): the task runs here, before start returns
    fn(0, 1);
    return;
  }
  fn_ = std::move(fn);
  post();
}

void CopyPool::join() {
  if (n_ == 1) return;
  wait_all();
  fn_ = nullptr;
}

void CopyPool::part(int i) {
  size_t per = (len_ / n_ + 63) & ~size_t(63);
  size_t b = std::min(len_, per * (size_t)i);
  size_t e = (i == n_ - 1) ? len_ : std::min(len_, b + per);
  if (e > b) std::memcpy(dst_ + b, src_ + b, e - b);
}

void CopyPool::run(int i) {
  uint32_t seen = 0;  // the generation the pool was built with: a task posted before this thread ran is still seen
  for (;;) {
    uint32_t g;
    while ((g = gen_.load(std::memory_order_acquire)) == seen) futex_wait(&gen_, seen);
    seen = g;
    if (stop_.load(std::memory_order_relaxed)) return;
    if (fn_) fn_(i - 1, n_ - 1);
    else part(i);
    if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) futex_wake(&pending_, 1);
  }
}

// ---- engine: construction --------------------------------------------------------------------

Engine::~Engine() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  (void)hipSetDevice(device_);
  if (s_in_) (void)hipStreamSynchronize(s_in_);
  if (s_out_) (void)hipStreamSynchronize(s_out_);
  if (s_map_) (void)hipStreamSynchronize(s_map_);
  for (auto &s : slots_) {
    for (hipEvent_t e : {s.h0, s.k0, s.k1, s.done})
      if (e) (void)hipEventDestroy(e);
    (void)numa_pinned_free(s.pin_in);
    (void)numa_pinned_free(s.pin_out);
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_out) (void)hipFree(s.d_out);
  }
  for (hipEvent_t e : free_events_) (void)hipEventDestroy(e);
  (void)numa_pinned_free(stg_in_);
  (void)numa_pinned_free(stg_out_);
  (void)numa_pinned_free(stg_flags_);
  if (stg_frontier_) (void)hipFree(stg_frontier_);
  if (s_in_) (void)hipStreamDestroy(s_in_);
  if (s_out_) (void)hipStreamDestroy(s_out_);
  if (s_map_) (void)hipStreamDestroy(s_map_);
}

hipError_t Engine::init(int device, int nslots, size_t slot_bytes, const LaunchCfg &cfg,
                        std::string *err) {
  device_ = device;
  cfg_ = cfg;
  slot_bytes_ = slot_bytes;
  pool_.reset(new CopyPool((int)env_or("VF_HOST_THREADS", 8)));
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    *err = std::string("hipSetDevice failed: ") + hipGetErrorString(e);
    return e;
  }
  zero_copy_ = env_or("VF_ZEROCOPY", 1) != 0;
  slots_.resize((size_t)nslots);
  for (auto &s : slots_) {
    if ((e = hipEventCreate(&s.h0)) != hipSuccess || (e = hipEventCreate(&s.k0)) != hipSuccess ||
        (e = hipEventCreate(&s.k1)) != hipSuccess || (e = hipEventCreate(&s.done)) != hipSuccess) {
      *err = std::string("event creation failed: ") + hipGetErrorString(e);
      return e;
    }
    const int node = device_numa_node(device);  // staging on the GPU's own socket
    if ((e = numa_pinned_alloc((void **)&s.pin_in, slot_bytes, node)) != hipSuccess ||
        (e = numa_pinned_alloc((void **)&s.pin_out, slot_bytes, node)) != hipSuccess ||
        (e = hipMalloc((void **)&s.d_in, slot_bytes)) != hipSuccess ||
        (e = hipMalloc((void **)&s.d_out, slot_bytes)) != hipSuccess) {
      char buf[160];
      std::snprintf(buf, sizeof buf, "slot allocation of %zu bytes failed: %s", slot_bytes,
                    hipGetErrorString(e));
      *err = buf;
      return e;
    }
  }
  thread_ = std::thread([this] { run(); });
  return hipSuccess;
}

// The engine's three streams are created with its first job, not with the context: HIP maps
// streams onto a few hardware queues per process (GPU_MAX_HW_QUEUES, 4 by default), and a
// process that only runs JPEG batches would otherwise lose three of them to idle streams and
// put its two codecs' streams on one queue, where each batch's copies and event waits stall
// the other's kernels (1080p worker form 15.0-15.3 k fps on 4 queues, 19.9 k on 8:
// profiles/r02_jpeg_hwq.jsonl).
hipError_t Engine::ensure_streams() {
  if (streams_ready_.load(std::memory_order_acquire)) return hipSuccess;
  std::lock_guard<std::mutex> lk(stream_mu_);
  if (streams_ready_.load(std::memory_order_relaxed)) return hipSuccess;
  hipError_t e = hipSetDevice(device_);
  if (e == hipSuccess && !s_in_) e = hipStreamCreateWithFlags(&s_in_, hipStreamNonBlocking);
  if (e == hipSuccess && !s_out_) e = hipStreamCreateWithFlags(&s_out_, hipStreamNonBlocking);
  if (e == hipSuccess && !s_map_) e = hipStreamCreateWithFlags(&s_map_, hipStreamNonBlocking);
  if (e == hipSuccess) streams_ready_.store(true, std::memory_order_release);
  return e;
}

// ---- page-locked range registry (so `direct` needs no runtime query per frame) ----------------

void Engine::note_pinned(const void *p, size_t n) {
  // the device address of the range (page-locked memory is mapped into the GPU's address
  // space; the runtime says where), or 0 if the runtime does not know the range as mapped
  void *dev = nullptr;
  if (hipHostGetDevicePointer(&dev, const_cast<void *>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    dev = nullptr;
  }
  std::lock_guard<std::mutex> lk(pin_mu_);
  pinned_.push_back(PinRange{(uintptr_t)p, n, (uintptr_t)dev});
}

void Engine::forget_pinned(const void *p) {
  std::lock_guard<std::mutex> lk(pin_mu_);
  pinned_.erase(std::remove_if(pinned_.begin(), pinned_.end(),
                               [p](const PinRange &r) { return r.host == (uintptr_t)p; }),
                pinned_.end());
}

bool Engine::is_pinned(const void *p, size_t len) {
  {
    std::lock_guard<std::mutex> lk(pin_mu_);
    const uintptr_t a = (uintptr_t)p;
    for (const auto &r : pinned_)
      if (a >= r.host && a + len <= r.host + r.len) return true;
  }
  hipPointerAttribute_t attr;
  std::memset(&attr, 0, sizeof attr);
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable pointers report an error on some runtimes
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

uint8_t *Engine::mapped(const void *p, size_t len) {
  std::lock_guard<std::mutex> lk(pin_mu_);
  const uintptr_t a = (uintptr_t)p;
  for (const auto &r : pinned_)
    if (r.dev && a >= r.host && a + len <= r.host + r.len) return reinterpret_cast<uint8_t *>(r.dev + (a - r.host));
  return nullptr;
}

// ---- engine: caller side ---------------------------------------------------------------------

uint64_t Engine::submit(std::vector<Seg> &&segs) {
  auto job = std::make_unique<Job>();
  job->mapped = zero_copy_;
  for (const Seg &s : segs) {
    job->total += s.len;
    if (!s.len) continue;
    if (job->mapped) {
      uint8_t *ds = mapped(s.src, s.len), *dd = mapped(s.dst, s.len);
      if (ds && dd) job->dsegs.push_back(Seg{ds, dd, s.len});
      else job->mapped = false;
    }
    if (job->direct && !(is_pinned(s.src, s.len) && is_pinned(s.dst, s.len))) job->direct = false;
  }
  if (!job->mapped) job->dsegs.clear();
  // Chunk size: the slot size for big jobs; small jobs still get >= 2 chunks per slot so the
  // ring fills (480p x 32 = 29 MB in 16 MiB chunks is only 2 chunks).
  const size_t kMinChunk = (size_t)1 << 20;
  size_t chunk = (job->total / (2 * slots_.size()) + 65535) & ~(size_t)65535;
  job->chunk = std::min(slot_bytes_, std::max(kMinChunk, chunk));
  job->segs = std::move(segs);
  std::lock_guard<std::mutex> lk(mu_);
  const uint64_t id = next_id_++;
  job->id = id;
  if (broken_ || job->total == 0) {
    JobResult r;
    if (broken_) {
      r.status = kStatusHip;
      r.msg = "the context's pipeline failed earlier; destroy and recreate the context";
    }
    results_[id] = std::move(r);
    done_cv_.notify_all();
    return id;
  }
  unfinished_.insert(id);
  pending_.push_back(std::move(job));
  cv_.notify_all();
  return id;
}

bool Engine::run_now(const std::vector<Seg> &segs, JobResult *out) {
  if (!zero_copy_) return false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (broken_) return false;  // the engine path reports it
  }
  std::vector<Seg> dsegs;
  size_t total = 0;
  bool all_mapped = true;
  for (const Seg &s : segs) {
    if (!s.len) continue;
    uint8_t *ds = mapped(s.src, s.len), *dd = mapped(s.dst, s.len);
    all_mapped = all_mapped && ds && dd;
    dsegs.push_back(Seg{ds, dd, s.len});
    total += s.len;
  }
  if (dsegs.empty() || (!all_mapped && total > kStagedMax)) return false;
  if (hipSetDevice(device_) != hipSuccess || ensure_streams() != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (!all_mapped) {
    if (segs.size() == 1) {
      const int g = run_gated(segs[0], out);
      if (g >= 0) return g != 0;
    }
    return run_staged(segs, total, out);
  }
  hipEvent_t a = take_event(), b = take_event();
  if (!a || !b) {
    give_event(a);
    give_event(b);
    return false;
  }
  hipError_t e = hipEventRecord(a, s_map_);
  MappedBatch mb;
  for (size_t i = 0; i < dsegs.size() && e == hipSuccess; i += kMappedMax) {
    const int n = (int)std::min<size_t>(kMappedMax, dsegs.size() - i);
    size_t bytes = 0;
    for (int k = 0; k < n; ++k) {
      mb.src[k] = dsegs[i + k].src;
      mb.dst[k] = dsegs[i + k].dst;
      mb.n[k] = dsegs[i + k].len;
      bytes += dsegs[i + k].len;
    }
    e = launch_invert_mapped(mb, n, bytes, s_map_);
  }
  if (e == hipSuccess) e = hipEventRecord(b, s_map_);
  if (e == hipSuccess) e = hipEventSynchronize(b);
  *out = JobResult();
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(s_map_);  // nothing may land in the caller's buffers later
    (void)hipGetLastError();
    out->status = kStatusHip;
    out->hip = e;
    out->msg = std::string("zero-copy launch failed: ") + hipGetErrorString(e);
  } else {
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = -1.f;
    out->kernel_ms = out->gpu_ms = ms;
    out->zero_copy = true;
    out->timeline.push_back(ChunkTime{total, 0.f, 0.f, ms, ms});
  }
  give_event(a);
  give_event(b);
  return true;
}

hipError_t Engine::ensure_staging() {
  if (stg_ready_) return hipSuccess;
  const int node = device_numa_node(device_);
  hipError_t e;
  if ((!stg_in_ && (e = numa_pinned_alloc((void **)&stg_in_, kStagedMax, node)) != hipSuccess) ||
      (!stg_out_ && (e = numa_pinned_alloc((void **)&stg_out_, kStagedMax, node)) != hipSuccess) ||
      (!stg_flags_ && (e = numa_pinned_alloc((void **)&stg_flags_, kGateFlagBytes, node)) != hipSuccess))
    return e;
  void *di = nullptr, *dout = nullptr, *dfl = nullptr;
  if ((e = hipHostGetDevicePointer(&di, stg_in_, 0)) != hipSuccess ||
      (e = hipHostGetDevicePointer(&dout, stg_out_, 0)) != hipSuccess ||
      (e = hipHostGetDevicePointer(&dfl, stg_flags_, 0)) != hipSuccess)
    return e;
  stg_dflags_ = static_cast<uint32_t *>(dfl);
  if (!stg_frontier_) {
    if ((e = hipMalloc((void **)&stg_frontier_, 256)) != hipSuccess) return e;
    if ((e = hipMemset(stg_frontier_, 0, 256)) != hipSuccess) return e;
  }
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_) == hipSuccess && khz > 0)
    clock_khz_ = (uint64_t)khz;
  (void)hipGetLastError();
  stg_din_ = static_cast<uint8_t *>(di);
  stg_dout_ = static_cast<uint8_t *>(dout);
  if (!cpool_) cpool_.reset(new CopyPool((int)env_or("VF_HOST_THREADS", 8) + 1, (size_t)256 << 10));
  stg_ready_ = true;
  return hipSuccess;
}

// The drop-in's own shape, one pageable frame (vfilter.bitwise_not(frame) for
// cv2.bitwise_not(frame), inverter.py:41), with the copy overlapped by the launch: the kernel
// is queued first and its tiles wait for their piece of the staging copy (invert_gated_kernel),
// while the pool's workers copy the pieces in order and count each one in page-locked memory.
// run_staged instead launches after the copy (one piece up to 8 MiB), so the frame paid
// copy + launch + PCIe in series.  -1: not this shape (a mapped source, an unaligned side, more
// than kStagedMax bytes, VF_STAGE_GATED=0, or the staging is busy on another thread).
int Engine::run_gated(const Seg &sg, JobResult *out) {
  // Read per call (tools/r6/gated_ab.py, the tests).  Frames above 8 MiB only by default: a 4K
  // frame takes 0.60-0.66 ms instead of 0.73-0.76 (run_staged copies it whole, then launches 3
  // pieces), within 2-12 % of a page-locked source; at 480p and 1080p the two forms measured
  // within noise of each other (profiles/r06_dropin_gated_ab.txt).
  const bool enabled = env_or("VF_STAGE_GATED", 1) != 0;
  const size_t min_len = env_or("VF_STAGE_GATE_MIN", (size_t)8 << 20);
  if (!enabled || sg.len == 0 || sg.len <= min_len || sg.len > kStagedMax || mapped(sg.src, sg.len)) return -1;
  uint8_t *dd = mapped(sg.dst, sg.len);
  const bool stage_out = dd == nullptr;
  if ((((uintptr_t)sg.dst) & 15) != 0) return -1;
  std::unique_lock<std::mutex> lk(stg_mu_, std::try_to_lock);
  if (!lk.owns_lock()) return -1;
  if (ensure_staging() != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if (stage_out) dd = stg_dout_;
  // pieces of 32 KiB and up, at most 254 (the relay reads their marks in one round trip; 255 is
  // its give-up mark)
  uint32_t shift = kGateMinShift;
  while (((sg.len - 1) >> shift) >= 254) ++shift;
  const size_t piece = (size_t)1 << shift;
  const size_t np = ((sg.len - 1) >> shift) + 1;
  volatile uint32_t *flags = stg_flags_;
  for (size_t i = 0; i < np; ++i) flags[i] = 0;
  flags[kGateStatus] = 0;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  // The pieces go to whichever thread asks next: the pool's workers are woken before the launch
  // and join as they wake (a wake-up costs microseconds to tens of them), this thread right after
  // the launch; each copies whole pieces and marks each one landed.  Also after a failed launch:
  // the copy completes either way, and nothing waits on it.
  const uint8_t *src = sg.src;
  uint8_t *stg = stg_in_;
  uint32_t *cnt = stg_flags_;
  const size_t len = sg.len;
  std::atomic<size_t> next{0};
  // (non-temporal stores for this copy, so the GPU's reads would not be served from the copying
  // cores' caches, measured the same: profiles/r06_dropin_gated_ab.txt)
  auto copy_pieces = [&next, src, stg, cnt, len, piece, shift, np] {
    for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < np;) {
      const size_t off = i << shift;
      std::memcpy(stg + off, src + off, std::min(piece, len - off));
      __atomic_store_n(cnt + i, 1u, __ATOMIC_RELEASE);
    }
  };
  cpool_->start([&copy_pieces](int, int) { copy_pieces(); });  // wakes the workers first
  hipEvent_t a = take_event(), b = take_event();
  hipError_t e = (a && b) ? hipEventRecord(a, s_map_) : hipErrorOutOfMemory;
  // 100 ms without a piece: the copy stalled (it never waits on the GPU); the kernel gives up.
  // VF_STAGE_GATE_BUDGET_US overrides (tests drive the give-up path with 0).
  const uint64_t budget_us = env_or("VF_STAGE_GATE_BUDGET_US", 100000);
  const uint64_t budget = clock_khz_ * budget_us / 1000;
  if (e == hipSuccess) {
    gate_gen_ = (gate_gen_ + 1) & 0xFFFFFFu;
    if (gate_gen_ == 0) gate_gen_ = 1;
    e = launch_invert_gated(stg_din_, dd, sg.len, stg_dflags_, shift, 1u, stg_frontier_, gate_gen_,
                            stg_dflags_ + kGateStatus, budget, s_map_);
  }
  if (e == hipSuccess) e = hipEventRecord(b, s_map_);
  copy_pieces();
  // the GPU first, then the pool: a worker that woke late (after the pieces ran out) still has to
  // check in before this frame's task may go out of scope, and that wait now overlaps the kernel
  if (e == hipSuccess) e = hipEventSynchronize(b);
  cpool_->join();
  bool gave_up = false;
  if (e == hipSuccess && flags[kGateStatus] != 0) {  // a wave gave up: the staging copy is complete now
    gave_up = true;
    MappedBatch mb;
    mb.src[0] = stg_din_;
    mb.dst[0] = dd;
    mb.n[0] = sg.len;
    e = launch_invert_mapped(mb, 1, sg.len, s_map_);
    if (e == hipSuccess) e = hipEventRecord(b, s_map_);
    if (e == hipSuccess) e = hipEventSynchronize(b);
  }
  if (e == hipSuccess && stage_out) cpool_->copy(sg.dst, stg_out_, sg.len);
  *out = JobResult();
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(s_map_);  // nothing may land in the caller's buffers later
    (void)hipGetLastError();
    out->status = kStatusHip;
    out->hip = e;
    out->msg = std::string("gated zero-copy launch failed: ") + hipGetErrorString(e);
  } else {
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = -1.f;
    out->kernel_ms = out->gpu_ms = ms;
    out->zero_copy = true;
    out->timeline.push_back(ChunkTime{sg.len, 0.f, 0.f, ms, ms});
    if (env_or("VF_STAGE_TRACE", 0) != 0)  // read per call: tests switch it on
      std::fprintf(stderr, "vf_stage: gated %zu B, %zu pieces, %d pool workers, GPU %.1f us%s\n", sg.len, np, cpool_->workers(),
                   ms * 1000.f, gave_up ? ", re-run ungated after a give-up" : "");
  }
  give_event(a);
  give_event(b);
  return 1;
}

// A small synchronous job with a side outside the mapped ranges (a pageable frame: the
// drop-in's own shape, vfilter.bitwise_not(frame) for cv2.bitwise_not(frame), inverter.py:41)
// on the calling thread.  The job is cut into pieces (below); an unmapped source is copied into the
// mapped staging input by the copy pool's workers -- woken once, they copy the pieces in order,
// each worker a 1/n share of each piece, and count every piece as it lands -- while this
// thread launches invert_mapped_kernel on each piece as soon as it is complete, so the copy of
// piece i + 1 overlaps piece i's launch over PCIe.  A mapped side is read or written in place;
// an unmapped destination is written into the staging output and copied out by the pool at
// the end.  1080p pageable -> pinned: 0.44-0.49 ms per call through the slot ring
// (profiles/r02_per_frame.jsonl).
bool Engine::run_staged(const std::vector<Seg> &segs, size_t total, JobResult *out) {
  std::unique_lock<std::mutex> lk(stg_mu_, std::try_to_lock);
  if (!lk.owns_lock()) return false;  // another thread is staging: the engine path takes it
  if (ensure_staging() != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  struct P {
    const uint8_t *src;   // caller's source
    uint8_t *dst;         // caller's destination
    size_t off, len;      // position in the staging buffers
    const uint8_t *ds;    // device address of the source (mapped, or the staging input)
    uint8_t *dd;          // device address of the destination (mapped, or the staging output)
    bool stage_in, stage_out;
  };
  // Pieces: a hot frame's copy runs at ~250 GB/s on the pool (6.2 MB in ~25 us) while each
  // extra launch over PCIe costs more than the overlap gains, so a frame up to 8 MiB is one
  // piece (1080p: 0.223 ms per call at 1 piece, 0.235 at 2, 0.240 at 3, 0.267 at 6;
  // profiles/r03_per_frame_pieces.txt); larger jobs take 3.  VF_STAGE_PIECES overrides.
  static const size_t kPieces = env_or("VF_STAGE_PIECES", 0);
  const size_t npieces = kPieces ? kPieces : total <= ((size_t)8 << 20) ? 1 : 3;
  const size_t piece = std::max<size_t>((size_t)256 << 10, (total / npieces + 65535) & ~(size_t)65535);
  std::vector<P> ps;
  size_t at = 0;
  bool any_in = false, any_out = false;
  for (const Seg &sg : segs)
    for (size_t o = 0; o < sg.len; o += piece) {
      const size_t n = std::min(piece, sg.len - o);
      P p{sg.src + o, sg.dst + o, at, n, mapped(sg.src + o, n), mapped(sg.dst + o, n), false, false};
      if (!p.ds) p.ds = stg_din_ + at, p.stage_in = any_in = true;
      if (!p.dd) p.dd = stg_dout_ + at, p.stage_out = any_out = true;
      ps.push_back(p);
      at += n;
    }
  const size_t np = ps.size();
  std::unique_ptr<std::atomic<int>[]> landed(new std::atomic<int>[np]);
  for (size_t i = 0; i < np; ++i) landed[i].store(0, std::memory_order_relaxed);
  if (any_in)
    cpool_->start([&](int w, int nw) {
      for (size_t i = 0; i < np; ++i) {
        const P &p = ps[i];
        if (p.stage_in) {
          const size_t per = (p.len / nw + 63) & ~(size_t)63;
          const size_t b = std::min(p.len, per * (size_t)w), e = w == nw - 1 ? p.len : std::min(p.len, b + per);
          if (e > b) std::memcpy(stg_in_ + p.off + b, p.src + b, e - b);
        }
        landed[i].fetch_add(1, std::memory_order_release);
      }
    });
  const int nw = cpool_->workers();
  static const bool trace = env_or("VF_STAGE_TRACE", 0) != 0;  // per-call host timeline on stderr
  const auto t0 = std::chrono::steady_clock::now();
  auto us = [&] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(); };
  std::vector<double> tl;
  hipEvent_t a = take_event(), b = take_event();
  hipError_t e = (a && b) ? hipEventRecord(a, s_map_) : hipErrorOutOfMemory;
  MappedBatch mb;
  for (size_t i = 0; i < np && e == hipSuccess; ++i) {
    const P &p = ps[i];
    if (p.stage_in)
      while (landed[i].load(std::memory_order_acquire) < nw) std::this_thread::yield();
    if (trace) tl.push_back(us());
    mb.src[0] = p.ds;
    mb.dst[0] = p.dd;
    mb.n[0] = p.len;
    e = launch_invert_mapped(mb, 1, p.len, s_map_);
  }
  if (any_in) cpool_->join();  // also on a failed launch: the workers read the caller's buffers
  if (trace) tl.push_back(us());
  if (e == hipSuccess) e = hipEventRecord(b, s_map_);
  if (e == hipSuccess) e = hipEventSynchronize(b);
  if (trace) {
    tl.push_back(us());
    std::string line = "vf_stage: " + std::to_string(total) + " B, " + std::to_string(np) + " pieces; launch at";
    for (size_t i = 0; i + 2 < tl.size(); ++i) line += " " + std::to_string((int)tl[i]);
    line += " us; copy-in joined " + std::to_string((int)tl[tl.size() - 2]) + ", GPU done " + std::to_string((int)tl.back()) + " us";
    std::fprintf(stderr, "%s\n", line.c_str());
  }
  if (e == hipSuccess && any_out)
    for (const P &p : ps)
      if (p.stage_out) cpool_->copy(p.dst, stg_out_ + p.off, p.len);
  *out = JobResult();
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(s_map_);  // nothing may land in the caller's buffers later
    (void)hipGetLastError();
    out->status = kStatusHip;
    out->hip = e;
    out->msg = std::string("staged zero-copy launch failed: ") + hipGetErrorString(e);
  } else {
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = -1.f;
    out->kernel_ms = out->gpu_ms = ms;
    out->zero_copy = true;
    out->timeline.push_back(ChunkTime{total, 0.f, 0.f, ms, ms});
  }
  give_event(a);
  give_event(b);
  return true;
}

bool Engine::wait(uint64_t id, JobResult *out) {
  std::unique_lock<std::mutex> lk(mu_);
  if (id == 0 || id >= next_id_) return false;
  done_cv_.wait(lk, [&] { return unfinished_.count(id) == 0; });
  auto it = results_.find(id);
  if (it != results_.end()) {
    if (out) *out = std::move(it->second);
    results_.erase(it);
  } else if (out) {
    *out = JobResult();  // collected before, or trimmed after kMaxResults newer jobs
  }
  return true;
}

bool Engine::query(uint64_t id, bool *done) {
  std::lock_guard<std::mutex> lk(mu_);
  if (id == 0 || id >= next_id_) return false;
  *done = unfinished_.count(id) == 0;
  return true;
}

void Engine::drain() {
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return unfinished_.empty(); });
}

// ---- engine thread -----------------------------------------------------------------------

void Engine::fail_all(hipError_t e, const char *what) {
  // copies already queued for direct (caller-pinned) jobs may still be moving: let them land
  // before the callers hear of the failure and free or reuse their buffers
  for (hipStream_t st : {s_in_, s_out_, s_map_})
    if (st) (void)hipStreamSynchronize(st);
  (void)hipGetLastError();
  char buf[256];
  std::snprintf(buf, sizeof buf, "%s failed: %s (%s)", what, hipGetErrorString(e), hipGetErrorName(e));
  std::lock_guard<std::mutex> lk(mu_);
  broken_ = true;
  for (uint64_t id : unfinished_) {
    JobResult r;
    r.status = kStatusHip;
    r.hip = e;
    r.msg = buf;
    results_[id] = std::move(r);
  }
  unfinished_.clear();
  for (auto &s : slots_) {
    s.state = Slot::kFree;
    s.job = nullptr;
  }
  pending_.clear();
  live_.clear();
  mapped_live_.clear();
  done_cv_.notify_all();
}

// Bytes of the job's next chunk.  A job's first H2D and its last D2H overlap nothing, so the
// chunks ramp up (1, 2, 4, ... MiB up to the job's chunk size) and down (never more than half
// of what is left): the exposed ends shrink from a whole chunk each (16 MiB, ~0.35 ms at
// 48 GB/s, ~15 % of a 199 MB batch) to about 1 MiB.
size_t Engine::chunk_size(const Job &job) const {
  constexpr size_t kRamp = (size_t)1 << 20, kAlign = (size_t)1 << 16;
  const size_t left = job.total - job.queued;
  size_t want = std::min(job.chunk, kRamp << std::min(job.chunks_submitted, 16));
  if (left > kRamp) want = std::min(want, std::max(kRamp, (left / 2 + kAlign - 1) & ~(kAlign - 1)));
  return std::min(want, left);
}

bool Engine::step_fill() {
  Slot &s = slots_[fill_];
  Job *job = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (pending_.empty()) return false;
    job = pending_.front().get();
  }
  if (job->mapped) return launch_mapped(job);
  if (s.state != Slot::kFree) return false;
  hipError_t e = hipSuccess;
  if (!job->started) {
    job->start = take_event();
    if (!job->start) {
      fail_all(hipErrorOutOfMemory, "hipEventCreate");
      return true;
    }
    e = hipEventRecord(job->start, s_in_);
    job->started = true;
  }
  s.pieces.clear();
  size_t filled = 0;
  const size_t want = chunk_size(*job);
  job->queued += want;
  while (job->seg < job->segs.size() && filled < want) {
    const Seg &g = job->segs[job->seg];
    const size_t take = std::min(g.len - job->seg_off, want - filled);
    if (take) {
      if (!job->direct) pool_->copy(s.pin_in + filled, g.src + job->seg_off, take);
      s.pieces.push_back(Piece{g.src + job->seg_off, g.dst + job->seg_off, filled, take});
      filled += take;
      job->seg_off += take;
    }
    if (job->seg_off == g.len) {
      ++job->seg;
      job->seg_off = 0;
    }
  }
  if (e == hipSuccess) e = hipEventRecord(s.h0, s_in_);
  if (job->direct) {
    for (size_t i = 0; i < s.pieces.size() && e == hipSuccess; ++i)
      e = hipMemcpyAsync(s.d_in + s.pieces[i].off, s.pieces[i].src, s.pieces[i].len,
                         hipMemcpyHostToDevice, s_in_);
  } else if (e == hipSuccess) {
    e = hipMemcpyAsync(s.d_in, s.pin_in, filled, hipMemcpyHostToDevice, s_in_);
  }
  if (e == hipSuccess) e = hipEventRecord(s.k0, s_in_);
  if (e == hipSuccess) e = launch_invert(s.d_in, s.d_out, filled, cfg_, s_in_);
  if (e == hipSuccess) e = hipEventRecord(s.k1, s_in_);
  if (e != hipSuccess) {
    fail_all(e, "chunk submit");
    return true;
  }
  s.job = job;
  s.bytes = filled;
  s.state = Slot::kIn;
  ++job->chunks_submitted;
  fill_ = (fill_ + 1) % slots_.size();
  if (job->seg >= job->segs.size()) {  // every byte of the job is in a slot
    std::lock_guard<std::mutex> lk(mu_);
    job->all_submitted = true;
    live_.push_back(std::move(pending_.front()));
    pending_.pop_front();
  }
  return true;
}

bool Engine::step_d2h() {
  Slot &s = slots_[d2h_];
  if (s.state != Slot::kIn) return false;
  hipError_t err = hipSuccess;
  if (!fired(s.k1, &err)) {
    if (err != hipSuccess) fail_all(err, "hipEventQuery");
    return err != hipSuccess;
  }
  hipError_t e = hipSuccess;
  if (s.job->direct) {
    for (size_t i = 0; i < s.pieces.size() && e == hipSuccess; ++i)
      e = hipMemcpyAsync(s.pieces[i].dst, s.d_out + s.pieces[i].off, s.pieces[i].len,
                         hipMemcpyDeviceToHost, s_out_);
  } else {
    e = hipMemcpyAsync(s.pin_out, s.d_out, s.bytes, hipMemcpyDeviceToHost, s_out_);
  }
  if (e == hipSuccess) e = hipEventRecord(s.done, s_out_);
  if (e != hipSuccess) {
    fail_all(e, "D2H submit");
    return true;
  }
  s.state = Slot::kOut;
  d2h_ = (d2h_ + 1) % slots_.size();
  return true;
}

bool Engine::step_retire() {
  Slot &s = slots_[retire_];
  if (s.state != Slot::kOut) return false;
  hipError_t err = hipSuccess;
  if (!fired(s.done, &err)) {
    if (err != hipSuccess) fail_all(err, "hipEventQuery");
    return err != hipSuccess;
  }
  Job *job = s.job;
  if (!job->direct)
    for (const Piece &p : s.pieces) pool_->copy(p.dst, s.pin_out + p.off, p.len);
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, s.k0, s.k1) == hipSuccess) job->kernel_ms += ms;
  ChunkTime ct{s.bytes, -1.f, -1.f, -1.f, -1.f};
  hipEvent_t evs[4] = {s.h0, s.k0, s.k1, s.done};
  float *at[4] = {&ct.h2d_start, &ct.kernel_start, &ct.kernel_end, &ct.d2h_end};
  for (int i = 0; i < 4; ++i)
    if (hipEventElapsedTime(at[i], job->start, evs[i]) != hipSuccess) *at[i] = -1.f;
  job->timeline.push_back(ct);
  ++job->chunks_done;
  s.state = Slot::kFree;
  s.job = nullptr;
  retire_ = (retire_ + 1) % slots_.size();
  if (job->all_submitted && job->chunks_done == job->chunks_submitted) {
    JobResult r;
    r.kernel_ms = job->kernel_ms;
    r.gpu_ms = job->timeline.back().d2h_end;
    r.timeline = std::move(job->timeline);
    give_event(job->start);
    std::lock_guard<std::mutex> lk(mu_);
    results_[job->id] = std::move(r);
    while (results_.size() > kMaxResults) results_.erase(results_.begin());
    unfinished_.erase(job->id);
    for (auto it = live_.begin(); it != live_.end(); ++it)
      if (it->get() == job) {
        live_.erase(it);
        break;
      }
    done_cv_.notify_all();
  }
  return true;
}

// A zero-copy job: its ranges in launches of up to kMappedMax on the mapped stream, between a
// start and an end event; no slot, no staging.
bool Engine::launch_mapped(Job *job) {
  job->start = take_event();
  job->end = take_event();
  if (!job->start || !job->end) {
    fail_all(hipErrorOutOfMemory, "hipEventCreate");
    return true;
  }
  hipError_t e = hipEventRecord(job->start, s_map_);
  MappedBatch b;
  for (size_t i = 0; i < job->dsegs.size() && e == hipSuccess; i += kMappedMax) {
    const int n = (int)std::min<size_t>(kMappedMax, job->dsegs.size() - i);
    size_t bytes = 0;
    for (int k = 0; k < n; ++k) {
      const Seg &g = job->dsegs[i + k];
      b.src[k] = g.src;
      b.dst[k] = g.dst;
      b.n[k] = g.len;
      bytes += g.len;
    }
    e = launch_invert_mapped(b, n, bytes, s_map_);
  }
  if (e == hipSuccess) e = hipEventRecord(job->end, s_map_);
  if (e != hipSuccess) {
    fail_all(e, "zero-copy launch");
    return true;
  }
  job->started = job->all_submitted = true;
  std::lock_guard<std::mutex> lk(mu_);
  mapped_live_.push_back(job);
  live_.push_back(std::move(pending_.front()));
  pending_.pop_front();
  return true;
}

bool Engine::step_mapped_retire() {
  if (mapped_live_.empty()) return false;
  Job *job = mapped_live_.front();
  hipError_t err = hipSuccess;
  if (!fired(job->end, &err)) {
    if (err != hipSuccess) fail_all(err, "hipEventQuery");
    return err != hipSuccess;
  }
  float ms = -1.f;
  if (hipEventElapsedTime(&ms, job->start, job->end) != hipSuccess) ms = -1.f;
  JobResult r;
  r.kernel_ms = ms;
  r.gpu_ms = ms;
  r.zero_copy = true;
  r.timeline.push_back(ChunkTime{job->total, 0.f, 0.f, ms, ms});  // one launch does all of it
  give_event(job->start);
  give_event(job->end);
  std::lock_guard<std::mutex> lk(mu_);
  mapped_live_.pop_front();
  results_[job->id] = std::move(r);
  while (results_.size() > kMaxResults) results_.erase(results_.begin());
  unfinished_.erase(job->id);
  for (auto it = live_.begin(); it != live_.end(); ++it)
    if (it->get() == job) {
      live_.erase(it);
      break;
    }
  done_cv_.notify_all();
  return true;
}

// Called from the engine thread and from run_now on the caller's thread (a synchronous
// zero-copy call while async jobs are in flight), so the free list is locked.
hipEvent_t Engine::take_event() {
  {
    std::lock_guard<std::mutex> lk(ev_mu_);
    if (!free_events_.empty()) {
      hipEvent_t e = free_events_.back();
      free_events_.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

void Engine::give_event(hipEvent_t e) {
  if (!e) return;
  std::lock_guard<std::mutex> lk(ev_mu_);
  free_events_.push_back(e);
}

int Engine::busy_slots() const {
  int n = 0;
  for (const auto &s : slots_) n += s.state != Slot::kFree;
  return n;
}

void Engine::run() {
  (void)hipSetDevice(device_);
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !pending_.empty() || busy_slots() > 0 || !mapped_live_.empty(); });
      if (stop_ && pending_.empty() && busy_slots() == 0 && mapped_live_.empty()) return;
    }
    if (!streams_ready_.load(std::memory_order_acquire)) {
      const hipError_t e = ensure_streams();
      if (e != hipSuccess) {
        fail_all(e, "stream creation");
        continue;
      }
    }
    bool progress = false;
    // retire first (frees a slot), then start the D2H of finished kernels, then refill
    while (step_retire()) progress = true;
    while (step_mapped_retire()) progress = true;
    while (step_d2h()) progress = true;
    while (step_fill()) progress = true;
    if (!progress) std::this_thread::yield();
  }
}

}  // namespace vf
