// vf_api.hip — C ABI of libvfilter_hip.so (declared in include/vfilter.h).
//
// Host side of the MI355X frame filter.  What it replaces in the reference:
//   * InverterWorker per-process state          inverter.py:10-20   -> vf_create / vf_destroy
//   * cv2.bitwise_not(frame) on one frame       inverter.py:41      -> vf_invert_host
//   * the one-frame-per-iteration worker loop   worker.py:35-57     -> vf_invert_batch_host,
//                                                                      vf_invert_frames_host,
//                                                                      vf_invert_frames_async
// Every host->host call becomes a job of the context's Engine (vf_engine.hip): a thread that
// streams the job's bytes through a ring of device slots (H2D on one SDMA engine, the invert
// kernel, D2H on the other) without draining between jobs.  Synchronous entry points submit
// and wait; the asynchronous one returns a ticket.  Pageable caller memory is staged through
// pinned slot buffers by a host copy pool; page-locked caller memory (vf_alloc_host,
// vf_host_register — e.g. a shared-memory frame ring) is DMA'd directly with no host copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/vfilter.h"
#include "vf_host_mem.h"
#include "vf_internal.h"
#include "vf_jpeg_codec.h"

#define VF_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kMaxSlots = 8;

struct ErrState {
  int hip = 0;
  char msg[512] = "no error";
};
thread_local ErrState g_thread_err;

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
  vf::LaunchCfg cfg;
  vf::Engine *engine = nullptr;
  int hip = 0;
  char msg[512] = "no error";
  std::mutex err_mu;  // msg / hip: JPEG calls on one context may fail on two threads at once
  // results of the last host->host job waited on (vf_elapsed_ms / vf_last_timeline)
  float last_kernel_ms = 0.f;
  std::vector<vf::ChunkTime> timeline;
  // JPEG codecs (created on first use, at most VF_JPEG_CODECS, default 2): each has its own
  // stream and buffers, so JPEG calls from two host threads overlap one batch's host work
  // (parse, staging, copy-out) with the other's GPU work.
  std::mutex jpeg_mu;
  std::condition_variable jpeg_cv;
  std::vector<vf::jpeg::Codec *> jpeg_all, jpeg_free;
  vf::jpeg::ComputeGate jpeg_gate;
  // submitted vf_jpeg_invert_submit batches: ticket -> the codec that holds it until fetched
  std::map<uint64_t, vf::jpeg::Codec *> jpeg_jobs;
  uint64_t jpeg_next_ticket = 1;
  // decoder frame-size limit (vf_jpeg_set_max_pixels), applied to a codec whenever it is leased
  std::atomic<uint64_t> jpeg_max_pixels{vf::jpeg::kDefaultMaxPixels};
  // vf_bench_device_ring's region events, created once (not inside a caller's timed region)
  hipEvent_t bench_ev[2] = {nullptr, nullptr};
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
    std::lock_guard<std::mutex> lk(ctx->err_mu);
    ctx->hip = hip;
    std::snprintf(ctx->msg, sizeof ctx->msg, "%s", buf);
  }
  return status;
}

int fail_hip(vf_ctx *ctx, hipError_t e, const char *what, int line) {
  return set_err(ctx, VF_E_HIP, (int)e, "%s failed: %s (%s, vf_api.hip:%d)", what,
                 hipGetErrorString(e), hipGetErrorName(e), line);
}

#define VF_HIP(ctx, call)                                              \
  do {                                                                 \
    hipError_t e_ = (call);                                            \
    if (e_ != hipSuccess) return fail_hip((ctx), e_, #call, __LINE__); \
  } while (0)

#define VF_CHECK_CTX(ctx)                                                             \
  do {                                                                                \
    if (!(ctx)) return set_err(nullptr, VF_E_INVALID, 0, "%s: ctx is NULL", __func__); \
  } while (0)

bool overlaps_partially(const uint8_t *a, const uint8_t *b, size_t n) {
  if (a == b || n == 0) return false;
  return (a < b + n) && (b < a + n);
}

// Wait for a job and publish its result on the context.
int finish(vf_ctx *ctx, uint64_t id, float *gpu_ms) {
  vf::JobResult r;
  if (!ctx->engine->wait(id, &r))
    return set_err(ctx, VF_E_INVALID, 0, "vf_wait: unknown ticket %llu", (unsigned long long)id);
  if (gpu_ms) *gpu_ms = r.gpu_ms;
  ctx->last_kernel_ms = r.kernel_ms;
  ctx->timeline = std::move(r.timeline);
  if (r.status != VF_OK) return set_err(ctx, r.status, (int)r.hip, "%s", r.msg.c_str());
  return VF_OK;
}

// Validate a frame list into engine segments (empty frames dropped).
int frames_to_segs(vf_ctx *ctx, const char *fn, const uint8_t *const *srcs, uint8_t *const *dsts,
                   const size_t *nbytes, int n, std::vector<vf::Seg> *segs) {
  if (n < 0) return set_err(ctx, VF_E_INVALID, 0, "%s: n < 0", fn);
  if (n > 0 && (!srcs || !dsts || !nbytes)) return set_err(ctx, VF_E_INVALID, 0, "%s: NULL array", fn);
  segs->reserve((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (nbytes[i] == 0) continue;
    if (!srcs[i] || !dsts[i]) return set_err(ctx, VF_E_INVALID, 0, "%s: frame %d has a NULL buffer", fn, i);
    if (overlaps_partially(srcs[i], dsts[i], nbytes[i]))
      return set_err(ctx, VF_E_INVALID, 0, "%s: frame %d src/dst partially overlap", fn, i);
    segs->push_back(vf::Seg{srcs[i], dsts[i], nbytes[i]});
  }
  return VF_OK;
}

int run_sync(vf_ctx *ctx, std::vector<vf::Seg> &&segs) {
  if (segs.empty()) {
    ctx->last_kernel_ms = 0.f;
    ctx->timeline.clear();
    return VF_OK;
  }
  vf::JobResult r;
  if (ctx->engine->run_now(segs, &r)) {  // page-locked, device-mapped: launched from this thread
    ctx->last_kernel_ms = r.kernel_ms;
    ctx->timeline = std::move(r.timeline);
    if (r.status != VF_OK) return set_err(ctx, r.status, (int)r.hip, "%s", r.msg.c_str());
    return VF_OK;
  }
  return finish(ctx, ctx->engine->submit(std::move(segs)), nullptr);
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
    case VF_E_JPEG: return "VF_E_JPEG: malformed or unsupported JPEG";
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

VF_EXPORT int vf_device_pci_bus_id(int device, char *buf, int len) {
  if (!buf || len < 13) return set_err(nullptr, VF_E_INVALID, 0, "vf_device_pci_bus_id: buffer too small");
  buf[0] = 0;
  int ndev = 0;
  vf_device_count(&ndev);
  if (device < 0 || device >= ndev)
    return set_err(nullptr, VF_E_NODEVICE, 0, "vf_device_pci_bus_id: device %d not available (%d visible)",
                   device, ndev);
  hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
  if (e != hipSuccess) return fail_hip(nullptr, e, "hipDeviceGetPCIBusId", __LINE__);
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
  ctx->cfg.max_blocks = (int)env_size("VF_MAX_BLOCKS", (size_t)ctx->num_cus * 32);
  if (ctx->cfg.max_blocks < 1) ctx->cfg.max_blocks = ctx->num_cus * 32;
  const int nslots = (int)std::min<size_t>(kMaxSlots, std::max<size_t>(2, env_size("VF_SLOTS", 4)));
  size_t want = max_frame_bytes ? max_frame_bytes * (size_t)max_batch : (size_t)8 << 20;
  size_t slot = env_size("VF_SLOT_BYTES", std::min(want, (size_t)16 << 20));
  slot = std::max<size_t>(slot, (size_t)1 << 20);
  slot = std::min<size_t>(slot, (size_t)64 << 20);
  slot = (slot + 4095) & ~(size_t)4095;
  ctx->engine = new (std::nothrow) vf::Engine();
  std::string err;
  e = ctx->engine ? ctx->engine->init(device, nslots, slot, ctx->cfg, &err) : hipErrorOutOfMemory;
  if (e != hipSuccess) {
    int st = (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? VF_E_NOMEM : VF_E_HIP;
    set_err(nullptr, st, (int)e, "vf_create: %s", err.empty() ? hipGetErrorString(e) : err.c_str());
    delete ctx->engine;
    delete ctx;
    return st;
  }
  *out = ctx;
  return VF_OK;
}

VF_EXPORT int vf_destroy(vf_ctx *ctx) {
  if (!ctx) return VF_OK;
  for (vf::jpeg::Codec *c : ctx->jpeg_all) delete c;  // each synchronises its stream first
  delete ctx->engine;  // finishes queued jobs first
  for (hipEvent_t e : ctx->bench_ev)
    if (e) (void)hipEventDestroy(e);
  delete ctx;
  return VF_OK;
}

VF_EXPORT const char *vf_last_error(const vf_ctx *ctx) { return ctx ? ctx->msg : g_thread_err.msg; }

VF_EXPORT int vf_last_hip_error(const vf_ctx *ctx) { return ctx ? ctx->hip : g_thread_err.hip; }

VF_EXPORT int vf_ctx_device(const vf_ctx *ctx, int *out_device) {
  if (!ctx || !out_device) return set_err(nullptr, VF_E_INVALID, 0, "vf_ctx_device: NULL argument");
  *out_device = ctx->device;
  return VF_OK;
}

// ---- host -> host ----------------------------------------------------------------------

VF_EXPORT int vf_invert_host(vf_ctx *ctx, const uint8_t *src, uint8_t *dst, size_t nbytes) {
  VF_CHECK_CTX(ctx);
  if (nbytes && (!src || !dst)) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_host: NULL buffer");
  if (overlaps_partially(src, dst, nbytes))
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_host: src and dst partially overlap");
  std::vector<vf::Seg> segs;
  if (nbytes) segs.push_back(vf::Seg{src, dst, nbytes});
  return run_sync(ctx, std::move(segs));
}

VF_EXPORT int vf_invert_batch_host(vf_ctx *ctx, const uint8_t *src, uint8_t *dst,
                                   size_t frame_bytes, int n) {
  VF_CHECK_CTX(ctx);
  if (n < 0) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_batch_host: n < 0");
  if (n && frame_bytes > SIZE_MAX / (size_t)n)
    return set_err(ctx, VF_E_INVALID, 0, "vf_invert_batch_host: size overflow");
  return vf_invert_host(ctx, src, dst, frame_bytes * (size_t)n);
}

VF_EXPORT int vf_invert_frames_host(vf_ctx *ctx, const uint8_t *const *srcs, uint8_t *const *dsts,
                                    const size_t *nbytes, int n) {
  VF_CHECK_CTX(ctx);
  std::vector<vf::Seg> segs;
  int rc = frames_to_segs(ctx, "vf_invert_frames_host", srcs, dsts, nbytes, n, &segs);
  return rc != VF_OK ? rc : run_sync(ctx, std::move(segs));
}

VF_EXPORT int vf_invert_frames_async(vf_ctx *ctx, const uint8_t *const *srcs, uint8_t *const *dsts,
                                     const size_t *nbytes, int n, uint64_t *ticket) {
  VF_CHECK_CTX(ctx);
  if (!ticket) return set_err(ctx, VF_E_INVALID, 0, "vf_invert_frames_async: ticket is NULL");
  *ticket = 0;
  std::vector<vf::Seg> segs;
  int rc = frames_to_segs(ctx, "vf_invert_frames_async", srcs, dsts, nbytes, n, &segs);
  if (rc != VF_OK) return rc;
  *ticket = ctx->engine->submit(std::move(segs));
  return VF_OK;
}

VF_EXPORT int vf_wait(vf_ctx *ctx, uint64_t ticket, float *gpu_ms) {
  VF_CHECK_CTX(ctx);
  if (gpu_ms) *gpu_ms = -1.f;
  return finish(ctx, ticket, gpu_ms);
}

VF_EXPORT int vf_query(vf_ctx *ctx, uint64_t ticket, int *done) {
  VF_CHECK_CTX(ctx);
  if (!done) return set_err(ctx, VF_E_INVALID, 0, "vf_query: done is NULL");
  bool d = false;
  if (!ctx->engine->query(ticket, &d))
    return set_err(ctx, VF_E_INVALID, 0, "vf_query: unknown ticket %llu", (unsigned long long)ticket);
  *done = d ? 1 : 0;
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
  hipError_t e = vf::numa_pinned_alloc(out, nbytes ? nbytes : 1, vf::device_numa_node(ctx->device));
  if (e != hipSuccess)
    return set_err(ctx, VF_E_NOMEM, (int)e, "pinned allocation of %zu bytes failed: %s", nbytes, hipGetErrorString(e));
  ctx->engine->note_pinned(*out, nbytes ? nbytes : 1);
  return VF_OK;
}

VF_EXPORT int vf_free_host(vf_ctx *ctx, void *p) {
  VF_CHECK_CTX(ctx);
  if (!p) return VF_OK;
  ctx->engine->drain();  // a queued job may still read or write it
  ctx->engine->forget_pinned(p);
  VF_HIP(ctx, vf::numa_pinned_free(p));
  return VF_OK;
}

VF_EXPORT int vf_host_register(vf_ctx *ctx, void *p, size_t nbytes) {
  VF_CHECK_CTX(ctx);
  if (!p || !nbytes) return set_err(ctx, VF_E_INVALID, 0, "vf_host_register: empty range");
  VF_HIP(ctx, hipSetDevice(ctx->device));
  VF_HIP(ctx, hipHostRegister(p, nbytes, hipHostRegisterMapped));
  ctx->engine->note_pinned(p, nbytes);
  return VF_OK;
}

VF_EXPORT int vf_host_unregister(vf_ctx *ctx, void *p) {
  VF_CHECK_CTX(ctx);
  if (!p) return VF_OK;
  ctx->engine->drain();
  ctx->engine->forget_pinned(p);
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
    ctx->engine->drain();
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
    const vf::ChunkTime &t = ctx->timeline[(size_t)i];
    if (out4) {
      out4[4 * i + 0] = t.h2d_start;
      out4[4 * i + 1] = t.kernel_start;
      out4[4 * i + 2] = t.kernel_end;
      out4[4 * i + 3] = t.d2h_end;
    }
    if (chunk_bytes) chunk_bytes[i] = t.bytes;
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
  std::vector<hipEvent_t> ev(each ? 2 * (size_t)steps : 0, nullptr);
  int rc = VF_OK;
  for (auto &e : ev) {
    hipError_t h = hipEventCreate(&e);
    if (h != hipSuccess) { rc = fail_hip(ctx, h, "hipEventCreate", __LINE__); break; }
  }
  // the region pair is the context's, created by the first call (the warm-up): a timed call
  // then only records, launches and synchronises
  for (hipEvent_t &e : ctx->bench_ev) {
    if (rc != VF_OK || e) continue;
    hipError_t h = hipEventCreate(&e);
    if (h != hipSuccess) rc = fail_hip(ctx, h, "hipEventCreate", __LINE__);
  }
  hipEvent_t r0 = ctx->bench_ev[0], r1 = ctx->bench_ev[1];
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

// ---- JPEG (inverter.py:32 / :41 / :44 in the default use_jpeg=True mode) --------------------

namespace {

// A codec leased to one call for its duration (blocks while all codecs are busy).
class CodecLease {
 public:
  explicit CodecLease(vf_ctx *ctx) : ctx_(ctx) {
    static const size_t kMax = std::max<size_t>(1, env_size("VF_JPEG_CODECS", 2));
    std::unique_lock<std::mutex> lk(ctx->jpeg_mu);
    ctx->jpeg_cv.wait(lk, [&] { return !ctx->jpeg_free.empty() || ctx->jpeg_all.size() < kMax; });
    if (!ctx->jpeg_free.empty()) {
      c_ = ctx->jpeg_free.back();
      ctx->jpeg_free.pop_back();
    } else {
      static const bool gated = env_size("VF_JPEG_GATE", 0) != 0;
      c_ = new (std::nothrow) vf::jpeg::Codec(ctx->device, gated ? &ctx->jpeg_gate : nullptr);
      if (c_) ctx->jpeg_all.push_back(c_);
    }
    if (c_) c_->set_max_pixels(ctx->jpeg_max_pixels.load());
  }
  ~CodecLease() {
    if (!c_) return;
    c_->quiesce();  // a failed call may have left work queued (no-op after a success)
    {
      std::lock_guard<std::mutex> lk(ctx_->jpeg_mu);
      ctx_->jpeg_free.push_back(c_);
    }
    ctx_->jpeg_cv.notify_one();
  }
  CodecLease(const CodecLease &) = delete;
  CodecLease &operator=(const CodecLease &) = delete;
  vf::jpeg::Codec *get() const { return c_; }

 private:
  vf_ctx *ctx_;
  vf::jpeg::Codec *c_ = nullptr;
};

// A codec for an asynchronous batch: never blocks (the caller thread may be the one that would
// fetch the batches holding the others); a new codec when none is free, up to kMaxJpegJobs.
constexpr size_t kMaxJpegJobs = 8;
vf::jpeg::Codec *lease_nowait(vf_ctx *ctx) {
  std::lock_guard<std::mutex> lk(ctx->jpeg_mu);
  vf::jpeg::Codec *c = nullptr;
  if (!ctx->jpeg_free.empty()) {
    c = ctx->jpeg_free.back();
    ctx->jpeg_free.pop_back();
  } else if (ctx->jpeg_all.size() < kMaxJpegJobs) {
    static const bool gated = env_size("VF_JPEG_GATE", 0) != 0;
    c = new (std::nothrow) vf::jpeg::Codec(ctx->device, gated ? &ctx->jpeg_gate : nullptr);
    if (c) ctx->jpeg_all.push_back(c);
  }
  if (c) c->set_max_pixels(ctx->jpeg_max_pixels.load());
  return c;
}

void give_back(vf_ctx *ctx, vf::jpeg::Codec *c) {
  {
    std::lock_guard<std::mutex> lk(ctx->jpeg_mu);
    ctx->jpeg_free.push_back(c);
  }
  ctx->jpeg_cv.notify_one();
}

vf::jpeg::Codec *job_codec(vf_ctx *ctx, uint64_t ticket) {
  std::lock_guard<std::mutex> lk(ctx->jpeg_mu);
  auto it = ctx->jpeg_jobs.find(ticket);
  return it == ctx->jpeg_jobs.end() ? nullptr : it->second;
}

void end_job(vf_ctx *ctx, uint64_t ticket) {
  vf::jpeg::Codec *c = nullptr;
  {
    std::lock_guard<std::mutex> lk(ctx->jpeg_mu);
    auto it = ctx->jpeg_jobs.find(ticket);
    if (it == ctx->jpeg_jobs.end()) return;
    c = it->second;
    ctx->jpeg_jobs.erase(it);
  }
  c->quiesce();
  give_back(ctx, c);
}

int jpeg_codec(vf_ctx *ctx, const CodecLease &lease, vf::jpeg::Codec **out) {
  if (!lease.get()) return set_err(ctx, VF_E_NOMEM, 0, "JPEG codec: out of host memory");
  *out = lease.get();
  return VF_OK;
}

int jpeg_status(vf_ctx *ctx, int rc, const std::string &msg) {
  if (rc == VF_OK) return VF_OK;
  return set_err(ctx, rc, 0, "%s", msg.c_str());
}

}  // namespace

VF_EXPORT int vf_jpeg_header(const uint8_t *jpeg, size_t size, int *width, int *height, int *subsamp,
                             int *colorspace) {
  if (!width || !height || !subsamp || !colorspace)
    return set_err(nullptr, VF_E_INVALID, 0, "vf_jpeg_header: NULL output pointer");
  std::string err;
  const int rc = vf::jpeg::header_info(jpeg, size, width, height, subsamp, colorspace, &err);
  return rc == VF_OK ? VF_OK : set_err(nullptr, rc, 0, "vf_jpeg_header: %s", err.c_str());
}

VF_EXPORT int vf_jpeg_set_max_pixels(vf_ctx *ctx, uint64_t max_pixels) {
  if (!ctx) return set_err(nullptr, VF_E_INVALID, 0, "vf_jpeg_set_max_pixels: NULL context");
  ctx->jpeg_max_pixels.store(max_pixels ? max_pixels : vf::jpeg::kDefaultMaxPixels);
  return VF_OK;
}

VF_EXPORT size_t vf_jpeg_buffer_size(int width, int height, int subsamp) {
  return vf::jpeg::buffer_size(width, height, subsamp);
}

VF_EXPORT int vf_jpeg_encode(vf_ctx *ctx, const uint8_t *const *imgs, const int *widths, const int *heights, int n,
                             int pixel_format, int quality, int subsamp, int flags, uint8_t *const *outs,
                             const size_t *caps, size_t *sizes) {
  VF_CHECK_CTX(ctx);
  if (n < 0 || (n > 0 && (!imgs || !widths || !heights || !outs || !caps || !sizes)))
    return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_encode: bad arguments");
  if (n > 65535) return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_encode: at most 65535 frames per call");
  CodecLease lease(ctx);
  vf::jpeg::Codec *c = nullptr;
  int rc = jpeg_codec(ctx, lease, &c);
  if (rc) return rc;
  std::string err;
  rc = c->encode(imgs, widths, heights, n, pixel_format, quality, subsamp, flags, outs, caps, sizes, &err);
  return jpeg_status(ctx, rc, "vf_jpeg_encode: " + err);
}

VF_EXPORT int vf_jpeg_decode(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n,
                             int pixel_format, int flags, uint8_t *const *outs, const size_t *caps) {
  VF_CHECK_CTX(ctx);
  if (n < 0 || (n > 0 && (!jpegs || !jpeg_sizes || !outs || !caps)))
    return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_decode: bad arguments");
  if (n > 65535) return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_decode: at most 65535 frames per call");
  CodecLease lease(ctx);
  vf::jpeg::Codec *c = nullptr;
  int rc = jpeg_codec(ctx, lease, &c);
  if (rc) return rc;
  std::string err;
  rc = c->decode(jpegs, jpeg_sizes, n, pixel_format, flags, outs, caps, &err);
  return jpeg_status(ctx, rc, "vf_jpeg_decode: " + err);
}

VF_EXPORT int vf_jpeg_invert(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n, int quality,
                             int subsamp, int flags, uint8_t *const *outs, const size_t *caps, size_t *sizes) {
  VF_CHECK_CTX(ctx);
  if (n < 0 || (n > 0 && (!jpegs || !jpeg_sizes || !outs || !caps || !sizes)))
    return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert: bad arguments");
  if (n > 65535) return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert: at most 65535 frames per call");
  CodecLease lease(ctx);
  vf::jpeg::Codec *c = nullptr;
  int rc = jpeg_codec(ctx, lease, &c);
  if (rc) return rc;
  std::string err;
  rc = c->invert(jpegs, jpeg_sizes, n, quality, subsamp, flags, outs, caps, sizes, &err);
  return jpeg_status(ctx, rc, "vf_jpeg_invert: " + err);
}

VF_EXPORT int vf_jpeg_invert_submit(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n,
                                    int quality, int subsamp, int flags, uint64_t *ticket) {
  VF_CHECK_CTX(ctx);
  if (!ticket || n <= 0 || n > 65535 || !jpegs || !jpeg_sizes)
    return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert_submit: bad arguments");
  *ticket = 0;
  vf::jpeg::Codec *c = lease_nowait(ctx);
  if (!c)
    return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert_submit: %zu batches already in flight; fetch one first",
                   kMaxJpegJobs);
  std::string err;
  const int rc = c->submit_invert(jpegs, jpeg_sizes, n, quality, subsamp, flags, &err);
  if (rc != VF_OK) {
    c->quiesce();  // a submit that failed after queueing work must not hand the codec on mid-flight
    give_back(ctx, c);
    return jpeg_status(ctx, rc, "vf_jpeg_invert_submit: " + err);
  }
  std::lock_guard<std::mutex> lk(ctx->jpeg_mu);
  *ticket = ctx->jpeg_next_ticket++;
  ctx->jpeg_jobs[*ticket] = c;
  return VF_OK;
}

VF_EXPORT int vf_jpeg_invert_query(vf_ctx *ctx, uint64_t ticket, int *done) {
  VF_CHECK_CTX(ctx);
  vf::jpeg::Codec *c = job_codec(ctx, ticket);
  if (!c || !done) return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert_query: unknown ticket %llu",
                                  (unsigned long long)ticket);
  *done = c->done_invert() ? 1 : 0;
  return VF_OK;
}

VF_EXPORT int vf_jpeg_invert_wait(vf_ctx *ctx, uint64_t ticket, size_t *total) {
  VF_CHECK_CTX(ctx);
  vf::jpeg::Codec *c = job_codec(ctx, ticket);
  if (!c || !total) return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert_wait: unknown ticket %llu",
                                   (unsigned long long)ticket);
  std::string err;
  const int rc = c->wait_invert(total, &err);
  if (rc != VF_OK) end_job(ctx, ticket);  // a failed batch is over: its codec is free again
  return jpeg_status(ctx, rc, "vf_jpeg_invert_wait: " + err);
}

VF_EXPORT int vf_jpeg_invert_fetch(vf_ctx *ctx, uint64_t ticket, uint8_t *out, size_t cap, size_t *sizes,
                                   size_t *offsets) {
  VF_CHECK_CTX(ctx);
  vf::jpeg::Codec *c = job_codec(ctx, ticket);
  if (!c) return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert_fetch: unknown ticket %llu", (unsigned long long)ticket);
  std::string err;
  int rc = VF_OK;
  if (!c->waited()) {  // fetch without wait: wait here (out == NULL just releases the batch)
    size_t total = 0;
    rc = c->wait_invert(&total, &err);
  }
  if (rc == VF_OK) rc = c->fetch_invert(out, cap, sizes, offsets, &err);
  if (rc == VF_E_INVALID && out && cap) return jpeg_status(ctx, rc, "vf_jpeg_invert_fetch: " + err);  // retry with room
  end_job(ctx, ticket);
  return jpeg_status(ctx, rc, "vf_jpeg_invert_fetch: " + err);
}

VF_EXPORT int vf_jpeg_invert_scatter(vf_ctx *ctx, uint64_t ticket, uint8_t *const *outs, const size_t *caps,
                                     size_t *sizes, int *placed) {
  VF_CHECK_CTX(ctx);
  vf::jpeg::Codec *c = job_codec(ctx, ticket);
  if (!c || !outs || !caps || !sizes || !placed)
    return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert_scatter: unknown ticket %llu or NULL argument",
                   (unsigned long long)ticket);
  if (!c->waited()) return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_invert_scatter: call vf_jpeg_invert_wait first");
  return jpeg_status(ctx, c->scatter_invert(outs, caps, sizes, placed), "vf_jpeg_invert_scatter");
}

VF_EXPORT int vf_jpeg_bench_invert(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n,
                                   int quality, int subsamp, int flags, int iters, float *ms, float *stage_ms) {
  VF_CHECK_CTX(ctx);
  if (n <= 0 || n > 65535 || !jpegs || !jpeg_sizes || !ms || iters <= 0)
    return set_err(ctx, VF_E_INVALID, 0, "vf_jpeg_bench_invert: bad arguments");
  CodecLease lease(ctx);
  vf::jpeg::Codec *c = nullptr;
  int rc = jpeg_codec(ctx, lease, &c);
  if (rc) return rc;
  std::string err;
  rc = c->bench_invert(jpegs, jpeg_sizes, n, quality, subsamp, flags, iters, ms, stage_ms, &err);
  return jpeg_status(ctx, rc, "vf_jpeg_bench_invert: " + err);
}
