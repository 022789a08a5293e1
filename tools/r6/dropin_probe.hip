// dropin_probe.hip — where the per-frame drop-in's time goes above the PCIe floor.
//
// One 1080p frame (6,220,800 B) inverted host -> host by a zero-copy kernel (page-locked source
// and destination mapped into the GPU's address space, as vf_invert_host does for page-locked
// buffers).  Per variant, over `reps` calls: host wall per call (launch + wait), the hipEvent
// span around the launch, and the kernel's own span from wall_clock64() stamps written by every
// workgroup (first start, last end, and when 10 / 50 / 90 % of the workgroups had finished).
// Rows: an empty kernel (the launch + wait floor), the invert kernel over grid x unroll, the
// three ways of waiting (event synchronize, stream synchronize, spinning on event query),
// and the SDMA copies of the same frame one way each.
//
//   tools/r6/dropin_probe [reps]      (one JSON object per row on stdout)
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/vfilter.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void k_empty(unsigned long long *st) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && st) st[0] = wall_clock64();
}

// stamps: [2 * blockIdx.x] = start, [2 * blockIdx.x + 1] = end
typedef unsigned int v4 __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void k_zc(const v4 *__restrict__ s, v4 *__restrict__ d, size_t n16,
                                            unsigned long long *stamps) {
  const unsigned long long t0 = wall_clock64();
  const size_t stride = (size_t)gridDim.x * 256 * U;
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < n16; i += stride) {
    v4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(~v[u], d + i + u * 256);
  }
  for (; i < n16; i += 256) {
    const v4 v = __builtin_nontemporal_load(s + i);
    __builtin_nontemporal_store(~v, d + i);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = wall_clock64();
  }
}


// page-locked host memory of one kind: hipHostMalloc, or mmap + hipHostRegister on 4 KiB pages
// (the product's numa_pinned_alloc), or the same on transparent huge pages
static uint8_t *host_alloc(int kind, size_t n) {
  if (kind == 0) {
    void *p = nullptr;
    CK(hipHostMalloc(&p, n, hipHostMallocMapped));
    return (uint8_t *)p;
  }
  const size_t len = (n + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
  void *raw = mmap(nullptr, len + (2u << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (raw == MAP_FAILED) std::exit(2);
  uint8_t *p = (uint8_t *)(((uintptr_t)raw + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
  madvise(p, len, kind == 2 ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
  std::memset(p, 0, len);
  CK(hipHostRegister(p, len, hipHostRegisterMapped));
  return p;
}
static const char *kind_name(int k) { return k == 0 ? "hostmalloc" : k == 1 ? "registered_4k" : "registered_thp"; }

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
  if (v.empty()) return -1;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

enum Wait { kEventSync, kStreamSync, kSpin };
static const char *wait_name(Wait w) { return w == kEventSync ? "event_sync" : w == kStreamSync ? "stream_sync" : "spin_query"; }

static void wait_for(Wait w, hipEvent_t e, hipStream_t s) {
  if (w == kEventSync) CK(hipEventSynchronize(e));
  else if (w == kStreamSync) CK(hipStreamSynchronize(s));
  else
    while (hipEventQuery(e) == hipErrorNotReady) {
    }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const size_t nbytes = 1080ull * 1920 * 3;
  const size_t n16 = nbytes / 16;
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
  const double us_per_tick = 1000.0 / clk_khz;
  uint8_t *hs, *hd;
  CK(hipHostMalloc((void **)&hs, nbytes, hipHostMallocMapped));
  CK(hipHostMalloc((void **)&hd, nbytes, hipHostMallocMapped));
  for (size_t i = 0; i < nbytes; ++i) hs[i] = (uint8_t)(i * 2654435761u >> 13);
  uint8_t *ds, *dd, *dbuf;
  CK(hipHostGetDevicePointer((void **)&ds, hs, 0));
  CK(hipHostGetDevicePointer((void **)&dd, hd, 0));
  CK(hipMalloc((void **)&dbuf, nbytes));
  unsigned long long *stamps;
  CK(hipMalloc((void **)&stamps, 2 * 4096 * sizeof(unsigned long long)));
  std::vector<unsigned long long> hst(2 * 4096);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));

  // the launch + wait floor
  for (Wait w : {kEventSync, kStreamSync, kSpin}) {
    std::vector<double> wall, ev;
    for (int r = 0; r < reps + 10; ++r) {
      const double t = now_us();
      CK(hipEventRecord(a, s));
      hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, (unsigned long long *)nullptr);
      CK(hipEventRecord(b, s));
      wait_for(w, b, s);
      const double el = now_us() - t;
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r >= 10) wall.push_back(el), ev.push_back(ms * 1000.0);
    }
    std::printf("{\"row\": \"empty_kernel\", \"wait\": \"%s\", \"wall_us\": %.1f, \"event_us\": %.1f}\n", wait_name(w),
                median(wall), median(ev));
  }

  auto run_zc = [&](int grid, int unroll, Wait w, const char *tag) {
    std::vector<double> wall, ev, span, lat0, p10, p50, p90, first_end;
    bool ok = true;
    for (int r = 0; r < reps + 10; ++r) {
      const double t = now_us();
      CK(hipEventRecord(a, s));
      if (unroll == 1) hipLaunchKernelGGL(k_zc<1>, dim3(grid), dim3(256), 0, s, (const v4 *)ds, (v4 *)dd, n16, stamps);
      else if (unroll == 2) hipLaunchKernelGGL(k_zc<2>, dim3(grid), dim3(256), 0, s, (const v4 *)ds, (v4 *)dd, n16, stamps);
      else hipLaunchKernelGGL(k_zc<4>, dim3(grid), dim3(256), 0, s, (const v4 *)ds, (v4 *)dd, n16, stamps);
      CK(hipEventRecord(b, s));
      wait_for(w, b, s);
      const double el = now_us() - t;
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r < 10) continue;
      wall.push_back(el);
      ev.push_back(ms * 1000.0);
      CK(hipMemcpy(hst.data(), stamps, 2 * grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      unsigned long long s0 = ~0ull, e1 = 0;
      std::vector<unsigned long long> ends(grid);
      for (int g = 0; g < grid; ++g) {
        s0 = std::min(s0, hst[2 * g]);
        e1 = std::max(e1, hst[2 * g + 1]);
        ends[g] = hst[2 * g + 1];
      }
      std::sort(ends.begin(), ends.end());
      unsigned long long smax = 0;
      for (int g = 0; g < grid; ++g) smax = std::max(smax, hst[2 * g]);
      span.push_back((e1 - s0) * us_per_tick);
      lat0.push_back((smax - s0) * us_per_tick);  // last workgroup start after the first
      first_end.push_back((ends[0] - s0) * us_per_tick);
      p10.push_back((ends[grid / 10] - s0) * us_per_tick);
      p50.push_back((ends[grid / 2] - s0) * us_per_tick);
      p90.push_back((ends[grid * 9 / 10] - s0) * us_per_tick);
    }
    for (size_t i = 0; i < nbytes && ok; i += 4099) ok = hd[i] == (uint8_t)~hs[i];
    std::printf("{\"row\": \"%s\", \"grid\": %d, \"unroll\": %d, \"wait\": \"%s\", \"wall_us\": %.1f, \"event_us\": %.1f, "
                "\"kernel_span_us\": %.1f, \"last_wg_start_us\": %.1f, \"first_wg_end_us\": %.1f, \"wg_end_p10_us\": %.1f, "
                "\"wg_end_p50_us\": %.1f, \"wg_end_p90_us\": %.1f, \"span_GBps_each_way\": %.2f, \"ok\": %s}\n",
                tag, grid, unroll, wait_name(w), median(wall), median(ev), median(span), median(lat0), median(first_end),
                median(p10), median(p50), median(p90), nbytes / median(span) / 1e3, ok ? "true" : "false");
    std::fflush(stdout);
  };
  for (Wait w : {kEventSync, kStreamSync, kSpin}) run_zc(256, 1, w, "zc_wait");
  for (int grid : {128, 256, 512, 1024, 2048})
    for (int u : {1, 2, 4}) run_zc(grid, u, kSpin, "zc_grid");

  // allocation kinds under the best launch shapes
  for (int kind : {1, 2}) {
    uint8_t *ks = host_alloc(kind, nbytes), *kd = host_alloc(kind, nbytes);
    std::memcpy(ks, hs, nbytes);
    CK(hipHostGetDevicePointer((void **)&ds, ks, 0));
    CK(hipHostGetDevicePointer((void **)&dd, kd, 0));
    uint8_t *save_s = hs, *save_d = hd;
    hs = ks, hd = kd;
    char tag[64];
    std::snprintf(tag, sizeof tag, "zc_%s", kind_name(kind));
    for (int grid : {128, 256}) run_zc(grid, 1, kSpin, tag);
    hs = save_s, hd = save_d;
  }
  CK(hipHostGetDevicePointer((void **)&ds, hs, 0));
  CK(hipHostGetDevicePointer((void **)&dd, hd, 0));

  // the product: vf_invert_host on page-locked buffers (vf_alloc_host), and with a pageable
  // source (the drop-in's shape: an ordinary numpy frame in, a page-locked result out)
  {
    vf_ctx *ctx = nullptr;
    if (vf_create(0, nbytes, 1, &ctx) != 0) {
      std::fprintf(stderr, "vf_create: %s\n", vf_last_error(nullptr));
      return 1;
    }
    void *ps = nullptr, *pd = nullptr;
    if (vf_alloc_host(ctx, nbytes, &ps) != 0 || vf_alloc_host(ctx, nbytes, &pd) != 0) return 1;
    std::vector<uint8_t> pageable(hs, hs + nbytes);
    for (int src_kind = 0; src_kind < 2; ++src_kind) {
      const uint8_t *src = src_kind == 0 ? (const uint8_t *)ps : pageable.data();
      if (src_kind == 0) std::memcpy(ps, hs, nbytes);
      std::vector<double> wall;
      for (int r = 0; r < reps + 10; ++r) {
        const double t = now_us();
        if (vf_invert_host(ctx, src, (uint8_t *)pd, nbytes) != 0) {
          std::fprintf(stderr, "vf_invert_host: %s\n", vf_last_error(ctx));
          return 1;
        }
        if (r >= 10) wall.push_back(now_us() - t);
      }
      bool ok = true;
      for (size_t i = 0; i < nbytes && ok; i += 4099) ok = ((uint8_t *)pd)[i] == (uint8_t)~hs[i];
      std::printf("{\"row\": \"product_vf_invert_host\", \"src\": \"%s\", \"wall_us\": %.1f, \"ok\": %s}\n",
                  src_kind == 0 ? "pinned" : "pageable", median(wall), ok ? "true" : "false");
      std::fflush(stdout);
    }
    vf_free_host(ctx, ps);
    vf_free_host(ctx, pd);
    vf_destroy(ctx);
  }

  // SDMA one way each (same frame), the copy engines' fixed cost
  for (int dir = 0; dir < 2; ++dir) {
    std::vector<double> wall, ev;
    for (int r = 0; r < reps + 10; ++r) {
      const double t = now_us();
      CK(hipEventRecord(a, s));
      if (dir == 0) CK(hipMemcpyAsync(dbuf, hs, nbytes, hipMemcpyHostToDevice, s));
      else CK(hipMemcpyAsync(hd, dbuf, nbytes, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(b, s));
      wait_for(kSpin, b, s);
      const double el = now_us() - t;
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r >= 10) wall.push_back(el), ev.push_back(ms * 1000.0);
    }
    std::printf("{\"row\": \"sdma\", \"dir\": \"%s\", \"wall_us\": %.1f, \"event_us\": %.1f, \"GBps\": %.2f}\n",
                dir == 0 ? "h2d" : "d2h", median(wall), median(ev), nbytes / median(ev) / 1e3);
  }
  std::fflush(stdout);
  return 0;
}
