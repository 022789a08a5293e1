// zerocopy_probe.hip — can the invert kernel move a host->host batch over PCIe itself,
// faster than SDMA copies staged through HBM?  The kernel reads the page-locked source and
// writes the page-locked destination directly (both mapped into the GPU's address space), so
// each byte crosses PCIe once each way with no HBM staging, no chunk ring and no host
// polling between the directions.
//
//   tools/zerocopy_probe [total_bytes] [reps]
//
// Rows: SDMA ceilings (H2D alone, D2H alone, both at once on two streams, one big copy each),
// then the zero-copy kernel for host allocation kinds (hipHostMalloc default / non-coherent,
// mmap + hipHostRegister) x unroll x grid, and the one-direction kernels (host -> device
// memory, device memory -> host).  Every zero-copy result is checked against ~src.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

template <int U>
__global__ __launch_bounds__(256) void zc_invert(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n16) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < n16; i += stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * 256] = make_uint4(~v[u].x, ~v[u].y, ~v[u].z, ~v[u].w);
  }
  for (; i < n16; i += 256) {
    const uint4 v = s[i];
    d[i] = make_uint4(~v.x, ~v.y, ~v.z, ~v.w);
  }
}

template <int U>
__global__ __launch_bounds__(256) void zc_invert_nt(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(s) + i);
    __builtin_nontemporal_store(~v, reinterpret_cast<v4 *>(d) + i);
  }
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct HostBuf {
  uint8_t *p = nullptr;
  size_t len = 0;
  int kind = 0;  // 0 hipHostMalloc default, 1 non-coherent, 2 mmap + hipHostRegister
};

static HostBuf host_alloc(size_t n, int kind) {
  HostBuf b;
  b.kind = kind;
  b.len = (n + 4095) & ~(size_t)4095;
  if (kind == 0) CK(hipHostMalloc((void **)&b.p, b.len, hipHostMallocDefault));
  if (kind == 1) CK(hipHostMalloc((void **)&b.p, b.len, hipHostMallocNonCoherent));
  if (kind == 2) {
    void *p = mmap(nullptr, b.len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) std::exit(2);
    std::memset(p, 0, b.len);
    CK(hipHostRegister(p, b.len, hipHostRegisterMapped));
    b.p = (uint8_t *)p;
  }
  return b;
}

static void host_free(HostBuf &b) {
  if (b.kind == 2) {
    CK(hipHostUnregister(b.p));
    munmap(b.p, b.len);
  } else {
    CK(hipHostFree(b.p));
  }
}

static void *dev_ptr(void *h) {
  void *d = nullptr;
  CK(hipHostGetDevicePointer(&d, h, 0));
  return d;
}

template <int U, bool NT = false>
static float launch_time(const void *s, void *d, size_t n, int grid, hipStream_t st, hipEvent_t a, hipEvent_t b,
                         int reps) {
  const size_t n16 = n / 16;
  void (*k)(const uint4 *, uint4 *, size_t) = NT ? zc_invert_nt<U> : zc_invert<U>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (const uint4 *)s, (uint4 *)d, n16);  // warm
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, st));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (const uint4 *)s, (uint4 *)d, n16);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

static bool check_inverted(const uint8_t *src, const uint8_t *dst, size_t n) {
  for (size_t i = 0; i < n; i += 4093)
    if ((uint8_t)~src[i] != dst[i]) return false;
  return (uint8_t)~src[n - 1] == dst[n - 1];
}

int main(int argc, char **argv) {
  const size_t total = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (size_t)199065600;  // 1080p x 32
  const int reps = argc > 2 ? std::atoi(argv[2]) : 6;
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  uint8_t *d_in, *d_out;
  CK(hipMalloc(&d_in, total));
  CK(hipMalloc(&d_out, total));
  CK(hipMemset(d_in, 0x5a, total));
  const double gb = total / 1e9;

  {  // SDMA ceilings
    HostBuf hi = host_alloc(total, 0), ho = host_alloc(total, 0);
    for (size_t i = 0; i < total; i += 4096) hi.p[i] = (uint8_t)i;
    for (int mode = 0; mode < 3; ++mode) {
      double best = 1e30;
      for (int r = 0; r < reps; ++r) {
        const double t0 = now();
        if (mode != 1) CK(hipMemcpyAsync(d_in, hi.p, total, hipMemcpyHostToDevice, s1));
        if (mode != 0) CK(hipMemcpyAsync(ho.p, d_out, total, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
        const double dt = now() - t0;
        if (dt < best) best = dt;
      }
      const char *nm[3] = {"sdma_h2d", "sdma_d2h", "sdma_both"};
      std::printf("{\"row\": \"%s\", \"bytes\": %zu, \"ms\": %.3f, \"GBps_each_way\": %.2f}\n", nm[mode], total,
                  best * 1e3, gb / best);
    }
    host_free(hi);
    host_free(ho);
  }

  // round 2b: small grids, nontemporal, per size (hipHostMalloc default and registered)
  for (int kind : {0, 2}) {
    HostBuf hi = host_alloc(total, kind), ho = host_alloc(total, kind);
    for (size_t i = 0; i < total; ++i) hi.p[i] = (uint8_t)(i * 131 + (i >> 12));
    const uint8_t *ds = (const uint8_t *)dev_ptr(hi.p);
    uint8_t *dd = (uint8_t *)dev_ptr(ho.p);
    const char *kn[3] = {"hostmalloc", "noncoherent", "registered"};
    for (size_t n : {(size_t)6220800, (size_t)24883200, (size_t)49766400, total}) {
      if (n > total) continue;
      for (int grid : {32, 64, 96, 128, 192, 256, 384}) {
        for (int nt = 0; nt < 2; ++nt) {
          std::memset(ho.p, 0, n);
          const float ms = nt ? launch_time<1, true>(ds, dd, n, grid, s1, a, b, reps)
                              : launch_time<1>(ds, dd, n, grid, s1, a, b, reps);
          const bool ok = check_inverted(hi.p, ho.p, n);
          std::printf("{\"row\": \"zc_host_to_host\", \"alloc\": \"%s\", \"bytes\": %zu, \"grid\": %d, \"nt\": %d, "
                      "\"ms\": %.3f, \"GBps_each_way\": %.2f, \"ok\": %s}\n",
                      kn[kind], n, grid, nt, ms, n / 1e9 / (ms * 1e-3), ok ? "true" : "false");
          std::fflush(stdout);
        }
      }
    }
    host_free(hi);
    host_free(ho);
  }
  CK(hipFree(d_in));
  CK(hipFree(d_out));
  return 0;
}
