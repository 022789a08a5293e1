// hbm_ceiling.hip — what HBM3E gives a streaming kernel on this MI355X, by direction, to put
// the invert kernel's rate (a copy: one read + one write per byte) in context:
//   read    nt 16-B loads of the whole buffer, folded into one value per lane (never written)
//   write   nt 16-B stores of a constant over the whole buffer
//   copy    the library's kernel shape (U = 4 loads then 4 stores per lane, nt both ways)
// Each row rotates over a ring of buffers larger than the 256 MiB Infinity Cache, interleaved
// in rounds, grid-stride, 256-thread workgroups; GB/s counts the bytes each kernel must move.
//   tools/hbm_ceiling [bytes_per_buffer] [ring] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

typedef unsigned int v4 __attribute__((ext_vector_type(4)));
constexpr int kB = 256, U = 4;

__global__ __launch_bounds__(kB) void k_read(const v4 *__restrict__ s, v4 *__restrict__ sink, size_t n16) {
  v4 acc = {0, 0, 0, 0};
  const size_t stride = (size_t)gridDim.x * kB * U;
  for (size_t t0 = (size_t)blockIdx.x * kB * U; t0 < n16; t0 += stride) {
    v4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const size_t i = t0 + (size_t)j * kB + threadIdx.x;
      v[j] = i < n16 ? __builtin_nontemporal_load(s + i) : v4{0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < U; ++j) acc ^= v[j];
  }
  // keeps the loads without writing: the fold of uniform 0x3c bytes is 0 or 0x3c3c3c3c
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[(size_t)blockIdx.x * kB + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kB) void k_write(v4 *__restrict__ d, size_t n16, unsigned seed) {
  const size_t stride = (size_t)gridDim.x * kB * U;
  const v4 c = {seed, ~seed, seed * 3u, seed ^ 0x5a5a5a5au};
  for (size_t t0 = (size_t)blockIdx.x * kB * U; t0 < n16; t0 += stride) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const size_t i = t0 + (size_t)j * kB + threadIdx.x;
      if (i < n16) __builtin_nontemporal_store(c, d + i);
    }
  }
}

__global__ __launch_bounds__(kB) void k_copy(const v4 *__restrict__ s, v4 *__restrict__ d, size_t n16) {
  const size_t stride = (size_t)gridDim.x * kB * U;
  for (size_t t0 = (size_t)blockIdx.x * kB * U; t0 < n16; t0 += stride) {
    v4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const size_t i = t0 + (size_t)j * kB + threadIdx.x;
      v[j] = i < n16 ? __builtin_nontemporal_load(s + i) : v4{0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const size_t i = t0 + (size_t)j * kB + threadIdx.x;
      if (i < n16) __builtin_nontemporal_store(~v[j], d + i);
    }
  }
}

int main(int argc, char **argv) {
  const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (size_t)199065600;
  const int ring = argc > 2 ? std::atoi(argv[2]) : 12;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 5;
  const size_t n16 = bytes / 16;
  std::vector<v4 *> buf((size_t)ring);
  for (auto &b : buf) {
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(b, 0x3c, bytes));
  }
  v4 *sink;
  CK(hipMalloc(&sink, (size_t)16384 * kB * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grids[] = {2048, 4096, 8192, 16384};
  const char *names[] = {"read", "write", "copy"};
  std::printf("{\"bytes_per_buffer\": %zu, \"ring\": %d, \"rounds\": %d}\n", bytes, ring, rounds);
  for (int g : grids) {
    for (int k = 0; k < 3; ++k) {
      std::vector<float> per;
      for (int r = 0; r < rounds; ++r) {
        const int steps = ring;  // one pass over the ring (copy: buffer i -> i+1)
        CK(hipEventRecord(a, 0));
        for (int s = 0; s < steps; ++s) {
          v4 *x = buf[(size_t)s], *y = buf[(size_t)((s + 1) % ring)];
          if (k == 0) hipLaunchKernelGGL(k_read, dim3(g), dim3(kB), 0, 0, x, sink, n16);
          if (k == 1) hipLaunchKernelGGL(k_write, dim3(g), dim3(kB), 0, 0, x, n16, (unsigned)s);
          if (k == 2) hipLaunchKernelGGL(k_copy, dim3(g), dim3(kB), 0, 0, x, y, n16);
        }
        CK(hipGetLastError());
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        per.push_back(ms / steps);
      }
      std::sort(per.begin(), per.end());
      const double moved = (k == 2 ? 2.0 : 1.0) * (double)bytes;
      std::printf("{\"kernel\": \"%s\", \"grid\": %d, \"ms_median\": %.4f, \"GBps_median\": %.1f, \"GBps_best\": %.1f}\n",
                  names[k], g, per[per.size() / 2], moved / (per[per.size() / 2] * 1e-3) / 1e9,
                  moved / (per[0] * 1e-3) / 1e9);
      std::fflush(stdout);
    }
  }
  return 0;
}
