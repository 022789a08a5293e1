// tune_invert.hip — kernel-variant sweep for the invert kernel on MI355X.
//
// Runs every (variant, grid cap) pair in interleaved rounds inside ONE process (guide §5.4
// rule 24) over a ring of HBM buffers far larger than the 256 MiB Infinity Cache, so the
// numbers are HBM rates, not cache rates.  Prints median / min / max algorithmic GB/s
// (2 bytes moved per byte filtered) per pair, and checks every variant's output bytes.
//
//   tools/tune_invert [batch_bytes] [ring] [rounds] [launches]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "vf_internal.h"
#include "vf_stream.h"

// The variants (the library ships U4-NT, vf_kernels.hip).  Un = n independent 16-B loads in
// flight per lane; NT = nontemporal loads and stores, NTL / NTS = on one side only; CHUNK =
// contiguous tiles per workgroup instead of grid-stride.
enum { kU4NT, kU2NT, kU8NT, kU1NT, kU4NTL, kU4NTS, kU4, kU2, kU8, kU1, kU4NTChunk, kU8NTChunk, kVariantCount };

static const char *vname(int v) {
  static const char *names[kVariantCount] = {"u4-nt", "u2-nt", "u8-nt", "u1-nt", "u4-ntl", "u4-nts",
                                             "u4",    "u2",    "u8",    "u1",    "u4-nt-chunk", "u8-nt-chunk"};
  return (v >= 0 && v < kVariantCount) ? names[v] : "?";
}

static hipError_t launch_variant(int v, const uint8_t *s, uint8_t *d, size_t n, int mb, hipStream_t st) {
  using vf::launch_stream;
  switch (v) {
    case kU4NT: return launch_stream<4, true, true>(s, d, n, mb, st);
    case kU2NT: return launch_stream<2, true, true>(s, d, n, mb, st);
    case kU8NT: return launch_stream<8, true, true>(s, d, n, mb, st);
    case kU1NT: return launch_stream<1, true, true>(s, d, n, mb, st);
    case kU4NTL: return launch_stream<4, true, false>(s, d, n, mb, st);
    case kU4NTS: return launch_stream<4, false, true>(s, d, n, mb, st);
    case kU4: return launch_stream<4, false, false>(s, d, n, mb, st);
    case kU2: return launch_stream<2, false, false>(s, d, n, mb, st);
    case kU8: return launch_stream<8, false, false>(s, d, n, mb, st);
    case kU1: return launch_stream<1, false, false>(s, d, n, mb, st);
    case kU4NTChunk: return launch_stream<4, true, true, true>(s, d, n, mb, st);
    case kU8NTChunk: return launch_stream<8, true, true, true>(s, d, n, mb, st);
    default: return hipErrorInvalidValue;
  }
}

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__global__ void fill_kernel(uint8_t *p, size_t n, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (uint8_t)x;
  }
}

__global__ void check_kernel(const uint8_t *a, const uint8_t *b, size_t n, int *bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride)
    if ((uint8_t)~a[i] != b[i]) atomicAdd(bad, 1);
}

// Large single-buffer experiment (configs[4]): one src of `bytes`, dst at several offsets
// from a bigger allocation, and the same bytes as one launch vs sub-range launches.
static int large_mode(size_t bytes, int reps, size_t pad) {
  vf::LaunchCfg lc;
  uint8_t *src, *dst;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes + pad));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, src, bytes, 77u);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("large-buffer mode: %zu B, dst alloc pad %zu, src %p dst %p (dst-src = %lld)\n", bytes, pad,
              (void *)src, (void *)dst, (long long)(dst - src));
  const size_t offs[] = {0, 4096, 65536, (size_t)1 << 20, (size_t)2 << 20, (size_t)8 << 20,
                         (size_t)32 << 20};
  const size_t subs[] = {0, (size_t)64 << 20, (size_t)128 << 20, (size_t)192 << 20, (size_t)199065600,
                         (size_t)256 << 20, (size_t)512 << 20, (size_t)1 << 30};
  for (size_t sub : subs) {
    for (size_t off : offs) {
      if (off > pad) continue;  // dst + off + bytes must stay inside the dst allocation
      std::vector<double> v;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        const size_t step = sub ? sub : bytes;
        for (size_t o = 0; o < bytes; o += step)
          CK(vf::launch_invert(src + o, dst + off + o, std::min(step, bytes - o), lc, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.push_back(2.0 * bytes / (ms * 1e-3) / 1e9);
      }
      std::sort(v.begin(), v.end());
      std::printf("sub-launch %12zu  dst offset %10zu : median %7.1f GB/s (min %7.1f max %7.1f)\n", sub,
                  off, v[v.size() / 2], v.front(), v.back());
    }
  }
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 2 && std::strcmp(argv[1], "large") == 0)
    return large_mode(std::strtoull(argv[2], nullptr, 0), argc > 3 ? std::atoi(argv[3]) : 5,
                      (argc > 4 ? std::strtoull(argv[4], nullptr, 0) : 64) << 20);
  size_t batch = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (size_t)32 * 1920 * 1080 * 3;
  int ring = argc > 2 ? std::atoi(argv[2]) : 6;
  int rounds = argc > 3 ? std::atoi(argv[3]) : 7;
  int launches = argc > 4 ? std::atoi(argv[4]) : 24;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::printf("device %s, %d CUs, batch %zu B, ring %d (%.2f GB in+out)\n", prop.gcnArchName, cus,
              batch, ring, 2.0 * batch * ring / 1e9);
  std::vector<uint8_t *> src(ring), dst(ring);
  for (int r = 0; r < ring; ++r) {
    CK(hipMalloc(&src[r], batch));
    CK(hipMalloc(&dst[r], batch));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, src[r], batch, 1234u + r);
  }
  int *bad;
  CK(hipMalloc(&bad, sizeof(int)));
  CK(hipDeviceSynchronize());

  struct Cfg { int variant; int blocks; };
  std::vector<Cfg> cfgs;
  const int mults[] = {2, 4, 8, 16, 32, 1 << 20};  // blocks per CU cap; huge = one tile per block
  const char *only = std::getenv("TUNE_VARIANTS");  // e.g. "0,1,2"
  for (int v = 0; v < kVariantCount; ++v) {
    if (only && !std::strstr(only, std::to_string(v).c_str())) continue;
    for (int m : mults) cfgs.push_back({v, (int)std::min<long>((long)cus * m, 1 << 30)});
  }

  // correctness of every variant (unaligned tail exercised with batch - 7 bytes)
  for (const Cfg &c : cfgs) {
    CK(hipMemset(dst[0], 0, batch));
    CK(launch_variant(c.variant, src[0] + 3, dst[0] + 3, batch - 7, c.blocks, 0));
    CK(hipMemset(bad, 0, sizeof(int)));
    hipLaunchKernelGGL(check_kernel, dim3(4096), dim3(256), 0, 0, src[0] + 3, dst[0] + 3,
                       batch - 7, bad);
    int h = 0;
    CK(hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost));
    if (h) {
      std::printf("MISMATCH variant %s blocks %d: %d bad bytes\n", vname(c.variant), c.blocks, h);
      return 2;
    }
  }
  std::printf("all %zu variants bit-exact\n", cfgs.size());

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> gbs(cfgs.size());
  int slot = 0;
  for (int rd = 0; rd < rounds; ++rd) {
    for (size_t ci = 0; ci < cfgs.size(); ++ci) {
      const int v = cfgs[ci].variant, mb = cfgs[ci].blocks;
      CK(launch_variant(v, src[slot], dst[slot], batch, mb, 0));  // warm
      slot = (slot + 1) % ring;
      CK(hipEventRecord(e0, 0));
      for (int l = 0; l < launches; ++l) {
        CK(launch_variant(v, src[slot], dst[slot], batch, mb, 0));
        slot = (slot + 1) % ring;
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      gbs[ci].push_back(2.0 * batch * launches / (ms * 1e-3) / 1e9);
    }
  }
  std::printf("%-8s %10s %10s %10s %10s %8s\n", "variant", "blocks", "median", "min", "max", "frac");
  for (size_t ci = 0; ci < cfgs.size(); ++ci) {
    auto v = gbs[ci];
    std::sort(v.begin(), v.end());
    std::printf("%-8s %10d %10.1f %10.1f %10.1f %8.3f\n", vname(cfgs[ci].variant), cfgs[ci].blocks,
                v[v.size() / 2], v.front(), v.back(), v[v.size() / 2] / 8000.0);
  }
  // reference point: hipMemcpyDtoD of the same bytes (same traffic as the filter)
  std::vector<double> cp;
  for (int rd = 0; rd < rounds; ++rd) {
    CK(hipEventRecord(e0, 0));
    for (int l = 0; l < launches; ++l) {
      CK(hipMemcpyAsync(dst[slot], src[slot], batch, hipMemcpyDeviceToDevice, 0));
      slot = (slot + 1) % ring;
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    cp.push_back(2.0 * batch * launches / (ms * 1e-3) / 1e9);
  }
  std::sort(cp.begin(), cp.end());
  std::printf("%-8s %10s %10.1f %10.1f %10.1f %8.3f\n", "hipMemcpyD2D", "-", cp[cp.size() / 2],
              cp.front(), cp.back(), cp[cp.size() / 2] / 8000.0);
  return 0;
}
