// pcie_probe.hip — host<->device copy ceilings on this box, to put the end-to-end
// (host->host) invert rate in context: H2D alone, D2H alone, and both at once on two
// streams, with pinned host memory, as one big copy and as a train of chunk copies.
//   tools/pcie_probe [total_bytes] [chunk_bytes]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  size_t total = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (size_t)1 << 30;
  size_t chunk = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : (size_t)8 << 20;
  uint8_t *h_in, *h_out, *d_in, *d_out;
  CK(hipHostMalloc((void **)&h_in, total, hipHostMallocDefault));
  CK(hipHostMalloc((void **)&h_out, total, hipHostMallocDefault));
  CK(hipMalloc(&d_in, total));
  CK(hipMalloc(&d_out, total));
  for (size_t i = 0; i < total; i += 4096) h_in[i] = (uint8_t)i;
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  auto run = [&](const char *name, bool h2d, bool d2h, size_t ck) {
    double best = 1e30;
    for (int rep = 0; rep < 4; ++rep) {
      double t0 = now();
      for (size_t o = 0; o < total; o += ck) {
        size_t n = (o + ck <= total) ? ck : total - o;
        if (h2d) CK(hipMemcpyAsync(d_in + o, h_in + o, n, hipMemcpyHostToDevice, s1));
        if (d2h) CK(hipMemcpyAsync(h_out + o, d_out + o, n, hipMemcpyDeviceToHost, s2));
      }
      CK(hipStreamSynchronize(s1));
      CK(hipStreamSynchronize(s2));
      double dt = now() - t0;
      if (dt < best) best = dt;
    }
    std::printf("%-28s chunk %10zu : %7.2f GB/s per direction\n", name, ck, total / best / 1e9);
  };
  for (size_t ck : {total, chunk}) {
    run("H2D alone", true, false, ck);
    run("D2H alone", false, true, ck);
    run("H2D + D2H concurrent", true, true, ck);
  }
  return 0;
}
