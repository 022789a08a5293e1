// Host cost of queuing one JPEG batch's launches directly vs through a hipGraph.
// A batch is modelled as the codec's submit sequence at 512 x 512 x 64: 6 small H2D copies from
// page-locked memory, 18 kernel launches of assorted grids, 1 D2H copy and an event record.
//   direct   every call issued on the stream (the codec today)
//   replay   the batch captured once, instantiated, then hipGraphLaunch per batch (only valid when
//            every argument and grid is the same from batch to batch)
//   update   each batch captured again and pushed into the instantiated graph with
//            hipGraphExecUpdate, then launched (what per-batch sizes would need)
// Per mode: host microseconds to queue one batch (median of 2000) and batches/s with 3 in flight.
// argv[1] "nocopy" leaves the copies out (kernels only).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/r6/graph_probe tools/r6/graph_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ void k_touch(unsigned *p, unsigned n, unsigned salt) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 3u + salt;
}

struct Batch {
  hipStream_t s;
  unsigned *dev;
  unsigned char *host_in, *host_out, *dev_in;
  hipEvent_t done;
};

static const int kGrids[18] = {64, 64, 1, 128, 512, 512, 64, 1, 256, 1024, 1024, 512, 64, 1, 64, 256, 128, 64};

static int g_copies = 1;  // argv[1] == "nocopy": kernels only

static void queue_batch(const Batch &b, unsigned salt) {
  if (!g_copies) {
    for (int k = 0; k < 18; ++k) {
      unsigned n = (unsigned)kGrids[k] * 256u;
      hipLaunchKernelGGL(k_touch, dim3(kGrids[k]), dim3(256), 0, b.s, b.dev, n, salt + k);
    }
    return;
  }
  size_t off = 0;
  const size_t sz[6] = {4096, 50688, 2048, 1024, 8192, 2097152};  // descriptors, tables, segments, input
  for (int c = 0; c < 6; ++c) {
    CK(hipMemcpyAsync(b.dev_in + off, b.host_in + off, sz[c], hipMemcpyHostToDevice, b.s));
    off += sz[c];
  }
  for (int k = 0; k < 18; ++k) {
    unsigned n = (unsigned)kGrids[k] * 256u;
    hipLaunchKernelGGL(k_touch, dim3(kGrids[k]), dim3(256), 0, b.s, b.dev, n, salt + k);
  }
  CK(hipMemcpyAsync(b.host_out, b.dev, 2097152, hipMemcpyDeviceToHost, b.s));
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  const int iters = 2000, depth = 3;
  if (argc > 1 && std::string(argv[1]) == "nocopy") g_copies = 0;
  std::vector<Batch> bs(depth);
  for (auto &b : bs) {
    CK(hipStreamCreateWithFlags(&b.s, hipStreamNonBlocking));
    CK(hipMalloc(&b.dev, 1024 * 256 * 4 + 2097152));
    CK(hipMalloc(&b.dev_in, 4 << 20));
    CK(hipHostMalloc(&b.host_in, 4 << 20));
    CK(hipHostMalloc(&b.host_out, 4 << 20));
    CK(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
  }
  for (int mode = 0; mode < 3; ++mode) {
    const char *name[3] = {"direct", "replay", "update"};
    std::vector<hipGraphExec_t> ex(depth, nullptr);
    if (mode > 0)
      for (int d = 0; d < depth; ++d) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(bs[d].s, hipStreamCaptureModeThreadLocal));
        queue_batch(bs[d], 0);
        CK(hipStreamEndCapture(bs[d].s, &g));
        CK(hipGraphInstantiate(&ex[d], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
      }
    std::vector<double> q;
    q.reserve(iters);
    for (int w = 0; w < 2; ++w) {  // pass 0 warms up
      q.clear();
      double t0 = now_us();
      for (int i = 0; i < iters; ++i) {
        Batch &b = bs[i % depth];
        CK(hipEventSynchronize(b.done));  // this slot's previous batch
        double a = now_us();
        if (mode == 0) {
          queue_batch(b, (unsigned)i);
        } else if (mode == 1) {
          CK(hipGraphLaunch(ex[i % depth], b.s));
        } else {
          hipGraph_t g;
          CK(hipStreamBeginCapture(b.s, hipStreamCaptureModeThreadLocal));
          queue_batch(b, (unsigned)i);
          CK(hipStreamEndCapture(b.s, &g));
          hipGraphExecUpdateResult r;
          hipGraphNode_t bad;
          CK(hipGraphExecUpdate(ex[i % depth], g, &bad, &r));
          CK(hipGraphDestroy(g));
          CK(hipGraphLaunch(ex[i % depth], b.s));
        }
        CK(hipEventRecord(b.done, b.s));
        q.push_back(now_us() - a);
      }
      for (auto &b : bs) CK(hipStreamSynchronize(b.s));
      double t = now_us() - t0;
      if (w == 1) {
        std::sort(q.begin(), q.end());
        std::printf("{\"copies\": %d, \"mode\": \"%s\", \"queue_us_median\": %.2f, \"queue_us_p90\": %.2f, \"batches_per_s\": %.0f}\n",
                    g_copies, name[mode], q[q.size() / 2], q[q.size() * 9 / 10], iters / (t * 1e-6));
      }
    }
    for (auto e : ex)
      if (e) CK(hipGraphExecDestroy(e));
  }
  return 0;
}
