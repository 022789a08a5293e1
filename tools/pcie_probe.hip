// pcie_probe.hip — host<->device copy ceilings on this box, to put the end-to-end
// (host->host) invert rate in context: H2D alone, D2H alone, and both at once on two
// streams, with pinned host memory, as one big copy and as a train of chunk copies.
//   tools/pcie_probe [total_bytes] [chunk_bytes]
#include <hip/hip_runtime.h>

#include <chrono>
#include <thread>
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

__global__ void probe_invert_kernel(const uint4 *s, uint4 *d, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = s[i];
    d[i] = make_uint4(~v.x, ~v.y, ~v.z, ~v.w);
  }
}

static hipError_t vf_probe_invert(const uint8_t *s, uint8_t *d, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(probe_invert_kernel, dim3(2048), dim3(256), 0, st, (const uint4 *)s, (uint4 *)d, n / 16);
  return hipGetLastError();
}

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

  // Pipelines of H2D -> kernel -> D2H over `nslots` device slots of `chunk` bytes:
  //  "devwait": IN stream H2D+kernel, OUT stream waits the kernel event (hipStreamWaitEvent),
  //             slot reuse waits on the device too; the host only enqueues.
  //  "hostdrive": no device-side cross-stream waits: the host polls each slot's kernel event
  //             and only then enqueues its D2H; a slot is refilled once its D2H event is done.
  auto pipeline = [&](const char *name, bool devwait, int nslots, bool timing = false) {
    std::vector<uint8_t *> din(nslots), dout(nslots);
    std::vector<hipEvent_t> ek(nslots), ed(nslots);
    const unsigned flags = timing ? hipEventDefault : hipEventDisableTiming;
    for (int s = 0; s < nslots; ++s) {
      CK(hipMalloc(&din[s], chunk));
      CK(hipMalloc(&dout[s], chunk));
      CK(hipEventCreateWithFlags(&ek[s], flags));
      CK(hipEventCreateWithFlags(&ed[s], flags));
    }
    const size_t nch = total / chunk;
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      double t0 = now();
      if (devwait) {
        std::vector<bool> used(nslots, false);
        for (size_t c = 0; c < nch; ++c) {
          int s = c % nslots;
          if (used[s]) CK(hipStreamWaitEvent(s1, ed[s], 0));
          CK(hipMemcpyAsync(din[s], h_in + c * chunk, chunk, hipMemcpyHostToDevice, s1));
          CK(vf_probe_invert(din[s], dout[s], chunk, s1));
          CK(hipEventRecord(ek[s], s1));
          CK(hipStreamWaitEvent(s2, ek[s], 0));
          CK(hipMemcpyAsync(h_out + c * chunk, dout[s], chunk, hipMemcpyDeviceToHost, s2));
          CK(hipEventRecord(ed[s], s2));
          used[s] = true;
        }
      } else {
        // per slot: 0 free, 1 H2D+kernel queued, 2 D2H queued; chunks retire in order
        std::vector<int> st(nslots, 0);
        std::vector<size_t> ch(nslots, 0);
        size_t next = 0, d2h_next = 0, done_next = 0;
        while (done_next < nch) {
          bool progress = false;
          int s = next % nslots;
          if (next < nch && st[s] == 0) {
            CK(hipMemcpyAsync(din[s], h_in + next * chunk, chunk, hipMemcpyHostToDevice, s1));
            CK(vf_probe_invert(din[s], dout[s], chunk, s1));
            CK(hipEventRecord(ek[s], s1));
            st[s] = 1; ch[s] = next++; progress = true;
          }
          int sd = d2h_next % nslots;
          if (d2h_next < next && st[sd] == 1 && hipEventQuery(ek[sd]) == hipSuccess) {
            CK(hipMemcpyAsync(h_out + ch[sd] * chunk, dout[sd], chunk, hipMemcpyDeviceToHost, s2));
            CK(hipEventRecord(ed[sd], s2));
            st[sd] = 2; ++d2h_next; progress = true;
          }
          int sf = done_next % nslots;
          if (done_next < d2h_next && st[sf] == 2 && hipEventQuery(ed[sf]) == hipSuccess) {
            st[sf] = 0; ++done_next; progress = true;
          }
          (void)hipGetLastError();  // hipErrorNotReady from the queries
          if (!progress) std::this_thread::yield();
        }
      }
      CK(hipDeviceSynchronize());
      double dt = now() - t0;
      if (dt < best) best = dt;
    }
    std::printf("%-10s slots %d chunk %9zu : %7.2f GB/s per direction\n", name, nslots, chunk,
                nch * chunk / best / 1e9);
    for (int s = 0; s < nslots; ++s) {
      CK(hipFree(din[s]));
      CK(hipFree(dout[s]));
      CK(hipEventDestroy(ek[s]));
      CK(hipEventDestroy(ed[s]));
    }
  };
  for (int ns : {2, 4, 8}) {
    pipeline("devwait", true, ns);
    pipeline("hostdrive", false, ns);
  }
  pipeline("devwait+timing-events", true, 4, true);
  pipeline("hostdrive+timing-events", false, 4, true);

  // The library's asynchronous pattern: batches of `per` chunks enqueued devwait-style, the
  // host keeping `depth` batches in flight and waiting for the oldest batch's end event
  // (hipEventSynchronize, or a hipEventQuery poll loop).
  auto batches = [&](int depth, bool poll, int per) {
    const int nslots = 4;
    std::vector<uint8_t *> din(nslots), dout(nslots);
    std::vector<hipEvent_t> ek(nslots), ed(nslots);
    for (int s = 0; s < nslots; ++s) {
      CK(hipMalloc(&din[s], chunk));
      CK(hipMalloc(&dout[s], chunk));
      CK(hipEventCreateWithFlags(&ek[s], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&ed[s], hipEventDisableTiming));
    }
    const size_t nch = total / chunk;
    const size_t nb = nch / per;
    std::vector<hipEvent_t> be(nb);
    for (auto &ev : be) CK(hipEventCreate(&ev));
    CK(hipDeviceSynchronize());
    double t0 = now();
    std::vector<bool> used(nslots, false);
    size_t waited = 0;
    int sl = 0;
    for (size_t b = 0; b < nb; ++b) {
      for (int j = 0; j < per; ++j) {
        size_t c = b * per + j;
        int s = sl;
        sl = (sl + 1) % nslots;
        if (used[s]) CK(hipStreamWaitEvent(s1, ed[s], 0));
        CK(hipMemcpyAsync(din[s], h_in + c * chunk, chunk, hipMemcpyHostToDevice, s1));
        CK(vf_probe_invert(din[s], dout[s], chunk, s1));
        CK(hipEventRecord(ek[s], s1));
        CK(hipStreamWaitEvent(s2, ek[s], 0));
        CK(hipMemcpyAsync(h_out + c * chunk, dout[s], chunk, hipMemcpyDeviceToHost, s2));
        CK(hipEventRecord(ed[s], s2));
        used[s] = true;
      }
      CK(hipEventRecord(be[b], s2));
      while (b + 1 - waited >= (size_t)depth) {
        if (poll) {
          while (hipEventQuery(be[waited]) != hipSuccess) std::this_thread::yield();
          (void)hipGetLastError();
        } else {
          CK(hipEventSynchronize(be[waited]));
        }
        ++waited;
      }
    }
    CK(hipDeviceSynchronize());
    double dt = now() - t0;
    std::printf("batches depth %d %-9s %d chunks/batch : %7.2f GB/s per direction\n", depth,
                poll ? "poll" : "eventsync", per, nb * per * chunk / dt / 1e9);
    for (auto &ev : be) CK(hipEventDestroy(ev));
    for (int s = 0; s < nslots; ++s) {
      CK(hipFree(din[s]));
      CK(hipFree(dout[s]));
      CK(hipEventDestroy(ek[s]));
      CK(hipEventDestroy(ed[s]));
    }
  };
  for (int depth : {1, 2, 4})
    for (bool poll : {false, true}) batches(depth, poll, 8);
  return 0;
}
