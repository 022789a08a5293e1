// vf_host_mem.h — page-locked host memory on the NUMA node of the GPU that DMAs it.
// Not installed.
//
// Every host->host path of the library moves each byte across PCIe twice (H2D, D2H) through
// page-locked buffers: the engine's slot staging buffers, vf_alloc_host memory, the JPEG
// codecs' staging and output buffers.  On a two-socket host a buffer on the other socket's
// DRAM makes every DMA cross the socket link.  hipHostMalloc places pages by the allocating
// thread's policy; here the buffer is mapped, bound to the GPU's node (MPOL_PREFERRED, so a
// full node falls back instead of failing), faulted in and then page-locked with
// hipHostRegister.  The node comes from the device's PCI address in sysfs.  Where any step is
// unavailable the allocation falls back to hipHostMalloc.  VF_NUMA=0 forces the fallback.
#pragma once
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

namespace vf {

inline int device_numa_node(int device) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  int node = -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) == hipSuccess) {
    for (char *c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
    char path[160];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    if (FILE *f = std::fopen(path, "r")) {
      if (std::fscanf(f, "%d", &node) != 1) node = -1;
      std::fclose(f);
    }
  } else {
    (void)hipGetLastError();
  }
  cache[device] = node;
  return node;
}

struct PinnedRegistry {
  std::mutex mu;
  std::map<void *, size_t> mapped;  // buffers from the mmap + hipHostRegister path
  static PinnedRegistry &get() {
    static PinnedRegistry r;
    return r;
  }
};

// Page-locked buffer of n bytes on `node` (< 0: wherever hipHostMalloc puts it).
inline hipError_t numa_pinned_alloc(void **out, size_t n, int node) {
  *out = nullptr;
  if (n == 0) n = 1;
  static const bool enabled = [] {
    const char *v = std::getenv("VF_NUMA");
    return !(v && v[0] == '0');
  }();
#if defined(__x86_64__) && defined(SYS_mbind)
  if (enabled && node >= 0 && node < 1024) {
    const size_t len = (n + 4095) & ~(size_t)4095;
    void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p != MAP_FAILED) {
      unsigned long mask[16] = {0};
      mask[node / 64] = 1ul << (node % 64);
      const long rc = syscall(SYS_mbind, p, len, 1 /* MPOL_PREFERRED */, mask, 16ul * 64 + 1, 0u);
      if (rc == 0) {
        std::memset(p, 0, len);  // fault the pages in on the node before locking them
        if (hipHostRegister(p, len, hipHostRegisterMapped) == hipSuccess) {
          std::lock_guard<std::mutex> lk(PinnedRegistry::get().mu);
          PinnedRegistry::get().mapped[p] = len;
          *out = p;
          return hipSuccess;
        }
        (void)hipGetLastError();
      }
      munmap(p, len);
    }
  }
#else
  (void)node;
  (void)enabled;
#endif
  return hipHostMalloc(out, n, hipHostMallocDefault);
}

inline hipError_t numa_pinned_free(void *p) {
  if (!p) return hipSuccess;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> lk(PinnedRegistry::get().mu);
    auto it = PinnedRegistry::get().mapped.find(p);
    if (it != PinnedRegistry::get().mapped.end()) {
      len = it->second;
      PinnedRegistry::get().mapped.erase(it);
    }
  }
  if (!len) return hipHostFree(p);
  const hipError_t e = hipHostUnregister(p);
  munmap(p, len);
  return e;
}

}  // namespace vf
