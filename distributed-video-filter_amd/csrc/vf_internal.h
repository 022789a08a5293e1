// vf_internal.h — shared between the kernel, engine and C-ABI translation units (not installed).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace vf {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

struct LaunchCfg {
  int max_blocks = 8192;  // grid cap: 32 workgroups per CU on 256 CUs
};

hipError_t launch_invert(const void *dsrc, void *ddst, size_t nbytes, const LaunchCfg &cfg,
                         hipStream_t stream);

hipError_t launch_invert_frames(const void *const *dsrcs, void *const *ddsts,
                                const size_t *nbytes, int n, size_t total_bytes,
                                const LaunchCfg &cfg, hipStream_t stream);

// Up to kMappedMax page-locked host ranges, by their device addresses, inverted in place over
// PCIe by one launch (vf_kernels.hip invert_mapped_kernel; passed by value as kernel arguments).
constexpr int kMappedMax = 64;
struct MappedBatch {
  const uint8_t *src[kMappedMax];
  uint8_t *dst[kMappedMax];
  uint64_t n[kMappedMax];
  uint32_t tile0[kMappedMax + 1];  // first 4-KiB tile of each range (set by the launcher)
};
hipError_t launch_invert_mapped(const MappedBatch &b, int n, size_t total_bytes, hipStream_t stream);
// One mapped range whose source is still being copied into it by the host: tile t waits until
// landed[piece of t] == nw, relayed through the device word `frontier` tagged with gen (24 bits,
// not 0) (vf_kernels.hip invert_gated_kernel); src and dst 16-B aligned, at most 254 pieces.
hipError_t launch_invert_gated(const uint8_t *src, uint8_t *dst, size_t n, const uint32_t *landed,
                               uint32_t piece_shift, uint32_t nw, uint32_t *frontier, uint32_t gen, uint32_t *status,
                               uint64_t budget_ticks, hipStream_t stream);

// ---- host -> host pipeline (vf_engine.hip) --------------------------------------------------

// memcpy of large staging chunks split over a few persistent threads: one core moves
// ~10 GB/s, well under one PCIe Gen5 x16 direction (1080p x 32 pageable: 30.5 GB/s each way
// with 4 threads, 40.5 with 8; pinned, i.e. no staging: 42.9).
class CopyPool {
 public:
  explicit CopyPool(int nthreads, size_t split_min = (size_t)1 << 20);
  ~CopyPool();
  void copy(uint8_t *dst, const uint8_t *src, size_t len);
  // fn(i, n) on each of the pool's n = threads() - 1 worker threads (i = 0 .. n-1), without
  // the caller: start() returns at once, join() waits for every fn to return.  A pool with no
  // worker threads runs fn(0, 1) on the caller inside start() (a staged job must
  // never launch before its bytes are copied); workers() is the number of fn calls either way.
  int workers() const { return n_ > 1 ? n_ - 1 : 1; }
  void start(std::function<void(int, int)> fn);
  void join();

 private:
  const size_t split_min_;  // shorter copies run on the calling thread alone
  std::function<void(int, int)> fn_;  // start(): the workers' task
  void part(int i);
  void run(int i);
  void post();
  void wait_all();
  int n_;
  std::vector<std::thread> threads_;
  // one task at a time: the caller sets the task fields, then post() bumps gen_ (futex) and
  // the workers count pending_ down (futex for the caller's wait)
  std::atomic<uint32_t> gen_{0}, pending_{0};
  std::atomic<bool> stop_{false};
  uint8_t *dst_ = nullptr;
  const uint8_t *src_ = nullptr;
  size_t len_ = 0;
};

// A contiguous run of a job's byte stream: src[0..len) -> dst[0..len).
struct Seg {
  const uint8_t *src;
  uint8_t *dst;
  size_t len;
};

// One chunk's GPU timeline, ms after its job's start event.
struct ChunkTime {
  size_t bytes;
  float h2d_start, kernel_start, kernel_end, d2h_end;
};

struct JobResult {
  int status = 0;  // VF_OK or a VF_E_* code
  hipError_t hip = hipSuccess;
  std::string msg;
  float kernel_ms = 0.f;  // sum of the job's kernel durations
  float gpu_ms = -1.f;    // job start -> last D2H done
  bool zero_copy = false; // inverted in place over PCIe (no slot ring)
  std::vector<ChunkTime> timeline;
};

class Engine {
 public:
  Engine() = default;
  ~Engine();  // finishes queued jobs, joins the thread, frees the slots
  hipError_t init(int device, int nslots, size_t slot_bytes, const LaunchCfg &cfg, std::string *err);

  uint64_t submit(std::vector<Seg> &&segs);  // returns the job id (> 0); never blocks on the GPU
  // Synchronous zero-copy on the calling thread (no hand-off to the engine thread and back):
  // false, with nothing done, unless every byte lies in noted device-mapped ranges.
  // Otherwise, for a job of at most kStagedMax bytes, the same launches on the calling thread
  // with the unmapped side staged through a small mapped ring (run_staged).
  bool run_now(const std::vector<Seg> &segs, JobResult *out);
  bool wait(uint64_t id, JobResult *out);    // false: unknown id
  bool query(uint64_t id, bool *done);       // false: unknown id
  void drain();                              // wait for every submitted job

  void note_pinned(const void *p, size_t n);
  void forget_pinned(const void *p);
  bool is_pinned(const void *p, size_t len);
  // device address of [p, p + len) when it lies inside one range noted above and that range is
  // mapped into the device's address space; else nullptr
  uint8_t *mapped(const void *p, size_t len);

 private:
  struct Piece {
    const uint8_t *src;
    uint8_t *dst;
    size_t off;  // offset in the slot
    size_t len;
  };
  struct Job {
    uint64_t id = 0;
    std::vector<Seg> segs;
    bool direct = true;  // every byte page-locked: DMA straight from/to the caller
    bool mapped = false;  // every byte in a noted, device-mapped range: inverted in place over PCIe
    std::vector<Seg> dsegs;  // mapped: the segments by their device addresses
    hipEvent_t end = nullptr;  // mapped: after the job's last launch
    size_t total = 0, chunk = 0;
    size_t queued = 0;            // bytes put into slots so far
    size_t seg = 0, seg_off = 0;  // fill cursor
    int chunks_submitted = 0, chunks_done = 0;
    bool started = false, all_submitted = false;
    hipEvent_t start = nullptr;
    float kernel_ms = 0.f;
    std::vector<ChunkTime> timeline;
  };
  struct Slot {
    enum State { kFree, kIn, kOut } state = kFree;
    hipEvent_t h0 = nullptr, k0 = nullptr, k1 = nullptr, done = nullptr;
    uint8_t *pin_in = nullptr, *pin_out = nullptr;
    uint8_t *d_in = nullptr, *d_out = nullptr;
    Job *job = nullptr;
    size_t bytes = 0;
    std::vector<Piece> pieces;
  };
  static constexpr size_t kMaxResults = 1024;

  void run();
  hipError_t ensure_streams();
  size_t chunk_size(const Job &job) const;
  bool step_fill();
  bool step_d2h();
  bool step_retire();
  bool launch_mapped(Job *job);
  bool run_staged(const std::vector<Seg> &segs, size_t total, JobResult *out);
  int run_gated(const Seg &sg, JobResult *out);  // -1: not this job's shape (run_staged takes it)
  hipError_t ensure_staging();
  bool step_mapped_retire();
  void fail_all(hipError_t e, const char *what);
  int busy_slots() const;
  hipEvent_t take_event();
  void give_event(hipEvent_t e);

  int device_ = 0;
  LaunchCfg cfg_;
  size_t slot_bytes_ = 0;
  hipStream_t s_in_ = nullptr, s_out_ = nullptr;
  hipStream_t s_map_ = nullptr;  // zero-copy launches (beside the slot ring's two streams)
  std::mutex stream_mu_;         // creation of the three streams (engine thread or run_now)
  std::atomic<bool> streams_ready_{false};
  bool zero_copy_ = true;        // VF_ZEROCOPY=0: caller-pinned jobs take the slot ring
  std::deque<Job *> mapped_live_;  // launched zero-copy jobs, in launch order
  std::vector<Slot> slots_;
  size_t fill_ = 0, d2h_ = 0, retire_ = 0;
  std::unique_ptr<CopyPool> pool_;
  // run_staged: page-locked, device-mapped staging for the unmapped side of a job (one input
  // and one output buffer of kStagedMax) and a copy pool of its own (the engine thread's pool_
  // is not reentrant)
  static constexpr size_t kStagedMax = (size_t)32 << 20;
  uint8_t *stg_in_ = nullptr, *stg_out_ = nullptr;    // host addresses
  uint8_t *stg_din_ = nullptr, *stg_dout_ = nullptr;  // their device addresses
  bool stg_ready_ = false;
  // run_gated: per-piece landed counts (host-written) and the kernel's give-up flag, page-locked
  uint32_t *stg_flags_ = nullptr, *stg_dflags_ = nullptr;
  uint32_t *stg_frontier_ = nullptr;  // device memory: the relay's published piece count
  uint32_t gate_gen_ = 0;
  uint64_t clock_khz_ = 100000;  // wall_clock64() rate
  std::mutex stg_mu_;                           // one staged job at a time
  std::unique_ptr<CopyPool> cpool_;
  std::mutex ev_mu_;             // free_events_: the engine thread and run_now's caller both take and give
  std::vector<hipEvent_t> free_events_;

  std::mutex mu_;  // guards everything below
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  bool broken_ = false;
  uint64_t next_id_ = 1;
  std::deque<std::unique_ptr<Job>> pending_;  // jobs with bytes not yet in a slot
  std::vector<std::unique_ptr<Job>> live_;    // fully queued, not yet retired
  std::set<uint64_t> unfinished_;
  std::map<uint64_t, JobResult> results_;     // finished, not yet collected by wait()

  struct PinRange {
    uintptr_t host;
    size_t len;
    uintptr_t dev;  // 0: not mapped into the device's address space
  };
  std::mutex pin_mu_;
  std::vector<PinRange> pinned_;
  std::thread thread_;
};

}  // namespace vf
