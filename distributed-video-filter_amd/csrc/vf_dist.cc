// vf_dist.cc -- the distributor's control plane in native code (include/vfdist.h).
//
// Reference: distributor.py:173-344.  Its dispatch thread (:205-251) answers one READY per
// 10 ms poll and its collect thread (:253-289) books one result per poll; reassembly (:291-344)
// keeps a dict of results.  The Python Distributor of this build (vfilter/distributor.py) keeps
// that API and its semantics; this file is the same state machine for the lossless ring
// deployment, built for 8 GPUs' worth of frames through one process:
//
//   * one I/O thread owns both listeners and every peer socket (epoll, non-blocking); a
//     dispatch is built and booked under the engine lock and queued on the peer's connection,
//     and written by whichever thread queued it or by the I/O thread when the socket is full --
//     no socket call ever blocks, so no lock holder can wait on a peer;
//   * frames are records in per-worker / per-shard index-ordered lanes, a dispatch is one
//     message per batch (wire v2 binary records, or v1 JSON, or the reference's v0), results are
//     booked per message, and in-order release is a ring keyed by frame index;
//   * frames live in one shared-memory slice per worker (created here, NUMA-bound to the
//     worker's GPU node before any page exists), so only slot numbers cross the sockets.
//
// Worker loss follows the Python engine rule for rule (distributor.py docstring): eviction on
// batch_timeout or disconnect, re-queue of in-flight frames as copies moved into a live worker's
// slice, quarantine of the evicted copies' slots until their late result / disconnect / one more
// batch_timeout, duplicates dropped, a frame counted lost after max_attempts dispatches, shards
// re-homed and re-taken.
#include "vfdist.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "vf_json.h"

namespace {

constexpr uint32_t kMaxParts = 1u << 16;
constexpr size_t kReadBurst = 8u << 20;  // bytes read from one connection before parsing
constexpr int64_t kDefaultMaxPart = int64_t(1) << 30;
constexpr size_t kRecord = 40;  // wire.COLS: index i64, nbytes i64, slot i32, ndim i32, shape i32[4]
constexpr uint64_t kEvListenD = 1, kEvListenC = 2, kEvWake = 3, kEvListenDU = 4, kEvListenCU = 5, kFirstConn = 16;

double mono() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string sys_err(const char* what) {
    char b[256];
    std::snprintf(b, sizeof b, "%s: %s", what, std::strerror(errno));
    return b;
}

// ---- framing -----------------------------------------------------------------------------
// "tcp" transport framing (vfilter/transport.py): u32 nparts, then per part u64 length + bytes.

struct OutMsg {
    std::string own;  // framing and small parts
    struct Seg {
        const uint8_t* ext;  // nullptr: own[off, off + len)
        size_t off, len;
    };
    std::vector<Seg> segs;
};

class MsgBuilder {
  public:
    explicit MsgBuilder(uint32_t nparts) {
        m_.own.append((const char*)&nparts, 4);
        mark_ = 0;
    }
    void part(const void* p, size_t n) {  // copied into the message
        uint64_t len = n;
        m_.own.append((const char*)&len, 8);
        m_.own.append((const char*)p, n);
    }
    void part(const std::string& s) { part(s.data(), s.size()); }
    void ext(const uint8_t* p, size_t n) {  // referenced (a ring slot): not copied
        uint64_t len = n;
        m_.own.append((const char*)&len, 8);
        cut();
        if (n) m_.segs.push_back({p, 0, n});
    }
    OutMsg done() {
        cut();
        return std::move(m_);
    }

  private:
    void cut() {
        if (m_.own.size() > mark_) m_.segs.push_back({nullptr, mark_, m_.own.size() - mark_});
        mark_ = m_.own.size();
    }
    OutMsg m_;
    size_t mark_;
};

struct Conn {
    int fd = -1;
    uint64_t id = 0;
    int role = 0;  // 0: dispatch (ROUTER side), 1: collect (PULL side)
    // reading: I/O thread only
    std::vector<uint8_t> rbuf;
    size_t rlen = 0;
    // writing
    std::mutex wmu;
    std::deque<OutMsg> out;
    size_t seg = 0, off = 0;  // progress inside out.front()
    bool want_out = false;
    bool closed = false;
    ~Conn() {
        if (fd >= 0) ::close(fd);
    }
};

// ---- state -------------------------------------------------------------------------------

struct Batch {
    double t;
    int remaining;
};

struct Frame {  // one copy of a frame (queued, in flight, or quarantined)
    int64_t index = 0;
    int64_t nbytes = 0;
    int32_t ndim = -1;
    int32_t shape[4] = {0, 0, 0, 0};
    int32_t slot = -1;      // global slot id it reads from
    int32_t src_slot = -1;  // a re-queued copy still reading from a quarantined slot
    int attempts = 0;
    double queued_at = 0.0, evicted_at = 0.0;
    std::shared_ptr<Batch> batch;
};

using Lane = std::deque<Frame*>;

struct Peer {
    uint64_t cid = 0;
    std::string wid;
    int version = 1, wire = 1, numa = -1, order = 0;
    bool shm = false;
    std::deque<int> requests;
    int64_t frames_sent = 0, batches_sent = 0, results = 0, errors = 0;
    int home_shard = -1, slice = -1, evictions = 0;
    Lane queue;
    std::unordered_map<int64_t, Frame*> inflight, quarantine;
    std::deque<std::shared_ptr<Batch>> batches;
    bool alive = true, gone = false;
    double last_seen = 0.0, waiting_since = -1.0;
    std::string v2_head;  // FRAMES2 head: {"ring": {...}} for a ring reader, {} otherwise
    std::string ring_json;
};

struct Slice {
    std::string name;
    uint8_t* base = nullptr;
    size_t bytes = 0;
    int numa = -1;
    bool bound = false;
    uint64_t owner = 0;
    std::vector<int> free;
};

struct Entry {  // reorder window entry
    uint8_t state = 0;  // 0 empty, 1 result, 2 lost
    int64_t index = 0;
    vfd_frame f{};
    double t_in = 0.0;
};

struct Held {
    int32_t slot;
    std::unique_ptr<std::vector<uint8_t>> heap;
};

struct ResMeta {  // one frame of a result message, whatever its wire form
    int64_t index = 0, nbytes = 0;
    int32_t slot = -1, ndim = -1, shape[4] = {0, 0, 0, 0};
    double start = 0.0, end = 0.0;
    bool error = false;
    const uint8_t* payload = nullptr;
    size_t plen = 0;
};

struct Span {
    const uint8_t* p;
    size_t n;
};

int64_t pid_of(const std::string& s) {
    if (s.empty() || s.size() > 18) return 0;
    int64_t v = 0;
    for (char c : s) {
        if (c < '0' || c > '9') return 0;
        v = v * 10 + (c - '0');
    }
    return v;
}

bool parse_i64(const Span& sp, int64_t& v) {
    if (sp.n == 0 || sp.n > 20) return false;
    std::string t((const char*)sp.p, sp.n);
    char* e = nullptr;
    errno = 0;
    long long x = std::strtoll(t.c_str(), &e, 10);
    if (errno || *e) return false;
    v = x;
    return true;
}

bool parse_f64(const Span& sp, double& v) {
    if (sp.n == 0 || sp.n > 64) return false;
    std::string t((const char*)sp.p, sp.n);
    char* e = nullptr;
    v = std::strtod(t.c_str(), &e);
    return *e == 0;
}

bool span_is(const Span& sp, const char* tag) {
    size_t n = std::strlen(tag);
    return sp.n == n && std::memcmp(sp.p, tag, n) == 0;
}

void shape_from_json(const vfjson::Value* v, int32_t& ndim, int32_t* shape) {
    ndim = -1;
    if (!v || v->type != vfjson::Value::Arr || v->arr.size() > 4) return;
    ndim = (int32_t)v->arr.size();
    for (int k = 0; k < ndim; ++k) shape[k] = (int32_t)v->arr[k].as_int();
}

void put_shape(std::string& o, int32_t ndim, const int32_t* shape) {
    if (ndim < 0) {
        o += "null";
        return;
    }
    o += '[';
    for (int k = 0; k < ndim; ++k) {
        if (k) o += ", ";
        vfjson::put_int(o, shape[k]);
    }
    o += ']';
}

long mbind_preferred(void* addr, size_t len, int node) {
#ifdef SYS_mbind
    unsigned long mask[4] = {0, 0, 0, 0};
    if (node < 0 || node >= 256) return -1;
    mask[node / 64] = 1UL << (node % 64);
    return syscall(SYS_mbind, addr, len, 1 /* MPOL_PREFERRED */, mask, 257UL, 0U);
#else
    (void)addr; (void)len; (void)node;
    return -1;
#endif
}

std::atomic<int> g_engine_seq{0};

}  // namespace

// ==========================================================================================

struct vfd_engine {
    vfd_config cfg{};
    std::string host;
    int64_t slot_bytes = 0;
    int64_t max_part = kDefaultMaxPart;
    int seq = 0;
    bool copy_results = false;  // zero_copy=False: results copied out, slots freed on arrival
    bool unix_too = true;       // also listen on "\0vfd-tcp-<port>" for same-host peers

    std::mutex mu;
    std::condition_variable cv_in, cv_out;
    bool started = false;
    std::atomic<bool> stopping{false};
    std::string err;

    // ingest and lanes
    int64_t counter = 0;
    std::unordered_map<int32_t, int64_t> reserved;
    std::unordered_map<int32_t, Frame*> clone_src;
    std::unordered_map<int64_t, int> copies;
    std::unordered_set<int64_t> settled;
    std::vector<Slice> slices;
    std::vector<std::unique_ptr<Peer>> peers;  // registration order
    std::unordered_map<uint64_t, Peer*> by_cid;
    std::unordered_map<std::string, Peer*> by_wid;
    std::vector<uint64_t> shard_home, shard_owner;  // 0: none
    std::vector<Lane> shard_lanes;
    Lane orphans;
    uint64_t rr = 0;
    double fill_deadline = 0.0;

    // counters
    int64_t results_received = 0, result_errors = 0, frames_lost = 0, frames_requeued = 0, duplicates = 0,
            evictions = 0, departures = 0, quarantine_expired = 0, dispatches = 0, result_messages = 0;

    // reassembly
    std::vector<Entry> win;
    int64_t next_index = 0;
    int64_t buffered = 0, max_depth = 0, out_of_order = 0, released_n = 0, lost_count = 0;
    double wait_total = 0.0, wait_max = 0.0;
    std::deque<vfd_frame> released;
    std::unordered_map<int64_t, Held> held;
    std::unordered_map<int64_t, std::unique_ptr<std::vector<uint8_t>>> pending_heap;  // by index, until release

    // I/O
    int epfd = -1, evfd = -1, lfd[2] = {-1, -1}, ufd[2] = {-1, -1};
    int port[2] = {0, 0};
    std::thread io;
    std::unordered_map<uint64_t, std::shared_ptr<Conn>> conns;     // under mu
    std::unordered_map<uint64_t, std::shared_ptr<Conn>> io_conns;  // I/O thread only
    uint64_t next_cid = kFirstConn;
    std::vector<std::shared_ptr<Conn>> dirty;  // under mu: connections with queued messages

    // ---------------------------------------------------------------------------------------
    // small helpers (mu held)

    Peer* peer_of_cid(uint64_t cid) {
        auto it = by_cid.find(cid);
        return it == by_cid.end() ? nullptr : it->second;
    }
    uint8_t* in_addr(int32_t slot) {
        const int rs = cfg.ring_slots;
        Slice& s = slices[(size_t)(slot / rs)];
        return s.base + (size_t)(slot % rs) * 2 * (size_t)slot_bytes;
    }
    uint8_t* out_addr(int32_t slot) { return in_addr(slot) + slot_bytes; }
    bool slot_valid(int32_t slot) const {
        return slot >= 0 && (size_t)(slot / cfg.ring_slots) < slices.size();
    }

    void free_slot(int32_t slot, bool notify = true) {
        if (slot < 0 || !slot_valid(slot)) return;
        auto c = clone_src.find(slot);
        if (c != clone_src.end()) {
            Frame* clone = c->second;
            clone_src.erase(c);
            if (clone->slot < 0) {  // the re-queued copy now owns it
                clone->slot = slot;
                clone->src_slot = -1;
                return;
            }
        }
        slices[(size_t)(slot / cfg.ring_slots)].free.push_back(slot % cfg.ring_slots);
        if (notify) cv_in.notify_all();
    }

    int32_t alloc_slot(int sid) {
        Slice& s = slices[(size_t)sid];
        if (s.free.empty()) return -1;
        int k = s.free.back();
        s.free.pop_back();
        return sid * cfg.ring_slots + k;
    }

    void copy_done(int64_t idx) {
        auto it = copies.find(idx);
        int n = (it == copies.end() ? 0 : it->second) - 1;
        if (n > 0) {
            it->second = n;
        } else {
            if (it != copies.end()) copies.erase(it);
            settled.erase(idx);
        }
    }
    void settle(int64_t idx) {
        auto it = copies.find(idx);
        if (it != copies.end() && it->second > 0) settled.insert(idx);
    }

    // forget a frame copy that leaves every queue (lock held)
    void drop_frame(Frame* f) {
        if (f->src_slot >= 0) {
            auto c = clone_src.find(f->src_slot);
            if (c != clone_src.end() && c->second == f) clone_src.erase(c);
        }
        delete f;
    }

    void release_copy(Frame* it) {  // a queued copy whose frame is settled: not dispatched
        if (it->slot >= 0) {
            free_slot(it->slot);
            it->slot = -1;
        }
        copy_done(it->index);
    }

    // ---- reassembly (reorder.OrderedBuffer, lossless) ---------------------------------------
    Entry& entry(int64_t idx) {
        size_t cap = win.size();
        if ((uint64_t)(idx - next_index) >= cap) {
            size_t ncap = cap ? cap : 1024;
            while ((uint64_t)(idx - next_index) >= ncap) ncap *= 2;
            std::vector<Entry> nw(ncap);
            for (size_t k = 0; k < cap; ++k) {
                Entry& e = win[k];
                if (e.state) nw[(size_t)e.index & (ncap - 1)] = e;
            }
            win.swap(nw);
        }
        return win[(size_t)idx & (win.size() - 1)];
    }
    bool present(int64_t idx) {
        if (idx < next_index || win.empty() || (uint64_t)(idx - next_index) >= win.size()) return false;
        Entry& e = win[(size_t)idx & (win.size() - 1)];
        return e.state != 0 && e.index == idx;
    }
    bool push_result(const vfd_frame& f) {
        int64_t idx = f.index;
        if (idx < next_index || present(idx)) return false;  // duplicate, lost or already released
        Entry& e = entry(idx);
        e.state = 1;
        e.index = idx;
        e.f = f;
        e.t_in = mono();
        if (idx != next_index) ++out_of_order;
        if (++buffered > max_depth) max_depth = buffered;
        return true;
    }
    void mark_lost(int64_t idx) {
        if (idx < next_index || present(idx)) return;
        Entry& e = entry(idx);
        e.state = 2;
        e.index = idx;
    }
    void release_ready() {
        if (win.empty()) return;
        double now = mono();
        bool any = false;
        for (;;) {
            Entry& e = win[(size_t)next_index & (win.size() - 1)];
            if (!e.state || e.index != next_index) break;
            if (e.state == 2) {
                ++lost_count;
            } else {
                double w = now - e.t_in;
                wait_total += w;
                if (w > wait_max) wait_max = w;
                ++released_n;
                --buffered;
                released.push_back(e.f);
                any = true;
            }
            e.state = 0;
            ++next_index;
        }
        if (any) cv_out.notify_all();
    }
    void lose(int64_t idx) {
        ++frames_lost;
        settle(idx);
        mark_lost(idx);
        release_ready();
        cv_in.notify_all();
    }

    // ---- lanes ----------------------------------------------------------------------------
    int chunk_owner(int64_t idx) const {
        return (int)((idx / cfg.shard_chunk) % cfg.shard_workers);
    }
    size_t waiting() const {
        size_t n = 0;
        if (cfg.policy == VFD_POLICY_PULL) {
            n = orphans.size();
            for (auto& p : peers) n += p->queue.size();
        } else {
            for (auto& ln : shard_lanes) n += ln.size();
        }
        return n;
    }
    Lane* lane_for(Frame* it) {
        if (cfg.policy == VFD_POLICY_SHARD) return &shard_lanes[(size_t)chunk_owner(it->index)];
        if (it->slot >= 0) {
            Peer* o = peer_of_cid(slices[(size_t)(it->slot / cfg.ring_slots)].owner);
            if (o && o->alive) return &o->queue;
        }
        Peer* best = nullptr;
        for (auto& up : peers) {
            Peer* p = up.get();
            if (!p->alive || p->slice < 0) continue;
            if (!best || p->queue.size() + p->inflight.size() < best->queue.size() + best->inflight.size())
                best = p;
        }
        return best ? &best->queue : &orphans;
    }
    static void insert_ordered(Lane& ln, Frame* it) {
        if (ln.empty() || ln.back()->index < it->index) {
            ln.push_back(it);
            return;
        }
        auto at = ln.end();
        while (at != ln.begin() && (*(at - 1))->index > it->index) --at;
        ln.insert(at, it);
    }
    void relane(std::vector<Frame*>& items) {
        std::vector<std::pair<Lane*, std::vector<Frame*>>> groups;
        for (Frame* it : items) {
            Lane* ln = lane_for(it);
            auto g = std::find_if(groups.begin(), groups.end(), [&](auto& x) { return x.first == ln; });
            if (g == groups.end()) {
                groups.push_back({ln, {}});
                g = groups.end() - 1;
            }
            g->second.push_back(it);
        }
        for (auto& g : groups) {
            std::vector<Frame*> merged(g.first->begin(), g.first->end());
            merged.insert(merged.end(), g.second.begin(), g.second.end());
            std::stable_sort(merged.begin(), merged.end(), [](Frame* a, Frame* b) { return a->index < b->index; });
            g.first->assign(merged.begin(), merged.end());
        }
        cv_in.notify_all();
    }
    std::vector<Lane*> lanes_of(Peer* p) {
        std::vector<Lane*> out;
        if (cfg.policy == VFD_POLICY_PULL) {
            if (!p->queue.empty()) out.push_back(&p->queue);
        } else {
            for (int k = 0; k < cfg.shard_workers; ++k)
                if (shard_owner[(size_t)k] == p->cid && !shard_lanes[(size_t)k].empty())
                    out.push_back(&shard_lanes[(size_t)k]);
        }
        return out;
    }

    // ---- peers ----------------------------------------------------------------------------
    bool make_slice(Peer* p) {
        const size_t bytes = (size_t)cfg.ring_slots * 2 * (size_t)slot_bytes;
        struct statvfs sv;
        if (statvfs("/dev/shm", &sv) == 0 && (uint64_t)sv.f_bavail * sv.f_frsize < bytes) {
            err = "no room in /dev/shm for a ring slice of " + std::to_string(bytes) + " B";
            return false;
        }
        char nm[96];
        std::snprintf(nm, sizeof nm, "vfd-%d-%d-%zu", (int)getpid(), seq, slices.size());
        std::string path = std::string("/") + nm;
        int fd = shm_open(path.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) {
            err = sys_err("shm_open");
            return false;
        }
        if (ftruncate(fd, (off_t)bytes) != 0) {
            err = sys_err("ftruncate");
            ::close(fd);
            shm_unlink(path.c_str());
            return false;
        }
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        ::close(fd);
        if (m == MAP_FAILED) {
            err = sys_err("mmap");
            shm_unlink(path.c_str());
            return false;
        }
        Slice s;
        s.name = nm;
        s.base = (uint8_t*)m;
        s.bytes = bytes;
        s.numa = p->numa;
        // the policy sits on the shared object, so pages follow it whoever faults them in first
        s.bound = p->numa >= 0 && mbind_preferred(m, bytes, p->numa) == 0;
        s.owner = p->cid;
        for (int k = cfg.ring_slots - 1; k >= 0; --k) s.free.push_back(k);
        slices.push_back(std::move(s));
        p->slice = (int)slices.size() - 1;
        p->ring_json = "{\"name\": ";
        vfjson::put_str(p->ring_json, nm);
        p->ring_json += ", \"slot_bytes\": ";
        vfjson::put_int(p->ring_json, slot_bytes);
        p->ring_json += "}";
        return true;
    }

    Peer* register_peer(uint64_t cid, int version, bool shm, const std::string& wid, int numa, int wire) {
        auto up = std::make_unique<Peer>();
        Peer* p = up.get();
        p->cid = cid;
        p->version = version;
        p->shm = shm;
        p->wid = wid;
        p->numa = numa;
        p->wire = wire;
        p->order = (int)peers.size();
        p->last_seen = mono();
        if (!make_slice(p)) {
            std::printf("Distributor: no ring slice for worker %010llx: %s\n", (unsigned long long)cid, err.c_str());
            std::fflush(stdout);
            return nullptr;
        }
        p->v2_head = shm ? "{\"ring\": " + p->ring_json + "}" : std::string("{}");
        peers.push_back(std::move(up));
        by_cid[cid] = p;
        if (!wid.empty()) by_wid[wid] = p;
        if (cfg.policy == VFD_POLICY_SHARD) {
            rebalance_shards();
        } else if (!orphans.empty()) {
            std::vector<Frame*> items(orphans.begin(), orphans.end());
            orphans.clear();
            relane(items);
        }
        cv_in.notify_all();
        return p;
    }

    void revive(Peer* p) {
        p->alive = true;
        if (cfg.verbose) {
            std::printf("Distributor: worker %010llx is back\n", (unsigned long long)p->cid);
            std::fflush(stdout);
        }
        if (cfg.policy == VFD_POLICY_SHARD && p->home_shard >= 0) {
            Peer* other = peer_of_cid(shard_home[(size_t)p->home_shard]);
            if (other && other != p) other->home_shard = -1;
            shard_home[(size_t)p->home_shard] = p->cid;
            rebalance_shards();
        } else if (cfg.policy == VFD_POLICY_PULL && !orphans.empty()) {
            std::vector<Frame*> items(orphans.begin(), orphans.end());  // frames no live worker had
            orphans.clear();
            relane(items);
        }
        cv_in.notify_all();
    }

    void rebalance_shards() {
        std::vector<Peer*> live;
        for (auto& up : peers)
            if (up->alive) live.push_back(up.get());  // registration order
        for (int k = 0; k < cfg.shard_workers; ++k) {
            Peer* home = peer_of_cid(shard_home[(size_t)k]);
            if (!home || !home->alive) {
                Peer* spare = nullptr;
                for (Peer* q : live)
                    if (q->home_shard < 0) {
                        spare = q;
                        break;
                    }
                if (spare) {
                    if (home) home->home_shard = -1;
                    spare->home_shard = k;
                    shard_home[(size_t)k] = spare->cid;
                    home = spare;
                }
            }
            if (home && home->alive) {
                shard_owner[(size_t)k] = home->cid;
                continue;
            }
            Peer* cur = peer_of_cid(shard_owner[(size_t)k]);
            if (cur && cur->alive) continue;
            if (live.empty()) {
                shard_owner[(size_t)k] = 0;
                continue;
            }
            Peer* best = nullptr;
            int best_load = 0;
            for (Peer* q : live) {
                int load = 0;
                for (int j = 0; j < cfg.shard_workers; ++j)
                    if (j != k && shard_owner[(size_t)j] == q->cid) ++load;
                if (!best || load < best_load) {
                    best = q;
                    best_load = load;
                }
            }
            shard_owner[(size_t)k] = best->cid;
        }
    }

    void evict(Peer* p, const char* reason, bool gone) {
        bool was_alive = p->alive;
        p->alive = false;
        p->gone = p->gone || gone;
        p->requests.clear();
        if (was_alive && gone && p->inflight.empty() && p->queue.empty()) {
            ++departures;
        } else if (was_alive) {
            ++p->evictions;
            ++evictions;
            if (cfg.verbose) {
                std::printf("Distributor: worker %010llx evicted (%s); %zu frames in flight re-queued\n",
                            (unsigned long long)p->cid, reason, p->inflight.size());
                std::fflush(stdout);
            }
        }
        std::vector<int64_t> idxs;
        for (auto& kv : p->inflight) idxs.push_back(kv.first);
        std::sort(idxs.begin(), idxs.end());
        std::vector<Frame*> requeue;
        double now = mono();
        for (int64_t idx : idxs) {
            Frame* it = p->inflight[idx];
            it->batch.reset();
            it->evicted_at = now;
            p->quarantine[idx] = it;  // its slot stays out of use until a result frees it
            if (it->attempts >= cfg.max_attempts) {
                lose(idx);
                continue;
            }
            Frame* clone = new Frame(*it);
            clone->slot = -1;
            clone->src_slot = it->slot;
            if (it->slot >= 0) clone_src[it->slot] = clone;
            ++copies[idx];
            ++frames_requeued;
            requeue.push_back(clone);
        }
        p->inflight.clear();
        p->batches.clear();
        for (Frame* f : p->queue) requeue.push_back(f);
        p->queue.clear();
        if (cfg.policy == VFD_POLICY_SHARD) rebalance_shards();
        if (!requeue.empty()) relane(requeue);
        if (p->gone) {  // nothing can come back from it: its quarantined slots are free again
            for (auto& kv : p->quarantine) {
                free_slot(kv.second->slot);
                copy_done(kv.first);
                delete kv.second;
            }
            p->quarantine.clear();
        }
        cv_in.notify_all();
    }

    void expire_quarantine(Peer* p, double now) {
        // per-worker slices: only the worker itself writes its slots, in dispatch order, so
        // after one more batch_timeout the slot can go to its next frame (Python engine rule)
        std::vector<int64_t> done;
        for (auto& kv : p->quarantine)
            if (now - kv.second->evicted_at > cfg.batch_timeout) done.push_back(kv.first);
        for (int64_t idx : done) {
            Frame* it = p->quarantine[idx];
            p->quarantine.erase(idx);
            free_slot(it->slot);
            copy_done(idx);
            ++quarantine_expired;
            delete it;
        }
    }

    void check_deadlines(double now) {
        if (cfg.batch_timeout <= 0) return;
        for (auto& up : peers) {
            Peer* p = up.get();
            if (!p->quarantine.empty()) expire_quarantine(p, now);
            if (!p->alive) continue;
            if (!p->batches.empty() && now - p->batches.front()->t > cfg.batch_timeout) {
                char why[96];
                std::snprintf(why, sizeof why, "no result within %g s", cfg.batch_timeout);
                evict(p, why, false);
                continue;
            }
            bool idle = p->batches.empty() && p->requests.empty() && !lanes_of(p).empty();
            if (!idle) {
                p->waiting_since = -1.0;
            } else if (p->waiting_since < 0) {
                p->waiting_since = now;
            } else if (now - p->waiting_since > cfg.batch_timeout) {
                char why[96];
                std::snprintf(why, sizeof why, "frames waiting, no request for %g s", cfg.batch_timeout);
                evict(p, why, false);
            }
        }
    }

    // ---- dispatch -------------------------------------------------------------------------
    bool fill_pending(Peer* p, int credit, double now) {
        if (p->version == 0 || credit <= 1 || p->inflight.empty() || cfg.batch_wait <= 0) return false;
        auto lanes = lanes_of(p);
        if (lanes.empty()) return false;
        size_t n = 0;
        double oldest = 1e300;
        for (Lane* ln : lanes) {
            n += ln->size();
            oldest = std::min(oldest, ln->front()->queued_at);
        }
        if ((int)n >= credit) return false;
        if (now - oldest < cfg.batch_wait) {
            double dl = oldest + cfg.batch_wait;
            if (fill_deadline == 0.0 || dl < fill_deadline) fill_deadline = dl;
            return true;
        }
        return false;
    }

    bool place(Frame* it, Peer* p) {  // make sure the copy sits in p's slice
        if (it->slot >= 0 && it->slot / cfg.ring_slots == p->slice) return true;
        int32_t src = it->slot >= 0 ? it->slot : it->src_slot;
        if (src < 0) return true;
        int32_t nw = alloc_slot(p->slice);
        if (nw < 0) return false;
        std::memcpy(in_addr(nw), in_addr(src), (size_t)it->nbytes);
        if (it->slot >= 0) {
            free_slot(it->slot);
        } else {
            auto c = clone_src.find(src);
            if (c != clone_src.end() && c->second == it) clone_src.erase(c);
        }
        it->slot = nw;
        it->src_slot = -1;
        return true;
    }

    void take(Peer* p, int credit, std::vector<Frame*>& out) {
        if (p->version == 0) credit = 1;
        auto lanes = lanes_of(p);
        if (lanes.empty()) return;
        if (lanes.size() == 1) {
            Lane& ln = *lanes[0];
            std::vector<Frame*> skipped;
            bool took = false;
            while (!ln.empty() && (int)out.size() < credit) {
                Frame* it = ln.front();
                ln.pop_front();
                took = true;
                if (settled.count(it->index)) {
                    release_copy(it);
                    drop_frame(it);
                } else if (place(it, p) || it->slot >= 0) {
                    // a copy that finds no free slot in p's slice but owns one elsewhere (a lost
                    // worker's) travels as a socket part: waiting for room could wait for ever
                    // when p's slots hold later results the consumer cannot take before this one
                    out.push_back(it);
                } else {
                    skipped.push_back(it);  // still reading from a quarantined slot: not waited on
                }
            }
            for (auto r = skipped.rbegin(); r != skipped.rend(); ++r) ln.push_front(*r);
            if (took) cv_in.notify_all();
            return;
        }
        std::vector<Frame*> all;
        for (Lane* ln : lanes) all.insert(all.end(), ln->begin(), ln->end());
        std::stable_sort(all.begin(), all.end(), [](Frame* a, Frame* b) { return a->index < b->index; });
        std::unordered_set<Frame*> taken, dead;
        for (Frame* it : all) {
            if ((int)out.size() >= credit) break;
            if (settled.count(it->index)) {
                release_copy(it);
                taken.insert(it);
                dead.insert(it);
                continue;
            }
            if (place(it, p) || it->slot >= 0) {
                out.push_back(it);
                taken.insert(it);
            }
        }
        if (!taken.empty()) {
            for (Lane* ln : lanes) {
                Lane keep;
                for (Frame* it : *ln)
                    if (!taken.count(it)) keep.push_back(it);
                ln->swap(keep);
            }
            for (Frame* it : dead) drop_frame(it);
            cv_in.notify_all();
        }
    }

    // a frame p reads from its own ring slice (else it travels as a socket part)
    bool in_ring(Peer* p, Frame* it) const { return p->shm && it->slot / cfg.ring_slots == p->slice; }

    void queue_dispatch(Peer* p, std::vector<Frame*>& items) {
        auto cit = conns.find(p->cid);
        std::shared_ptr<Conn> c = cit == conns.end() ? nullptr : cit->second;
        OutMsg msg;
        const int rs = cfg.ring_slots;
        if (p->version == 0) {  // distributor.py:236-238: [index, frame]
            Frame* it = items[0];
            MsgBuilder b(2);
            std::string idx = std::to_string(it->index);
            b.part(idx);
            b.ext(in_addr(it->slot), (size_t)it->nbytes);
            msg = b.done();
        } else if (p->wire >= 2) {
            size_t npay = 0;
            for (Frame* it : items) npay += in_ring(p, it) ? 0 : 1;
            MsgBuilder b((uint32_t)(3 + npay));
            b.part("FRAMES2", 7);
            b.part(npay < items.size() ? p->v2_head : std::string("{}"));
            std::string cols(items.size() * kRecord, '\0');
            for (size_t i = 0; i < items.size(); ++i) {
                Frame* it = items[i];
                char* r = &cols[i * kRecord];
                int32_t slot = in_ring(p, it) ? it->slot % rs : -1;
                std::memcpy(r, &it->index, 8);
                std::memcpy(r + 8, &it->nbytes, 8);
                std::memcpy(r + 16, &slot, 4);
                std::memcpy(r + 20, &it->ndim, 4);
                std::memcpy(r + 24, it->shape, 16);
            }
            b.part(cols);
            for (Frame* it : items)
                if (!in_ring(p, it)) b.ext(in_addr(it->slot), (size_t)it->nbytes);
            msg = b.done();
        } else {  // v1, per-frame JSON
            std::string head = "{\"frames\": [";
            for (size_t i = 0; i < items.size(); ++i) {
                Frame* it = items[i];
                if (i) head += ", ";
                head += "{\"index\": ";
                vfjson::put_int(head, it->index);
                head += ", \"nbytes\": ";
                vfjson::put_int(head, it->nbytes);
                head += ", \"shape\": ";
                put_shape(head, it->ndim, it->shape);
                head += ", \"slot\": ";
                if (in_ring(p, it)) vfjson::put_int(head, it->slot % rs);
                else head += "null";
                head += "}";
            }
            head += "]";
            size_t npay = 0;
            for (Frame* it : items) npay += in_ring(p, it) ? 0 : 1;
            if (npay < items.size()) head += ", \"ring\": " + p->ring_json;
            head += "}";
            MsgBuilder b((uint32_t)(2 + npay));
            b.part("FRAMES1", 7);
            b.part(head);
            for (Frame* it : items)
                if (!in_ring(p, it)) b.ext(in_addr(it->slot), (size_t)it->nbytes);
            msg = b.done();
        }
        // book before the bytes leave: a result can never arrive before its dispatch record
        p->frames_sent += (int64_t)items.size();
        ++p->batches_sent;
        ++dispatches;
        auto batch = std::make_shared<Batch>(Batch{mono(), (int)items.size()});
        for (Frame* it : items) {
            ++it->attempts;
            it->batch = batch;
            p->inflight[it->index] = it;
        }
        p->batches.push_back(batch);
        if (!c) {  // its connection is gone (the I/O thread evicts it): back to the queues
            unsend(p, items);
            return;
        }
        {
            std::lock_guard<std::mutex> wl(c->wmu);
            if (c->closed) {
                c.reset();
            } else {
                c->out.push_back(std::move(msg));
            }
        }
        if (!c) {
            unsend(p, items);
            return;
        }
        dirty.push_back(c);
    }

    void unsend(Peer* p, std::vector<Frame*>& items) {
        std::vector<Frame*> mine;
        for (Frame* it : items) {
            auto f = p->inflight.find(it->index);
            if (f != p->inflight.end() && f->second == it) {
                p->inflight.erase(f);
                it->batch.reset();
                --it->attempts;
                mine.push_back(it);
            }
        }
        p->frames_sent -= (int64_t)mine.size();
        relane(mine);
        evict(p, "dispatch refused (worker disconnected)", true);
    }

    void serve_waiting() {
        double now = mono();
        fill_deadline = 0.0;
        for (auto& up : peers) {
            Peer* p = up.get();
            while (p->alive && !p->requests.empty()) {
                if (fill_pending(p, p->requests.front(), now)) break;
                std::vector<Frame*> items;
                take(p, p->requests.front(), items);
                if (items.empty()) break;
                p->requests.pop_front();
                queue_dispatch(p, items);
            }
        }
    }

    // ---- requests and results ---------------------------------------------------------------
    void on_request(uint64_t cid, const std::vector<Span>& parts) {
        if (parts.empty()) return;
        int version;
        int credit = 1, numa = -1, wire = 1;
        bool shm = false;
        std::string wid;
        if (span_is(parts[0], "READY")) {  // worker.py:39
            version = 0;
        } else if (span_is(parts[0], "READY1") && parts.size() >= 2) {
            vfjson::Value v;
            if (!vfjson::parse(parts[1].p, parts[1].n, v) || v.type != vfjson::Value::Obj) return;
            version = 1;
            if (auto x = v.get("credit")) credit = (int)std::max<int64_t>(1, std::min<int64_t>(x->as_int(1), 1 << 20));
            if (auto x = v.get("shm")) shm = x->type == vfjson::Value::Bool && x->b;
            if (auto x = v.get("wid"); x && x->type == vfjson::Value::Str) wid = x->s;
            if (auto x = v.get("numa"); x && x->type == vfjson::Value::Num) numa = (int)x->as_int(-1);
            if (auto x = v.get("wire")) wire = (int)x->as_int(1);
        } else {
            return;
        }
        Peer* p = peer_of_cid(cid);
        if (!p) {
            p = register_peer(cid, version, shm, wid, numa, wire);
            if (!p) return;
        } else if (!p->alive && !p->gone) {
            revive(p);
        }
        p->last_seen = mono();
        p->wire = wire;
        if (version == 0 && p->requests.size() >= 2) return;  // a reference worker re-sends READY every 10 ms
        p->requests.push_back(credit);
    }

    bool parse_result(const std::vector<Span>& parts, std::vector<ResMeta>& metas, std::string& wid,
                      int64_t& pid) {
        metas.clear();
        if (parts.empty()) return false;
        if (span_is(parts[0], "RESULT2")) {
            if (parts.size() < 3 || parts[2].n % kRecord) return false;
            vfjson::Value d;
            if (!vfjson::parse(parts[1].p, parts[1].n, d) || d.type != vfjson::Value::Obj) return false;
            const vfjson::Value* x;
            if ((x = d.get("pid")) && x->type == vfjson::Value::Str) pid = pid_of(x->s);
            if ((x = d.get("wid")) && x->type == vfjson::Value::Str) wid = x->s;
            size_t n = parts[2].n / kRecord;
            metas.resize(n);
            const vfjson::Value* st = d.get("starts");
            const vfjson::Value* en = d.get("ends");
            double s0 = (x = d.get("start")) ? x->as_num() : 0.0, e0 = (x = d.get("end")) ? x->as_num() : 0.0;
            for (size_t i = 0; i < n; ++i) {
                ResMeta& m = metas[i];
                const uint8_t* r = parts[2].p + i * kRecord;
                std::memcpy(&m.index, r, 8);
                std::memcpy(&m.nbytes, r + 8, 8);
                std::memcpy(&m.slot, r + 16, 4);
                std::memcpy(&m.ndim, r + 20, 4);
                std::memcpy(m.shape, r + 24, 16);
                if (m.ndim > 4) m.ndim = 4;
                m.start = st && st->type == vfjson::Value::Arr && i < st->arr.size() ? st->arr[i].as_num() : s0;
                m.end = en && en->type == vfjson::Value::Arr && i < en->arr.size() ? en->arr[i].as_num() : e0;
            }
            if ((x = d.get("errors")) && x->type == vfjson::Value::Obj)
                for (auto& kv : x->obj) {
                    long k = std::strtol(kv.first.c_str(), nullptr, 10);
                    if (k >= 0 && (size_t)k < n) metas[(size_t)k].error = true;
                }
            size_t pi = 3;
            for (auto& m : metas) {
                if (m.slot >= 0 || m.error) continue;
                if (pi >= parts.size()) return false;
                m.payload = parts[pi].p;
                m.plen = parts[pi].n;
                m.nbytes = (int64_t)parts[pi].n;
                ++pi;
            }
            return true;
        }
        if (span_is(parts[0], "RESULT1")) {
            if (parts.size() < 2) return false;
            vfjson::Value d;
            if (!vfjson::parse(parts[1].p, parts[1].n, d) || d.type != vfjson::Value::Obj) return false;
            const vfjson::Value* x;
            if ((x = d.get("pid")) && x->type == vfjson::Value::Str) pid = pid_of(x->s);
            if ((x = d.get("wid")) && x->type == vfjson::Value::Str) wid = x->s;
            if ((x = d.get("frames")) && x->type == vfjson::Value::Arr) {  // per-frame form
                for (auto& f : x->arr) {
                    ResMeta m;
                    const vfjson::Value* y;
                    if (!(y = f.get("index"))) return false;
                    m.index = y->as_int();
                    if ((y = f.get("nbytes"))) m.nbytes = y->as_int();
                    if ((y = f.get("slot")) && !y->null()) m.slot = (int32_t)y->as_int(-1);
                    shape_from_json(f.get("shape"), m.ndim, m.shape);
                    if ((y = f.get("start"))) m.start = y->as_num();
                    if ((y = f.get("end"))) m.end = y->as_num();
                    if ((y = f.get("error")) && !y->null()) m.error = true;
                    metas.push_back(m);
                }
            } else {  // round 4's columnar form
                const vfjson::Value* idx = d.get("index");
                const vfjson::Value* nb = d.get("nbytes");
                if (!idx || !nb || idx->type != vfjson::Value::Arr || nb->type != vfjson::Value::Arr ||
                    idx->arr.size() != nb->arr.size())
                    return false;
                size_t n = idx->arr.size();
                const vfjson::Value* sl = d.get("slot");
                const vfjson::Value* sh = d.get("shape");
                const vfjson::Value* sh1 = d.get("shape1");
                const vfjson::Value* st = d.get("starts");
                const vfjson::Value* en = d.get("ends");
                double s0 = (x = d.get("start")) ? x->as_num() : 0.0, e0 = (x = d.get("end")) ? x->as_num() : 0.0;
                for (size_t i = 0; i < n; ++i) {
                    ResMeta m;
                    m.index = idx->arr[i].as_int();
                    m.nbytes = nb->arr[i].as_int();
                    if (sl && sl->type == vfjson::Value::Arr && i < sl->arr.size() && !sl->arr[i].null())
                        m.slot = (int32_t)sl->arr[i].as_int(-1);
                    if (sh && sh->type == vfjson::Value::Arr && i < sh->arr.size())
                        shape_from_json(&sh->arr[i], m.ndim, m.shape);
                    else
                        shape_from_json(sh1, m.ndim, m.shape);
                    m.start = st && st->type == vfjson::Value::Arr && i < st->arr.size() ? st->arr[i].as_num() : s0;
                    m.end = en && en->type == vfjson::Value::Arr && i < en->arr.size() ? en->arr[i].as_num() : e0;
                    metas.push_back(m);
                }
                if ((x = d.get("errors")) && x->type == vfjson::Value::Obj)
                    for (auto& kv : x->obj) {
                        long k = std::strtol(kv.first.c_str(), nullptr, 10);
                        if (k >= 0 && (size_t)k < n) metas[(size_t)k].error = true;
                    }
            }
            size_t pi = 2;
            for (auto& m : metas) {
                if (m.slot >= 0 || m.error) continue;
                if (pi >= parts.size()) return false;
                m.payload = parts[pi].p;
                m.plen = parts[pi].n;
                ++pi;
            }
            return true;
        }
        if (parts.size() == 5) {  // v0, worker.py:63-67: [index, pid, start, end, frame]
            ResMeta m;
            if (!parse_i64(parts[0], m.index) || !parse_f64(parts[2], m.start) || !parse_f64(parts[3], m.end))
                return false;
            int64_t pv = 0;
            if (parse_i64(parts[1], pv)) pid = pv;
            m.payload = parts[4].p;
            m.plen = parts[4].n;
            m.nbytes = (int64_t)parts[4].n;
            metas.push_back(m);
            return true;
        }
        return false;
    }

    // (worker, dispatched copy) of a result; the copy leaves the worker's in-flight set
    Frame* find_copy(Peer* sender, int64_t idx, Peer*& q_out) {
        auto try_peer = [&](Peer* q) -> Frame* {
            auto f = q->inflight.find(idx);
            if (f != q->inflight.end()) {
                Frame* it = f->second;
                q->inflight.erase(f);
                if (it->batch) {
                    --it->batch->remaining;
                    it->batch.reset();
                }
                while (!q->batches.empty() && q->batches.front()->remaining <= 0) q->batches.pop_front();
                return it;
            }
            auto g = q->quarantine.find(idx);
            if (g != q->quarantine.end()) {
                Frame* it = g->second;
                q->quarantine.erase(g);
                return it;
            }
            return nullptr;
        };
        q_out = nullptr;
        if (sender) {
            Frame* it = try_peer(sender);
            if (it) q_out = sender;
            return it;
        }
        for (auto& up : peers) {
            Frame* it = try_peer(up.get());
            if (it) {
                q_out = up.get();
                return it;
            }
        }
        return nullptr;
    }

    void deliver(int64_t idx, int32_t slot, const ResMeta& m, int64_t pid) {
        vfd_frame f{};
        f.index = idx;
        f.slot = slot;
        f.ndim = m.ndim;
        std::memcpy(f.shape, m.shape, sizeof f.shape);
        f.pid = pid;
        f.start = m.start;
        f.end = m.end;
        std::unique_ptr<std::vector<uint8_t>> heap;
        if (copy_results) {  // zero_copy=False: the result is copied out and its slot freed now
            const uint8_t* src = m.payload ? m.payload : out_addr(slot);
            size_t n = m.payload ? m.plen : (size_t)m.nbytes;
            heap = std::make_unique<std::vector<uint8_t>>(src, src + n);
            f.nbytes = (int64_t)n;
            f.data = (uint64_t)(uintptr_t)heap->data();
            f.slot = -1;
            ++results_received;
            free_slot(slot);
            if (push_result(f)) held[idx] = Held{-1, std::move(heap)};
            return;
        }
        if (m.payload) {  // a result that came back as a socket part
            f.nbytes = (int64_t)m.plen;
            if (slot >= 0 && (int64_t)m.plen <= slot_bytes) {
                if (m.plen) std::memcpy(out_addr(slot), m.payload, m.plen);
                f.data = (uint64_t)(uintptr_t)out_addr(slot);
            } else {
                heap = std::make_unique<std::vector<uint8_t>>(m.payload, m.payload + m.plen);
                f.data = (uint64_t)(uintptr_t)heap->data();
            }
        } else {
            f.nbytes = m.nbytes;
            f.data = (uint64_t)(uintptr_t)out_addr(slot);
        }
        ++results_received;
        if (!push_result(f)) {  // index already released, lost or buffered: nothing to hand out
            free_slot(slot);
            return;
        }
        held[idx] = Held{slot, std::move(heap)};
    }

    void on_result(const std::vector<Span>& parts) {
        std::vector<ResMeta> metas;
        std::string wid;
        int64_t pid = 0;
        if (!parse_result(parts, metas, wid, pid)) {
            std::printf("Error receiving inverted frame: malformed result message\n");
            std::fflush(stdout);
            return;
        }
        ++result_messages;
        Peer* sender = nullptr;
        if (!wid.empty()) {
            auto w = by_wid.find(wid);
            if (w != by_wid.end()) sender = w->second;
        }
        if (sender) sender->last_seen = mono();
        // the common message: every frame a ring result of the sender's own dispatch, in flight
        // once, no error, indices strictly increasing (so none repeats) -- booked in one pass;
        // anything else (a repeated index included) takes the per-record path below
        bool fast = sender != nullptr;
        if (fast)
            for (size_t i = 0; i < metas.size(); ++i) {
                const ResMeta& m = metas[i];
                if (i && m.index <= metas[i - 1].index) {
                    fast = false;
                    break;
                }
                auto f = sender->inflight.find(m.index);
                if (m.error || m.slot < 0 || f == sender->inflight.end() || f->second->slot < 0 ||
                    settled.count(m.index) || m.nbytes < 0 || m.nbytes > slot_bytes) {
                    fast = false;
                    break;
                }
                auto c = copies.find(m.index);
                if (c == copies.end() || c->second != 1) {
                    fast = false;
                    break;
                }
            }
        if (fast) {
            for (auto& m : metas) {
                auto f = sender->inflight.find(m.index);
                if (f == sender->inflight.end()) continue;  // unreachable after the pre-check
                Frame* it = f->second;
                sender->inflight.erase(f);
                if (it->batch) --it->batch->remaining;
                copies.erase(m.index);
                deliver(m.index, it->slot, m, pid);
                delete it;
            }
            while (!sender->batches.empty() && sender->batches.front()->remaining <= 0) sender->batches.pop_front();
            sender->results += (int64_t)metas.size();
            release_ready();
            return;
        }
        for (auto& m : metas) {
            Peer* q = nullptr;
            Frame* it = find_copy(sender, m.index, q);
            int32_t slot = it ? it->slot : -1;
            if (q) {
                ++q->results;
                if (m.error) ++q->errors;
            }
            bool tracked = it != nullptr;
            if (tracked && settled.count(m.index)) {  // a re-queued frame's second result
                ++duplicates;
                free_slot(slot);
                copy_done(m.index);
                delete it;
                continue;
            }
            if (tracked) {
                copy_done(m.index);
                settle(m.index);
            }
            bool bad_len = !m.payload && (m.nbytes < 0 || m.nbytes > slot_bytes);
            if (m.error || bad_len) {
                ++result_errors;
                free_slot(slot);
                mark_lost(m.index);
                release_ready();
                delete it;
                continue;
            }
            if (!m.payload && slot < 0) {  // a ring result with no dispatch record
                delete it;
                continue;
            }
            deliver(m.index, slot, m, pid);
            delete it;
        }
        release_ready();
    }

    void on_disconnect(uint64_t cid) {
        Peer* p = peer_of_cid(cid);
        if (p) evict(p, "connection closed", true);
    }

    // ---- sockets ------------------------------------------------------------------------------
    void flush(const std::shared_ptr<Conn>& c) {
        std::lock_guard<std::mutex> wl(c->wmu);
        if (c->closed) return;
        while (!c->out.empty()) {
            iovec iov[64];
            int n = 0;
            size_t seg = c->seg, off = c->off;
            for (auto mi = c->out.begin(); mi != c->out.end() && n < 64; ++mi) {
                for (; seg < mi->segs.size() && n < 64; ++seg) {
                    const auto& s = mi->segs[seg];
                    const uint8_t* base = s.ext ? s.ext : (const uint8_t*)mi->own.data() + s.off;
                    iov[n].iov_base = (void*)(base + off);
                    iov[n].iov_len = s.len - off;
                    ++n;
                    off = 0;
                }
                seg = 0;
            }
            msghdr mh{};
            mh.msg_iov = iov;
            mh.msg_iovlen = (size_t)n;
            ssize_t w = ::sendmsg(c->fd, &mh, MSG_NOSIGNAL | MSG_DONTWAIT);
            if (w < 0) {
                if (errno == EINTR) continue;
                if (errno == EAGAIN || errno == EWOULDBLOCK) break;
                c->out.clear();  // broken: the read side reports the disconnect
                c->seg = c->off = 0;
                break;
            }
            size_t left = (size_t)w;
            while (left && !c->out.empty()) {
                OutMsg& m = c->out.front();
                size_t avail = m.segs[c->seg].len - c->off;
                if (left < avail) {
                    c->off += left;
                    left = 0;
                    break;
                }
                left -= avail;
                c->off = 0;
                if (++c->seg == m.segs.size()) {
                    c->out.pop_front();
                    c->seg = 0;
                }
            }
        }
        bool want = !c->out.empty();
        if (want != c->want_out) {
            epoll_event ev{};
            ev.events = (uint32_t)(EPOLLIN | EPOLLRDHUP) | (want ? (uint32_t)EPOLLOUT : 0u);
            ev.data.u64 = c->id;
            epoll_ctl(epfd, EPOLL_CTL_MOD, c->fd, &ev);
            c->want_out = want;
        }
    }

    void flush_dirty(std::unique_lock<std::mutex>& lk) {
        // called with mu held; sends happen after it is released
        std::vector<std::shared_ptr<Conn>> todo;
        todo.swap(dirty);
        lk.unlock();
        std::sort(todo.begin(), todo.end());
        todo.erase(std::unique(todo.begin(), todo.end()), todo.end());
        for (auto& c : todo) flush(c);
    }

    void wake_io() {
        uint64_t one = 1;
        ssize_t r = ::write(evfd, &one, 8);
        (void)r;
    }

    int open_listener(int which) {
        int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
        if (fd < 0) {
            err = sys_err("socket");
            return VFD_E_SYS;
        }
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)(which == 0 ? cfg.distribute_port : cfg.collect_port));
        if (host.empty() || host == "*" || host == "0.0.0.0") {
            a.sin_addr.s_addr = htonl(INADDR_ANY);
        } else {
            std::string h = host == "localhost" ? "127.0.0.1" : host;
            if (inet_pton(AF_INET, h.c_str(), &a.sin_addr) != 1) {
                err = "bind address must be an IPv4 address, '*' or 'localhost': " + host;
                ::close(fd);
                return VFD_E_INVALID;
            }
        }
        if (::bind(fd, (sockaddr*)&a, sizeof a) != 0 || ::listen(fd, 128) != 0) {
            err = sys_err("bind/listen");
            ::close(fd);
            return VFD_E_SYS;
        }
        socklen_t len = sizeof a;
        getsockname(fd, (sockaddr*)&a, &len);
        port[which] = ntohs(a.sin_port);
        lfd[which] = fd;
        return VFD_OK;
    }

    // Same-host peers: each listener also answers on an abstract Unix socket named after its TCP
    // port ("\0vfd-tcp-<port>"), which vfilter/transport.py tries first for 127.0.0.1 / localhost
    // (the stdlib transport's framing over AF_UNIX: no TCP stack per message; VF_TCP_UNIX=0 skips it).
    void open_unix(int which) {
        int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
        if (fd < 0) return;
        sockaddr_un a{};
        a.sun_family = AF_UNIX;
        int n = std::snprintf(a.sun_path + 1, sizeof a.sun_path - 1, "vfd-tcp-%d", port[which]);
        socklen_t len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
        if (::bind(fd, (sockaddr*)&a, len) != 0 || ::listen(fd, 128) != 0) {
            ::close(fd);  // another process holds the name: TCP only
            return;
        }
        ufd[which] = fd;
    }

    void accept_all(int which, bool unix_side = false) {
        for (;;) {
            int fd = ::accept4(unix_side ? ufd[which] : lfd[which], nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
            if (fd < 0) return;
            int one = 1;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
            auto c = std::make_shared<Conn>();
            c->fd = fd;
            c->role = which;
            c->rbuf.resize(64 << 10);
            {
                std::lock_guard<std::mutex> lk(mu);
                c->id = next_cid++;
                conns[c->id] = c;
            }
            io_conns[c->id] = c;
            epoll_event ev{};
            ev.events = EPOLLIN | EPOLLRDHUP;
            ev.data.u64 = c->id;
            epoll_ctl(epfd, EPOLL_CTL_ADD, fd, &ev);
        }
    }

    void close_conn(const std::shared_ptr<Conn>& c, const char* why) {
        if (why && cfg.verbose) {
            std::printf("transport: dropping peer %010llx: %s\n", (unsigned long long)c->id, why);
            std::fflush(stdout);
        }
        epoll_ctl(epfd, EPOLL_CTL_DEL, c->fd, nullptr);
        ::shutdown(c->fd, SHUT_RDWR);
        {
            std::lock_guard<std::mutex> wl(c->wmu);
            c->closed = true;
            c->out.clear();
        }
        io_conns.erase(c->id);
        std::unique_lock<std::mutex> lk(mu);
        conns.erase(c->id);
        if (c->role == 0) {
            on_disconnect(c->id);
            serve_waiting();
        }
        flush_dirty(lk);
    }

    // read what the socket has, handle every complete message (one lock hold per read burst)
    void on_readable(const std::shared_ptr<Conn>& c) {
        bool closed = false;
        for (;;) {
            if (c->rlen == c->rbuf.size()) {
                // a full buffer past the burst cap is parsed before reading more (epoll is
                // level-triggered, so the rest is read on the next wakeup): a peer that writes
                // without pause cannot grow the buffer past max(burst, its pending message)
                // or hold the I/O thread; a pending message's size is reserved below
                if (c->rbuf.size() >= kReadBurst) break;
                c->rbuf.resize(std::min(c->rbuf.size() * 2, kReadBurst));
            }
            ssize_t r = ::recv(c->fd, c->rbuf.data() + c->rlen, c->rbuf.size() - c->rlen, MSG_DONTWAIT);
            if (r > 0) {
                c->rlen += (size_t)r;
                if (c->rlen < c->rbuf.size()) break;  // drained
                continue;
            }
            if (r == 0) {
                closed = true;
                break;
            }
            if (errno == EINTR) continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK) closed = true;
            break;
        }
        // parse complete messages
        std::vector<std::vector<Span>> msgs;
        size_t pos = 0;
        const char* bad = nullptr;
        size_t need = 0;
        for (;;) {
            size_t avail = c->rlen - pos;
            if (avail < 4) break;
            uint32_t np;
            std::memcpy(&np, c->rbuf.data() + pos, 4);
            if (np > kMaxParts) {
                bad = "malformed message (part count)";
                break;
            }
            size_t off = pos + 4;
            std::vector<Span> parts;
            bool complete = true;
            for (uint32_t k = 0; k < np; ++k) {
                if (c->rlen - off < 8) {
                    complete = false;
                    need = off + 8 - pos;
                    break;
                }
                uint64_t len;
                std::memcpy(&len, c->rbuf.data() + off, 8);
                if (len > (uint64_t)max_part) {
                    bad = "malformed message (part length)";
                    break;
                }
                off += 8;
                if (c->rlen - off < len) {
                    complete = false;
                    need = off + len - pos;
                    break;
                }
                parts.push_back({c->rbuf.data() + off, (size_t)len});
                off += len;
            }
            if (bad || !complete) break;
            msgs.push_back(std::move(parts));
            pos = off;
        }
        if (!msgs.empty()) {
            std::unique_lock<std::mutex> lk(mu);
            for (auto& m : msgs) {
                if (c->role == 0) on_request(c->id, m);
                else on_result(m);
            }
            serve_waiting();
            flush_dirty(lk);
        }
        if (pos) {
            std::memmove(c->rbuf.data(), c->rbuf.data() + pos, c->rlen - pos);
            c->rlen -= pos;
        }
        if (need > c->rbuf.size()) c->rbuf.resize(need);
        if (bad) {
            close_conn(c, bad);
            return;
        }
        if (closed) close_conn(c, nullptr);
    }

    void io_loop() {
        epoll_event evs[64];
        double next_check = 0.0;
        while (!stopping.load()) {
            int timeout_ms;
            bool fill_due;  // a busy worker's request waits for its batch to fill (read under mu)
            {
                std::lock_guard<std::mutex> lk(mu);
                double now = mono();
                double t = cfg.batch_timeout > 0 ? 0.002 : 0.05;
                fill_due = fill_deadline > 0.0;
                if (fill_due) t = std::min(t, std::max(0.0, fill_deadline - now));
                timeout_ms = (int)(t * 1000.0 + 0.999);
            }
            int n = epoll_wait(epfd, evs, 64, timeout_ms);
            if (n < 0 && errno != EINTR) break;
            for (int i = 0; i < n; ++i) {
                uint64_t id = evs[i].data.u64;
                if (id == kEvListenD) {
                    accept_all(0);
                } else if (id == kEvListenC) {
                    accept_all(1);
                } else if (id == kEvListenDU) {
                    accept_all(0, true);
                } else if (id == kEvListenCU) {
                    accept_all(1, true);
                } else if (id == kEvWake) {
                    uint64_t v;
                    ssize_t r = ::read(evfd, &v, 8);
                    (void)r;
                } else {
                    auto it = io_conns.find(id);
                    if (it == io_conns.end()) continue;
                    std::shared_ptr<Conn> c = it->second;
                    if (evs[i].events & EPOLLOUT) flush(c);
                    if (evs[i].events & (EPOLLIN | EPOLLERR | EPOLLHUP | EPOLLRDHUP)) on_readable(c);
                }
            }
            double now = mono();
            if (now >= next_check || fill_due) {
                std::unique_lock<std::mutex> lk(mu);
                check_deadlines(now);
                serve_waiting();
                flush_dirty(lk);
                next_check = now + 0.001;
            }
        }
    }

    // ---- stats --------------------------------------------------------------------------------
    void counters(int64_t* o) {
        o[VFD_C_RELEASED] = released_n;
        o[VFD_C_LOST] = lost_count;
        o[VFD_C_BUFFERED] = buffered;
        o[VFD_C_MAX_DEPTH] = max_depth;
        o[VFD_C_OUT_OF_ORDER] = out_of_order;
        o[VFD_C_NEXT_INDEX] = next_index;
        o[VFD_C_RESULTS] = results_received;
        o[VFD_C_RESULT_ERRORS] = result_errors;
        o[VFD_C_FRAMES_LOST] = frames_lost;
        o[VFD_C_REQUEUED] = frames_requeued;
        o[VFD_C_DUPLICATES] = duplicates;
        o[VFD_C_EVICTIONS] = evictions;
        o[VFD_C_DEPARTURES] = departures;
        o[VFD_C_QUARANTINE_EXPIRED] = quarantine_expired;
        o[VFD_C_FRAME_COUNTER] = counter;
        int64_t w = 0;
        for (auto& p : peers) w += p->alive ? 1 : 0;
        o[VFD_C_WORKERS] = w;
        int64_t fr = 0;
        for (auto& s : slices) fr += (int64_t)s.free.size();
        o[VFD_C_FREE_SLOTS] = fr;
        o[VFD_C_TOTAL_SLOTS] = (int64_t)slices.size() * cfg.ring_slots;
        o[VFD_C_DISPATCHES] = dispatches;
        o[VFD_C_RESULT_MESSAGES] = result_messages;
    }

    std::string stats_json() {
        using namespace vfjson;
        std::string o = "{";
        auto kv = [&](const char* k, int64_t v) {
            put_str(o, k);
            o += ": ";
            put_int(o, v);
            o += ", ";
        };
        kv("released", released_n);
        kv("lost", lost_count);
        kv("buffered", buffered);
        kv("max_depth", max_depth);
        kv("out_of_order", out_of_order);
        kv("next_index", next_index);
        o += "\"reorder_wait_mean_ms\": ";
        put_num(o, released_n ? 1e3 * wait_total / (double)released_n : 0.0);
        o += ", \"reorder_wait_max_ms\": ";
        put_num(o, 1e3 * wait_max);
        o += ", ";
        kv("frames_dropped", 0);
        kv("results_received", results_received);
        kv("result_errors", result_errors);
        kv("frames_lost", frames_lost);
        kv("frames_requeued", frames_requeued);
        kv("duplicates", duplicates);
        kv("evictions", evictions);
        kv("departures", departures);
        kv("dispatches", dispatches);
        kv("result_messages", result_messages);
        o += "\"workers\": {";
        bool first = true;
        for (auto& up : peers) {
            Peer* p = up.get();
            if (!first) o += ", ";
            first = false;
            char key[32];
            std::snprintf(key, sizeof key, "%010llx", (unsigned long long)p->cid);
            put_str(o, key);
            o += ": {";
            kv("sent", p->frames_sent);
            kv("batches", p->batches_sent);
            kv("results", p->results);
            o += "\"alive\": ";
            o += p->alive ? "true" : "false";
            o += ", \"home_shard\": ";
            if (p->home_shard < 0) o += "null";
            else put_int(o, p->home_shard);
            o += ", \"shards\": [";
            bool f2 = true;
            for (int k = 0; k < (int)shard_owner.size(); ++k)
                if (shard_owner[(size_t)k] == p->cid) {
                    if (!f2) o += ", ";
                    f2 = false;
                    put_int(o, k);
                }
            o += "], ";
            kv("in_flight", (int64_t)p->inflight.size());
            kv("evictions", p->evictions);
            o += "\"wid\": ";
            put_str(o, p->wid);
            o += ", \"wire\": ";
            put_int(o, p->version == 0 ? 0 : p->wire);
            o += ", \"slice\": ";
            if (p->slice < 0) {
                o += "null";
            } else {
                Slice& s = slices[(size_t)p->slice];
                o += "{\"name\": ";
                put_str(o, s.name);
                o += ", \"bytes\": ";
                put_int(o, (int64_t)s.bytes);
                o += ", \"numa\": ";
                if (s.numa < 0) o += "null";
                else put_int(o, s.numa);
                o += ", \"numa_bound\": ";
                o += s.bound ? "true" : "false";
                o += ", \"free\": ";
                put_int(o, (int64_t)s.free.size());
                o += "}";
            }
            o += ", \"slice_id\": ";
            if (p->slice < 0) o += "null";
            else put_int(o, p->slice);
            o += "}";
        }
        o += "}}";
        return o;
    }

    void teardown() {
        for (auto& kv : io_conns) {
            epoll_ctl(epfd, EPOLL_CTL_DEL, kv.second->fd, nullptr);
            ::shutdown(kv.second->fd, SHUT_RDWR);
        }
        io_conns.clear();
        conns.clear();
        dirty.clear();
        for (int w = 0; w < 2; ++w) {
            if (lfd[w] >= 0) ::close(lfd[w]);
            if (ufd[w] >= 0) ::close(ufd[w]);
        }
        if (evfd >= 0) ::close(evfd);
        if (epfd >= 0) ::close(epfd);
        auto kill_lane = [&](Lane& ln) {
            for (Frame* f : ln) delete f;
            ln.clear();
        };
        for (auto& up : peers) {
            kill_lane(up->queue);
            for (auto& kv : up->inflight) delete kv.second;
            for (auto& kv : up->quarantine) delete kv.second;
        }
        for (auto& ln : shard_lanes) kill_lane(ln);
        kill_lane(orphans);
        held.clear();
        for (auto& s : slices) {
            if (s.base) munmap(s.base, s.bytes);
            shm_unlink(("/" + s.name).c_str());
        }
        slices.clear();
    }
};

// ==========================================================================================
// C ABI (the only symbols the library exports; it is built with -fvisibility=hidden)

#pragma GCC visibility push(default)
extern "C" {

int vfd_abi_version(void) { return VFD_ABI_VERSION; }

int vfd_create(const vfd_config* cfg, vfd_engine** out) {
    if (!out) return VFD_E_INVALID;
    *out = nullptr;
    if (!cfg || (cfg->policy != VFD_POLICY_PULL && cfg->policy != VFD_POLICY_SHARD) || cfg->ring_slots < 1 ||
        cfg->ring_slot_bytes < 1 || cfg->queue_size < 1 ||
        (cfg->policy == VFD_POLICY_SHARD && (cfg->shard_workers < 1 || cfg->shard_chunk < 1)))
        return VFD_E_INVALID;
    auto* e = new (std::nothrow) vfd_engine();
    if (!e) return VFD_E_NOMEM;
    e->cfg = *cfg;
    e->host = cfg->host ? cfg->host : "";
    e->cfg.host = nullptr;
    if (e->cfg.max_attempts < 1) e->cfg.max_attempts = 1;
    if (e->cfg.shard_chunk < 1) e->cfg.shard_chunk = 1;
    if (e->cfg.policy == VFD_POLICY_PULL) e->cfg.shard_workers = std::max(1, e->cfg.shard_workers);
    e->slot_bytes = (cfg->ring_slot_bytes + 4095) / 4096 * 4096;
    e->max_part = cfg->max_part > 0 ? cfg->max_part : kDefaultMaxPart;
    e->copy_results = cfg->copy_results != 0;
    e->unix_too = cfg->no_unix == 0;
    e->seq = g_engine_seq.fetch_add(1);
    if (e->cfg.policy == VFD_POLICY_SHARD) {
        e->shard_home.assign((size_t)e->cfg.shard_workers, 0);
        e->shard_owner.assign((size_t)e->cfg.shard_workers, 0);
        e->shard_lanes.resize((size_t)e->cfg.shard_workers);
    }
    e->epfd = epoll_create1(EPOLL_CLOEXEC);
    e->evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    int rc = VFD_OK;
    if (e->epfd < 0 || e->evfd < 0) {
        e->err = sys_err("epoll/eventfd");
        rc = VFD_E_SYS;
    }
    if (rc == VFD_OK) rc = e->open_listener(0);
    if (rc == VFD_OK) rc = e->open_listener(1);
    if (rc != VFD_OK) {
        std::fprintf(stderr, "vfd_create: %s\n", e->err.c_str());
        e->teardown();
        delete e;
        return rc;
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = kEvListenD;
    epoll_ctl(e->epfd, EPOLL_CTL_ADD, e->lfd[0], &ev);
    ev.data.u64 = kEvListenC;
    epoll_ctl(e->epfd, EPOLL_CTL_ADD, e->lfd[1], &ev);
    ev.data.u64 = kEvWake;
    epoll_ctl(e->epfd, EPOLL_CTL_ADD, e->evfd, &ev);
    if (e->unix_too) {
        e->open_unix(0);
        e->open_unix(1);
        for (int w = 0; w < 2; ++w) {
            if (e->ufd[w] < 0) continue;
            ev.data.u64 = w == 0 ? kEvListenDU : kEvListenCU;
            epoll_ctl(e->epfd, EPOLL_CTL_ADD, e->ufd[w], &ev);
        }
    }
    *out = e;
    return VFD_OK;
}

int vfd_ports(vfd_engine* e, int* dport, int* cport) {
    if (!e) return VFD_E_INVALID;
    if (dport) *dport = e->port[0];
    if (cport) *cport = e->port[1];
    return VFD_OK;
}

int vfd_start(vfd_engine* e) {
    if (!e) return VFD_E_INVALID;
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->started) return VFD_OK;
    if (e->stopping.load()) return VFD_E_STOPPED;
    try {
        e->io = std::thread([e] { e->io_loop(); });
    } catch (...) {
        e->err = "could not start the I/O thread";
        return VFD_E_SYS;
    }
    e->started = true;
    return VFD_OK;
}

int vfd_stop(vfd_engine* e) {
    if (!e) return VFD_E_INVALID;
    e->stopping.store(true);
    e->wake_io();
    std::lock_guard<std::mutex> lk(e->mu);
    e->cv_in.notify_all();
    e->cv_out.notify_all();
    return VFD_OK;
}

int vfd_destroy(vfd_engine* e) {
    if (!e) return VFD_OK;
    vfd_stop(e);
    if (e->io.joinable()) e->io.join();
    {
        std::lock_guard<std::mutex> lk(e->mu);
        e->teardown();
    }
    delete e;
    return VFD_OK;
}

const char* vfd_last_error(vfd_engine* e) {
    if (!e) return "engine is NULL";
    // err is written under the engine lock (by any thread); the caller gets its own copy, valid
    // until its next call
    thread_local std::string copy;
    std::lock_guard<std::mutex> lk(e->mu);
    copy = e->err;
    return copy.c_str();
}

int vfd_reserve(vfd_engine* e, int64_t nbytes, int n, double timeout_s, int32_t* slots, int64_t* indices) {
    if (!e || n < 0 || (n > 0 && (!slots || !indices))) return VFD_E_INVALID;
    std::unique_lock<std::mutex> lk(e->mu);
    if (nbytes < 0 || nbytes > e->slot_bytes) {
        e->err = "frame of " + std::to_string(nbytes) + " B exceeds ring slot of " + std::to_string(e->slot_bytes) + " B";
        return VFD_E_INVALID;
    }
    auto deadline = std::chrono::steady_clock::now() +
                    std::chrono::microseconds((int64_t)(std::max(0.0, timeout_s) * 1e6));
    int got = 0;
    for (;;) {
        if (e->stopping.load()) return got ? got : VFD_E_STOPPED;
        if (n == 0) return 0;
        if (e->waiting() < (size_t)e->cfg.queue_size) {
            if (e->cfg.policy == VFD_POLICY_PULL) {
                // one target worker and one run of indices per call: the worker with the most free
                // slots (a slower worker gets fewer frames), ties in turn
                std::vector<Peer*> best;
                size_t most = 0;
                for (auto& up : e->peers) {
                    Peer* p = up.get();
                    if (!p->alive || p->slice < 0) continue;
                    size_t fr = e->slices[(size_t)p->slice].free.size();
                    if (!fr) continue;
                    if (fr > most) {
                        most = fr;
                        best.clear();
                    }
                    if (fr == most) best.push_back(p);
                }
                if (!best.empty()) {
                    Peer* p = best[(size_t)(++e->rr % best.size())];
                    int k = (int)std::min<size_t>((size_t)n, most);
                    for (int j = 0; j < k; ++j) {
                        int32_t s = e->alloc_slot(p->slice);
                        slots[j] = s;
                        indices[j] = e->counter + j;
                        e->reserved[s] = e->counter + j;
                    }
                    e->counter += k;
                    return k;
                }
            } else {
                while (got < n) {
                    int64_t idx = e->counter;
                    Peer* p = e->peer_of_cid(e->shard_owner[(size_t)e->chunk_owner(idx)]);
                    if (!p || !p->alive || p->slice < 0) break;
                    int32_t s = e->alloc_slot(p->slice);
                    if (s < 0) break;
                    slots[got] = s;
                    indices[got] = idx;
                    e->reserved[s] = idx;
                    ++e->counter;
                    ++got;
                }
                if (got) return got;
            }
        }
        if (timeout_s == 0.0) return 0;
        if (timeout_s < 0) {
            e->cv_in.wait_for(lk, std::chrono::milliseconds(50));
        } else if (e->cv_in.wait_until(lk, std::min(deadline, std::chrono::steady_clock::now() +
                                                                     std::chrono::milliseconds(50))) ==
                       std::cv_status::timeout &&
                   std::chrono::steady_clock::now() >= deadline) {
            return 0;
        }
    }
}

int vfd_commit(vfd_engine* e, int n, const int32_t* slots, const int64_t* nbytes, const int32_t* ndims,
               const int32_t* shapes, int64_t* out_indices) {
    if (!e || n < 0 || (n > 0 && (!slots || !nbytes))) return VFD_E_INVALID;
    std::unique_lock<std::mutex> lk(e->mu);
    std::unordered_set<int32_t> seen;
    for (int i = 0; i < n; ++i) {
        if (!e->reserved.count(slots[i]) || !seen.insert(slots[i]).second) {
            e->err = "slot " + std::to_string(slots[i]) + " was not reserved";
            return VFD_E_INVALID;
        }
        if (nbytes[i] < 0 || nbytes[i] > e->slot_bytes) {
            e->err = "frame of " + std::to_string(nbytes[i]) + " B exceeds its ring slot";
            return VFD_E_INVALID;
        }
    }
    double now = mono();
    for (int i = 0; i < n; ++i) {
        auto r = e->reserved.find(slots[i]);
        Frame* f = new Frame();
        f->index = r->second;
        if (out_indices) out_indices[i] = f->index;
        e->reserved.erase(r);
        f->nbytes = nbytes[i];
        f->slot = slots[i];
        f->queued_at = now;
        if (ndims && ndims[i] >= 0 && ndims[i] <= 4 && shapes) {
            f->ndim = ndims[i];
            std::memcpy(f->shape, shapes + 4 * i, 16);
        }
        e->copies[f->index] = 1;
        // lanes stay in index order; several producers may commit out of order
        e->insert_ordered(*e->lane_for(f), f);
    }
    e->serve_waiting();
    e->flush_dirty(lk);
    return VFD_OK;
}

int vfd_cancel(vfd_engine* e, int32_t slot) {
    if (!e) return VFD_E_INVALID;
    std::lock_guard<std::mutex> lk(e->mu);
    auto r = e->reserved.find(slot);
    if (r == e->reserved.end()) {
        e->err = "slot " + std::to_string(slot) + " was not reserved";
        return VFD_E_INVALID;
    }
    int64_t idx = r->second;
    e->reserved.erase(r);
    e->free_slot(slot);
    e->lose(idx);
    return VFD_OK;
}

int vfd_reserved_index(vfd_engine* e, int32_t slot, int64_t* index) {
    if (!e || !index) return VFD_E_INVALID;
    std::lock_guard<std::mutex> lk(e->mu);
    auto r = e->reserved.find(slot);
    if (r == e->reserved.end()) return VFD_E_INVALID;
    *index = r->second;
    return VFD_OK;
}

int vfd_fill(vfd_engine* e, int n, const int32_t* slots, const uint64_t* src_addrs, const int64_t* nbytes) {
    if (!e || n < 0 || (n > 0 && (!slots || !src_addrs || !nbytes))) return VFD_E_INVALID;
    std::vector<uint8_t*> dst((size_t)n);
    {
        std::lock_guard<std::mutex> lk(e->mu);
        for (int i = 0; i < n; ++i) {
            if (!e->reserved.count(slots[i])) {
                e->err = "slot " + std::to_string(slots[i]) + " was not reserved";
                return VFD_E_INVALID;
            }
            if (nbytes[i] < 0 || nbytes[i] > e->slot_bytes || (nbytes[i] > 0 && !src_addrs[i])) {
                e->err = "frame " + std::to_string(i) + " of " + std::to_string(nbytes[i]) + " B does not fit a slot of " +
                         std::to_string(e->slot_bytes) + " B";
                return VFD_E_INVALID;
            }
            dst[(size_t)i] = e->in_addr(slots[i]);
        }
    }
    // the reservations are the caller's until vfd_commit: the copies run outside the lock
    for (int i = 0; i < n; ++i)
        if (nbytes[i] > 0) std::memcpy(dst[(size_t)i], reinterpret_cast<const void*>((uintptr_t)src_addrs[i]), (size_t)nbytes[i]);
    return VFD_OK;
}

int vfd_next(vfd_engine* e, int max_n, double timeout_s, vfd_frame* out) {
    if (!e || max_n < 0 || (max_n > 0 && !out)) return VFD_E_INVALID;
    std::unique_lock<std::mutex> lk(e->mu);
    auto deadline = std::chrono::steady_clock::now() +
                    std::chrono::microseconds((int64_t)(std::max(0.0, timeout_s) * 1e6));
    while (e->released.empty()) {
        if (e->stopping.load() || timeout_s == 0.0) return 0;
        if (timeout_s < 0) {
            e->cv_out.wait(lk);
        } else if (e->cv_out.wait_until(lk, deadline) == std::cv_status::timeout && e->released.empty()) {
            return 0;
        }
    }
    int k = 0;
    while (k < max_n && !e->released.empty()) {
        out[k++] = e->released.front();
        e->released.pop_front();
    }
    return k;
}

int vfd_release(vfd_engine* e, int n, const int64_t* indices) {
    if (!e || n < 0 || (n > 0 && !indices)) return VFD_E_INVALID;
    std::lock_guard<std::mutex> lk(e->mu);
    for (int i = 0; i < n; ++i) {
        auto h = e->held.find(indices[i]);
        if (h == e->held.end()) continue;
        e->free_slot(h->second.slot, false);
        e->held.erase(h);
    }
    e->cv_in.notify_all();  // one wake-up for the group
    return VFD_OK;
}

int vfd_slot_addr(vfd_engine* e, int32_t slot, uint64_t* in_addr, uint64_t* out_addr) {
    if (!e) return VFD_E_INVALID;
    std::lock_guard<std::mutex> lk(e->mu);
    if (!e->slot_valid(slot)) return VFD_E_INVALID;
    if (in_addr) *in_addr = (uint64_t)(uintptr_t)e->in_addr(slot);
    if (out_addr) *out_addr = (uint64_t)(uintptr_t)e->out_addr(slot);
    return VFD_OK;
}

int vfd_slice(vfd_engine* e, int sid, uint64_t* base, int64_t* bytes, char* name, int name_cap, int* numa,
              int* bound) {
    if (!e) return VFD_E_INVALID;
    std::lock_guard<std::mutex> lk(e->mu);
    if (sid < 0 || (size_t)sid >= e->slices.size()) return VFD_E_INVALID;
    const Slice& s = e->slices[(size_t)sid];
    if (base) *base = (uint64_t)(uintptr_t)s.base;
    if (bytes) *bytes = (int64_t)s.bytes;
    if (name && name_cap > 0) {
        std::snprintf(name, (size_t)name_cap, "%s", s.name.c_str());
    }
    if (numa) *numa = s.numa;
    if (bound) *bound = s.bound ? 1 : 0;
    return VFD_OK;
}

int vfd_counters(vfd_engine* e, int64_t* out, int n) {
    if (!e || !out || n < 0) return VFD_E_INVALID;
    int64_t all[VFD_C_COUNT];
    {
        std::lock_guard<std::mutex> lk(e->mu);
        e->counters(all);
    }
    for (int i = 0; i < n && i < VFD_C_COUNT; ++i) out[i] = all[i];
    return VFD_OK;
}

int vfd_stats_json(vfd_engine* e, char* buf, int64_t cap) {
    if (!e) return VFD_E_INVALID;
    std::string s;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        s = e->stats_json();
    }
    if (buf && cap > 0) std::snprintf(buf, (size_t)cap, "%s", s.c_str());
    return (int)s.size();
}

}  // extern "C"
#pragma GCC visibility pop
