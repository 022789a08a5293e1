// vfd_load.cc -- the native control plane's own ceiling: libvfdist.so driven from C++ alone.
//
// tools/distributor_overhead.py measures the distributor with Python echo worker processes and a
// Python producer / consumer (the system as deployed).  This drives the same engine with N worker
// threads that speak wire v2 over real loopback TCP (READY1 requests, FRAMES2 dispatches, RESULT2
// results that leave every frame in place, like --no-copy), one producer thread (vfd_reserve /
// vfd_commit, groups of --group) and the consumer on the main thread (vfd_next / vfd_release), so
// the rate is the engine's: sockets, dispatch, booking, in-order release.
//
//   g++ -O2 -std=c++17 -Iinclude tools/vfd_load.cc -o tools/vfd_load \
//       -Ldistributed-video-filter_amd/vfilter -lvfdist -Wl,-rpath,$PWD/distributed-video-filter_amd/vfilter -pthread
//   tools/vfd_load --workers 8 --batch 32 --bytes 181876 --frames 2000000
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstddef>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "vfdist.h"

static bool g_unix = false;

static int connect_to(int port) {
    if (g_unix) {  // the listeners' abstract Unix socket (vf_dist.cc open_unix)
        int fd = socket(AF_UNIX, SOCK_STREAM, 0);
        sockaddr_un a{};
        a.sun_family = AF_UNIX;
        int n = snprintf(a.sun_path + 1, sizeof a.sun_path - 1, "vfd-tcp-%d", port);
        if (connect(fd, (sockaddr*)&a, (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n)) == 0) return fd;
        perror("connect unix");
        exit(1);
    }
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr*)&a, sizeof a) != 0) {
        perror("connect");
        exit(1);
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    return fd;
}

static bool read_exact(int fd, void* p, size_t n) {
    uint8_t* b = (uint8_t*)p;
    while (n) {
        ssize_t r = recv(fd, b, n, 0);
        if (r <= 0) return false;
        b += r;
        n -= (size_t)r;
    }
    return true;
}

static void send_parts(int fd, const std::vector<std::string>& parts) {
    std::string m;
    uint32_t np = (uint32_t)parts.size();
    m.append((const char*)&np, 4);
    for (auto& p : parts) {
        uint64_t n = p.size();
        m.append((const char*)&n, 8);
        m += p;
    }
    size_t off = 0;
    while (off < m.size()) {
        ssize_t w = send(fd, m.data() + off, m.size() - off, MSG_NOSIGNAL);
        if (w <= 0) return;
        off += (size_t)w;
    }
}

static bool recv_parts(int fd, std::vector<std::string>& parts) {
    uint32_t np;
    if (!read_exact(fd, &np, 4)) return false;
    parts.resize(np);
    for (uint32_t k = 0; k < np; ++k) {
        uint64_t n;
        if (!read_exact(fd, &n, 8)) return false;
        parts[k].resize(n);
        if (n && !read_exact(fd, &parts[k][0], n)) return false;
    }
    return true;
}

int main(int argc, char** argv) {
    int workers = 8, batch = 32, group = 32, depth = 4;
    // --chaos 1: worker 0 closes its connections after 40 batches (a crash), worker 1 stops
    // answering after 60 (a hang; the engine's batch deadline evicts it): the survivors must
    // still deliver every frame in order (re-queue, quarantine, shard-free pull policy)
    bool chaos = false;
    double timeout_s = 0.2;  // --chaos: the batch deadline that evicts the hung worker
    long long frames = 1000000;
    long long bytes = 181876;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string k = argv[i];
        if (k == "--workers") workers = atoi(argv[i + 1]);
        else if (k == "--batch") batch = atoi(argv[i + 1]);
        else if (k == "--group") group = atoi(argv[i + 1]);
        else if (k == "--depth") depth = atoi(argv[i + 1]);
        else if (k == "--frames") frames = atoll(argv[i + 1]);
        else if (k == "--bytes") bytes = atoll(argv[i + 1]);
        else if (k == "--unix") g_unix = atoi(argv[i + 1]) != 0;
        else if (k == "--chaos") chaos = atoi(argv[i + 1]) != 0;
        else if (k == "--timeout") timeout_s = atof(argv[i + 1]);
    }
    vfd_config cfg{};
    cfg.policy = VFD_POLICY_PULL;
    cfg.shard_workers = 1;
    cfg.shard_chunk = 1;
    cfg.queue_size = 3 * batch * workers;
    cfg.ring_slots = 4 * batch;
    cfg.ring_slot_bytes = bytes;
    cfg.batch_timeout = chaos ? timeout_s : 30.0;
    cfg.batch_wait = 0.002;
    cfg.max_attempts = 3;
    cfg.host = "127.0.0.1";
    vfd_engine* e = nullptr;
    if (vfd_create(&cfg, &e) != VFD_OK) return 1;
    int dport, cport;
    vfd_ports(e, &dport, &cport);
    vfd_start(e);
    std::atomic<bool> stop{false};
    std::vector<std::thread> ws;
    for (int w = 0; w < workers; ++w) {
        ws.emplace_back([&, w] {
            int d = connect_to(dport), c = connect_to(cport);
            char head[160];
            snprintf(head, sizeof head, "{\"credit\": %d, \"shm\": true, \"wid\": \"L%d\", \"wire\": 2}", batch, w);
            std::vector<std::string> req = {"READY1", head};
            for (int k = 0; k < depth; ++k) send_parts(d, req);
            snprintf(head, sizeof head, "{\"pid\": \"%d\", \"wid\": \"L%d\", \"start\": 0.0, \"end\": 0.0}", 1000 + w, w);
            std::string rhead = head;
            std::vector<std::string> parts;
            int nb = 0;
            while (!stop.load() && recv_parts(d, parts)) {
                if (parts.size() < 3 || parts[0] != "FRAMES2") continue;
                ++nb;
                if (chaos && w == 0 && nb == 40) break;  // crash: both connections close
                if (chaos && w == 1 && nb >= 60) continue;  // hang: keeps reading, never answers
                // echo: the records as dispatched; frames sent as parts (slot -1: a re-queued frame
                // that found no room in this worker's slice) go back as parts
                std::vector<std::string> res = {"RESULT2", rhead, parts[2]};
                for (size_t k = 3; k < parts.size(); ++k) res.push_back(parts[k]);
                send_parts(c, res);
                send_parts(d, req);
            }
            close(d);
            close(c);
        });
    }
    int64_t cnt[VFD_C_COUNT];
    do {
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
        vfd_counters(e, cnt, VFD_C_COUNT);
    } while (cnt[VFD_C_WORKERS] < workers);
    const long long warm = 8LL * batch * workers, total = warm + frames;
    std::thread prod([&] {
        std::vector<int32_t> slots(group);
        std::vector<int64_t> idx(group), nb(group, bytes);
        long long done = 0;
        while (done < total) {
            int n = (int)std::min<long long>(group, total - done);
            int k = vfd_reserve(e, bytes, n, -1.0, slots.data(), idx.data());
            if (k <= 0) break;
            vfd_commit(e, k, slots.data(), nb.data(), nullptr, nullptr, nullptr);
            done += k;
        }
    });
    std::vector<vfd_frame> out(256);
    std::vector<int64_t> rel(256);
    long long got = 0, calls = 0;
    auto t0 = std::chrono::steady_clock::now();
    while (got < total) {
        if (got >= warm && calls == 0) t0 = std::chrono::steady_clock::now();
        int k = vfd_next(e, 256, 10.0, out.data());
        if (k <= 0) {
            fprintf(stderr, "stalled at %lld\n", got);
            _exit(2);
        }
        for (int j = 0; j < k; ++j) {
            if (out[j].index != got + j) {
                fprintf(stderr, "order: %lld at %lld\n", (long long)out[j].index, got + j);
                _exit(3);
            }
            rel[j] = out[j].index;
        }
        vfd_release(e, k, rel.data());
        if (got >= warm) ++calls;
        got += k;
    }
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    prod.join();
    stop.store(true);
    vfd_counters(e, cnt, VFD_C_COUNT);
    if (chaos)
        printf("{\"chaos\": true, \"evictions\": %lld, \"requeued\": %lld, \"lost\": %lld, \"duplicates\": %lld}\n",
               (long long)cnt[VFD_C_EVICTIONS], (long long)cnt[VFD_C_REQUEUED], (long long)cnt[VFD_C_FRAMES_LOST],
               (long long)cnt[VFD_C_DUPLICATES]);
    printf("{\"kind\": \"vfd_load\", \"workers\": %d, \"batch\": %d, \"group\": %d, \"frame_bytes\": %lld, "
           "\"frames\": %lld, \"fps\": %.1f, \"dispatches\": %lld, \"frames_per_dispatch\": %.1f, "
           "\"unix\": %d, \"host_cpus\": %u}\n",
           workers, batch, group, bytes, frames, (double)frames / el, (long long)cnt[VFD_C_DISPATCHES],
           (double)total / (double)std::max<int64_t>(1, cnt[VFD_C_DISPATCHES]), g_unix ? 1 : 0,
           std::thread::hardware_concurrency());
    fflush(stdout);
    vfd_destroy(e);  // closes the sockets: the worker threads' reads end
    for (auto& t : ws) t.join();
    return 0;
}
