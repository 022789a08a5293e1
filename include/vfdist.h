/* vfdist.h -- C ABI of libvfdist.so: the distributor's control plane in native code.
 *
 * The reference's Distributor (distributor.py:8-376) runs its fan-out in two Python threads:
 * handle_distribute_requests (:205-251) answers one READY per loop and check_inverter_output
 * (:253-289) books one result per loop, with reassembly by frame index (:291-344).  This build's
 * Python Distributor keeps that API (vfilter/distributor.py); for the lossless ring deployment
 * (policy "pull" or "shard", ordered reassembly, "tcp" transport, one shared-memory ring slice
 * per worker) it hands the whole loop to this library: one I/O thread (epoll, non-blocking
 * sockets, per-peer output queues, so no send ever blocks a lock holder), per-batch
 * bookkeeping in plain arrays, and in-order release -- no Python per frame and no GIL between
 * a worker's request and its dispatch.  Workers are unchanged: they speak wire v1 (JSON) or v2
 * (binary columns, vfilter/wire.py), negotiated per worker, and v0 (the reference's own
 * messages) over the same "tcp" framing.
 *
 * Every call returns VFD_OK (0) or a negative VFD_E_* status (vfd_last_error says why), unless
 * noted.  No C++ exception crosses the boundary.  All calls are thread-safe; blocking calls
 * (vfd_reserve, vfd_next) wait on condition variables and return early on vfd_stop.
 * The Python binding is vfilter/native.py (ctypes; the GIL is released during each call).
 */
#ifndef VFDIST_H
#define VFDIST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VFD_ABI_VERSION 1

#define VFD_OK 0
#define VFD_E_INVALID -1   /* bad argument or state (e.g. a slot that was not reserved) */
#define VFD_E_SYS -2       /* a system call failed (socket, shm, mmap) */
#define VFD_E_NOMEM -3     /* no room in /dev/shm for a worker's ring slice */
#define VFD_E_STOPPED -4   /* the engine was stopped */

#define VFD_POLICY_PULL 1   /* distributor.py policy="pull": lossless, any worker, batched */
#define VFD_POLICY_SHARD 2  /* policy="shard": index chunk c goes to shard c % shard_workers */

typedef struct vfd_engine vfd_engine;

/* Distributor(...) keyword arguments of the lossless ring deployment. */
typedef struct vfd_config {
    int policy;                /* VFD_POLICY_* */
    int shard_workers;         /* shard: number of shards (>= 1) */
    int shard_chunk;           /* shard: frames per index chunk (>= 1) */
    int queue_size;            /* frames waiting for dispatch before vfd_reserve blocks */
    int ring_slots;            /* slots per worker slice */
    int64_t ring_slot_bytes;   /* largest frame (rounded up to 4 KiB); a slot is [input | output] */
    double batch_timeout;      /* s: a worker whose oldest batch is older is evicted (<= 0: never) */
    double batch_wait;         /* s: a busy worker's request waits this long to be filled */
    int max_attempts;          /* dispatches of one frame before it is counted lost */
    int verbose;               /* print evictions and refused peers */
    int distribute_port;       /* 0: any free port (vfd_ports tells which) */
    int collect_port;
    const char* host;          /* bind address ("*", "" or NULL: all interfaces) */
    int64_t max_part;          /* largest message part a peer may announce (0: 1 GiB) */
    int copy_results;          /* 1 (zero_copy=False): a result is copied out of its slot on
                                  arrival and the slot freed at once; 0: the result is read in
                                  place and its slot held until vfd_release */
    int no_unix;               /* 0: each listener also answers on the abstract Unix socket
                                  "\0vfd-tcp-<port>", which same-host workers try first
                                  (vfilter/transport.py); 1: TCP only */
} vfd_config;

/* One released result, in index order (vfd_next). */
typedef struct vfd_frame {
    int64_t index;
    int64_t nbytes;            /* the result's own length */
    uint64_t data;             /* address of the result bytes (the slot's output half, or an
                                  engine buffer for a result that came back as a socket part) */
    int32_t slot;              /* global slot id (slice * ring_slots + k); -1 if none */
    int32_t ndim;              /* -1: no shape */
    int32_t shape[4];
    int64_t pid;               /* worker process id (0 if not numeric) */
    double start;              /* worker-side begin / end of the frame (worker.py:47,59) */
    double end;
} vfd_frame;

/* Counters, in this order, for vfd_counters. */
enum {
    VFD_C_RELEASED, VFD_C_LOST, VFD_C_BUFFERED, VFD_C_MAX_DEPTH, VFD_C_OUT_OF_ORDER, VFD_C_NEXT_INDEX,
    VFD_C_RESULTS, VFD_C_RESULT_ERRORS, VFD_C_FRAMES_LOST, VFD_C_REQUEUED, VFD_C_DUPLICATES,
    VFD_C_EVICTIONS, VFD_C_DEPARTURES, VFD_C_QUARANTINE_EXPIRED, VFD_C_FRAME_COUNTER, VFD_C_WORKERS,
    VFD_C_FREE_SLOTS, VFD_C_TOTAL_SLOTS, VFD_C_DISPATCHES, VFD_C_RESULT_MESSAGES, VFD_C_COUNT
};

int vfd_abi_version(void);

/* Bind both listeners (the reference's ROUTER distributor.py:30-31 and PULL :34-35).  No
 * thread runs yet. */
int vfd_create(const vfd_config* cfg, vfd_engine** out);
int vfd_ports(vfd_engine* e, int* distribute_port, int* collect_port);
/* Start the I/O thread (Distributor.start, distributor.py:53-57). */
int vfd_start(vfd_engine* e);
/* Stop serving and wake every blocked call (Distributor.stop, distributor.py:59-61). */
int vfd_stop(vfd_engine* e);
/* Stop, join, close every socket, unmap and unlink every ring slice, free everything. */
int vfd_destroy(vfd_engine* e);
/* The engine's last error message, copied for the calling thread (valid until its next call). */
const char* vfd_last_error(vfd_engine* e);

/* Ingest (distributor.py:173-203, lossless): reserve up to n ring slots for frames of at most
 * nbytes and fix their indices; fill the input halves in place (vfd_slot_addr), then
 * vfd_commit.  Waits up to timeout_s (< 0: until stopped) for the first one while queue_size
 * frames wait or no worker has room.  Returns the number reserved (>= 0) or a status. */
int vfd_reserve(vfd_engine* e, int64_t nbytes, int n, double timeout_s, int32_t* slots, int64_t* indices);
/* Queue n filled reservations for dispatch (shapes: n x 4, ndims: -1 = none; either may be
 * NULL) and write their indices to out_indices (may be NULL).  Returns VFD_OK. */
int vfd_commit(vfd_engine* e, int n, const int32_t* slots, const int64_t* nbytes, const int32_t* ndims,
               const int32_t* shapes, int64_t* out_indices);
/* Columnar fill of n reservations (a producer at hundreds of thousands of small frames per
 * second, e.g. 512 x 512 JPEGs, cannot afford a per-frame call): copy nbytes[i] from src_addrs[i]
 * into slot slots[i]'s input half.  Every slot must be reserved and every size fit a slot, else
 * VFD_E_INVALID and nothing is copied.  Replaces the per-frame copy of distributor.py:173-203. */
int vfd_fill(vfd_engine* e, int n, const int32_t* slots, const uint64_t* src_addrs, const int64_t* nbytes);
/* Give back a reservation that will not be committed; its index is counted lost. */
int vfd_cancel(vfd_engine* e, int32_t slot);
/* The index a reservation carries. */
int vfd_reserved_index(vfd_engine* e, int32_t slot, int64_t* index);

/* In-order release (distributor.py:291-344, lossless form): up to max_n results whose
 * predecessors have all been released or counted lost, waiting up to timeout_s (< 0: until
 * stopped) for the first.  Returns the number written to out (0 on timeout). */
int vfd_next(vfd_engine* e, int max_n, double timeout_s, vfd_frame* out);
/* Return the slots of consumed results (zero-copy: a result stays valid until released). */
int vfd_release(vfd_engine* e, int n, const int64_t* indices);

/* Addresses of a slot's input and output halves. */
int vfd_slot_addr(vfd_engine* e, int32_t slot, uint64_t* in_addr, uint64_t* out_addr);
/* Ring slice sid: base address, bytes, shm name (NUL-terminated into name[name_cap]), NUMA
 * node (-1 unknown) and whether it was bound there.  VFD_E_INVALID past the last slice. */
int vfd_slice(vfd_engine* e, int sid, uint64_t* base, int64_t* bytes, char* name, int name_cap, int* numa,
              int* bound);
/* VFD_C_COUNT counters (the enum above) into out[0 .. n). */
int vfd_counters(vfd_engine* e, int64_t* out, int n);
/* Distributor.ordering_stats() as a JSON object (per-worker details included), NUL-terminated
 * into buf[cap].  Returns the length it needs (excluding the NUL) or a status. */
int vfd_stats_json(vfd_engine* e, char* buf, int64_t cap);

#ifdef __cplusplus
}
#endif

#endif /* VFDIST_H */
