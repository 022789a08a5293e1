"""Distributor: frame fan-out to worker processes and in-order reassembly
(reference: distributor.py:8-376).

Public API of the reference, same names, arguments and behaviour:
  Distributor(distribute_port=5555, collect_port=5556, frame_delay=5, enable_trace_export=False)
  start / stop / cleanup, add_frame_for_distribution(frame, timestamp=None),
  update_display_frame / get_frame_to_display / get_frame_stats / cleanup_old_frames,
  log_frame_timing / log_frame_complete_timing / export_perfetto_trace,
  handle_distribute_requests / check_inverter_output (the two thread bodies).
With the defaults it reproduces the reference: a bounded ingest queue that drops the
oldest frame (distributor.py:173-203), a latest-wins dispatch slot that sends each frame at
most once in increasing index order (:205-251), and the lossy display policy (:253-344),
checked against traces of the real reference in tests/golden.

Additions for GPU workers (keyword-only):
  policy="pull"    lossless: every frame is dispatched, in index order, in batches of up to a
                   worker's credit (contiguous index runs -> contiguous device batches); ingest
                   blocks instead of dropping when ``queue_size`` frames are waiting.
  policy="shard"   lossless, deterministic: index chunk c = [c*shard_chunk, (c+1)*shard_chunk)
                   goes to shard c % shard_workers; shard k belongs to the k-th worker to
                   register — frame-index sharding across 1/2/4/8 GPUs.
  reassembly="ordered"  every result released exactly once in index order
                   (``get_next_frame``), with ordering-overhead statistics.
  ring_slots>0     same-node shared-memory data plane (``vfilter.shm``): frames are written once
                   into a ring slot and only slot numbers travel on the sockets.
                   ring_layout="per_worker" (default for pull/shard): every worker gets its own
                   slice of ``ring_slots`` slots, bound to the NUMA node of its GPU
                   (``vfilter.numa``); it page-locks only that slice.  A frame is written into
                   the slice of the worker that will filter it (shard: the shard's owner; pull:
                   the worker with the most free slots, so a slower worker gets fewer frames).
                   ring_layout="shared": one ring every worker maps (the latest policy's).
Worker loss (lossless policies).  Every dispatched frame is tracked per worker.  A worker
whose oldest outstanding batch is older than ``batch_timeout`` seconds, or whose connection
closes (tcp transport), is evicted: its frames are re-queued to the others (copied into their
slices), its shards move to a spare or to the least-loaded live worker, and a frame that has
been dispatched ``max_attempts`` times is counted lost (``OrderedBuffer.mark_lost``), so
``get_next_frame`` never waits forever.  A result that still arrives from an evicted worker is
a duplicate and is dropped; its ring slot is kept out of use until then.  An evicted worker
that asks again is taken back and re-takes its home shard.  (The reference tolerates workers
coming and going through READY and loses a failed frame, worker.py:74-76.)
Batch filling (lossless policies).  A v1 request asks for up to ``credit`` frames.  While the
worker still has a batch in flight, a request is answered only once it can be filled, or once
the oldest frame waiting for that worker has waited ``batch_wait`` seconds; an idle worker is
served at once.  Answering every request with whatever had just arrived gave a fast worker
batches of 2-10 frames and let fixed per-batch costs dominate (JPEG 480p through the system:
the GPU codec's per-call host work ran at 55 % of the worker's time).
All shared state sits behind one lock (the reference relies on the GIL).
"""
from __future__ import annotations

import collections
import ctypes
import json
import os
import queue
import sys
import threading
import time
from typing import Sequence, Deque, Dict, List, Optional

import numpy as np

from . import numa
from . import transport as tp
from . import wire
from .reorder import DisplayBuffer, OrderedBuffer
from .sharding import chunk_owner
from .shm import FrameRing, copy_into


class ListBatch:
    """Released results as columns (``index``, ``nbytes``) over ``get_next_frames``' tuples."""

    def __init__(self, items: list):
        self._items = items
        self.index = np.asarray([it[0] for it in items], np.int64)
        self.nbytes = np.asarray([len(memoryview(it[1]).cast("B")) for it in items], np.int64)

    def __len__(self) -> int:
        return len(self._items)

    def view(self, i: int):
        return self._items[i][1]

    def info(self, i: int) -> dict:
        return self._items[i][2]

    def items(self) -> list:
        return list(self._items)


def _native_serves(args, kw) -> bool:
    """True when engine="auto" should pick the native control plane for these arguments."""
    from . import native
    try:
        transport = tp.resolve(kw.get("transport", "auto"))
    except ValueError:
        return False
    trace = kw.get("enable_trace_export", args[3] if len(args) > 3 else False)
    if native.supports(kw.get("policy", "latest"), kw.get("reassembly", "display"), transport,
                       int(kw.get("ring_slots", 0)), kw.get("ring_layout", "auto"), bool(trace)) is not None:
        return False
    if not native.available():  # auto never fails for a missing library: the Python engine serves
        global _auto_notice_shown
        if not _auto_notice_shown:
            _auto_notice_shown = True
            print(f"vfilter.distributor: engine='auto' uses the Python engine ({native.LIB_NAME} not loadable "
                  f"at {native.library_path()}; `make lib` builds it)", file=sys.stderr, flush=True)
        return False
    return True


_auto_notice_shown = False


class _Peer:
    __slots__ = ("pid", "version", "wid", "requests", "frames_sent", "batches_sent", "results", "errors", "home_shard", "shm",
                 "numa", "slice", "queue", "inflight", "quarantine", "batches", "alive", "gone", "evictions",
                 "order", "last_seen", "waiting_since", "wire", "outbox", "send_lock")

    def __init__(self, pid: bytes, req: wire.Request, order: int):
        self.pid = pid
        self.version = req.version
        self.wid = req.wid
        self.shm = bool(req.shm)
        self.numa = req.numa
        self.order = order                    # registration order
        self.requests: Deque[int] = collections.deque()  # credits of outstanding requests
        self.frames_sent = 0
        self.batches_sent = 0
        self.results = 0
        self.errors = 0
        self.home_shard: Optional[int] = None
        self.slice: Optional[int] = None      # ring slice (per_worker layout)
        self.queue: Deque[dict] = collections.deque()   # pull + per_worker: frames in this slice
        self.inflight: Dict[int, dict] = {}   # index -> dispatched copy awaiting its result
        self.quarantine: Dict[int, dict] = {}  # copies dispatched before an eviction
        self.batches: Deque[list] = collections.deque()  # [t_dispatch, {indices}] oldest first
        self.alive = True
        self.gone = False                     # connection closed: no result can come any more
        self.evictions = 0
        self.last_seen = time.monotonic()     # last request or result
        self.waiting_since: Optional[float] = None  # frames wait for it, it has not asked
        self.wire = req.wire                  # newest dispatch form it reads (wire.py)
        # dispatches built and booked under the distributor's lock, sent outside it (no socket
        # I/O under the lock: a worker blocked sending its results must never stall a thread that
        # holds the lock its result reader needs); send_lock keeps one peer's sends in order
        self.outbox: Deque[tuple] = collections.deque()
        self.send_lock = threading.Lock()


class _Slice:
    __slots__ = ("ring", "free", "numa", "bound", "owner")

    def __init__(self, ring: FrameRing, node: Optional[int], bound: bool, owner: Optional[bytes]):
        self.ring = ring
        self.free: List[int] = list(range(ring.nslots - 1, -1, -1))
        self.numa = node
        self.bound = bound
        self.owner = owner


class Distributor:
    QUARANTINE_HOLD = 4  # batch timeouts a shared-ring slot of an evicted worker is held without a disconnect notice
    engine = "python"

    def __new__(cls, *args, **kw):
        """``engine="native"`` -- or ``"auto"`` (the default) for the lossless ring deployment it
        serves -- gives a ``vfilter.native.NativeDistributor``: the same API over the C++ control
        plane (libvfdist.so).  ``"python"``, and every configuration the native engine does not
        serve (the reference's latest-wins / display policy, ZeroMQ, socket payloads, trace
        export), is this class."""
        if cls is Distributor:
            eng = kw.get("engine", "auto")
            if eng == "native" or (eng == "auto" and _native_serves(args, kw)):
                from .native import NativeDistributor
                return super().__new__(NativeDistributor)
        return super().__new__(cls)

    def __init__(self, distribute_port: int = 5555, collect_port: int = 5556, frame_delay: int = 5,
                 enable_trace_export: bool = False, *, policy: str = "latest", reassembly: str = "display",
                 transport: str = "auto", host: str = "*", queue_size: int = 10, frame_buffer_size: int = 50,
                 ring_slots: int = 0, ring_slot_bytes: int = 0, ring_layout: str = "auto", shard_workers: int = 0,
                 shard_chunk: int = 1, batch_timeout: float = 30.0, max_attempts: int = 3, batch_wait: float = 0.002,
                 trace_file: str = "webcam_frame_timing.pftrace", verbose: bool = True, zero_copy: bool = False,
                 engine: str = "auto"):
        if engine not in ("auto", "python", "native"):
            raise ValueError("engine must be auto | python | native")
        if zero_copy and (ring_slots < 1 or reassembly != "ordered"):
            raise ValueError("zero_copy needs ring_slots > 0 and reassembly='ordered'")
        self.zero_copy = zero_copy
        if policy not in ("latest", "pull", "shard"):
            raise ValueError("policy must be latest | pull | shard")
        if reassembly not in ("display", "ordered"):
            raise ValueError("reassembly must be display | ordered")
        if policy == "shard" and shard_workers < 1:
            raise ValueError("policy='shard' needs shard_workers >= 1")
        if ring_layout == "auto":
            ring_layout = "shared" if policy == "latest" else "per_worker"
        if ring_layout not in ("shared", "per_worker"):
            raise ValueError("ring_layout must be auto | shared | per_worker")
        if ring_layout == "per_worker" and policy == "latest":
            raise ValueError("the latest policy serves any worker from one slot: use ring_layout='shared'")
        self.policy = policy
        self.reassembly = reassembly
        self.verbose = verbose
        # ingest (distributor.py:11-14)
        self.frame_queue: "queue.Queue[dict]" = queue.Queue(maxsize=queue_size)
        self.frame_index_counter = 0
        self.last_frame_sent = -1                   # distributor.py:17
        self.current_frame_data: Optional[dict] = None
        self._pending: Deque[dict] = collections.deque()   # pull without per-worker slices
        self._shard_pending: Dict[int, Deque[dict]] = collections.defaultdict(collections.deque)
        self._orphans: Deque[dict] = collections.deque()   # pull + per_worker, no live worker
        self.queue_size = queue_size
        self.shard_workers = shard_workers
        self.shard_chunk = max(1, shard_chunk)
        self.batch_timeout = float(batch_timeout)
        self.batch_wait = max(0.0, float(batch_wait))
        self.max_attempts = max(1, int(max_attempts))
        # reassembly (distributor.py:19-24)
        self._display = DisplayBuffer(frame_delay, frame_buffer_size)
        self._ordered = OrderedBuffer(0)
        self._released: Deque[tuple] = collections.deque()
        self._lock = threading.RLock()
        # two conditions on the one lock: producers wait on _cv (a free slot, room in the
        # queue), the in-order consumer on _cv_out (a released result), so a freed slot does
        # not wake the consumer and a released result does not wake the producers
        self._cv = threading.Condition(self._lock)
        self._cv_out = threading.Condition(self._lock)
        # transport (distributor.py:26-35)
        self.transport = tp.resolve(transport)
        self._zctx = tp.make_context(self.transport)
        self.distribute_socket = tp.RouterEnd(self.transport, host, distribute_port, self._zctx)
        self._wakeable = self.distribute_socket.wakeable
        self._inline = False  # set by start(): messages handled on the reader threads
        self.collect_socket = tp.PullEnd(self.transport, host, collect_port, self._zctx)
        self.distribute_port = self.distribute_socket.port
        self.collect_port = self.collect_socket.port
        # shared-memory ring: slices of ring_slots slots; global slot id = slice * ring_slots + k
        self.ring_slots = int(ring_slots)
        self.ring_slot_bytes = int(ring_slot_bytes)
        self.ring_layout = ring_layout if ring_slots > 0 else None
        self._slices: List[_Slice] = []
        self.ring: Optional[FrameRing] = None       # the shared ring (ring_layout="shared")
        if ring_slots > 0:
            if ring_slot_bytes < 1:
                raise ValueError("ring_slots needs ring_slot_bytes (largest frame)")
            if ring_layout == "shared":
                self.ring = FrameRing(ring_slots, ring_slot_bytes)
                self._slices.append(_Slice(self.ring, None, False, None))
        self._reserved: Dict[int, Optional[int]] = {}   # reserved slot -> its frame index (per_worker)
        self._clone_src: Dict[int, dict] = {}   # quarantined slot -> re-queued copy reading from it
        self._held: Dict[int, int] = {}         # zero_copy: index -> slot of its released result
        self._copies: Dict[int, int] = {}       # index -> copies queued or in flight
        self._settled = set()                   # indices delivered/lost while copies remain
        # tracing (distributor.py:37-40)
        self.enable_trace_export = enable_trace_export
        self.frame_timings: List[dict] = []
        self.trace_start_time = time.time()
        self.trace_file = trace_file
        # peers and counters
        self._peers: Dict[bytes, _Peer] = {}
        self._dirty = set()                       # peers with dispatches queued for sending
        self._by_wid: Dict[str, _Peer] = {}
        self._shard_home: Dict[int, bytes] = {}   # shard -> the worker it belongs to
        self._shard_owner: Dict[int, bytes] = {}  # shard -> the worker serving it now
        self._rr = 0
        self.frames_dropped = 0
        self.frames_lost = 0
        self.frames_requeued = 0
        self.duplicates = 0
        self.evictions = 0
        self.departures = 0
        self.results_received = 0
        self.result_errors = 0
        self.quarantine_expired = 0   # slots of evicted workers' frames freed after the grace period
        self.quarantine_forced = 0    # of which shared-ring slots freed with no disconnect notice (zmq)
        self._disconnect_notices = self.transport == "tcp"  # zmq reports no peer disconnects
        # threads (distributor.py:42-51)
        self.running = False
        self.distribute_thread = threading.Thread(target=self.handle_distribute_requests, daemon=True)
        self.inverter_thread = threading.Thread(target=self.check_inverter_output, daemon=True)

    # ---- reference properties kept as attributes ------------------------------------------
    @property
    def received_frames(self) -> dict:
        return self._display.received_frames

    @property
    def current_display_frame(self) -> int:
        return self._display.current_display_frame

    @property
    def latest_received_frame(self) -> int:
        return self._display.latest_received_frame

    @property
    def frame_delay(self) -> int:
        return self._display.frame_delay

    @property
    def frame_buffer_size(self) -> int:
        return self._display.frame_buffer_size

    # ---- lifecycle (distributor.py:53-61, 356-376) --------------------------------------
    def start(self):
        self.running = True
        # "tcp" with a lossless policy: requests and results are handled on the socket reader
        # threads as they arrive, and committed frames are served on the committing thread, so a
        # batch costs no hand-off to the dispatch / collect threads (which then only keep the
        # timers: batch-fill deadlines and worker deadlines).  The GIL makes every hand-off a
        # thread switch: round 3's polling threads cost ~35 us of CPU per 1080p JPEG frame here.
        # zmq and the reference's "latest" policy keep the reference's two polling threads.
        self._inline = (self.policy != "latest" and self.distribute_socket.set_handler(self._inline_request)
                        and self.collect_socket.set_handler(self._inline_result))
        self.distribute_thread.start()
        self.inverter_thread.start()

    def _inline_request(self, pid: bytes, parts) -> None:
        try:
            if parts is None:
                with self._cv:
                    p = self._peers.get(pid)
                    if p is not None:
                        self._evict(p, "connection closed", gone=True)
            else:
                req = wire.decode_request(parts)
                if req is not None:
                    self._on_request(pid, req)
            self._serve_waiting()
        except Exception as e:  # as the dispatch loop: report and keep serving
            print(f"Error handling distribute request: {e}")

    def _inline_result(self, parts) -> None:
        try:
            self._on_result(wire.decode_result(parts))
        except Exception as e:  # distributor.py:287-289
            print(f"Error receiving inverted frame: {e}")

    def stop(self):
        self.running = False
        with self._cv:
            self._cv.notify_all()
            self._cv_out.notify_all()

    def cleanup(self):
        self.stop()
        for t in (self.distribute_thread, self.inverter_thread):
            if t.is_alive():
                t.join(timeout=1.0)
        self.distribute_socket.close()
        self.collect_socket.close()
        if self._zctx is not None:
            self._zctx.term()
        for sl in self._slices:
            sl.ring.close()
        self._slices = []
        self.ring = None
        if self.verbose:
            print("ZeroMQ connections closed" if self.transport == "zmq" else "Connections closed")
            print("Frame reordering statistics:")
            print(f"  Latest received frame: {self.latest_received_frame}")
            print(f"  Current display frame: {self.current_display_frame}")
            print(f"  Frames in buffer: {len(self.received_frames)}")
            print(f"  Frame delay: {self.frame_delay} frames")
        if self.enable_trace_export and self.frame_timings:
            if self.verbose:
                print("Exporting Perfetto trace on cleanup...")
            self.export_perfetto_trace()

    # ---- tracing (distributor.py:63-171) ------------------------------------------------
    def log_frame_timing(self, frame_index, timestamp, event_type="frame_captured"):
        if not self.enable_trace_export:
            return
        self.frame_timings.append({"frame_index": frame_index, "timestamp": timestamp, "event_type": event_type,
                                   "relative_time": timestamp - self.trace_start_time, "event_ph": "i"})

    def log_frame_complete_timing(self, frame_index, begin_time, end_time, event_type="frame_processed", pid=None):
        if not self.enable_trace_export:
            return
        self.frame_timings.append({"frame_index": frame_index, "begin_time": begin_time, "end_time": end_time,
                                   "event_type": event_type, "begin_relative_time": begin_time - self.trace_start_time,
                                   "end_relative_time": end_time - self.trace_start_time, "event_ph": "X",
                                   "pid": pid})

    GPU_TIDS = {"H2D": 1, "kernel": 2, "D2H": 3, "batch": 4}  # "batch" = H2D..D2H of an async batch

    def log_gpu_span(self, name: str, begin_time: float, end_time: float, pid, nbytes: int = 0):
        """A GPU span of a worker batch (H2D / kernel / D2H), shown on its own track under
        the worker's pid next to the reference's per-frame events."""
        if not self.enable_trace_export:
            return
        self.frame_timings.append({"event_ph": "G", "name": name, "begin_time": begin_time, "end_time": end_time,
                                   "begin_relative_time": begin_time - self.trace_start_time,
                                   "end_relative_time": end_time - self.trace_start_time, "pid": pid,
                                   "bytes": nbytes})

    def trace_events(self) -> List[dict]:
        """Chrome-trace events in the reference's schema (distributor.py:107-138), plus GPU
        spans ("ph": "X" on tids 1-3 of the worker's pid, named by "M" metadata events)."""
        tid = threading.get_ident()
        ev = []
        named = set()
        for t in self.frame_timings:
            if t["event_ph"] == "G":
                gtid = self.GPU_TIDS.get(t["name"], 9)
                if (t["pid"], gtid) not in named:
                    named.add((t["pid"], gtid))
                    ev.append({"name": "thread_name", "ph": "M", "pid": t["pid"], "tid": gtid,
                               "args": {"name": f"GPU {t['name']}"}})
                dur = t["end_relative_time"] - t["begin_relative_time"]
                ev.append({"name": f"GPU {t['name']}", "cat": "gpu", "ph": "X",
                           "ts": int(t["begin_relative_time"] * 1e6), "dur": max(0, int(dur * 1e6)),
                           "pid": t["pid"], "tid": gtid,
                           "args": {"bytes": t["bytes"], "GBps": (t["bytes"] / dur / 1e9) if dur > 0 else None}})
                continue
            if t["event_ph"] == "i":
                ev.append({"name": f"Frame {t['frame_index']} - {t['event_type']}", "cat": "video_frames",
                           "ph": "i", "ts": int(t["relative_time"] * 1e6), "pid": os.getpid(), "tid": tid,
                           "args": {"frame_index": t["frame_index"], "event_type": t["event_type"],
                                    "absolute_timestamp": t["timestamp"]}})
            else:
                dur = t["end_relative_time"] - t["begin_relative_time"]
                ev.append({"name": f"Frame {t['frame_index']} - {t['event_type']}", "ph": "X",
                           "ts": int(t["begin_relative_time"] * 1e6), "dur": int(dur * 1e6),
                           "pid": t.get("pid") if t.get("pid") is not None else os.getpid(), "tid": tid,
                           "args": {"frame_index": t["frame_index"], "event_type": t["event_type"],
                                    "begin_timestamp": t["begin_time"], "end_timestamp": t["end_time"],
                                    "duration_ms": dur * 1000}})
        return ev

    def trace_summary(self) -> dict:
        """The statistics the reference prints after an export (distributor.py:151-171): the
        mean interval between capture instants and the mean worker processing span.  GPU spans
        are summarised per stage beside them (bytes and GB/s)."""
        out: dict = {}
        inst = [t for t in self.frame_timings if t["event_ph"] == "i"]
        comp = [t for t in self.frame_timings if t["event_ph"] == "X"]
        if len(inst) > 1:
            ts = [t["timestamp"] for t in inst]
            iv = [ts[i + 1] - ts[i] for i in range(len(ts) - 1)]
            avg = sum(iv) / len(iv)
            out["avg_capture_interval_ms"] = avg * 1000
            out["capture_fps"] = (1 / avg) if avg > 0 else float("inf")
        if comp:
            ds = [t["end_time"] - t["begin_time"] for t in comp]
            avg = sum(ds) / len(ds)
            out["avg_processing_ms"] = avg * 1000
            out["processing_fps"] = (1 / avg) if avg > 0 else float("inf")
            out["frames_processed"] = len(comp)
        gpu: Dict[str, dict] = {}
        for t in self.frame_timings:
            if t["event_ph"] == "G":
                g = gpu.setdefault(t["name"], {"spans": 0, "seconds": 0.0, "bytes": 0})
                g["spans"] += 1
                g["seconds"] += max(0.0, t["end_time"] - t["begin_time"])
                g["bytes"] += int(t["bytes"])
        for g in gpu.values():
            g["GBps"] = g["bytes"] / g["seconds"] / 1e9 if g["seconds"] > 0 else None
        if gpu:
            out["gpu"] = gpu
        return out

    def export_perfetto_trace(self):
        if not self.enable_trace_export:
            print("Trace export is disabled")
            return
        if not self.frame_timings:
            print("No frame timing data to export")
            return
        with open(self.trace_file, "w") as f:
            json.dump({"traceEvents": self.trace_events()}, f)
        print(f"Perfetto trace exported to: {self.trace_file}")
        print(f"Total frames logged: {len(self.frame_timings)}")
        s = self.trace_summary()                    # distributor.py:151-171
        if "avg_capture_interval_ms" in s:
            print(f"Average frame capture interval: {s['avg_capture_interval_ms']:.2f}ms")
            print(f"Frame capture rate: {s['capture_fps']:.1f} FPS")
        if "avg_processing_ms" in s:
            print(f"Average processing duration: {s['avg_processing_ms']:.2f}ms")
            print(f"Processing rate: {s['processing_fps']:.1f} FPS")
            print(f"Total frames processed: {s['frames_processed']}")
        for name, g in s.get("gpu", {}).items():
            rate = f", {g['GBps']:.1f} GB/s" if g["GBps"] else ""
            print(f"GPU {name}: {g['spans']} spans, {g['seconds'] * 1000:.2f}ms, {g['bytes']} bytes{rate}")

    # ---- ring slots -----------------------------------------------------------------------
    def in_view(self, slot: int, nbytes: int) -> np.ndarray:
        """Input half of ring slot ``slot`` (a global slot id)."""
        sid, k = divmod(slot, self.ring_slots)
        return self._slices[sid].ring.in_view(k, nbytes)

    def out_view(self, slot: int, nbytes: int) -> np.ndarray:
        sid, k = divmod(slot, self.ring_slots)
        return self._slices[sid].ring.out_view(k, nbytes)

    frame_view = in_view

    def free_slots(self) -> int:
        with self._lock:
            return sum(len(sl.free) for sl in self._slices)

    def total_slots(self) -> int:
        with self._lock:
            return len(self._slices) * self.ring_slots

    def _alloc_slot(self, sid: int) -> Optional[int]:
        sl = self._slices[sid]
        return sid * self.ring_slots + sl.free.pop() if sl.free else None

    def _free_slot(self, slot: Optional[int], notify: bool = True) -> None:
        if slot is None or not self._slices:
            return
        if self._clone_src:
            clone = self._clone_src.pop(slot, None)
            if clone is not None and clone.get("slot") is None:
                clone["slot"], clone["src_slot"] = slot, None  # the re-queued copy now owns it
                return
        sid, k = divmod(slot, self.ring_slots)
        self._slices[sid].free.append(k)
        if notify:
            self._cv.notify_all()

    def _make_slice(self, p: _Peer) -> None:
        ring = FrameRing(self.ring_slots, self.ring_slot_bytes)
        bound = numa.bind(ring.base_address, ring.nbytes, p.numa) if p.numa is not None else False
        self._slices.append(_Slice(ring, p.numa, bound, p.pid))
        p.slice = len(self._slices) - 1

    # ---- ingest (distributor.py:173-203) -------------------------------------------------
    def add_frame_for_distribution(self, frame, timestamp=None, shape=None, block: bool = True) -> int:
        """Queue one frame; returns its index.  ``frame`` is bytes-like (or an ndarray).
        latest policy: drop-oldest when full (reference).  pull/shard: block while
        ``queue_size`` frames wait (or return -1 when ``block`` is False)."""
        if timestamp is None:
            timestamp = time.time()
        if isinstance(frame, np.ndarray):
            shape = list(frame.shape) if shape is None else shape
            frame = np.ascontiguousarray(frame)
        nbytes = frame.nbytes if isinstance(frame, np.ndarray) else len(frame)
        if self._slices or self.ring_layout == "per_worker":
            slot = self.reserve_frame(nbytes, block)
            if slot is None:
                return -1
            copy_into(self.in_view(slot, nbytes), frame)
            return self.commit_frame(slot, nbytes, shape, timestamp, block)
        idx = self._enqueue(frame, nbytes, shape, None, timestamp, block)
        self._kick()
        return idx

    # ---- zero-copy ingest (ring mode) ------------------------------------------------------
    def reserve_frame(self, nbytes: int, block: bool = True) -> Optional[int]:
        """Reserve a ring slot for a frame of ``nbytes``; fill ``frame_view(slot, nbytes)`` in
        place (e.g. decode or capture straight into it), then ``commit_frame`` (or
        ``cancel_frame``).  Returns None when no slot is free and ``block`` is False.  With
        per-worker slices the frame's index is fixed here (it decides the slice)."""
        if self.ring_layout is None:
            raise RuntimeError("reserve_frame needs ring_slots > 0")
        if nbytes > self.ring_slot_bytes:
            raise ValueError(f"frame of {nbytes} B exceeds ring slot of {self.ring_slot_bytes} B")
        with self._cv:
            while True:
                if self.ring_layout == "shared":
                    slot = self._alloc_slot(0)
                    if slot is None and self.policy == "latest":
                        slot = self._evict_oldest_queued_slot()
                    if slot is not None:
                        self._reserved[slot] = None
                        return slot
                elif self.policy == "latest" or self._waiting() < self.queue_size:
                    idx = self.frame_index_counter
                    p = self._target_peer(idx)
                    if p is not None:
                        slot = self._alloc_slot(p.slice)
                        if slot is not None:
                            self.frame_index_counter += 1
                            self._reserved[slot] = idx
                            return slot
                if not block or not self.running:
                    return None
                self._cv.wait(0.05)

    def reserve_frames(self, nbytes: int, n: int, block: bool = True) -> List[int]:
        """Up to ``n`` reservations under one lock hold (at least one when ``block``), each as
        ``reserve_frame``: a producer of many small frames (JPEG) pays the lock once per group."""
        out: List[int] = []
        if self.ring_layout == "per_worker" and self.policy == "pull":
            # one target worker and one run of indices per call (what reserve_frame decides per
            # frame: the worker with the most free slots, while fewer than queue_size wait)
            if nbytes > self.ring_slot_bytes:
                raise ValueError(f"frame of {nbytes} B exceeds ring slot of {self.ring_slot_bytes} B")
            with self._cv:
                while True:
                    if self._waiting() < self.queue_size:
                        idx = self.frame_index_counter
                        p = self._target_peer(idx)
                        if p is not None:
                            free = self._slices[p.slice].free
                            k = min(n, len(free))
                            base = p.slice * self.ring_slots
                            for j in range(k):
                                slot = base + free.pop()
                                self._reserved[slot] = idx + j
                                out.append(slot)
                            self.frame_index_counter = idx + k
                            return out
                    if not block or not self.running:
                        return out
                    self._cv.wait(0.05)
        with self._cv:
            while len(out) < n:
                slot = self.reserve_frame(nbytes, block=block and not out)
                if slot is None:
                    break
                out.append(slot)
        return out

    def reserved_index(self, slot: int) -> Optional[int]:
        """The frame index a reservation already carries (per-worker slices fix it at
        ``reserve_frame``), else None (it is taken at ``commit_frame``)."""
        with self._lock:
            return self._reserved.get(slot)

    def commit_frame(self, slot: int, nbytes: int, shape=None, timestamp=None, block: bool = True) -> int:
        """Queue the frame written into ``slot``; returns its index (as add_frame_for_distribution)."""
        idx = self._enqueue(None, nbytes, shape, slot, time.time() if timestamp is None else timestamp, block)
        self._kick()
        return idx

    def commit_frames(self, slots: Sequence[int], nbytes: Sequence[int], shapes=None, timestamp=None) -> List[int]:
        """``commit_frame`` for a group of filled reservations, under one lock hold."""
        ts = time.time() if timestamp is None else timestamp
        with self._cv:
            out = [self._enqueue(None, nb, shapes[i] if shapes is not None else None, s_, ts, True)
                   for i, (s_, nb) in enumerate(zip(slots, nbytes))]
        self._kick()
        return out

    def _kick(self) -> None:
        """Frames were queued: serve waiting requests now (inline mode), or wake the dispatch
        thread's socket wait ("tcp"), so a worker holding unserved credit is answered now rather
        than at the end of the poll."""
        if self._inline:
            self._serve_waiting()
        elif self.policy != "latest" and self._wakeable:
            self.distribute_socket.wake()

    def cancel_frame(self, slot: int) -> None:
        """Give back a reserved slot that will not be committed (its index, if one was fixed at
        reservation, is counted lost so the in-order consumer does not wait for it)."""
        with self._cv:
            idx = self._reserved.pop(slot, None)
            self._free_slot(slot)
            if idx is not None:
                self._lose(idx)

    def _target_peer(self, idx: int) -> Optional[_Peer]:
        """The worker whose slice frame ``idx`` goes into (per_worker layout)."""
        if self.policy == "shard":
            pid = self._shard_owner.get(chunk_owner(idx, self.shard_chunk, self.shard_workers))
            p = self._peers.get(pid) if pid is not None else None
            return p if p is not None and p.alive and p.slice is not None else None
        live = [p for p in self._peers.values() if p.alive and p.slice is not None
                and self._slices[p.slice].free]
        if not live:
            return None
        most = max(len(self._slices[p.slice].free) for p in live)
        best = [p for p in live if len(self._slices[p.slice].free) == most]
        self._rr += 1
        return best[self._rr % len(best)]

    def _enqueue(self, frame, nbytes: int, shape, slot: Optional[int], timestamp: float, block: bool) -> int:
        with self._cv:
            idx = self._reserved.pop(slot, None) if slot is not None else None
            if idx is None:
                if self.policy != "latest":
                    # wait for room BEFORE taking an index: a rejected frame must not leave a
                    # hole in the index sequence (the ordered consumer would wait for it)
                    while block and self.running and self._waiting() >= self.queue_size:
                        self._cv.wait(0.05)
                    if self._waiting() >= self.queue_size:
                        self._free_slot(slot)
                        return -1
                idx = self.frame_index_counter          # distributor.py:179-180
                self.frame_index_counter += 1
            item = {"frame": None if slot is not None else frame, "frame_index": idx, "timestamp": timestamp,
                    "nbytes": nbytes, "shape": shape, "slot": slot, "src_slot": None, "attempts": 0,
                    "queued_at": time.monotonic()}
            self._copies[idx] = 1
            if self.policy == "latest":
                self._ingest_latest(item)
            else:
                # lanes stay in index order (_take serves lowest indices first from the left);
                # several producers may commit out of order
                ln = self._lane_for(item)
                if ln and ln[-1]["frame_index"] > idx:
                    at = len(ln)
                    while at > 0 and ln[at - 1]["frame_index"] > idx:
                        at -= 1
                    ln.insert(at, item)
                else:
                    ln.append(item)
            self.log_frame_timing(idx, timestamp, "frame_captured")
        return idx

    def _lane_for(self, item: dict) -> Deque[dict]:
        """Queue a (re-)queued frame waits in."""
        if self.policy == "shard":
            return self._shard_pending[chunk_owner(item["frame_index"], self.shard_chunk, self.shard_workers)]
        if self.ring_layout != "per_worker":
            return self._pending
        if item["slot"] is not None:
            owner = self._peers.get(self._slices[item["slot"] // self.ring_slots].owner)
            if owner is not None and owner.alive:
                return owner.queue
        live = [p for p in self._peers.values() if p.alive and p.slice is not None]
        if not live:
            return self._orphans
        return min(live, key=lambda p: (len(p.queue) + len(p.inflight), p.order)).queue

    def _waiting(self) -> int:
        if self.policy == "pull":
            return len(self._pending) + len(self._orphans) + sum(len(p.queue) for p in self._peers.values())
        return sum(len(q) for q in self._shard_pending.values())

    def _ingest_latest(self, item):
        try:
            self.frame_queue.put_nowait(item)
        except queue.Full:                                   # distributor.py:193-203
            try:
                old = self.frame_queue.get_nowait()
                self._drop(old)
                self.frame_queue.put_nowait(item)
                if self.verbose:
                    print(f"Replaced old frame with new frame {item['frame_index']}")
            except queue.Full:
                self._drop(item)
                if self.verbose:
                    print(f"Frame {item['frame_index']} dropped due to queue overflow")

    def _drop(self, item, keep_slot: bool = False) -> Optional[int]:
        """A frame the latest policy discards (queue overflow, or overwritten in the dispatch
        slot before any worker took it).  Returns its slot when ``keep_slot``."""
        self.frames_dropped += 1
        slot = item.get("slot")
        if not keep_slot:
            self._free_slot(slot)
        self._copy_done(item["frame_index"])
        if self.reassembly == "ordered":
            self._ordered.mark_lost(item["frame_index"])
            self._release_ready()
        return slot if keep_slot else None

    def _evict_oldest_queued_slot(self) -> Optional[int]:
        try:
            old = self.frame_queue.get_nowait()
        except queue.Empty:
            return None
        return self._drop(old, keep_slot=True)

    # ---- copies and losses -----------------------------------------------------------------
    def _copy_done(self, idx: int) -> None:
        n = self._copies.get(idx, 0) - 1
        if n > 0:
            self._copies[idx] = n
        else:
            self._copies.pop(idx, None)
            self._settled.discard(idx)

    def _settle(self, idx: int) -> None:
        if self._copies.get(idx, 0) > 0:
            self._settled.add(idx)

    def _lose(self, idx: int) -> None:
        self.frames_lost += 1
        self._settle(idx)
        if self.reassembly == "ordered":
            self._ordered.mark_lost(idx)
            self._release_ready()
        self._cv.notify_all()

    def _release_ready(self) -> None:
        """Move results that are next in index order to the consumer's queue (lock held)."""
        ready = self._ordered.pop_ready()
        if ready:
            self._released.extend(ready)
            self._cv_out.notify_all()

    # ---- dispatch (distributor.py:205-251) ------------------------------------------------
    def handle_distribute_requests(self):
        while self.running:
            # while a worker holds unserved credit, frames committed during the socket wait
            # must not wait out a whole poll: with "tcp" a commit wakes the wait (``_kick``), so
            # it is 1 ms (batch-fill deadlines and worker deadlines are checked at that pace);
            # with "zmq" (whole-millisecond polls, no wake) it is 0.2 ms, and 1 ms otherwise;
            # the reference's 10 ms under "latest"
            if self.policy == "latest":
                poll_ms = 10
            elif self._wakeable:
                poll_ms = 1
            else:
                with self._lock:
                    hungry = any(p.alive and p.requests for p in self._peers.values())
                poll_ms = 0.2 if hungry else 1
            try:
                self.dispatch_step(poll_ms)
            except BlockingIOError:
                continue
            except Exception as e:
                print(f"Error handling distribute request: {e}")
                continue

    def dispatch_step(self, poll_ms: float = 0) -> None:
        """One iteration of the dispatch loop (distributor.py:209-248): move at most one queued
        frame into the latest-wins slot, poll the dispatch socket for ``poll_ms`` and answer
        what arrived, evict workers past their deadline, serve outstanding requests."""
        if self.policy == "latest":
            try:                                          # distributor.py:210-221
                item = self.frame_queue.get_nowait()
                with self._lock:
                    prev = self.current_frame_data
                    self.current_frame_data = item
                    if prev is not None and prev["frame_index"] > self.last_frame_sent:
                        self._drop(prev)  # overwritten before any READY took it
            except queue.Empty:
                pass
        if self.distribute_socket.poll(poll_ms):
            pid, parts = self.distribute_socket.recv()
            if parts is None:
                with self._cv:
                    p = self._peers.get(pid)
                    if p is not None:
                        self._evict(p, "connection closed", gone=True)
            else:
                req = wire.decode_request(parts)
                if req is not None:
                    self._on_request(pid, req)
        self._check_deadlines()
        self._serve_waiting()

    def _on_request(self, pid: bytes, req: wire.Request):
        with self._cv:
            p = self._peers.get(pid)
            if p is None:
                p = self._register(pid, req)
                if p is None:
                    return
            elif not p.alive and not p.gone:
                self._revive(p)
            p.last_seen = time.monotonic()
            p.wire = req.wire
            if req.version == 0 and self.policy == "latest":
                self._serve_latest_v0(p)                      # distributor.py:229-241
                return
            if req.version == 0 and len(p.requests) >= 2:
                return  # a reference worker re-sends READY every 10 ms; keep at most 2
            p.requests.append(req.credit)

    def _register(self, pid: bytes, req: wire.Request) -> Optional[_Peer]:
        p = _Peer(pid, req, len(self._peers))
        if self.ring_layout == "per_worker":
            try:
                self._make_slice(p)
            except (MemoryError, OSError) as e:
                print(f"Distributor: no ring slice for worker {pid.hex()}: {e}")
                return None
        self._peers[pid] = p
        if p.wid:
            self._by_wid[p.wid] = p
        if self.policy == "shard":
            self._rebalance_shards()
        elif self._orphans:
            self._relane(list(self._orphans))
            self._orphans.clear()
        self._cv.notify_all()
        return p

    def _revive(self, p: _Peer) -> None:
        """An evicted worker asked again: take it back; it re-takes its home shard."""
        p.alive = True
        if self.verbose:
            print(f"Distributor: worker {p.pid.hex()} is back")
        if self.policy == "shard" and p.home_shard is not None:
            other = self._peers.get(self._shard_home.get(p.home_shard))
            if other is not None and other is not p:
                other.home_shard = None
            self._shard_home[p.home_shard] = p.pid
            self._rebalance_shards()
        elif self._orphans:  # frames that found no live worker while it was out
            self._relane(list(self._orphans))
            self._orphans.clear()
        self._cv.notify_all()

    def _rebalance_shards(self) -> None:
        """Shard k is served by its home worker while that one is alive; an orphaned shard is
        adopted (as home) by a live worker that has none, else served by the live worker with
        the fewest shards."""
        live = sorted((p for p in self._peers.values() if p.alive), key=lambda p: p.order)
        for k in range(self.shard_workers):
            home = self._peers.get(self._shard_home.get(k))
            if home is None or not home.alive:
                spare = next((p for p in live if p.home_shard is None), None)
                if spare is not None:
                    if home is not None:
                        home.home_shard = None
                    spare.home_shard = k
                    self._shard_home[k] = spare.pid
                    home = spare
            if home is not None and home.alive:
                self._shard_owner[k] = home.pid
                continue
            cur = self._peers.get(self._shard_owner.get(k))
            if cur is not None and cur.alive:
                continue
            if live:
                load = collections.Counter(self._shard_owner.get(j) for j in range(self.shard_workers)
                                           if j != k)
                self._shard_owner[k] = min(live, key=lambda p: (load[p.pid], p.order)).pid
            else:
                self._shard_owner.pop(k, None)

    def _serve_latest_v0(self, p: _Peer):
        cur = self.current_frame_data
        if cur is not None and cur.get("frame_index") is not None and cur["frame_index"] > self.last_frame_sent:
            self._queue_dispatch(p, [cur])
            self.last_frame_sent = cur["frame_index"]

    def _fill_pending(self, p: _Peer, credit: int) -> bool:
        """True while request ``credit`` of busy worker ``p`` should wait for more frames
        (see "Batch filling" above)."""
        if self.policy == "latest" or p.version == 0 or credit <= 1 or not p.inflight or self.batch_wait <= 0:
            return False
        lanes = [ln for ln in self._lanes_of(p) if ln]
        if not lanes or sum(len(ln) for ln in lanes) >= credit:
            return False
        oldest = min(ln[0].get("queued_at", 0.0) for ln in lanes)
        return time.monotonic() - oldest < self.batch_wait

    def _serve_waiting(self):
        with self._lock:
            for p in list(self._peers.values()):
                while p.alive and p.requests:
                    if self._fill_pending(p, p.requests[0]):
                        break
                    items = self._take(p, p.requests[0])
                    if not items:
                        break
                    p.requests.popleft()
                    self._queue_dispatch(p, items)
        self._flush_dirty()

    def _lanes_of(self, p: _Peer) -> List[Deque[dict]]:
        if self.policy == "pull":
            return [p.queue] if self.ring_layout == "per_worker" else [self._pending]
        return [self._shard_pending[k] for k in range(self.shard_workers) if self._shard_owner.get(k) == p.pid]

    def _take(self, p: _Peer, credit: int) -> List[dict]:
        if self.policy == "latest":
            cur = self.current_frame_data
            if cur is not None and cur["frame_index"] > self.last_frame_sent:
                self.last_frame_sent = cur["frame_index"]
                return [cur]
            return []
        if p.version == 0:
            credit = 1
        lanes = [ln for ln in self._lanes_of(p) if ln]
        if not lanes:
            return []
        out: List[dict] = []
        if len(lanes) == 1:  # one lane, kept in index order: take from the left
            ln, settled, skipped, took = lanes[0], self._settled, [], False
            while ln and len(out) < credit:
                it = ln.popleft()
                took = True
                if it["frame_index"] in settled:  # delivered from another copy
                    self._release_copy(it)
                elif self._place(it, p):
                    out.append(it)
                else:  # no free slot in this worker's slice for the copy: not waited on
                    skipped.append(it)
            for it in reversed(skipped):
                ln.appendleft(it)
            if took:
                self._cv.notify_all()  # ingest may be waiting for room
            return out
        taken = set()
        # lowest indices first; a copy that must move into this worker's slice but finds no
        # free slot there is skipped, not waited on (the slots may be held by the frames
        # queued behind it)
        for it in sorted((it for ln in lanes for it in ln), key=lambda x: x["frame_index"]):
            if len(out) >= credit:
                break
            if it["frame_index"] in self._settled:  # delivered from another copy
                self._release_copy(it)
                taken.add(id(it))
                continue
            if self._place(it, p):
                out.append(it)
                taken.add(id(it))
        if taken:
            for ln in lanes:
                keep = [it for it in ln if id(it) not in taken]
                if len(keep) != len(ln):
                    ln.clear()
                    ln.extend(keep)
            self._cv.notify_all()  # ingest may be waiting for room
        return out

    def _place(self, it: dict, p: _Peer) -> bool:
        """Make sure frame copy ``it`` sits in a slot ``p`` can read (its own slice, or any
        slot of the shared ring for a copy that does not own one yet)."""
        if self.ring_layout is None:
            return True
        sid = 0 if self.ring_layout == "shared" else p.slice
        slot = it["slot"]
        if slot is None and it["src_slot"] is None:
            return True  # travels as a socket payload
        if slot is not None and (self.ring_layout == "shared" or slot // self.ring_slots == sid):
            return True
        new = self._alloc_slot(sid)
        if new is None:
            return False
        src = slot if slot is not None else it["src_slot"]
        self.in_view(new, it["nbytes"])[:] = self.in_view(src, it["nbytes"])
        if slot is not None:
            self._free_slot(slot)
        else:
            self._clone_src.pop(src, None)
        it["slot"], it["src_slot"] = new, None
        return True

    def _release_copy(self, it: dict) -> None:
        """A queued copy that will not be dispatched (its frame is settled)."""
        if it.get("slot") is not None:
            self._free_slot(it["slot"])
        elif it.get("src_slot") is not None:
            self._clone_src.pop(it["src_slot"], None)
        self._copy_done(it["frame_index"])

    def _dispatch_parts(self, p: _Peer, items: List[dict]) -> list:
        """The dispatch message for ``items`` in the form ``p`` reads (lock held)."""
        if p.version == 0:
            it = items[0]
            payload = it["frame"] if it["slot"] is None else bytes(self.in_view(it["slot"], it["nbytes"]))
            return wire.encode_dispatch_v0(it["frame_index"], payload)
        ring = None
        rs = self.ring_slots
        use_ring = p.shm and any(it["slot"] is not None for it in items)
        if use_ring:
            sid = next(it["slot"] for it in items if it["slot"] is not None) // rs
            ring = {"name": self._slices[sid].ring.name, "slot_bytes": self._slices[sid].ring.slot_bytes}
        payloads = [None if (use_ring and it["slot"] is not None) else
                    (it["frame"] if it["slot"] is None else bytes(self.in_view(it["slot"], it["nbytes"])))
                    for it in items]
        if p.wire >= 2 and all(wire.v2_shape_ok(it["shape"]) for it in items):
            cols = np.zeros(len(items), wire.COLS)
            cols["index"] = [it["frame_index"] for it in items]
            cols["nbytes"] = [it["nbytes"] for it in items]
            cols["slot"] = [it["slot"] % rs if pl is None else -1 for it, pl in zip(items, payloads)]
            cols["ndim"] = -1
            for i, it in enumerate(items):
                sh = it["shape"]
                if sh is not None:
                    cols["ndim"][i] = len(sh)
                    cols["shape"][i, :len(sh)] = sh
            return wire.encode_dispatch2(cols, [pl for pl in payloads if pl is not None], ring)
        metas = [wire.FrameMeta(index=it["frame_index"], nbytes=it["nbytes"], shape=it["shape"],
                                slot=it["slot"] % rs if pl is None else None) for it, pl in zip(items, payloads)]
        return wire.encode_dispatch(metas, payloads, ring)

    def _queue_dispatch(self, p: _Peer, items: List[dict]) -> None:
        """Build and book a dispatch of ``items`` to ``p`` and queue it for sending (lock held):
        the frames are in flight from here, so a result can never arrive before its booking."""
        parts = self._dispatch_parts(p, items)
        p.frames_sent += len(items)
        p.batches_sent += 1
        batch = [time.monotonic(), set()]
        for it in items:
            it["attempts"] += 1
            it["_batch"] = batch
            p.inflight[it["frame_index"]] = it
            batch[1].add(it["frame_index"])
        p.batches.append(batch)
        p.outbox.append((parts, items))
        self._dirty.add(p)

    def _flush_dirty(self) -> None:
        """Send every queued dispatch, outside the distributor's lock."""
        if not self._dirty:
            return
        with self._lock:
            peers = list(self._dirty)
            self._dirty.clear()
        for p in peers:
            self._flush(p)

    def _flush(self, p: _Peer) -> None:
        """Drain ``p``'s outbox in order.  One thread at a time sends to a peer (``send_lock``);
        another thread finding the lock held leaves its messages to the holder, which checks
        the outbox again after letting go of the lock."""
        while True:
            if not p.send_lock.acquire(blocking=False):
                return
            try:
                while True:
                    with self._lock:
                        if not p.outbox:
                            break
                        parts, items = p.outbox.popleft()
                    if not self.distribute_socket.send(p.pid, parts):
                        with self._cv:
                            self._unsend(p, items)
            finally:
                p.send_lock.release()
            with self._lock:
                if not p.outbox:
                    return

    def _unsend(self, p: _Peer, items: List[dict]) -> None:
        """The transport refused a dispatch (the worker is gone): that dispatch and every one
        still queued behind it are un-booked and go back to the queues (lock held)."""
        for _, more in p.outbox:
            items = items + more
        p.outbox.clear()
        # only copies still booked to p: an eviction since the booking has re-queued the others
        items = [it for it in items if p.inflight.get(it["frame_index"]) is it]
        for it in items:
            idx = it["frame_index"]
            del p.inflight[idx]
            b = it.pop("_batch", None)
            if b is not None:
                b[1].discard(idx)
            it["attempts"] -= 1
        while p.batches and not p.batches[0][1]:
            p.batches.popleft()
        p.frames_sent -= len(items)
        if self.policy == "latest":
            cur = self.current_frame_data
            for it in items:
                if it is cur and it["frame_index"] == self.last_frame_sent:
                    # the reference books last_frame_sent only after a successful send
                    # (distributor.py:238-241): the frame still in the dispatch slot stays there
                    # for the next READY instead of being dropped
                    self.last_frame_sent = it["frame_index"] - 1
                else:
                    self._drop(it)
        else:
            self._relane(items)
        self._evict(p, "dispatch refused (worker disconnected)", gone=True)

    def _relane(self, items: List[dict]) -> None:
        """Put frame copies back at the front of their queues, in index order."""
        by_lane: Dict[int, list] = {}
        lanes: Dict[int, Deque[dict]] = {}
        for it in items:
            ln = self._lane_for(it)
            lanes[id(ln)] = ln
            by_lane.setdefault(id(ln), []).append(it)
        for key, its in by_lane.items():
            ln = lanes[key]
            merged = sorted(its + list(ln), key=lambda x: x["frame_index"])
            ln.clear()
            ln.extend(merged)
        self._cv.notify_all()

    # ---- worker loss -----------------------------------------------------------------------
    def _check_deadlines(self) -> None:
        """Evict a worker whose oldest batch is past ``batch_timeout``, and one that has frames
        waiting for it but has neither asked for them nor had anything in flight for as long
        (it stopped asking without closing its connection; ZeroMQ reports no disconnects)."""
        if self.batch_timeout <= 0:
            return
        now = time.monotonic()
        with self._cv:
            for p in list(self._peers.values()):
                if p.quarantine:
                    self._expire_quarantine(p, now)
                if not p.alive:
                    continue
                if p.batches and now - p.batches[0][0] > self.batch_timeout:
                    self._evict(p, f"no result within {self.batch_timeout:g} s")
                    continue
                idle = (self.policy != "latest" and not p.batches and not p.requests
                        and any(self._lanes_of(p)))
                if not idle:
                    p.waiting_since = None
                elif p.waiting_since is None:
                    p.waiting_since = now
                elif now - p.waiting_since > self.batch_timeout:
                    self._evict(p, f"frames waiting, no request for {self.batch_timeout:g} s")

    def _expire_quarantine(self, p: _Peer, now: float) -> None:
        """Slots of frames an evicted worker still held come back after a grace period of one
        more ``batch_timeout``: ZeroMQ reports no disconnects, so a worker that died or hung
        would otherwise keep them out of use for ever and every eviction would shrink the ring
        (ADVICE r02).  A result that still arrives later finds no dispatch record and is
        dropped (``_find_copy``), so it cannot be mistaken for the slot's next frame.

        Its BYTES are another matter: a worker that was only slow may still write
        the stale result into the slot's output half after the slot has a new owner.  That is
        harmless only where the new owner's result comes from the same worker, written after
        the stale one: a slot of the evicted worker's own slice (``per_worker`` layout) is only
        ever dispatched to that worker, which writes its results in dispatch order (one in-order
        zero-copy stream; JPEG results are scattered in FIFO order), so its late write lands
        before any later dispatch's.  A slot of the shared ring could go to any worker, so it
        stays out of use until the late result frees it or the worker is known gone."""
        for idx in [i for i, it in p.quarantine.items() if now - it.get("_evicted_at", now) > self.batch_timeout]:
            it = p.quarantine[idx]
            slot = it.get("slot")
            if slot is not None and not (self.ring_layout == "per_worker" and p.slice is not None
                                         and slot // self.ring_slots == p.slice):
                # shared ring: held until the result or the disconnect -- and where the transport
                # reports no disconnects (ZeroMQ), for at most QUARANTINE_HOLD batch timeouts, so a
                # dead worker cannot shrink the ring for ever.  A worker that was only
                # hung that long and then writes its stale result into the slot's output half is
                # the documented risk of that bound.
                if self._disconnect_notices or now - it["_evicted_at"] <= self.QUARANTINE_HOLD * self.batch_timeout:
                    continue
                self.quarantine_forced += 1
            p.quarantine.pop(idx)
            self._free_slot(it.get("slot"))
            self._copy_done(it["frame_index"])
            self.quarantine_expired += 1

    def _evict(self, p: _Peer, reason: str, gone: bool = False) -> None:
        """Take ``p`` out of service: re-queue (or lose, after ``max_attempts``) what it holds."""
        was_alive = p.alive
        p.alive = False
        p.gone = p.gone or gone
        p.requests.clear()
        if was_alive and gone and not p.inflight and not p.queue:
            self.departures += 1            # left with nothing outstanding
        elif was_alive:
            p.evictions += 1
            self.evictions += 1
            if self.verbose:
                print(f"Distributor: worker {p.pid.hex()} evicted ({reason}); "
                      f"{len(p.inflight)} frames in flight re-queued")
        requeue = []
        for idx in sorted(p.inflight):
            it = p.inflight[idx]
            it.pop("_batch", None)
            it["_evicted_at"] = time.monotonic()
            p.quarantine[idx] = it          # its slot stays out of use until a result frees it
            if self.policy == "latest" or it["attempts"] >= self.max_attempts:
                self._lose(idx)
                continue
            clone = dict(it, slot=None, src_slot=it["slot"])
            if it["slot"] is not None:
                self._clone_src[it["slot"]] = clone
            self._copies[idx] = self._copies.get(idx, 0) + 1
            self.frames_requeued += 1
            requeue.append(clone)
        p.inflight.clear()
        p.batches.clear()
        if p.queue:
            requeue.extend(p.queue)
            p.queue.clear()
        if self.policy == "shard":
            self._rebalance_shards()
        if requeue:
            self._relane(requeue)
        if p.gone:  # nothing can come back from it: its quarantined slots are free again
            for it in p.quarantine.values():
                self._free_slot(it.get("slot"))
                self._copy_done(it["frame_index"])
            p.quarantine.clear()
        self._cv.notify_all()

    # ---- collect (distributor.py:253-289) ------------------------------------------------
    def check_inverter_output(self):
        while self.running:
            try:
                if self.collect_socket.poll(10):
                    res = wire.decode_result(self.collect_socket.recv())
                    self._on_result(res)
            except BlockingIOError:
                continue
            except Exception as e:
                print(f"Error receiving inverted frame: {e}")
                continue

    def _find_copy(self, p: Optional[_Peer], idx: int):
        """(worker, dispatched copy) of a result; the worker's copy leaves its in-flight set."""
        cands = [p] if p is not None else list(self._peers.values())
        for q in cands:
            it = q.inflight.pop(idx, None)
            if it is not None:
                b = it.pop("_batch", None)
                if b is not None:
                    b[1].discard(idx)
                while q.batches and not q.batches[0][1]:
                    q.batches.popleft()
                return q, it
            it = q.quarantine.pop(idx, None)
            if it is not None:
                return q, it
        return None, None

    def _on_result_fast(self, res: wire.Result, pid_val) -> bool:
        """The common result message -- every frame a zero-copy ring result of the sender's own
        dispatch, in flight once, no error, ordered reassembly, no trace -- booked in one pass
        under one lock hold: what ``_on_result``'s general path does for it, with the per-frame
        helper calls inlined.  False (nothing done) for any other message."""
        if not (self.zero_copy and self.reassembly == "ordered" and res.wid and not self.enable_trace_export):
            return False
        with self._cv:
            sender = self._by_wid.get(res.wid)
            if sender is None:
                return False
            inflight, copies, settled = sender.inflight, self._copies, self._settled
            for m in res.metas:
                if (m.error is not None or m.slot is None or m.index not in inflight or m.index in settled
                        or copies.get(m.index) != 1 or inflight[m.index].get("slot") is None):
                    return False
            sender.last_seen = time.monotonic()
            sid_of, rs = self.ring_slots, self._slices
            held, push = self._held, self._ordered.push
            pid = res.pid
            for m in res.metas:
                idx = m.index
                it = inflight.pop(idx)
                b = it.pop("_batch", None)
                if b is not None:
                    b[1].discard(idx)
                copies.pop(idx, None)
                slot = it["slot"]
                sid, k = divmod(slot, sid_of)
                held[idx] = slot
                push(idx, rs[sid].ring.out_view(k, m.nbytes),
                     {"process_id": pid, "start_time": m.start, "end_time": m.end, "shape": m.shape, "slot": slot})
            bq = sender.batches
            while bq and not bq[0][1]:
                bq.popleft()
            n = len(res.metas)
            sender.results += n
            self.results_received += n
            self._release_ready()
        return True

    def _on_result(self, res: wire.Result):
        """One result message (a batch): bookkeeping for all its frames under one lock hold,
        the result bytes read outside it (each copy and its slot are this thread's alone once
        taken out of the in-flight set), then one hold to hand them to the reassembly."""
        pid_val = int(res.pid) if res.pid.isdigit() else res.pid
        for sp in res.spans:
            self.log_gpu_span(sp.get("name", "?"), float(sp["begin"]), float(sp["end"]), pid_val,
                              int(sp.get("bytes", 0)))
        if self._on_result_fast(res, pid_val):
            return
        reads = []
        with self._cv:
            sender = self._by_wid.get(res.wid) if res.wid else None
            if sender is not None:
                sender.last_seen = time.monotonic()
            for m, payload in zip(res.metas, res.payloads):
                self.log_frame_complete_timing(m.index, m.start, m.end, "frame_inverted_received", pid_val)
                q, it = self._find_copy(sender, m.index)
                slot = it.get("slot") if it is not None else None
                if q is not None:
                    q.results += 1
                    if m.error is not None:
                        q.errors += 1
                tracked = it is not None
                if tracked and m.index in self._settled:    # a re-queued frame's second result
                    self.duplicates += 1
                    self._free_slot(slot)
                    self._copy_done(m.index)
                    continue
                if tracked:
                    self._copy_done(m.index)
                    self._settle(m.index)
                if m.error is not None:
                    self.result_errors += 1
                    self._free_slot(slot)
                    if self.reassembly == "ordered":
                        self._ordered.mark_lost(m.index)
                        self._release_ready()
                    continue
                if m.slot is not None and slot is None:
                    continue  # a ring result with no dispatch record: nothing to read it from
                reads.append((m, payload, slot, self.zero_copy and m.slot is not None))
        if not reads:
            return
        out = []
        for m, payload, slot, keep in reads:
            if m.slot is not None:
                view = self.out_view(slot, m.nbytes)
                out.append((m, view if keep else bytes(view), slot, keep))
            else:
                out.append((m, payload, slot, keep))
        with self._cv:
            for m, data, slot, keep in out:
                if keep:
                    self._held[m.index] = slot
                else:
                    self._free_slot(slot)
                self.results_received += 1
                if self.reassembly == "display":
                    self._display.receive(m.index, data, res.pid, m.start, m.end)
                else:
                    self._ordered.push(m.index, data, {"process_id": res.pid, "start_time": m.start,
                                                       "end_time": m.end, "shape": m.shape,
                                                       "slot": slot if keep else None})
            if self.reassembly != "display":
                self._release_ready()

    # ---- reassembly API (distributor.py:291-354) ---------------------------------------
    def cleanup_old_frames(self):
        with self._lock:
            self._display.cleanup_old_frames()

    def get_frame_to_display(self):
        with self._lock:
            return self._display.get_frame_to_display()

    def update_display_frame(self):
        with self._lock:
            return self._display.update_display_frame()

    def get_frame_stats(self):
        with self._lock:
            return {"buffer_size": len(self.received_frames),
                    "current_display_frame": self.current_display_frame,
                    "latest_received_frame": self.latest_received_frame,
                    "frame_delay": self.frame_delay,
                    "total_frames_processed": self.frame_index_counter}

    def get_next_frame(self, timeout: Optional[float] = None):
        """reassembly='ordered': the next result in index order as (index, data, info),
        or None on timeout."""
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while not self._released:
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    return None
                if not self.running and not self._released:
                    return None
                self._cv_out.wait(rem if rem is not None else 0.1)
            return self._released.popleft()

    def get_next_frames(self, max_n: int, timeout: Optional[float] = None) -> list:
        """reassembly='ordered': up to ``max_n`` next results in index order (at least one, or
        an empty list on timeout), taken under one lock hold."""
        first = self.get_next_frame(timeout)
        if first is None:
            return []
        out = [first]
        with self._cv:
            while self._released and len(out) < max_n:
                out.append(self._released.popleft())
        return out

    def get_next_batch(self, max_n: int, timeout: Optional[float] = None) -> "ListBatch":
        """``get_next_frames`` in the columnar form of the native engine's ``get_next_batch``."""
        return ListBatch(self.get_next_frames(max_n, timeout))

    def reserve_frames_array(self, nbytes: int, n: int, block: bool = True):
        """``reserve_frames`` as arrays: (slots, indices)."""
        slots = self.reserve_frames(nbytes, n, block)
        idx = [self.reserved_index(s_) for s_ in slots]
        return np.asarray(slots, np.int32), np.asarray([-1 if i is None else i for i in idx], np.int64)

    def fill_frames(self, slots, src_addrs, nbytes) -> None:
        """The native engine's columnar copy (vfd_fill) for this engine: frame i's ``nbytes[i]``
        bytes at address ``src_addrs[i]`` into reserved slot ``slots[i]`` (one copy per frame)."""
        if not (len(slots) == len(src_addrs) == len(nbytes)):
            raise ValueError("fill_frames: slots, src_addrs and nbytes differ in length")
        cols = list(zip(np.asarray(slots).tolist(), np.asarray(src_addrs, np.uint64).tolist(),
                        np.asarray(nbytes).tolist()))
        for s_, a, nb in cols:  # refused before anything is copied, as vfd_fill
            if self.reserved_index(s_) is None:
                raise ValueError(f"fill_frames: slot {s_} was not reserved")
            if nb < 0 or nb > self.ring_slot_bytes:
                raise ValueError(f"fill_frames: a frame of {nb} B does not fit a slot of {self.ring_slot_bytes} B")
        for s_, a, nb in cols:
            if nb:
                src = np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(a))
                self.in_view(s_, nb)[:] = src

    def release_frame(self, index: int) -> None:
        """zero_copy: return frame ``index``'s ring slot once its result view is consumed."""
        with self._cv:
            self._free_slot(self._held.pop(index, None))

    def release_frames(self, indices: Sequence[int]) -> None:
        """``release_frame`` for a group of consumed results, under one lock hold."""
        with self._cv:
            held = self._held
            for i in indices:
                self._free_slot(held.pop(i, None), notify=False)
            self._cv.notify_all()  # one wake-up for the group

    def num_workers(self) -> int:
        with self._lock:
            return sum(1 for p in self._peers.values() if p.alive)

    def ordering_stats(self) -> dict:
        with self._lock:
            s = self._ordered.stats()
            s.update({"frames_dropped": self.frames_dropped, "results_received": self.results_received,
                      "result_errors": self.result_errors, "frames_lost": self.frames_lost,
                      "frames_requeued": self.frames_requeued, "duplicates": self.duplicates,
                      "evictions": self.evictions, "departures": self.departures,
                      "workers": {p.pid.hex(): {"sent": p.frames_sent, "batches": p.batches_sent,
                                                "results": p.results, "alive": p.alive,
                                                "home_shard": p.home_shard,
                                                "shards": sorted(k for k, o in self._shard_owner.items()
                                                                 if o == p.pid),
                                                "in_flight": len(p.inflight), "evictions": p.evictions,
                                                "slice": self._slice_info(p.slice), "slice_id": p.slice}
                                  for p in self._peers.values()}})
            return s

    def _slice_info(self, sid: Optional[int]) -> Optional[dict]:
        if sid is None:
            return None
        sl = self._slices[sid]
        return {"name": sl.ring.name, "bytes": sl.ring.nbytes, "numa": sl.numa, "numa_bound": sl.bound,
                "free": len(sl.free)}
