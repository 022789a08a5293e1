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
                   goes to the (c % shard_workers)-th worker to register — frame-index sharding
                   across 1/2/4/8 GPUs.
  reassembly="ordered"  every result released exactly once in index order
                   (``get_next_frame``), with ordering-overhead statistics.
  ring_slots>0     same-node shared-memory data plane (``vfilter.shm``): frames are written once
                   into a ring slot and only slot numbers travel on the sockets.
All shared state sits behind one lock (the reference relies on the GIL).
"""
from __future__ import annotations

import collections
import json
import os
import queue
import threading
import time
from typing import Deque, Dict, List, Optional

import numpy as np

from . import transport as tp
from . import wire
from .reorder import DisplayBuffer, OrderedBuffer
from .sharding import chunk_owner
from .shm import FrameRing


class _Peer:
    __slots__ = ("pid", "version", "requests", "frames_sent", "results", "errors", "shard")

    def __init__(self, pid: bytes, version: int):
        self.pid = pid
        self.version = version
        self.requests: Deque[int] = collections.deque()  # credits of outstanding requests
        self.frames_sent = 0
        self.results = 0
        self.errors = 0
        self.shard: Optional[int] = None


class Distributor:
    def __init__(self, distribute_port: int = 5555, collect_port: int = 5556, frame_delay: int = 5,
                 enable_trace_export: bool = False, *, policy: str = "latest", reassembly: str = "display",
                 transport: str = "auto", host: str = "*", queue_size: int = 10, frame_buffer_size: int = 50,
                 ring_slots: int = 0, ring_slot_bytes: int = 0, shard_workers: int = 0, shard_chunk: int = 1,
                 trace_file: str = "webcam_frame_timing.pftrace", verbose: bool = True, zero_copy: bool = False):
        if zero_copy and (ring_slots < 1 or reassembly != "ordered"):
            raise ValueError("zero_copy needs ring_slots > 0 and reassembly='ordered'")
        self.zero_copy = zero_copy
        if policy not in ("latest", "pull", "shard"):
            raise ValueError("policy must be latest | pull | shard")
        if reassembly not in ("display", "ordered"):
            raise ValueError("reassembly must be display | ordered")
        if policy == "shard" and shard_workers < 1:
            raise ValueError("policy='shard' needs shard_workers >= 1")
        self.policy = policy
        self.reassembly = reassembly
        self.verbose = verbose
        # ingest (distributor.py:11-14)
        self.frame_queue: "queue.Queue[dict]" = queue.Queue(maxsize=queue_size)
        self.frame_index_counter = 0
        self.last_frame_sent = -1                   # distributor.py:17
        self.current_frame_data: Optional[dict] = None
        self._pending: Deque[dict] = collections.deque()   # lossless policies
        self._shard_pending: Dict[int, Deque[dict]] = collections.defaultdict(collections.deque)
        self.queue_size = queue_size
        self.shard_workers = shard_workers
        self.shard_chunk = max(1, shard_chunk)
        # reassembly (distributor.py:19-24)
        self._display = DisplayBuffer(frame_delay, frame_buffer_size)
        self._ordered = OrderedBuffer(0)
        self._released: Deque[tuple] = collections.deque()
        self._lock = threading.RLock()
        self._cv = threading.Condition(self._lock)
        # transport (distributor.py:26-35)
        self.transport = tp.resolve(transport)
        self._zctx = tp.make_context(self.transport)
        self.distribute_socket = tp.RouterEnd(self.transport, host, distribute_port, self._zctx)
        self.collect_socket = tp.PullEnd(self.transport, host, collect_port, self._zctx)
        self.distribute_port = self.distribute_socket.port
        self.collect_port = self.collect_socket.port
        # shared-memory ring
        self.ring: Optional[FrameRing] = None
        if ring_slots > 0:
            if ring_slot_bytes < 1:
                raise ValueError("ring_slots needs ring_slot_bytes (largest frame)")
            self.ring = FrameRing(ring_slots, ring_slot_bytes)
        self._slot_of: Dict[int, int] = {}
        # tracing (distributor.py:37-40)
        self.enable_trace_export = enable_trace_export
        self.frame_timings: List[dict] = []
        self.trace_start_time = time.time()
        self.trace_file = trace_file
        # peers and counters
        self._peers: Dict[bytes, _Peer] = {}
        self._shard_owner: Dict[int, bytes] = {}
        self.frames_dropped = 0
        self.results_received = 0
        self.result_errors = 0
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
        self.distribute_thread.start()
        self.inverter_thread.start()

    def stop(self):
        self.running = False
        with self._cv:
            self._cv.notify_all()

    def cleanup(self):
        self.stop()
        for t in (self.distribute_thread, self.inverter_thread):
            if t.is_alive():
                t.join(timeout=1.0)
        self.distribute_socket.close()
        self.collect_socket.close()
        if self._zctx is not None:
            self._zctx.term()
        if self.ring is not None:
            self.ring.close()
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
        slot = None
        if self.ring is not None:
            slot = self.reserve_frame(nbytes, block)
            if slot is None:
                return -1
            self.ring.in_view(slot, nbytes)[:] = np.frombuffer(frame, dtype=np.uint8) \
                if not isinstance(frame, np.ndarray) else frame.reshape(-1).view(np.uint8)
        return self._enqueue(None if slot is not None else frame, nbytes, shape, slot, timestamp, block)

    # ---- zero-copy ingest (ring mode) ------------------------------------------------------
    def reserve_frame(self, nbytes: int, block: bool = True) -> Optional[int]:
        """Reserve a ring slot for a frame of ``nbytes``; fill ``frame_view(slot, nbytes)`` in
        place (e.g. decode or capture straight into it), then ``commit_frame``.  Returns None
        when no slot is free and ``block`` is False."""
        if self.ring is None:
            raise RuntimeError("reserve_frame needs ring_slots > 0")
        if nbytes > self.ring.slot_bytes:
            raise ValueError(f"frame of {nbytes} B exceeds ring slot of {self.ring.slot_bytes} B")
        slot = self.ring.acquire(timeout=None if (block and self.policy != "latest") else 0)
        if slot is None and self.policy == "latest":
            slot = self._evict_oldest_queued_slot()
        return slot

    def frame_view(self, slot: int, nbytes: int) -> np.ndarray:
        return self.ring.in_view(slot, nbytes)

    def commit_frame(self, slot: int, nbytes: int, shape=None, timestamp=None, block: bool = True) -> int:
        """Queue the frame written into ``slot``; returns its index (as add_frame_for_distribution)."""
        return self._enqueue(None, nbytes, shape, slot, time.time() if timestamp is None else timestamp, block)

    def _enqueue(self, frame, nbytes: int, shape, slot: Optional[int], timestamp: float, block: bool) -> int:
        with self._cv:
            frame_index = self.frame_index_counter          # distributor.py:179-180
            self.frame_index_counter += 1
            item = {"frame": None if slot is not None else frame, "frame_index": frame_index,
                    "timestamp": timestamp, "nbytes": nbytes, "shape": shape, "slot": slot}
            if slot is not None:
                self._slot_of[frame_index] = slot
            if self.policy == "latest":
                self._ingest_latest(item)
            else:
                while block and self.running and self._waiting() >= self.queue_size:
                    self._cv.wait(0.05)
                if not block and self._waiting() >= self.queue_size:
                    if slot is not None:
                        self._free_slot(frame_index)
                    return -1
                if self.policy == "pull":
                    self._pending.append(item)
                else:
                    self._shard_pending[chunk_owner(frame_index, self.shard_chunk, self.shard_workers)].append(item)
                self._cv.notify_all()
            self.log_frame_timing(frame_index, timestamp, "frame_captured")
        return frame_index

    def _waiting(self) -> int:
        if self.policy == "pull":
            return len(self._pending)
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

    def _drop(self, item):
        self.frames_dropped += 1
        if item.get("slot") is not None:
            self._free_slot(item["frame_index"])

    def _evict_oldest_queued_slot(self) -> Optional[int]:
        with self._lock:
            try:
                old = self.frame_queue.get_nowait()
            except queue.Empty:
                return None
            self.frames_dropped += 1
            s = self._slot_of.pop(old["frame_index"], None)
            return s

    def _free_slot(self, index: int):
        s = self._slot_of.pop(index, None)
        if s is not None and self.ring is not None:
            self.ring.release(s)

    # ---- dispatch (distributor.py:205-251) ------------------------------------------------
    def handle_distribute_requests(self):
        poll_ms = 10 if self.policy == "latest" else 1
        while self.running:
            try:
                if self.policy == "latest":
                    try:                                      # distributor.py:210-221
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
                    req = wire.decode_request(parts)
                    if req is not None:
                        self._on_request(pid, req)
                self._serve_waiting()
            except BlockingIOError:
                continue
            except Exception as e:
                print(f"Error handling distribute request: {e}")
                continue

    def _peer(self, pid: bytes, version: int) -> _Peer:
        p = self._peers.get(pid)
        if p is None:
            p = self._peers[pid] = _Peer(pid, version)
            if self.policy == "shard":
                k = len(self._shard_owner)
                if k < self.shard_workers:
                    self._shard_owner[k] = pid
                    p.shard = k
        return p

    def _on_request(self, pid: bytes, req: wire.Request):
        with self._lock:
            p = self._peer(pid, req.version)
            if req.version == 0 and self.policy == "latest":
                self._serve_latest_v0(p)                      # distributor.py:229-241
                return
            if req.version == 0 and len(p.requests) >= 2:
                return  # a reference worker re-sends READY every 10 ms; keep at most 2
            p.requests.append(req.credit)

    def _serve_latest_v0(self, p: _Peer):
        cur = self.current_frame_data
        if cur is not None and cur.get("frame_index") is not None and cur["frame_index"] > self.last_frame_sent:
            if self._send(p, [cur]):
                self.last_frame_sent = cur["frame_index"]

    def _serve_waiting(self):
        with self._lock:
            for p in list(self._peers.values()):
                while p.requests:
                    items = self._take(p, p.requests[0])
                    if not items:
                        break
                    p.requests.popleft()
                    if not self._send(p, items):
                        break

    def _take(self, p: _Peer, credit: int) -> List[dict]:
        if self.policy == "latest":
            cur = self.current_frame_data
            if cur is not None and cur["frame_index"] > self.last_frame_sent:
                self.last_frame_sent = cur["frame_index"]
                return [cur]
            return []
        src = self._pending if self.policy == "pull" else (
            self._shard_pending.get(p.shard) if p.shard is not None else None)
        if not src:
            return []
        if p.version == 0:
            credit = 1
        out = []
        while src and len(out) < credit:
            out.append(src.popleft())
        self._cv.notify_all()  # ingest may be waiting for room
        return out

    def _send(self, p: _Peer, items: List[dict]) -> bool:
        if p.version == 0:
            it = items[0]
            payload = it["frame"] if it["slot"] is None else \
                bytes(self.ring.in_view(it["slot"], it["nbytes"]))
            ok = self.distribute_socket.send(p.pid, wire.encode_dispatch_v0(it["frame_index"], payload))
        else:
            metas = [wire.FrameMeta(index=it["frame_index"], nbytes=it["nbytes"], shape=it["shape"],
                                    slot=it["slot"]) for it in items]
            ring = None
            if any(m.slot is not None for m in metas):
                ring = {"name": self.ring.name, "slot_bytes": self.ring.slot_bytes}
            ok = self.distribute_socket.send(p.pid, wire.encode_dispatch(metas, [it["frame"] for it in items], ring))
        if ok:
            p.frames_sent += len(items)
        return ok

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

    def _on_result(self, res: wire.Result):
        pid_val = int(res.pid) if res.pid.isdigit() else res.pid
        for sp in res.spans:
            self.log_gpu_span(sp.get("name", "?"), float(sp["begin"]), float(sp["end"]), pid_val,
                              int(sp.get("bytes", 0)))
        for m, payload in zip(res.metas, res.payloads):
            self.log_frame_complete_timing(m.index, m.start, m.end, "frame_inverted_received",
                                           int(res.pid) if res.pid.isdigit() else res.pid)
            if m.error is not None:
                with self._cv:
                    self.result_errors += 1
                    self._free_slot(m.index)
                    if self.reassembly == "ordered":
                        self._ordered.mark_lost(m.index)
                        self._released.extend(self._ordered.pop_ready())
                        self._cv.notify_all()
                continue
            if m.slot is not None:
                # zero-copy: hand out the slot's output half; the consumer releases it
                data = self.ring.out_view(m.slot, m.nbytes) if self.zero_copy else \
                    bytes(self.ring.out_view(m.slot, m.nbytes))
            else:
                data = payload
            with self._cv:
                if not (self.zero_copy and m.slot is not None):
                    self._free_slot(m.index)
                self.results_received += 1
                if self.reassembly == "display":
                    self._display.receive(m.index, data, res.pid, m.start, m.end)
                else:
                    self._ordered.push(m.index, data, {"process_id": res.pid, "start_time": m.start,
                                                       "end_time": m.end, "shape": m.shape, "slot": m.slot})
                    self._released.extend(self._ordered.pop_ready())
                self._cv.notify_all()

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
                self._cv.wait(rem if rem is not None else 0.1)
            return self._released.popleft()

    def release_frame(self, index: int) -> None:
        """zero_copy: return frame ``index``'s ring slot once its result view is consumed."""
        with self._cv:
            self._free_slot(index)

    def num_workers(self) -> int:
        with self._lock:
            return len(self._peers)

    def ordering_stats(self) -> dict:
        with self._lock:
            s = self._ordered.stats()
            s.update({"frames_dropped": self.frames_dropped, "results_received": self.results_received,
                      "result_errors": self.result_errors,
                      "workers": {p.pid.hex(): {"sent": p.frames_sent, "shard": p.shard}
                                  for p in self._peers.values()}})
            return s
