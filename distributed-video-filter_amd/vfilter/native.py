"""The distributor's native control plane: ctypes binding to ``libvfdist.so`` (include/vfdist.h)
and ``NativeDistributor``, the ``Distributor`` API over it.

The reference distributes from two Python threads, one READY and one result per 10 ms poll
(distributor.py:205-289).  This build's Python engine (``vfilter.distributor``) batches that and
books each result message in one pass, and tops out near 100 k frames/s of JPEG-size frames at 8
workers -- about 2.5 GPUs' worth of the JPEG worker form.  The native engine runs
the whole loop in C++ on one I/O thread: workers' requests are answered, dispatches built and
sent, results booked and released in index order without Python or the GIL; Python touches
only its own calls (reserve / commit / next / release, a batch per call).

``Distributor(...)`` returns a ``NativeDistributor`` when ``engine="native"``, or with
``engine="auto"`` (the default) for the lossless ring deployment it implements: policy "pull" or
"shard", ``reassembly="ordered"``, the "tcp" transport, ``ring_slots > 0`` with per-worker slices,
no trace export.  Everything else (the reference's latest-wins policy and display reassembly,
ZeroMQ, frames as socket payloads, Perfetto export) stays on the Python engine.  The library is
host code (g++, no HIP): if it is missing, the native engine refuses loudly.
"""
from __future__ import annotations

import ctypes
import json
import os
import threading
import time
from typing import List, Optional, Sequence

import numpy as np

from .distributor import Distributor
from .shm import copy_into

LIB_NAME = "libvfdist.so"
ABI_VERSION = 1

VFD_OK = 0
VFD_E_INVALID = -1
VFD_E_SYS = -2
VFD_E_NOMEM = -3
VFD_E_STOPPED = -4
POLICY = {"pull": 1, "shard": 2}

C_NAMES = ("released", "lost", "buffered", "max_depth", "out_of_order", "next_index", "results_received",
           "result_errors", "frames_lost", "frames_requeued", "duplicates", "evictions", "departures",
           "quarantine_expired", "frame_index_counter", "workers", "free_slots", "total_slots", "dispatches",
           "result_messages")


class _Config(ctypes.Structure):
    _fields_ = [("policy", ctypes.c_int), ("shard_workers", ctypes.c_int), ("shard_chunk", ctypes.c_int),
                ("queue_size", ctypes.c_int), ("ring_slots", ctypes.c_int), ("ring_slot_bytes", ctypes.c_int64),
                ("batch_timeout", ctypes.c_double), ("batch_wait", ctypes.c_double),
                ("max_attempts", ctypes.c_int), ("verbose", ctypes.c_int), ("distribute_port", ctypes.c_int),
                ("collect_port", ctypes.c_int), ("host", ctypes.c_char_p), ("max_part", ctypes.c_int64),
                ("copy_results", ctypes.c_int), ("no_unix", ctypes.c_int)]


# vfd_frame, as a numpy record (72 bytes, the C struct's natural layout)
FRAME = np.dtype([("index", "<i8"), ("nbytes", "<i8"), ("data", "<u8"), ("slot", "<i4"), ("ndim", "<i4"),
                  ("shape", "<i4", (4,)), ("pid", "<i8"), ("start", "<f8"), ("end", "<f8")])
assert FRAME.itemsize == 72

_vp = ctypes.c_void_p
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_ip = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes); must list every entry point of include/vfdist.h
SIGNATURES = {
    "vfd_abi_version": (ctypes.c_int, []),
    "vfd_create": (ctypes.c_int, [ctypes.POINTER(_Config), ctypes.POINTER(_vp)]),
    "vfd_ports": (ctypes.c_int, [_vp, _ip, _ip]),
    "vfd_start": (ctypes.c_int, [_vp]),
    "vfd_stop": (ctypes.c_int, [_vp]),
    "vfd_destroy": (ctypes.c_int, [_vp]),
    "vfd_last_error": (ctypes.c_char_p, [_vp]),
    "vfd_reserve": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int, ctypes.c_double, _vp, _vp]),
    "vfd_commit": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    "vfd_fill": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp]),
    "vfd_cancel": (ctypes.c_int, [_vp, ctypes.c_int32]),
    "vfd_reserved_index": (ctypes.c_int, [_vp, ctypes.c_int32, _i64p]),
    "vfd_next": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double, _vp]),
    "vfd_release": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "vfd_slot_addr": (ctypes.c_int, [_vp, ctypes.c_int32, _u64p, _u64p]),
    "vfd_slice": (ctypes.c_int, [_vp, ctypes.c_int, _u64p, _i64p, ctypes.c_char_p, ctypes.c_int, _ip, _ip]),
    "vfd_counters": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    "vfd_stats_json": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int64]),
}


class NativeError(RuntimeError):
    def __init__(self, message: str, status: int = VFD_E_INVALID):
        super().__init__(message)
        self.status = status


_lib = None
_lib_lock = threading.Lock()


def library_path() -> str:
    return os.environ.get("VFDIST_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)


def load_library() -> ctypes.CDLL:
    """Load libvfdist.so once.  Raises if it is absent (build it with ``make``)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if not os.path.exists(path):
            raise NativeError(f"{LIB_NAME} not found at {path}; build it with `make lib` (g++, host code)")
        lib = ctypes.CDLL(path)
        for name, (restype, argtypes) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = restype
            fn.argtypes = argtypes
        if lib.vfd_abi_version() != ABI_VERSION:
            raise NativeError(f"{LIB_NAME} ABI {lib.vfd_abi_version()} != {ABI_VERSION}: rebuild it")
        _lib = lib
        return lib


def available() -> bool:
    try:
        load_library()
        return True
    except (NativeError, OSError):
        return False


def supports(policy: str, reassembly: str, transport: str, ring_slots: int, ring_layout: str,
             enable_trace_export: bool) -> Optional[str]:
    """None when the native engine implements this configuration, else why not."""
    if policy not in POLICY:
        return f"policy {policy!r} (the native engine is lossless: pull | shard)"
    if reassembly != "ordered":
        return f"reassembly {reassembly!r} (native: ordered)"
    if transport != "tcp":
        return f"transport {transport!r} (native: tcp)"
    if ring_slots <= 0:
        return "no shared-memory ring (native: frames travel in per-worker ring slices)"
    if ring_layout not in ("auto", "per_worker"):
        return f"ring_layout {ring_layout!r} (native: per_worker)"
    if enable_trace_export:
        return "trace export (the Python engine records Perfetto events)"
    return None


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_vp)


class _Scratch(threading.local):
    """Per-thread argument buffers whose addresses are taken once: ``ndarray.ctypes`` costs
    2.5-5.5 us per access, which at a few calls per 32-frame batch was most of the Python side's
    cost per frame (tools/distributor_overhead.py --profile)."""

    def __init__(self):
        self.cap = 0
        self._grow(256)

    def _grow(self, n: int) -> None:
        cap = max(n, 2 * self.cap)
        self.slots = np.empty(cap, np.int32)
        self.idx = np.empty(cap, np.int64)
        self.nbytes = np.empty(cap, np.int64)
        self.addr = np.empty(cap, np.uint64)
        self.ndim = np.empty(cap, np.int32)
        self.shape = np.empty((cap, 4), np.int32)
        self.rec = np.empty(cap, FRAME)
        self.p_slots, self.p_idx, self.p_nbytes = self.slots.ctypes.data, self.idx.ctypes.data, self.nbytes.ctypes.data
        self.p_ndim, self.p_shape, self.p_rec = self.ndim.ctypes.data, self.shape.ctypes.data, self.rec.ctypes.data
        self.p_addr = self.addr.ctypes.data
        self.cap = cap

    def need(self, n: int) -> "_Scratch":
        if n > self.cap:
            self._grow(n)
        return self


class ReleasedBatch:
    """Results released in index order by one call (``get_next_batch``): columns, not tuples --
    a consumer of 300 k frames/s cannot afford a Python object per frame.  ``view(i)`` is frame
    i's result bytes (valid until ``release_frames``), ``info(i)`` the reference-style dict."""

    def __init__(self, owner, rec: np.ndarray):
        self._owner = owner
        self.rec = rec
        self.index = rec["index"]
        self.nbytes = rec["nbytes"]
        self.slot = rec["slot"]

    def __len__(self) -> int:
        return len(self.rec)

    def view(self, i: int) -> np.ndarray:
        return self._owner._view_of(self.rec[i])

    def info(self, i: int) -> dict:
        return self._owner._info_of(self.rec[i])

    def items(self) -> list:
        return [(int(r["index"]), self._owner._view_of(r), self._owner._info_of(r)) for r in self.rec]


class NativeDistributor(Distributor):
    """``Distributor`` (vfilter/distributor.py, reference distributor.py:8-376) over libvfdist.so.
    Same constructor, same methods; see the module docstring for the configurations it serves."""

    engine = "native"

    def __init__(self, distribute_port: int = 5555, collect_port: int = 5556, frame_delay: int = 5,
                 enable_trace_export: bool = False, *, policy: str = "pull", reassembly: str = "ordered",
                 transport: str = "tcp", host: str = "*", queue_size: int = 10, frame_buffer_size: int = 50,
                 ring_slots: int = 0, ring_slot_bytes: int = 0, ring_layout: str = "auto", shard_workers: int = 0,
                 shard_chunk: int = 1, batch_timeout: float = 30.0, max_attempts: int = 3, batch_wait: float = 0.002,
                 trace_file: str = "webcam_frame_timing.pftrace", verbose: bool = True, zero_copy: bool = False,
                 engine: str = "native"):
        why = supports(policy, reassembly, transport, ring_slots, ring_layout, enable_trace_export)
        if why is not None:
            raise ValueError(f"engine='native' does not serve {why}; use engine='python'")
        if policy == "shard" and shard_workers < 1:
            raise ValueError("policy='shard' needs shard_workers >= 1")
        if ring_slot_bytes < 1:
            raise ValueError("ring_slots needs ring_slot_bytes (largest frame)")
        self._L = load_library()
        self.policy, self.reassembly, self.transport = policy, reassembly, "tcp"
        self.ring_layout = "per_worker"
        self.ring_slots = int(ring_slots)
        self.ring_slot_bytes = int(ring_slot_bytes)
        self.slot_bytes = (int(ring_slot_bytes) + 4095) // 4096 * 4096  # FrameRing's rounding
        self.zero_copy = zero_copy
        self.verbose = verbose
        self.queue_size = queue_size
        self.shard_workers = shard_workers
        self.shard_chunk = max(1, shard_chunk)
        self.batch_timeout, self.batch_wait, self.max_attempts = float(batch_timeout), float(batch_wait), max_attempts
        self.enable_trace_export = False
        self.frame_timings: List[dict] = []
        self.trace_start_time = time.time()
        self.trace_file = trace_file
        self._frame_delay, self._frame_buffer_size = frame_delay, frame_buffer_size
        self.running = False
        cfg = _Config(policy=POLICY[policy], shard_workers=max(1, shard_workers), shard_chunk=self.shard_chunk,
                      queue_size=max(1, queue_size), ring_slots=self.ring_slots, ring_slot_bytes=self.ring_slot_bytes,
                      batch_timeout=self.batch_timeout, batch_wait=max(0.0, self.batch_wait),
                      max_attempts=max(1, int(max_attempts)), verbose=1 if verbose else 0,
                      distribute_port=distribute_port, collect_port=collect_port,
                      host=("*" if host in ("*", "", None) else host).encode(),
                      max_part=max(64 << 20, 4 * self.slot_bytes + (1 << 20)), copy_results=0 if zero_copy else 1)
        e = _vp()
        rc = self._L.vfd_create(ctypes.byref(cfg), ctypes.byref(e))
        if rc != VFD_OK:
            raise NativeError(f"vfd_create failed ({rc}): see stderr", rc)
        self._e = e
        dp, cp = ctypes.c_int(), ctypes.c_int()
        self._L.vfd_ports(e, ctypes.byref(dp), ctypes.byref(cp))
        self.distribute_port, self.collect_port = dp.value, cp.value
        self._slices: dict = {}
        self._slices_lock = threading.Lock()
        self._scratch = _Scratch()
        self._closed = False
        self.current_frame_data = None
        self.last_frame_sent = -1

    # ---- errors ---------------------------------------------------------------------------
    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            if rc == VFD_E_STOPPED:
                return rc
            raise NativeError(f"{what}: {self._L.vfd_last_error(self._e).decode(errors='replace')} ({rc})", rc)
        return rc

    # ---- counters as the Python engine's attributes --------------------------------------------
    def _counters(self) -> dict:
        if self._closed:
            return dict(self._final)
        out = np.zeros(len(C_NAMES), np.int64)
        self._L.vfd_counters(self._e, _ptr(out), len(C_NAMES))
        return dict(zip(C_NAMES, out.tolist()))

    def _counter(name):  # noqa: N805 -- a property factory
        return property(lambda self: self._counters()[name])

    results_received = _counter("results_received")
    result_errors = _counter("result_errors")
    frames_lost = _counter("frames_lost")
    frames_requeued = _counter("frames_requeued")
    duplicates = _counter("duplicates")
    evictions = _counter("evictions")
    departures = _counter("departures")
    quarantine_expired = _counter("quarantine_expired")
    frame_index_counter = _counter("frame_index_counter")
    frames_dropped = property(lambda self: 0)
    quarantine_forced = property(lambda self: 0)
    del _counter

    @property
    def received_frames(self) -> dict:
        return {}

    @property
    def current_display_frame(self) -> int:
        return 0

    @property
    def latest_received_frame(self) -> int:
        return self._counters()["next_index"] - 1

    @property
    def frame_delay(self) -> int:
        return self._frame_delay

    @property
    def frame_buffer_size(self) -> int:
        return self._frame_buffer_size

    # ---- lifecycle ------------------------------------------------------------------------
    def start(self):
        self._check(self._L.vfd_start(self._e), "vfd_start")
        self.running = True

    def stop(self):
        self.running = False
        if not self._closed:
            self._L.vfd_stop(self._e)

    def cleanup(self):
        if self._closed:
            return
        st = self._counters()
        self._final_stats = self.ordering_stats()
        self.stop()
        self._final = st
        self._closed = True
        with self._slices_lock:
            self._slices.clear()
        self._L.vfd_destroy(self._e)
        if self.verbose:
            print("Connections closed")
            print("Frame reordering statistics:")
            print(f"  Next frame index: {st['next_index']}")
            print(f"  Frames released: {st['released']}, lost: {st['lost']}")

    def handle_distribute_requests(self):
        """The reference's dispatch thread body: the native I/O thread does this work."""

    def check_inverter_output(self):
        """The reference's collect thread body: the native I/O thread does this work."""

    # ---- ring views -----------------------------------------------------------------------
    def _slice_arr(self, sid: int) -> np.ndarray:
        a = self._slices.get(sid)
        if a is not None:
            return a
        with self._slices_lock:
            a = self._slices.get(sid)
            if a is None:
                base, nb = ctypes.c_uint64(), ctypes.c_int64()
                rc = self._L.vfd_slice(self._e, sid, ctypes.byref(base), ctypes.byref(nb), None, 0, None, None)
                self._check(rc, f"slice {sid}")
                a = np.ctypeslib.as_array((ctypes.c_uint8 * nb.value).from_address(base.value))
                self._slices[sid] = a
        return a

    def in_view(self, slot: int, nbytes: int) -> np.ndarray:
        sid, k = divmod(int(slot), self.ring_slots)
        o = k * 2 * self.slot_bytes
        return self._slice_arr(sid)[o:o + nbytes]

    def out_view(self, slot: int, nbytes: int) -> np.ndarray:
        sid, k = divmod(int(slot), self.ring_slots)
        o = k * 2 * self.slot_bytes + self.slot_bytes
        return self._slice_arr(sid)[o:o + nbytes]

    frame_view = in_view

    def free_slots(self) -> int:
        return self._counters()["free_slots"]

    def total_slots(self) -> int:
        return self._counters()["total_slots"]

    def num_workers(self) -> int:
        return self._counters()["workers"]

    # ---- ingest -----------------------------------------------------------------------------
    def _reserve(self, nbytes: int, n: int, block: bool):
        sc = self._scratch.need(n)
        while True:
            rc = self._L.vfd_reserve(self._e, int(nbytes), int(n), 0.1 if block else 0.0, sc.p_slots, sc.p_idx)
            if rc == VFD_E_STOPPED:
                rc = 0
            if rc < 0:
                msg = self._L.vfd_last_error(self._e).decode(errors="replace")
                raise ValueError(msg) if "exceeds" in msg else NativeError(f"vfd_reserve: {msg} ({rc})", rc)
            if rc > 0 or not block or not self.running:
                return sc.slots[:rc].copy(), sc.idx[:rc].copy()

    def reserve_frame(self, nbytes: int, block: bool = True) -> Optional[int]:
        slots, _ = self._reserve(nbytes, 1, block)
        return int(slots[0]) if len(slots) else None

    def reserve_frames(self, nbytes: int, n: int, block: bool = True) -> List[int]:
        slots, _ = self._reserve(nbytes, n, block)
        return slots.tolist()

    def reserve_frames_array(self, nbytes: int, n: int, block: bool = True):
        """``reserve_frames`` as arrays: (slots int32, indices int64)."""
        return self._reserve(nbytes, n, block)

    def reserved_index(self, slot: int) -> Optional[int]:
        v = ctypes.c_int64()
        rc = self._L.vfd_reserved_index(self._e, int(slot), ctypes.byref(v))
        return v.value if rc == VFD_OK else None

    def commit_frames(self, slots: Sequence[int], nbytes: Sequence[int], shapes=None, timestamp=None) -> List[int]:
        n = len(slots)
        if len(nbytes) != n:
            raise ValueError("commit_frames: slots and nbytes differ in length")
        sc = self._scratch.need(n)
        sc.slots[:n] = slots
        sc.nbytes[:n] = nbytes
        p_nd = p_sh = None
        if shapes is not None:
            sc.ndim[:n] = -1
            for i, x in enumerate(shapes):
                if x is not None:
                    k = len(x)
                    if k > 4:
                        raise ValueError(f"shape {x} has more than 4 dimensions")
                    sc.ndim[i] = k
                    sc.shape[i, :k] = x
            p_nd, p_sh = sc.p_ndim, sc.p_shape
        rc = self._L.vfd_commit(self._e, n, sc.p_slots, sc.p_nbytes, p_nd, p_sh, sc.p_idx)
        self._check(rc, "vfd_commit")
        return sc.idx[:n].tolist()

    def fill_frames(self, slots, src_addrs, nbytes) -> None:
        """Copy n frames into their reserved slots in one call (vfd_fill): ``src_addrs`` are the
        frames' addresses (uint64), ``nbytes`` their sizes.  The columnar form of the copy in
        distributor.py:173-203 for producers of small frames at high rates; then commit_frames."""
        n = len(slots)
        if len(src_addrs) != n or len(nbytes) != n:
            raise ValueError("fill_frames: slots, src_addrs and nbytes differ in length")
        sc = self._scratch.need(n)
        sc.slots[:n] = slots
        sc.addr[:n] = src_addrs
        sc.nbytes[:n] = nbytes
        self._check(self._L.vfd_fill(self._e, n, sc.p_slots, sc.p_addr, sc.p_nbytes), "vfd_fill")

    def commit_frame(self, slot: int, nbytes: int, shape=None, timestamp=None, block: bool = True) -> int:
        return self.commit_frames([slot], [nbytes], None if shape is None else [list(shape)])[0]

    def cancel_frame(self, slot: int) -> None:
        self._check(self._L.vfd_cancel(self._e, int(slot)), "vfd_cancel")

    def add_frame_for_distribution(self, frame, timestamp=None, shape=None, block: bool = True) -> int:
        """distributor.py:173-203, lossless: reserve a slot of the target worker, copy the frame
        in, commit.  Returns its index, or -1 when ``block`` is False and no slot is free."""
        if isinstance(frame, np.ndarray):
            shape = list(frame.shape) if shape is None else shape
            frame = np.ascontiguousarray(frame)
        nbytes = frame.nbytes if isinstance(frame, np.ndarray) else len(frame)
        slot = self.reserve_frame(nbytes, block)
        if slot is None:
            return -1
        copy_into(self.in_view(slot, nbytes), frame)
        return self.commit_frame(slot, nbytes, shape)

    # ---- in-order release ---------------------------------------------------------------------
    def _view_of(self, r) -> np.ndarray:
        n, slot, addr = int(r["nbytes"]), int(r["slot"]), int(r["data"])
        if slot >= 0:
            a = self._slice_arr(slot // self.ring_slots)
            o = addr - a.ctypes.data
            if 0 <= o and o + n <= a.nbytes:
                return a[o:o + n]
        if n == 0:
            return np.empty(0, np.uint8)
        return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(addr))

    def _info_of(self, r) -> dict:
        nd = int(r["ndim"])
        return {"process_id": str(int(r["pid"])), "start_time": float(r["start"]), "end_time": float(r["end"]),
                "shape": None if nd < 0 else [int(x) for x in r["shape"][:nd]],
                "slot": int(r["slot"]) if (self.zero_copy and int(r["slot"]) >= 0) else None}

    def _next(self, max_n: int, timeout: Optional[float]) -> np.ndarray:
        sc = self._scratch.need(max_n)
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            rem = 0.1 if deadline is None else max(0.0, min(0.1, deadline - time.monotonic()))
            k = self._L.vfd_next(self._e, int(max_n), rem, sc.p_rec)
            if k > 0:
                return sc.rec[:k].copy()
            if k < 0 or not self.running or (deadline is not None and time.monotonic() >= deadline):
                return sc.rec[:0].copy()

    def get_next_batch(self, max_n: int, timeout: Optional[float] = None) -> ReleasedBatch:
        """Up to ``max_n`` next results in index order, as columns (``ReleasedBatch``); empty on
        timeout.  Zero-copy: each stays valid until ``release_frames``."""
        rec = self._next(max_n, timeout)
        if not self.zero_copy and len(rec):
            raise RuntimeError("get_next_batch needs zero_copy=True (results are views into ring slots)")
        return ReleasedBatch(self, rec)

    def get_next_frames(self, max_n: int, timeout: Optional[float] = None) -> list:
        rec = self._next(max_n, timeout)
        out = []
        for r in rec:
            v = self._view_of(r)
            out.append((int(r["index"]), v if self.zero_copy else bytes(v), self._info_of(r)))
        if not self.zero_copy and len(rec):  # copied out: the slots go back at once
            self.release_frames(rec["index"])
        return out

    def get_next_frame(self, timeout: Optional[float] = None):
        got = self.get_next_frames(1, timeout)
        return got[0] if got else None

    def release_frames(self, indices) -> None:
        n = len(indices)
        if n:
            sc = self._scratch.need(n)
            sc.idx[:n] = indices
            self._L.vfd_release(self._e, n, sc.p_idx)

    def release_frame(self, index: int) -> None:
        self.release_frames([index])

    # ---- stats and the reference's display API ----------------------------------------------
    def ordering_stats(self) -> dict:
        if self._closed:
            return dict(self._final_stats)
        buf = ctypes.create_string_buffer(1 << 16)
        n = self._L.vfd_stats_json(self._e, buf, len(buf))
        if n >= len(buf):
            buf = ctypes.create_string_buffer(n + 1)
            self._L.vfd_stats_json(self._e, buf, len(buf))
        s = json.loads(buf.value)
        s["engine"] = "native"
        return s

    def get_frame_stats(self):
        c = self._counters()
        return {"buffer_size": c["buffered"], "current_display_frame": 0, "latest_received_frame": c["next_index"] - 1,
                "frame_delay": self._frame_delay, "total_frames_processed": c["frame_index_counter"]}

    def cleanup_old_frames(self):
        """Display policy (distributor.py:291-307): not used with ordered reassembly."""

    def get_frame_to_display(self):
        return None

    def update_display_frame(self):
        return False

    def export_perfetto_trace(self):
        print("Trace export is disabled")
