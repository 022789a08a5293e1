"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

Restates, on the CPU, what the reference (kylemcdonald/distributed-video-filter) computes
on the hot path, so tests can check the MI355X product path against it.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this module, and
only as the checker / the timed CPU baseline; the product (``vfilter`` + libvfilter_hip.so)
never imports it and has no CPU fallback.

Contents, each citing the reference lines it restates:
  * the filter: ``cv2.bitwise_not`` (inverter.py:41) = per-byte ``~x`` (numpy and plain C);
  * the raw framing of ``InverterWorker.__call__`` with ``use_jpeg=False`` (inverter.py:29-46);
  * the distributor's ingest queue (distributor.py:173-203), its latest-wins dispatch slot
    (distributor.py:205-251) and its reorder/display policy (distributor.py:253-344).
Pinning: tests/golden/ (KATs, seeded-frame digests, and traces of the real reference
distributor.py/worker.py captured under the survey container's pyzmq; see
tests/golden/capture_reference.py and DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes
import os
import queue
from typing import Dict, List, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(_HERE, "_build", "libvf_oracle.so")

# ---------------------------------------------------------------------------------------
# The filter (inverter.py:41): OpenCV bitwise_not on a CV_8UC3 Mat = per-byte NOT.
# ---------------------------------------------------------------------------------------


def invert(frame: np.ndarray) -> np.ndarray:
    """``cv2.bitwise_not(frame)``: a NEW array with every byte inverted (inverter.py:41)."""
    return np.bitwise_not(frame)


def invert_bytes(frame_bytes) -> bytes:
    return np.bitwise_not(np.frombuffer(frame_bytes, dtype=np.uint8)).tobytes()


_clib = None


def c_library() -> ctypes.CDLL:
    """The plain-C restatement (oracle/vf_oracle.c), built by ``make -C oracle``."""
    global _clib
    if _clib is None:
        if not os.path.exists(ORACLE_LIB):
            raise FileNotFoundError(f"{ORACLE_LIB} missing: run `make -C oracle`")
        lib = ctypes.CDLL(ORACLE_LIB)
        lib.vfo_invert.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.vfo_invert.restype = None
        lib.vfo_fnv1a64.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.vfo_fnv1a64.restype = ctypes.c_uint64
        _clib = lib
    return _clib


def c_invert(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src)
    out = np.empty_like(src)
    c_library().vfo_invert(src.ctypes.data, out.ctypes.data, src.nbytes)
    return out


def fnv1a64(a) -> int:
    a = np.ascontiguousarray(np.frombuffer(a, dtype=np.uint8) if not isinstance(a, np.ndarray) else a)
    return int(c_library().vfo_fnv1a64(a.ctypes.data, a.nbytes))


# ---------------------------------------------------------------------------------------
# Synthetic frames: uniform uint8 from a seeded default_rng.
# ---------------------------------------------------------------------------------------

SIZES = {
    "480sq": (480, 480),     # the reference raw path's hard-coded shape (inverter.py:34)
    "480p": (480, 640),
    "1080p": (1080, 1920),
    "4k": (2160, 3840),
}


def synthetic_frame(seed: int, h: int, w: int) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


# ---------------------------------------------------------------------------------------
# InverterWorker.__call__ raw path (inverter.py:29-46 with use_jpeg=False)
# ---------------------------------------------------------------------------------------

REF_RAW_SHAPE = (480, 480, 3)  # inverter.py:34 hard-codes this


def reference_raw_call(frame_bytes) -> bytes:
    """inverter.py:34 -> :41 -> :46.  Raises ValueError for any size but 480x480x3, as the
    reference's reshape does (the frame is then dropped by worker.py:74-76)."""
    frame = np.frombuffer(frame_bytes, dtype=np.uint8).reshape(*REF_RAW_SHAPE)
    return invert(frame).tobytes()


# ---------------------------------------------------------------------------------------
# Distributor policy (distributor.py).  Pure state machines, no sockets, no threads.
# ---------------------------------------------------------------------------------------


class RefIngestQueue:
    """``add_frame_for_distribution`` (distributor.py:173-203): global frame_index counter
    (:179-180), ``queue.Queue(maxsize=10)`` (:11), drop-oldest-and-retry-once when full
    (:193-203)."""

    def __init__(self, maxsize: int = 10):
        self.q: "queue.Queue[dict]" = queue.Queue(maxsize=maxsize)
        self.frame_index_counter = 0

    def add(self, frame, timestamp: float = 0.0) -> int:
        idx = self.frame_index_counter
        self.frame_index_counter += 1
        item = {"frame": frame, "frame_index": idx, "timestamp": timestamp}
        try:
            self.q.put_nowait(item)
        except queue.Full:
            try:
                self.q.get_nowait()
                self.q.put_nowait(item)
            except queue.Full:  # pragma: no cover - unreachable single-threaded
                pass
        return idx

    def get_nowait(self) -> Optional[dict]:
        try:
            return self.q.get_nowait()
        except queue.Empty:
            return None


class RefDispatchSlot:
    """The dispatch loop's frame selection (distributor.py:209-241) as a state machine: each
    loop iteration moves at most ONE queued frame into the single ``current_frame_data``
    slot (latest wins, :211-217); a READY is answered only if the slot's index is greater
    than ``last_frame_sent`` (:231-241), so every frame goes out at most once, in
    increasing index order, and frames overwritten in the slot are skipped."""

    def __init__(self):
        self.current: Optional[dict] = None
        self.last_frame_sent = -1

    def pull(self, item: Optional[dict]) -> None:
        if item is not None:
            self.current = {"frame": item["frame"], "frame_index": item["frame_index"]}

    def on_ready(self) -> Optional[dict]:
        cur = self.current
        if cur is not None and cur.get("frame_index") is not None and cur["frame_index"] > self.last_frame_sent:
            self.last_frame_sent = cur["frame_index"]
            return cur
        return None


class RefReorderBuffer:
    """Collect + reorder + display selection (distributor.py:253-344)."""

    def __init__(self, frame_delay: int = 5, frame_buffer_size: int = 50):
        self.received_frames: Dict[int, dict] = {}
        self.current_display_frame = 0          # :21
        self.latest_received_frame = -1         # :22
        self.frame_buffer_size = frame_buffer_size  # :23
        self.frame_delay = frame_delay          # :24

    def receive(self, frame_index: int, frame_data, process_id: str = "0",
                start_time: float = 0.0, end_time: float = 0.0) -> None:
        """check_inverter_output body (distributor.py:270-282)."""
        self.received_frames[frame_index] = {
            "frame_data": frame_data,
            "process_id": process_id,
            "start_time": float(start_time),
            "end_time": float(end_time),
        }
        self.latest_received_frame = max(self.latest_received_frame, frame_index)
        self.cleanup_old_frames()

    def cleanup_old_frames(self) -> None:
        """distributor.py:291-307: drop indices below the display index, then cap at the
        ``frame_buffer_size`` newest."""
        for idx in [i for i in self.received_frames if i < self.current_display_frame]:
            del self.received_frames[idx]
        if len(self.received_frames) > self.frame_buffer_size:
            keys = sorted(self.received_frames)
            for idx in keys[: len(keys) - self.frame_buffer_size]:
                del self.received_frames[idx]

    def get_frame_to_display(self):
        """distributor.py:309-322: the exact frame, else the nearest index (ties -> lower)."""
        target = self.current_display_frame
        if target in self.received_frames:
            return self.received_frames[target]["frame_data"]
        if self.received_frames:
            closest = min(sorted(self.received_frames), key=lambda x: abs(x - target))
            return self.received_frames[closest]["frame_data"]
        return None

    def update_display_frame(self) -> bool:
        """distributor.py:324-344."""
        if self.latest_received_frame >= self.frame_delay:
            self.current_display_frame = self.latest_received_frame - self.frame_delay
            return True
        if self.latest_received_frame > 0:
            if self.current_display_frame < self.latest_received_frame:
                self.current_display_frame = self.latest_received_frame
                return True
        return False

    def snapshot(self) -> dict:
        return {
            "keys": sorted(self.received_frames),
            "current_display_frame": self.current_display_frame,
            "latest_received_frame": self.latest_received_frame,
        }


def replay_display_ops(ops: List[list], frame_delay: int, frame_buffer_size: int = 50) -> List[dict]:
    """Run a captured op sequence through the restatement; returns one record per op in
    the same schema as tests/golden/ref_display_*.json."""
    rb = RefReorderBuffer(frame_delay, frame_buffer_size)
    out = []
    for op in ops:
        rec: dict = {"op": op}
        if op[0] == "recv":
            idx = op[1]
            rb.receive(idx, payload_for(idx))
        elif op[0] == "update":
            rec["ret"] = rb.update_display_frame()
        elif op[0] == "get":
            fd = rb.get_frame_to_display()
            rec["ret"] = None if fd is None else payload_index(fd)
        rec.update(rb.snapshot())
        out.append(rec)
    return out


def payload_for(idx: int) -> bytes:
    """Payload the capture script attaches to result ``idx`` (identifies the frame)."""
    return b"F" + int(idx).to_bytes(4, "little")


def payload_index(payload: bytes) -> int:
    return int.from_bytes(bytes(payload)[1:5], "little")
