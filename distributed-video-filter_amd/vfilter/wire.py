"""Wire format between the distributor and its workers.

v0 — the reference's own messages, byte for byte:
  request  (worker -> distributor, DEALER -> ROUTER)  ["READY"]                       worker.py:39
  dispatch (distributor -> worker, ROUTER -> DEALER)   [index:str, frame:bytes]        distributor.py:236-238
  result   (worker -> distributor, PUSH -> PULL)       [index:str, pid:str, start:str(float),
                                                        end:str(float), frame:bytes]   worker.py:63-67
  v0 has no shape: a raw frame is its bytes (the reference reshapes to 480x480x3,
  inverter.py:34; the invert itself needs no shape).

v1 — shape-carrying and batched.  Every v1 message starts with a
tag part that can never be a decimal index string, so a v1 peer can always tell v0 from v1:
  request  ["READY1", json{"credit": k, "shm": bool, "wid": worker id, "numa": node of its GPU,
                          "wire": 2 (the worker also reads v2 messages)}]
  dispatch ["FRAMES1", json{"frames": [{"index", "nbytes", "shape", "slot"}, ...],
                             "ring": {"name": shm name, "slot_bytes": n} (if any slot)},
            frame_0, ..., frame_{k-1}]
           (frames whose slot is set travel in the shared-memory ring and have no part)
  result   ["RESULT1", json{"pid": p, "wid": worker id, "frames": [{..., "start", "end", "error"}],
                            "spans": [{"name", "begin", "end", "bytes"}...] (GPU timeline)},
            out_0, ...]
  This per-frame form is what every earlier build of either side reads.  Decoders also accept
  round 4's columnar v1 form ({"index": [...], "nbytes": [...], ...} under the same tags).
  "wid" ties a result to the request stream it answers (the distributor tracks every dispatched
  frame per worker, re-queues a lost worker's frames and frees their ring slots); "numa" lets
  the distributor place the worker's ring slice on its GPU's NUMA node.  A result's "nbytes" is
  the RESULT's length (a JPEG differs from its input's).

v2 — binary columns, negotiated: a distributor sends v2 only to a worker whose request says
"wire": 2, and a worker answers v2 only to a v2 dispatch, so mixed builds keep talking v1.
  dispatch ["FRAMES2", json{"ring": {...}} (or {}), columns, frame parts of unslotted frames]
  result   ["RESULT2", json{"pid", "wid", "start", "end" (or "starts", "ends": [...]),
                            "errors": {"position": message}, "spans": [...]}, columns, parts]
  columns = one little-endian 40-byte record per frame (``COLS``): index i64, nbytes i64,
  slot i32 (-1: no slot), ndim i32 (-1: no shape), shape i32[4].  The metadata of a batch is
  what the distributor handles per message; fixed records cost the native control plane
  (csrc/vf_dist.cc) no parsing and the Python side one ``np.frombuffer``.
A worker run with protocol v0 against the reference distributor sends "READY" and reads 2
parts; this build's distributor answers a bare "READY" with a v0 dispatch.  Either side of the reference can
therefore be swapped for this build's independently.
"""
from __future__ import annotations

import json
from collections.abc import Sequence as _Seq
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

READY_V0 = b"READY"
READY_V1 = b"READY1"
FRAMES_V1 = b"FRAMES1"
RESULT_V1 = b"RESULT1"
FRAMES_V2 = b"FRAMES2"
RESULT_V2 = b"RESULT2"
WIRE = 2  # the newest message form this build reads

# v2 per-frame record (csrc/vf_dist.cc kColsRecord mirrors it)
COLS = np.dtype([("index", "<i8"), ("nbytes", "<i8"), ("slot", "<i4"), ("ndim", "<i4"), ("shape", "<i4", (4,))])
assert COLS.itemsize == 40


class FrameMeta:
    """One frame's metadata on the wire.  A slotted class (the control plane builds one per frame
    per message; ``dataclass(slots=True)`` needs Python 3.10, and the reference interop runs
    this module under the conda 3.9 that has pyzmq)."""
    __slots__ = ("index", "nbytes", "shape", "slot", "start", "end", "error")

    def __init__(self, index: int, nbytes: int, shape: Optional[List[int]] = None, slot: Optional[int] = None,
                 start: float = 0.0, end: float = 0.0, error: Optional[str] = None):
        self.index, self.nbytes, self.shape, self.slot = index, nbytes, shape, slot
        self.start, self.end, self.error = start, end, error

    def __eq__(self, other) -> bool:
        return isinstance(other, FrameMeta) and all(getattr(self, k) == getattr(other, k) for k in self.__slots__)

    def __repr__(self) -> str:
        return "FrameMeta(" + ", ".join(f"{k}={getattr(self, k)!r}" for k in self.__slots__) + ")"

    def to_json(self) -> dict:
        d = {"index": self.index, "nbytes": self.nbytes, "shape": self.shape, "slot": self.slot}
        if self.start or self.end:
            d["start"], d["end"] = self.start, self.end
        if self.error:
            d["error"] = self.error
        return d

    @classmethod
    def from_json(cls, d: dict) -> "FrameMeta":
        return cls(index=int(d["index"]), nbytes=int(d["nbytes"]), shape=d.get("shape"),
                   slot=d.get("slot"), start=float(d.get("start", 0.0)), end=float(d.get("end", 0.0)),
                   error=d.get("error"))


@dataclass
class Request:
    version: int
    credit: int = 1
    shm: bool = False
    wid: Optional[str] = None
    numa: Optional[int] = None
    wire: int = 1  # newest dispatch form the worker reads (v1 requests only)


@dataclass
class Dispatch:
    metas: Sequence[FrameMeta]
    payloads: List[Optional[bytes]] = field(default_factory=list)  # None where slot is set
    version: int = 1
    ring: Optional[dict] = None  # {"name": shm name, "slot_bytes": n} when any slot is set
    cols: Optional[np.ndarray] = None  # v2: the COLS records as received


@dataclass
class Result:
    pid: str
    metas: List[FrameMeta]
    payloads: List[Optional[bytes]] = field(default_factory=list)
    version: int = 1
    wid: Optional[str] = None
    # GPU spans of the batch: [{"name": "H2D"|"kernel"|"D2H", "begin": t, "end": t, "bytes": n}]
    # (wall-clock seconds, like start/end), for the distributor's Perfetto export
    spans: List[dict] = field(default_factory=list)


def _metas(d: dict) -> List[FrameMeta]:
    if "frames" in d:  # the per-frame form
        return [FrameMeta.from_json(x) for x in d["frames"]]
    idx, nb = d["index"], d["nbytes"]  # round 4's columnar v1 form
    n = len(idx)
    slots = d.get("slot") or [None] * n
    shapes = d["shape"] if "shape" in d else [d.get("shape1")] * n
    if "starts" in d:
        st, en = d["starts"], d["ends"]
    else:
        st, en = [float(d.get("start", 0.0))] * n, [float(d.get("end", 0.0))] * n
    out = [FrameMeta(int(idx[i]), int(nb[i]), shapes[i], slots[i], st[i], en[i], None) for i in range(n)]
    for k, msg in (d.get("errors") or {}).items():
        out[int(k)].error = msg
    return out


# ---- v2 columns -------------------------------------------------------------------------

def v2_shape_ok(shape) -> bool:
    """True when ``shape`` fits a v2 record (None, or up to 4 int32 dimensions)."""
    if shape is None:
        return True
    try:
        return len(shape) <= 4 and all(0 <= int(x) < 2 ** 31 for x in shape)
    except TypeError:
        return False


def columns(metas: Sequence[FrameMeta]) -> np.ndarray:
    """COLS records of ``metas`` (every shape must pass ``v2_shape_ok``)."""
    c = np.zeros(len(metas), COLS)
    c["slot"] = -1
    c["ndim"] = -1
    for i, m in enumerate(metas):
        c["index"][i] = m.index
        c["nbytes"][i] = m.nbytes
        if m.slot is not None:
            c["slot"][i] = m.slot
        if m.shape is not None:
            k = len(m.shape)
            c["ndim"][i] = k
            c["shape"][i, :k] = m.shape
    return c


def _shape_of(ndim: int, row) -> Optional[List[int]]:
    return None if ndim < 0 else [int(x) for x in row[:ndim]]


class ColumnMetas(_Seq):
    """The FrameMeta view of v2 records: built per frame on access (a worker that only needs the
    slots and sizes reads ``cols`` directly)."""

    def __init__(self, cols: np.ndarray, starts=None, ends=None, errors=None):
        self.cols = cols
        self._idx = cols["index"].tolist()
        self._nb = cols["nbytes"].tolist()
        self._slot = cols["slot"].tolist()
        self._ndim = cols["ndim"].tolist()
        self._starts, self._ends, self._errors = starts, ends, errors or {}

    def __len__(self) -> int:
        return len(self._idx)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        s = self._slot[i]
        return FrameMeta(self._idx[i], self._nb[i], _shape_of(self._ndim[i], self.cols["shape"][i]),
                         None if s < 0 else s,
                         self._starts[i] if self._starts is not None else 0.0,
                         self._ends[i] if self._ends is not None else 0.0, self._errors.get(i))


def _cols_from(part) -> np.ndarray:
    b = memoryview(part).cast("B")
    if len(b) % COLS.itemsize:
        raise ValueError(f"v2 columns of {len(b)} B are not whole {COLS.itemsize}-B records")
    return np.frombuffer(b, COLS)


# ---- requests -------------------------------------------------------------------------

def encode_request(credit: int = 1, shm: bool = False, version: int = 1, wid: Optional[str] = None,
                   numa: Optional[int] = None, wire: int = 1) -> List[bytes]:
    if version == 0:
        return [READY_V0]
    d = {"credit": int(credit), "shm": bool(shm)}
    if wid is not None:
        d["wid"] = str(wid)
    if numa is not None:
        d["numa"] = int(numa)
    if wire > 1:
        d["wire"] = int(wire)
    return [READY_V1, json.dumps(d).encode()]


def decode_request(parts: Sequence[bytes]) -> Optional[Request]:
    if not parts:
        return None
    tag = bytes(parts[0])
    if tag == READY_V0:                      # distributor.py:229
        return Request(version=0)
    if tag == READY_V1 and len(parts) >= 2:
        d = json.loads(bytes(parts[1]))
        numa = d.get("numa")
        return Request(version=1, credit=max(1, int(d.get("credit", 1))), shm=bool(d.get("shm", False)),
                       wid=None if d.get("wid") is None else str(d["wid"]),
                       numa=None if numa is None else int(numa), wire=int(d.get("wire", 1)))
    return None


# ---- dispatch -------------------------------------------------------------------------

def encode_dispatch_v0(index: int, frame) -> List:
    return [str(index).encode(), frame]      # distributor.py:237-238


def encode_dispatch(metas: Sequence[FrameMeta], payloads: Sequence, ring: Optional[dict] = None) -> List:
    """v1, per-frame form (readable by every build)."""
    d = {"frames": [{"index": m.index, "nbytes": m.nbytes, "shape": m.shape, "slot": m.slot} for m in metas]}
    if ring is not None:
        d["ring"] = ring
    head = json.dumps(d).encode()
    return [FRAMES_V1, head] + [p for m, p in zip(metas, payloads) if m.slot is None]


def encode_dispatch2(cols: np.ndarray, payloads: Sequence, ring: Optional[dict] = None) -> List:
    """v2: ``cols`` (COLS records) and the parts of the frames without a slot, in order."""
    head = json.dumps({"ring": ring} if ring is not None else {}).encode()
    return [FRAMES_V2, head, cols.tobytes()] + list(payloads)


def decode_dispatch(parts: Sequence) -> Dispatch:
    tag = bytes(parts[0])
    if tag == FRAMES_V2:
        head = json.loads(bytes(parts[1]))
        cols = _cols_from(parts[2])
        slots = cols["slot"].tolist()
        it = iter(parts[3:])
        payloads = [None if s >= 0 else next(it) for s in slots]
        return Dispatch(ColumnMetas(cols), payloads, version=2, ring=head.get("ring"), cols=cols)
    if tag != FRAMES_V1:                     # v0: [index, frame]   (worker.py:50-51)
        if len(parts) != 2:
            raise ValueError(f"v0 dispatch must have 2 parts, got {len(parts)}")
        frame = parts[1]
        return Dispatch([FrameMeta(index=int(bytes(parts[0])), nbytes=len(frame))], [frame], version=0)
    head = json.loads(bytes(parts[1]))
    metas = _metas(head)
    it = iter(parts[2:])
    payloads = [None if m.slot is not None else next(it) for m in metas]
    return Dispatch(metas, payloads, version=1, ring=head.get("ring"))


# ---- results --------------------------------------------------------------------------

def encode_result_v0(index: int, pid, start: float, end: float, frame) -> List:
    # worker.py:63-67: every part a str except the frame; floats via str()
    return [str(index).encode(), str(pid).encode(), str(start).encode(), str(end).encode(), frame]


def encode_result(pid, metas: Sequence[FrameMeta], payloads: Sequence, spans: Optional[List[dict]] = None,
                  wid: Optional[str] = None) -> List:
    """v1, per-frame form (readable by every build)."""
    d = {"pid": str(pid), "frames": [m.to_json() for m in metas]}
    if wid is not None:
        d["wid"] = str(wid)
    if spans:
        d["spans"] = spans
    head = json.dumps(d).encode()
    return [RESULT_V1, head] + [p for m, p in zip(metas, payloads) if m.slot is None and m.error is None]


def encode_result2(pid, cols: np.ndarray, payloads: Sequence, start: float, end: float,
                   wid: Optional[str] = None, errors: Optional[dict] = None, spans: Optional[List[dict]] = None,
                   starts: Optional[List[float]] = None, ends: Optional[List[float]] = None) -> List:
    """v2: ``cols`` as dispatched with each result's own nbytes / slot (-1: the result is a part),
    ``payloads`` the parts of unslotted, successful frames in order, ``errors`` {position: message}."""
    d = {"pid": str(pid)}
    if wid is not None:
        d["wid"] = str(wid)
    if starts is not None:
        d["starts"], d["ends"] = starts, ends
    else:
        d["start"], d["end"] = start, end
    if errors:
        d["errors"] = {str(k): v for k, v in errors.items()}
    if spans:
        d["spans"] = spans
    return [RESULT_V2, json.dumps(d).encode(), cols.tobytes()] + list(payloads)


def decode_result(parts: Sequence) -> Result:
    tag = bytes(parts[0])
    if tag == RESULT_V2:
        d = json.loads(bytes(parts[1]))
        cols = _cols_from(parts[2])
        n = len(cols)
        errors = {int(k): v for k, v in (d.get("errors") or {}).items()}
        if "starts" in d:
            st, en = [float(x) for x in d["starts"]], [float(x) for x in d["ends"]]
        else:
            st, en = [float(d.get("start", 0.0))] * n, [float(d.get("end", 0.0))] * n
        metas = list(ColumnMetas(cols, st, en, errors))
        it = iter(parts[3:])
        payloads = [None if (m.slot is not None or m.error is not None) else next(it) for m in metas]
        return Result(str(d["pid"]), metas, payloads, version=2, spans=list(d.get("spans", [])),
                      wid=None if d.get("wid") is None else str(d["wid"]))
    if tag != RESULT_V1:                     # distributor.py:260-264
        if len(parts) != 5:
            raise ValueError(f"v0 result must have 5 parts, got {len(parts)}")
        idx, pid, start, end, frame = parts
        m = FrameMeta(index=int(bytes(idx)), nbytes=len(frame), start=float(bytes(start)), end=float(bytes(end)))
        return Result(bytes(pid).decode(), [m], [frame], version=0)
    d = json.loads(bytes(parts[1]))
    metas = _metas(d)
    it = iter(parts[2:])
    payloads = [None if (m.slot is not None or m.error is not None) else next(it) for m in metas]
    return Result(str(d["pid"]), metas, payloads, version=1, spans=list(d.get("spans", [])),
                  wid=None if d.get("wid") is None else str(d["wid"]))
