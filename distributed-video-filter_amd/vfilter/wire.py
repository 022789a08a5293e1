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
  request  ["READY1", json{"credit": k, "shm": bool, "wid": worker id, "numa": node of its GPU}]
  dispatch ["FRAMES1", json{"index": [i, ...], "nbytes": [n, ...], "slot": [s | null, ...] | null,
                             "shape1": [h, w, c] | null  (every frame's)  or  "shape": [[h, w, c] | null, ...],
                             "ring": {"name": shm name, "slot_bytes": n} (if any slot)},
            frame_0, ..., frame_{k-1}]
           (frames whose slot is set travel in the shared-memory ring and have no part)
  result   ["RESULT1", json{"pid": p, "wid": worker id, "index", "nbytes", "slot", "shape1" | "shape" as
                            above, "start": t, "end": t (every frame's) or "starts", "ends": [t, ...],
                            "errors": {"position": message} (frames that failed, if any),
                            "spans": [{"name", "begin", "end", "bytes"}...] (GPU timeline)},
            out_0, ...]
  Columns, not a list of per-frame objects: one JSON list of ints per field encodes and parses
  ~4-6x faster than 32 small dicts, and the metadata of a batch is what the distributor's one
  Python process handles per message (round 3: ~6 us per frame of the control plane's ~17).
  A decoder also accepts the earlier per-frame form ({"frames": [{"index", ...}, ...]}).
  "wid" ties a result to the request stream it answers (the distributor tracks every dispatched
  frame per worker, re-queues a lost worker's frames and frees their ring slots); "numa" lets
  the distributor place the worker's ring slice on its GPU's NUMA node.  A result's "nbytes" is
  the RESULT's length (a JPEG differs from its input's).
A worker run with protocol v0 against the reference distributor sends "READY" and reads 2
parts; this build's distributor answers a bare "READY" with a v0 dispatch.  Either side of the reference can
therefore be swapped for this build's independently.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

READY_V0 = b"READY"
READY_V1 = b"READY1"
FRAMES_V1 = b"FRAMES1"
RESULT_V1 = b"RESULT1"


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


@dataclass
class Dispatch:
    metas: List[FrameMeta]
    payloads: List[Optional[bytes]] = field(default_factory=list)  # None where slot is set
    version: int = 1
    ring: Optional[dict] = None  # {"name": shm name, "slot_bytes": n} when any slot is set


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


def _columns(metas: Sequence[FrameMeta], timing: bool) -> dict:
    d = {"index": [m.index for m in metas], "nbytes": [m.nbytes for m in metas]}
    slots = [m.slot for m in metas]
    if any(x is not None for x in slots):
        d["slot"] = slots
    shapes = [m.shape for m in metas]
    if all(x == shapes[0] for x in shapes):
        d["shape1"] = shapes[0] if shapes else None
    else:
        d["shape"] = shapes
    if timing:
        st, en = [m.start for m in metas], [m.end for m in metas]
        if st and all(x == st[0] for x in st) and all(x == en[0] for x in en):
            d["start"], d["end"] = st[0], en[0]
        else:
            d["starts"], d["ends"] = st, en
        errs = {str(i): m.error for i, m in enumerate(metas) if m.error}
        if errs:
            d["errors"] = errs
    return d


def _metas(d: dict) -> List[FrameMeta]:
    if "frames" in d:  # the per-frame form
        return [FrameMeta.from_json(x) for x in d["frames"]]
    idx, nb = d["index"], d["nbytes"]
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


# ---- requests -------------------------------------------------------------------------

def encode_request(credit: int = 1, shm: bool = False, version: int = 1, wid: Optional[str] = None,
                   numa: Optional[int] = None) -> List[bytes]:
    if version == 0:
        return [READY_V0]
    d = {"credit": int(credit), "shm": bool(shm)}
    if wid is not None:
        d["wid"] = str(wid)
    if numa is not None:
        d["numa"] = int(numa)
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
                       numa=None if numa is None else int(numa))
    return None


# ---- dispatch -------------------------------------------------------------------------

def encode_dispatch_v0(index: int, frame) -> List:
    return [str(index).encode(), frame]      # distributor.py:237-238


def encode_dispatch(metas: Sequence[FrameMeta], payloads: Sequence, ring: Optional[dict] = None) -> List:
    d = _columns(metas, False)
    if ring is not None:
        d["ring"] = ring
    head = json.dumps(d).encode()
    return [FRAMES_V1, head] + [p for m, p in zip(metas, payloads) if m.slot is None]


def encode_dispatch_columns(index: List[int], nbytes: List[int], slots: Optional[List[Optional[int]]],
                            shapes: List, payloads: Sequence, ring: Optional[dict] = None) -> List:
    """``encode_dispatch`` from columns the caller already holds (the distributor's hot path:
    no FrameMeta per frame); ``payloads`` are the parts of the frames without a slot, in order."""
    d = {"index": index, "nbytes": nbytes}
    if slots is not None:
        d["slot"] = slots
    if all(x == shapes[0] for x in shapes):
        d["shape1"] = shapes[0] if shapes else None
    else:
        d["shape"] = shapes
    if ring is not None:
        d["ring"] = ring
    return [FRAMES_V1, json.dumps(d).encode()] + list(payloads)


def decode_dispatch(parts: Sequence) -> Dispatch:
    tag = bytes(parts[0])
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
    d = _columns(metas, True)
    d["pid"] = str(pid)
    if wid is not None:
        d["wid"] = str(wid)
    if spans:
        d["spans"] = spans
    head = json.dumps(d).encode()
    return [RESULT_V1, head] + [p for m, p in zip(metas, payloads) if m.slot is None and m.error is None]


def decode_result(parts: Sequence) -> Result:
    tag = bytes(parts[0])
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
