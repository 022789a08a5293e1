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
  dispatch ["FRAMES1", json{"frames": [{"index": i, "shape": [h, w, c] | null, "nbytes": n,
                                        "slot": s | null}, ...],
                             "ring": {"name": shm name, "slot_bytes": n} (if any slot)},
            frame_0, ..., frame_{k-1}]
           (frames whose "slot" is set travel in the shared-memory ring and have no part)
  result   ["RESULT1", json{"pid": p, "wid": worker id, "frames": [{"index", "shape", "nbytes",
                                                 "slot", "start", "end", "error"}...],
                            "spans": [{"name", "begin", "end", "bytes"}...] (GPU timeline)},
            out_0, ...]
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


@dataclass
class FrameMeta:
    index: int
    nbytes: int
    shape: Optional[List[int]] = None
    slot: Optional[int] = None
    start: float = 0.0
    end: float = 0.0
    error: Optional[str] = None

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
    d = {"frames": [m.to_json() for m in metas]}
    if ring is not None:
        d["ring"] = ring
    head = json.dumps(d).encode()
    return [FRAMES_V1, head] + [p for m, p in zip(metas, payloads) if m.slot is None]


def decode_dispatch(parts: Sequence) -> Dispatch:
    tag = bytes(parts[0])
    if tag != FRAMES_V1:                     # v0: [index, frame]   (worker.py:50-51)
        if len(parts) != 2:
            raise ValueError(f"v0 dispatch must have 2 parts, got {len(parts)}")
        frame = parts[1]
        return Dispatch([FrameMeta(index=int(bytes(parts[0])), nbytes=len(frame))], [frame], version=0)
    head = json.loads(bytes(parts[1]))
    metas = [FrameMeta.from_json(d) for d in head["frames"]]
    it = iter(parts[2:])
    payloads = [None if m.slot is not None else next(it) for m in metas]
    return Dispatch(metas, payloads, version=1, ring=head.get("ring"))


# ---- results --------------------------------------------------------------------------

def encode_result_v0(index: int, pid, start: float, end: float, frame) -> List:
    # worker.py:63-67: every part a str except the frame; floats via str()
    return [str(index).encode(), str(pid).encode(), str(start).encode(), str(end).encode(), frame]


def encode_result(pid, metas: Sequence[FrameMeta], payloads: Sequence, spans: Optional[List[dict]] = None,
                  wid: Optional[str] = None) -> List:
    d = {"pid": str(pid), "frames": [m.to_json() for m in metas]}
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
    metas = [FrameMeta.from_json(x) for x in d["frames"]]
    it = iter(parts[2:])
    payloads = [None if (m.slot is not None or m.error is not None) else next(it) for m in metas]
    return Result(str(d["pid"]), metas, payloads, version=1, spans=list(d.get("spans", [])),
                  wid=None if d.get("wid") is None else str(d["wid"]))
