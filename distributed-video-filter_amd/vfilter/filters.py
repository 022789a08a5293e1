"""The filter entry points: ``cv2.bitwise_not`` semantics on the MI355X.

Reference call site: ``inverted = cv2.bitwise_not(frame)`` (inverter.py:41), frame a
C-contiguous uint8 H x W x 3 ndarray (a read-only view from ``np.frombuffer`` on the raw
path, inverter.py:34).  ``bitwise_not`` keeps that signature: a new same-shape, same-dtype
array comes back and the input is never written.  The work runs in libvfilter_hip.so;
there is no CPU fallback.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np

from ._lib import Context, get_context

_PINNED_RESULTS = os.environ.get("VF_PINNED_RESULTS", "1") != "0"


def bitwise_not(src: np.ndarray, dst: Optional[np.ndarray] = None, mask=None,
                ctx: Optional[Context] = None) -> np.ndarray:
    """Drop-in for ``cv2.bitwise_not(src[, dst[, mask]])`` (inverter.py:41).

    Per-element bitwise NOT over the raw bytes of ``src`` (any dtype, any shape; the
    reference passes uint8 H x W x 3).  ``dst`` (optional) receives the result and is
    returned; it must have ``src``'s shape and dtype.  ``mask`` is not supported (the
    reference never passes one) and raises.
    """
    if mask is not None:
        raise NotImplementedError("bitwise_not: mask is not supported (inverter.py:41 passes none)")
    src = np.ascontiguousarray(src)
    ctx = ctx or get_context()
    if dst is None:
        # a result in the context's pinned arena: the kernel writes it directly over PCIe
        # (no staging copy out); it goes back to the arena when the array is dropped.  Past the
        # arena's cap of live results (VF_PINNED_RESULT_CAP, 1 GiB), when page-locking fails, or
        # with VF_PINNED_RESULTS=0, the result is an ordinary array, as cv2.bitwise_not's is
        dst = ctx._arena.try_empty(src.shape, src.dtype) if _PINNED_RESULTS else None
        if dst is None:
            dst = np.empty_like(src)
    elif dst.shape != src.shape or dst.dtype != src.dtype or not dst.flags.c_contiguous:
        raise ValueError("bitwise_not: dst must be C-contiguous with src's shape and dtype")
    ctx.invert_host(src, dst, src.nbytes)
    return dst


invert = bitwise_not


def invert_bytes(frame_bytes, ctx: Optional[Context] = None) -> bytes:
    """bytes -> inverted bytes (inverter.py:34 -> :41 -> :46 without the fixed reshape)."""
    src = np.frombuffer(frame_bytes, dtype=np.uint8)
    out = bytearray(src.nbytes)
    if src.nbytes:
        (ctx or get_context()).invert_host(src, np.frombuffer(out, dtype=np.uint8), src.nbytes)
    return bytes(out)


def invert_batch(frames: np.ndarray, out: Optional[np.ndarray] = None,
                 ctx: Optional[Context] = None) -> np.ndarray:
    """Invert a packed (N, H, W, 3) batch in one pipelined pass (replaces N iterations of
    worker.py:57 -> inverter.py:41)."""
    frames = np.ascontiguousarray(frames)
    if out is None:
        out = np.empty_like(frames)
    n = frames.shape[0] if frames.ndim else 1
    fb = frames.nbytes // max(n, 1)
    (ctx or get_context()).invert_batch_host(frames, out, fb, n)
    return out


def invert_frames(frames: Sequence, outs: Optional[List] = None,
                  ctx: Optional[Context] = None) -> List:
    """Invert separately stored frames (ndarrays or bytes-likes; mixed sizes allowed) with
    one gathered pipeline pass.  Returns ndarrays (or fills ``outs``)."""
    srcs = [np.ascontiguousarray(f) if isinstance(f, np.ndarray) else np.frombuffer(f, dtype=np.uint8)
            for f in frames]
    if outs is None:
        outs = [np.empty_like(s) for s in srcs]
    (ctx or get_context()).invert_frames_host(srcs, outs, [s.nbytes for s in srcs])
    return outs
