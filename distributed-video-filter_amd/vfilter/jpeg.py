"""``TurboJPEG`` on the MI355X: the JPEG half of the reference's default mode.

With ``use_jpeg=True`` (the default, inverter.py:10) the reference worker runs

    frame = self.jpeg.decode(frame_bytes)      # inverter.py:32
    inverted = cv2.bitwise_not(frame)          # inverter.py:41
    return self.jpeg.encode(inverted)          # inverter.py:44

with ``self.jpeg = TurboJPEG()`` from PyTurboJPEG (inverter.py:7,13; the app does the same at
webcam_app.py:9,24,110,140).  ``vfilter.jpeg.TurboJPEG`` keeps that class's method names,
arguments, defaults (quality 85, TJSAMP_422, TJPF_BGR) and return types, and runs them on
hand-written gfx950 kernels whose integer arithmetic is libjpeg-turbo's, so the bytes and
pixels are the ones libjpeg-turbo produces.  ``invert`` fuses the three reference lines on
the GPU (no host round trip of the pixels); ``*_batch`` forms take a list of frames and use one
batched GPU pass.

Which forward DCT libturbojpeg uses at quality < 96 depends on its version: 3.x uses the
accurate one unless ``TJFLAG_FASTDCT``; 2.x uses the fast one unless ``TJFLAG_ACCURATEDCT``.
The default here is 3.x behaviour; ``TurboJPEG(tj_version=2)`` reproduces 2.x.

No CPU fallback: without libvfilter_hip.so or a gfx950 device every call raises.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from ._lib import Context, get_context, jpeg_header

# TurboJPEG constants (turbojpeg.h / PyTurboJPEG)
TJPF_RGB, TJPF_BGR = 0, 1
TJSAMP_444, TJSAMP_422, TJSAMP_420, TJSAMP_GRAY, TJSAMP_440 = 0, 1, 2, 3, 4
TJCS_RGB, TJCS_YCbCr, TJCS_GRAY = 0, 1, 2
TJFLAG_BOTTOMUP = 2
TJFLAG_FASTUPSAMPLE = 256
TJFLAG_FASTDCT = 2048
TJFLAG_ACCURATEDCT = 4096

_SUPPORTED_FLAGS = TJFLAG_FASTUPSAMPLE | TJFLAG_FASTDCT | TJFLAG_ACCURATEDCT


class TurboJPEG:
    """Drop-in for PyTurboJPEG's ``TurboJPEG`` (inverter.py:13, webcam_app.py:24)."""

    def __init__(self, lib_path: Optional[str] = None, ctx: Optional[Context] = None, tj_version: int = 3):
        # lib_path is PyTurboJPEG's path to libturbojpeg; there is nothing to load here
        self._ctx = ctx
        self.tj_version = int(tj_version)

    @property
    def ctx(self) -> Context:
        if self._ctx is None:
            self._ctx = get_context()
        return self._ctx

    def _enc_flags(self, flags: int, quality: int) -> int:
        if flags & ~_SUPPORTED_FLAGS:
            raise NotImplementedError(f"TurboJPEG flags {flags:#x} not supported on the GPU path")
        fast = bool(flags & TJFLAG_FASTDCT) if self.tj_version >= 3 else \
            not (flags & TJFLAG_ACCURATEDCT) and quality < 96
        return (flags & TJFLAG_FASTUPSAMPLE) | (TJFLAG_FASTDCT if fast else 0)

    @staticmethod
    def _dec_flags(flags: int) -> int:
        if flags & ~_SUPPORTED_FLAGS:
            raise NotImplementedError(f"TurboJPEG flags {flags:#x} not supported on the GPU path")
        return flags & TJFLAG_FASTUPSAMPLE

    # -- PyTurboJPEG API -------------------------------------------------------------------
    def decode_header(self, jpeg_buf):
        """(width, height, jpeg_subsample, jpeg_colorspace)."""
        return jpeg_header(jpeg_buf)

    def decode(self, jpeg_buf, pixel_format: int = TJPF_BGR, scaling_factor=None, flags: int = 0) -> np.ndarray:
        """inverter.py:32 / webcam_app.py:140: JPEG bytes -> H x W x 3 uint8."""
        if scaling_factor not in (None, (1, 1)):
            raise NotImplementedError("scaling_factor is not supported on the GPU path")
        return self.ctx.jpeg_decode([jpeg_buf], pixel_format, self._dec_flags(flags))[0]

    def encode(self, img_array: np.ndarray, quality: int = 85, pixel_format: int = TJPF_BGR,
               jpeg_subsample: int = TJSAMP_422, flags: int = 0) -> bytes:
        """inverter.py:44 / webcam_app.py:110: H x W x 3 uint8 -> JPEG bytes."""
        return self.ctx.jpeg_encode([img_array], pixel_format, quality, jpeg_subsample,
                                    self._enc_flags(flags, quality))[0]

    # -- batched / fused extensions --------------------------------------------------------
    def decode_batch(self, jpeg_bufs: Sequence, pixel_format: int = TJPF_BGR, flags: int = 0) -> List[np.ndarray]:
        return self.ctx.jpeg_decode(list(jpeg_bufs), pixel_format, self._dec_flags(flags))

    def encode_batch(self, imgs: Sequence[np.ndarray], quality: int = 85, pixel_format: int = TJPF_BGR,
                     jpeg_subsample: int = TJSAMP_422, flags: int = 0) -> List[bytes]:
        return self.ctx.jpeg_encode(list(imgs), pixel_format, quality, jpeg_subsample,
                                    self._enc_flags(flags, quality))

    def invert(self, jpeg_buf, quality: int = 85, jpeg_subsample: int = TJSAMP_422, flags: int = 0) -> bytes:
        """``encode(bitwise_not(decode(jpeg_buf)))`` (inverter.py:32 -> :41 -> :44) fused on the GPU."""
        return self.invert_batch([jpeg_buf], quality, jpeg_subsample, flags)[0]

    def invert_batch(self, jpeg_bufs: Sequence, quality: int = 85, jpeg_subsample: int = TJSAMP_422,
                     flags: int = 0) -> List[bytes]:
        """One fused GPU pass over the batch (safe to call from several threads at once: each
        call leases its own codec)."""
        return self.ctx.jpeg_invert(list(jpeg_bufs), quality, jpeg_subsample, self._enc_flags(flags, quality))

    def invert_batch_submit(self, jpeg_bufs: Sequence, quality: int = 85, jpeg_subsample: int = TJSAMP_422,
                            flags: int = 0) -> int:
        """invert_batch, asynchronously: stage and queue the batch, return a ticket at once.
        One host thread can keep several batches in flight (each holds its own codec)."""
        return self.ctx.jpeg_invert_submit(list(jpeg_bufs), quality, jpeg_subsample, self._enc_flags(flags, quality))

    def invert_batch_submit_addrs(self, addrs, sizes, quality: int = 85, jpeg_subsample: int = TJSAMP_422,
                                  flags: int = 0) -> int:
        """``invert_batch_submit`` for JPEGs given by address and size arrays (a worker's ring
        slots; the memory stays valid until the result is collected)."""
        return self.ctx.jpeg_invert_submit_addrs(addrs, sizes, quality, jpeg_subsample, self._enc_flags(flags, quality))

    def invert_batch_result_into_addrs(self, ticket: int, out_addrs, cap: int):
        """(sizes, {i: JPEG that did not fit}): each result written at ``out_addrs[i]`` (``cap``
        writable bytes each) when it fits there."""
        return self.ctx.jpeg_invert_result_into_addrs(ticket, out_addrs, cap)

    def invert_batch_ready(self, ticket: int) -> bool:
        return self.ctx.jpeg_invert_ready(ticket)

    def invert_batch_result(self, ticket: int) -> List[np.ndarray]:
        """The inverted JPEGs of a submitted batch (bytes-like uint8 views), in batch order."""
        return self.ctx.jpeg_invert_result(ticket)

    def invert_batch_result_into(self, ticket: int, outs: Sequence) -> List[np.ndarray]:
        """The same, each JPEG written straight into ``outs[i]`` when it fits there (e.g. the
        output half of its ring slot); a frame without room comes back in a fresh buffer."""
        return self.ctx.jpeg_invert_result_into(ticket, outs)
