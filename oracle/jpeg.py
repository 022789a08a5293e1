"""CPU ORACLE — TEST INFRASTRUCTURE ONLY: the reference's default JPEG path.

In its default mode (``use_jpeg=True``) the reference decodes every frame, inverts it and
re-encodes it with PyTurboJPEG (inverter.py:32 -> :41 -> :44; the app encodes at
webcam_app.py:110 and decodes at :140).  This module wraps

  * ``oracle/vf_jpeg_oracle.c`` — a plain-C restatement of the libjpeg-turbo baseline codec
    with PyTurboJPEG's defaults (quality 85, TJSAMP_422, TJPF_BGR); and
  * ``oracle/jpeg_xcheck.c`` — the image's own libjpeg-turbo 2.1.2 (``libjpeg.so.8``, the codec
    libturbojpeg wraps) driven as TurboJPEG drives it, used only to pin the restatement and
    to make golden vectors.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg import it;
the product (``vfilter.jpeg`` + libvfilter_hip.so) never does.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(_HERE, "_build", "libvf_jpeg_oracle.so")
XCHECK_LIB = os.path.join(_HERE, "_build", "libjpeg_xcheck.so")

# TurboJPEG constants (turbojpeg.h), the values PyTurboJPEG exposes
TJPF_RGB, TJPF_BGR = 0, 1
TJSAMP_444, TJSAMP_422, TJSAMP_420, TJSAMP_GRAY, TJSAMP_440 = 0, 1, 2, 3, 4
TJFLAG_FASTUPSAMPLE = 256
TJFLAG_FASTDCT = 2048
TJFLAG_ACCURATEDCT = 4096

_lib = None
_xlib = None


def _oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            raise FileNotFoundError(f"{ORACLE_LIB} missing: run `make -C oracle`")
        lib = ctypes.CDLL(ORACLE_LIB)
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        lib.vfo_jpeg_encode.argtypes = [vp, ci, ci, ci, ci, ci, ci, vp, sz]
        lib.vfo_jpeg_encode.restype = sz
        lib.vfo_jpeg_encode_bound.argtypes = [ci, ci, ci]
        lib.vfo_jpeg_encode_bound.restype = sz
        lib.vfo_jpeg_decode.argtypes = [vp, sz, ci, ci, vp, sz]
        lib.vfo_jpeg_decode.restype = ci
        lib.vfo_jpeg_parse.argtypes = [vp, sz, vp]
        lib.vfo_jpeg_parse.restype = ci
        _lib = lib
    return _lib


class _Info(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("ncomp", ctypes.c_int),
                ("comp_id", ctypes.c_int * 3), ("h", ctypes.c_int * 3), ("v", ctypes.c_int * 3),
                ("tq", ctypes.c_int * 3), ("td", ctypes.c_int * 3), ("ta", ctypes.c_int * 3),
                ("max_h", ctypes.c_int), ("max_v", ctypes.c_int), ("restart_interval", ctypes.c_int),
                ("qt", (ctypes.c_uint16 * 64) * 4), ("qt_defined", ctypes.c_int),
                ("dc_defined", ctypes.c_int), ("ac_defined", ctypes.c_int),
                ("dc_bits", (ctypes.c_uint8 * 17) * 4), ("ac_bits", (ctypes.c_uint8 * 17) * 4),
                ("dc_vals", (ctypes.c_uint8 * 256) * 4), ("ac_vals", (ctypes.c_uint8 * 256) * 4),
                ("scan_offset", ctypes.c_size_t), ("scan_end", ctypes.c_size_t)]


def _buf(b) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else b)


def info(jpeg) -> dict:
    """Header fields of a baseline JPEG (jdmarker.c restated)."""
    a = _buf(jpeg)
    st = _Info()
    rc = _oracle().vfo_jpeg_parse(a.ctypes.data, a.nbytes, ctypes.byref(st))
    if rc:
        raise ValueError(f"not a supported baseline JPEG (oracle status {rc})")
    return {"width": st.width, "height": st.height, "ncomp": st.ncomp,
            "h": list(st.h)[:st.ncomp], "v": list(st.v)[:st.ncomp],
            "restart_interval": st.restart_interval}


def fast_dct(flags: int, quality: int, tj_version: int = 3) -> bool:
    """Forward DCT libturbojpeg picks: 3.x accurate unless TJFLAG_FASTDCT; 2.x fast unless
    TJFLAG_ACCURATEDCT or quality >= 96 (turbojpeg.c setCompDefaults)."""
    if tj_version >= 3:
        return bool(flags & TJFLAG_FASTDCT)
    return not (flags & TJFLAG_ACCURATEDCT) and quality < 96


def encode(img: np.ndarray, quality: int = 85, pixel_format: int = TJPF_BGR,
           jpeg_subsample: int = TJSAMP_422, flags: int = 0, tj_version: int = 3) -> bytes:
    """``TurboJPEG.encode`` restated (inverter.py:44, webcam_app.py:110)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    lib = _oracle()
    cap = lib.vfo_jpeg_encode_bound(w, h, jpeg_subsample)
    out = np.empty(cap, np.uint8)
    n = lib.vfo_jpeg_encode(img.ctypes.data, w, h, pixel_format, quality, jpeg_subsample,
                            int(fast_dct(flags, quality, tj_version)), out.ctypes.data, cap)
    if n == 0:
        raise ValueError("oracle encode failed")
    return out[:n].tobytes()


def decode(jpeg, pixel_format: int = TJPF_BGR, flags: int = 0) -> np.ndarray:
    """``TurboJPEG.decode`` restated (inverter.py:32, webcam_app.py:140): H x W x 3 uint8."""
    a = _buf(jpeg)
    hdr = info(a)
    out = np.empty((hdr["height"], hdr["width"], 3), np.uint8)
    rc = _oracle().vfo_jpeg_decode(a.ctypes.data, a.nbytes, pixel_format,
                                   int(bool(flags & TJFLAG_FASTUPSAMPLE)), out.ctypes.data, out.nbytes)
    if rc:
        raise ValueError(f"oracle decode failed ({rc})")
    return out


def invert_jpeg(jpeg, quality: int = 85, jpeg_subsample: int = TJSAMP_422, flags: int = 0,
                tj_version: int = 3) -> bytes:
    """``InverterWorker.__call__`` with use_jpeg=True (inverter.py:31-44): decode, bitwise_not,
    re-encode with the PyTurboJPEG defaults."""
    return encode(np.bitwise_not(decode(jpeg, TJPF_BGR, flags)), quality, TJPF_BGR, jpeg_subsample,
                  flags, tj_version)


# ---------------------------------------------------------------------------------------
# The image's libjpeg-turbo (the codec libturbojpeg wraps), for pinning the restatement.
# ---------------------------------------------------------------------------------------

def _x():
    global _xlib
    if _xlib is None:
        if not os.path.exists(XCHECK_LIB):
            raise FileNotFoundError(f"{XCHECK_LIB} missing: run `make -C oracle`")
        lib = ctypes.CDLL(XCHECK_LIB)
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        lib.xc_available.argtypes = [ctypes.c_char_p, sz]
        lib.xc_available.restype = ci
        lib.xc_encode.argtypes = [vp, ci, ci, ci, ci, ci, ci, vp, sz]
        lib.xc_encode.restype = sz
        lib.xc_encode_ex.argtypes = [vp, ci, ci, ci, ci, ci, ci, ci, ci, ci, vp, sz]
        lib.xc_encode_ex.restype = sz
        lib.xc_decode.argtypes = [vp, sz, ci, ci, ci, ci, ci, vp]
        lib.xc_decode.restype = ci
        _xlib = lib
    return _xlib


def libjpeg_available() -> Tuple[bool, str]:
    try:
        lib = _x()
    except OSError as e:
        return False, str(e)
    why = ctypes.create_string_buffer(256)
    ok = bool(lib.xc_available(why, 256))
    return ok, why.value.decode()


def libjpeg_encode(img: np.ndarray, quality: int = 85, pixel_format: int = TJPF_BGR,
                   jpeg_subsample: int = TJSAMP_422, fastdct: bool = False, restart_interval: int = 0,
                   restart_rows: int = 0, optimize: bool = False) -> bytes:
    """libjpeg-turbo as tjCompress2 drives it, plus libjpeg options TurboJPEG leaves at their
    defaults (restart markers, optimised Huffman tables) for decoder test inputs."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    cap = _oracle().vfo_jpeg_encode_bound(w, h, jpeg_subsample) + 2 * (w * h // 64 + 16) + 4096
    out = np.empty(cap, np.uint8)
    n = _x().xc_encode_ex(img.ctypes.data, w, h, int(pixel_format == TJPF_BGR), quality, jpeg_subsample,
                          int(fastdct), restart_interval, restart_rows, int(optimize), out.ctypes.data, cap)
    if n == 0:
        raise RuntimeError("libjpeg encode failed: " + libjpeg_available()[1])
    return out[:n].tobytes()


def libjpeg_decode(jpeg, pixel_format: int = TJPF_BGR, fast_upsample: bool = False) -> np.ndarray:
    a = _buf(jpeg)
    hdr = info(a)
    out = np.empty((hdr["height"], hdr["width"], 3), np.uint8)
    rc = _x().xc_decode(a.ctypes.data, a.nbytes, int(pixel_format == TJPF_BGR), int(fast_upsample),
                        hdr["width"], hdr["height"], hdr["ncomp"], out.ctypes.data)
    if rc:
        raise RuntimeError("libjpeg decode failed: " + libjpeg_available()[1])
    return out


# ---------------------------------------------------------------------------------------
# Synthetic camera-like frames (JPEG of uniform noise is the codec's worst case, not a
# video frame): smooth gradients, a few flat shapes with edges, texture and mild noise.
# ---------------------------------------------------------------------------------------

def synthetic_scene(seed: int, h: int, w: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    y = np.linspace(0.0, 1.0, h, dtype=np.float64)[:, None]
    x = np.linspace(0.0, 1.0, w, dtype=np.float64)[None, :]
    img = np.empty((h, w, 3), np.float64)
    for c in range(3):
        a, b, p = rng.uniform(-80, 80), rng.uniform(-80, 80), rng.uniform(0, 6.3)
        f = rng.uniform(1.0, 6.0)
        img[..., c] = 128 + a * x + b * y + 30 * np.sin(2 * np.pi * f * (x + 0.5 * y) + p)
    for _ in range(6):  # flat rectangles with hard edges
        y0, x0 = int(rng.integers(0, h)), int(rng.integers(0, w))
        y1, x1 = y0 + int(rng.integers(1, max(2, h // 3))), x0 + int(rng.integers(1, max(2, w // 3)))
        img[y0:y1, x0:x1, :] = rng.uniform(0, 255, 3)
    img += rng.normal(0.0, 3.0, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)
