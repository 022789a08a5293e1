"""Synthetic frames for benchmarks and demos: uniform uint8 from a seeded
``np.random.default_rng`` — the invert is data-independent, and uniform bytes exercise every
lane and byte position.  Frame sizes used by BASELINE.json's configs are named here."""
from __future__ import annotations

import numpy as np

SIZES = {
    "480sq": (480, 480),    # the reference raw path's hard-coded shape (inverter.py:34)
    "480p": (480, 640),
    "1080p": (1080, 1920),
    "4k": (2160, 3840),
}


def synthetic_frame(seed: int, h: int, w: int) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def synthetic_batch(n: int, h: int, w: int, seed0: int = 0) -> np.ndarray:
    out = np.empty((n, h, w, 3), np.uint8)
    for i in range(n):
        out[i] = synthetic_frame(seed0 + i, h, w)
    return out
