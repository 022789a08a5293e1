"""Synthetic frames for benchmarks and demos: uniform uint8 from a seeded
``np.random.default_rng`` — the invert is data-independent, and uniform bytes exercise every
lane and byte position.  Frame sizes used by BASELINE.json's configs are named here.

``synthetic_scene`` makes camera-like frames for the JPEG mode (the reference's default,
inverter.py:32-44): JPEG of uniform noise is the codec's worst case, not a video frame."""
from __future__ import annotations

import numpy as np

SIZES = {
    "480sq": (480, 480),    # the reference raw path's hard-coded shape (inverter.py:34)
    "512sq": (512, 512),    # the reference app's crop (webcam_app.py:17,97-101), JPEG-encoded at :110
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


def synthetic_scene(seed: int, h: int, w: int) -> np.ndarray:
    """Smooth gradients, a few flat shapes with hard edges, texture and mild noise."""
    rng = np.random.default_rng(seed)
    y = np.linspace(0.0, 1.0, h, dtype=np.float64)[:, None]
    x = np.linspace(0.0, 1.0, w, dtype=np.float64)[None, :]
    img = np.empty((h, w, 3), np.float64)
    for c in range(3):
        a, b, p = rng.uniform(-80, 80), rng.uniform(-80, 80), rng.uniform(0, 6.3)
        f = rng.uniform(1.0, 6.0)
        img[..., c] = 128 + a * x + b * y + 30 * np.sin(2 * np.pi * f * (x + 0.5 * y) + p)
    for _ in range(6):
        y0, x0 = int(rng.integers(0, h)), int(rng.integers(0, w))
        y1, x1 = y0 + int(rng.integers(1, max(2, h // 3))), x0 + int(rng.integers(1, max(2, w // 3)))
        img[y0:y1, x0:x1, :] = rng.uniform(0, 255, 3)
    img += rng.normal(0.0, 3.0, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def synthetic_noisy_scene(seed: int, h: int, w: int, amp: int = 40) -> np.ndarray:
    """A camera-like scene with strong sensor-like noise (uniform +-amp per sample): the hard
    content of tests/test_gpu_jpeg.py's sync tests at full size.  Encoded at q95 its blocks are
    long (~1 MB per 1080p frame vs ~0.18 MB for the smooth scenes), the Huffman-table cache and
    the speculative sync's links see dense, varied streams, and the encoder codes many more
    AC coefficients."""
    rng = np.random.default_rng(10_000 + seed)
    img = synthetic_scene(seed, h, w).astype(np.int16) + rng.integers(-amp, amp + 1, (h, w, 3), dtype=np.int16)
    return np.clip(img, 0, 255).astype(np.uint8)
