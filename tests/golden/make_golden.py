"""Generate the known-answer fixtures for the invert filter (run here; outputs committed).

    python tests/golden/make_golden.py tests/golden

Expected outputs are computed as ``255 - x`` in uint16 arithmetic — a formulation
independent of both the oracle (``np.bitwise_not`` / C ``~x``) and the HIP kernel — from
OpenCV's definition of ``bitwise_not`` on CV_8U data (dst = ~src), which the reference
calls at inverter.py:41.

  kat.json             small frames with full input and expected output bytes:
                       the all-256-values frame (16x16x3 = 768 B, every byte value 3x),
                       ragged sizes (17x13x3 = 663 B, 1x1x3, 0 bytes) and a 31-byte
                       odd buffer.
  seeded_digests.json  sha256 of input and expected output of
                       default_rng(seed).integers(0, 256, (H, W, 3), uint8) for seeds 0-3
                       at 480x480, 640x480, 1920x1080 and 3840x2160 (inputs are
                       regenerated on the GPU box; only digests are stored).
"""
import hashlib
import json
import os
import sys

import numpy as np


def expected(x: np.ndarray) -> np.ndarray:
    return (255 - x.astype(np.uint16)).astype(np.uint8)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main(out_dir: str) -> None:
    kats = []
    allv = (np.arange(768) % 256).astype(np.uint8).reshape(16, 16, 3)
    kats.append({"name": "all_values_16x16x3", "shape": [16, 16, 3],
                 "input_hex": allv.tobytes().hex(), "expected_hex": expected(allv).tobytes().hex()})
    rng = np.random.default_rng(7)
    for name, shape in (("ragged_17x13x3", (17, 13, 3)), ("tiny_1x1x3", (1, 1, 3)),
                        ("empty_0x0x3", (0, 0, 3)), ("odd_31", (31,))):
        x = rng.integers(0, 256, shape, dtype=np.uint8)
        kats.append({"name": name, "shape": list(shape), "input_hex": x.tobytes().hex(),
                     "expected_hex": expected(x).tobytes().hex()})
    with open(os.path.join(out_dir, "kat.json"), "w") as f:
        json.dump({"definition": "dst[i] = 255 - src[i] (OpenCV bitwise_not on CV_8U; inverter.py:41)",
                   "kats": kats}, f, indent=1)

    sizes = {"480sq": (480, 480), "480p": (480, 640), "1080p": (1080, 1920), "4k": (2160, 3840)}
    digests = []
    for tag, (h, w) in sizes.items():
        for seed in range(4):
            x = np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
            digests.append({"size": tag, "shape": [h, w, 3], "seed": seed,
                            "input_sha256": sha(x), "expected_sha256": sha(expected(x))})
    with open(os.path.join(out_dir, "seeded_digests.json"), "w") as f:
        json.dump({"generator": "np.random.default_rng(seed).integers(0, 256, (H, W, 3), dtype=np.uint8)",
                   "numpy": np.__version__, "frames": digests}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.abspath(__file__)))
