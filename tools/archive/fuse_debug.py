"""Which frames of test_invert_samplings_and_edges' batch differ from the oracle, per output
sampling, fused colour pass vs pixel round trip (debugging aid)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "distributed-video-filter_amd"))
from oracle import jpeg as J  # noqa: E402
from vfilter.jpeg import TurboJPEG  # noqa: E402

SIZES = [(1, 1), (7, 5), (8, 8), (16, 16), (17, 13), (33, 9), (64, 48), (130, 66), (31, 45), (480, 641), (23, 100)]


def img(kind, seed, h, w):
    if kind == "noise":
        return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    return J.synthetic_scene(seed, h, w)


tj = TurboJPEG()
jpgs = [J.encode(img("scene" if i % 2 else "noise", 200 + i, h, w), 80, J.TJPF_BGR, i % 5) for i, (h, w) in enumerate(SIZES)]
for out_ss in range(5):
    for fuse in ("1", "0"):
        os.environ["VF_JPEG_FUSE"] = fuse
        got = tj.invert_batch(jpgs, 85, out_ss, 0)
        bad = [(SIZES[i], i % 5) for i, (g, j) in enumerate(zip(got, jpgs)) if g != J.invert_jpeg(j, 85, out_ss, 0)]
        print("out_ss", out_ss, "fuse", fuse, "bad (h, w), in_ss:", bad, flush=True)
        # single-frame batches too
        if bad and fuse == "1":
            for i, j in enumerate(jpgs):
                g = tj.invert_batch([j], 85, out_ss, 0)[0]
                if g != J.invert_jpeg(j, 85, out_ss, 0):
                    print("   alone bad:", SIZES[i], i % 5, flush=True)
