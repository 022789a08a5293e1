#!/usr/bin/env python3
"""Host-side phase times of TurboJPEG.invert_batch (VF_JPEG_TRACE=1 makes the library print
prepare / queue / wait / fetch ms per call to stderr); Python-side wall time beside it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-video-filter_amd")]
from oracle import jpeg as J  # noqa: E402
from vfilter import Context  # noqa: E402
from vfilter.jpeg import TurboJPEG  # noqa: E402

size = sys.argv[1] if len(sys.argv) > 1 else "1080p"
h, w = {"512sq": (512, 512), "480p": (480, 640), "1080p": (1080, 1920), "4k": (2160, 3840)}[size]
ctx = Context(0)
tj = TurboJPEG(ctx=ctx)
frames = [J.synthetic_scene(s, h, w) for s in range(8)]
jpgs = [J.encode(frames[i % 8], 85, J.TJPF_BGR, 1) for i in range(32)]
for _ in range(3):
    tj.invert_batch(jpgs)
for _ in range(5):
    t0 = time.perf_counter()
    tj.invert_batch(jpgs)
    print(f"python wall {1e3 * (time.perf_counter() - t0):.3f} ms", file=sys.stderr, flush=True)
if len(sys.argv) > 2 and sys.argv[2] == "2threads":
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(2) as ex:
        list(ex.map(lambda _: tj.invert_batch(jpgs), range(2)))
        print("--- 2 threads", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        list(ex.map(lambda _: tj.invert_batch(jpgs), range(6)))
        print(f"2-thread wall {1e3 * (time.perf_counter() - t0) / 6:.3f} ms per batch", file=sys.stderr, flush=True)
ctx.close()
