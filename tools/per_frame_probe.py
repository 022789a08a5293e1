#!/usr/bin/env python3
"""One frame per call, the drop-in's own shape (``vfilter.bitwise_not(frame)`` in place of
``cv2.bitwise_not(frame)``, inverter.py:41): per-call latency at 480p / 1080p / 4K for
  cpu        numpy's bitwise_not on one core (the reference arithmetic)
  dropin     vfilter.bitwise_not(frame): an ordinary numpy frame in, the result in the context's
             pinned arena (the drop-in's own call: the source staged through the mapped ring
             piece by piece beside the launches, the result written in place over PCIe)
  pageable   vfilter.bitwise_not(frame, out) with an ordinary numpy destination as well
  pinned     vfilter.bitwise_not with src and dst in vf_alloc_host memory (zero-copy launch)
Prints one JSON line per size.
  python tools/per_frame_probe.py"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-video-filter_amd")]
import numpy as np  # noqa: E402

import vfilter  # noqa: E402


def timed(fn, reps):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ctx = vfilter.Context(int(os.environ.get("VF_DEVICE", "0")), max_frame_bytes=2160 * 3840 * 3, max_batch=4)
    for name, (h, w) in {"480p": (480, 640), "1080p": (1080, 1920), "4k": (2160, 3840)}.items():
        n = h * w * 3
        frame = np.random.default_rng(0).integers(0, 256, (h, w, 3), dtype=np.uint8)
        out = np.empty_like(frame)
        ps, pd = ctx.alloc_host(n), ctx.alloc_host(n)
        try:
            fs = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ps)).reshape(h, w, 3)
            fd = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pd)).reshape(h, w, 3)
            fs[:] = frame
            reps = 200 if h < 2000 else 60
            r = {"size": name, "frame_bytes": n}
            r["cpu_ms"] = timed(lambda: np.bitwise_not(frame), reps) * 1e3
            r["dropin_ms"] = timed(lambda: vfilter.bitwise_not(frame, ctx=ctx), reps) * 1e3
            r["pageable_ms"] = timed(lambda: vfilter.bitwise_not(frame, out, ctx=ctx), reps) * 1e3
            r["pinned_ms"] = timed(lambda: vfilter.bitwise_not(fs, fd, ctx=ctx), reps) * 1e3
            assert np.array_equal(vfilter.bitwise_not(frame, ctx=ctx), ~frame)
            assert np.array_equal(out, ~frame) and np.array_equal(fd, ~frame)
            for k in ("cpu", "dropin", "pageable", "pinned"):
                r[f"{k}_fps"] = round(1e3 / r[f"{k}_ms"], 1)
                r[f"{k}_ms"] = round(r[f"{k}_ms"], 4)
            print(json.dumps(r), flush=True)
        finally:
            ctx.free_host(ps)
            ctx.free_host(pd)
    ctx.close()


if __name__ == "__main__":
    main()
