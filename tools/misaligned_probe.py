#!/usr/bin/env python3
"""HBM rate of the invert kernels on resident buffers by relative alignment: equal offsets
(streaming kernel), unequal offsets (shifting kernel), and the descriptor kernel over 32
1080p frames (aligned and misaligned).  Rotates over > 2 GB so the Infinity Cache cannot
hold the stream; GB/s = 2 x bytes / mean launch time."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-video-filter_amd"))
import numpy as np  # noqa: E402

from vfilter import Context  # noqa: E402

ctx = Context(int(os.environ.get("VF_DEVICE", "0")))
fb = 1920 * 1080 * 3
bb = 32 * fb
ring = 6
srcs = [ctx.alloc_device(bb + 64) for _ in range(ring)]
dsts = [ctx.alloc_device(bb + 64) for _ in range(ring)]
for s in srcs:
    ctx.memset_device(s, 0x3C, bb + 64)
ctx.sync()
for soff, doff in ((0, 0), (5, 5), (3, 0), (0, 8), (1, 2), (15, 0)):
    ss = [s + soff for s in srcs]
    dd = [d + doff for d in dsts]
    ctx.bench_device_ring(ss, dd, bb, 12)
    ms, _ = ctx.bench_device_ring(ss, dd, bb, 60)
    gbs = 2 * bb / (ms / 60 * 1e-3) / 1e9
    print(json.dumps({"kernel": "stream" if soff % 16 == doff % 16 else "shift", "src_off": soff, "dst_off": doff,
                      "bytes": bb, "ms_per_launch": round(ms / 60, 4), "GBps": round(gbs, 1),
                      "frac": round(gbs / 8000, 4)}), flush=True)
# descriptor kernel: 32 frames per launch, per-frame pointers
for label, soff, doff in (("frames_aligned", 0, 0), ("frames_shifted", 3, 0)):
    tabs = []
    for r in range(ring):
        sp = np.array([srcs[r] + soff + i * fb for i in range(32)], np.uint64)
        dp = np.array([dsts[r] + doff + i * fb for i in range(32)], np.uint64)
        nb = np.full(32, fb, np.uint64)
        t = [ctx.alloc_device(256) for _ in range(3)]
        for tt, a in zip(t, (sp, dp, nb)):
            ctx.upload(tt, a, a.nbytes)
        tabs.append(t)
    ctx.sync()
    import time
    for _ in range(12):
        for t in tabs:
            ctx.invert_device_frames(t[0], t[1], t[2], 32, bb)
    ctx.sync()
    t0 = time.perf_counter()
    k = 0
    for _ in range(10):
        for t in tabs:
            ctx.invert_device_frames(t[0], t[1], t[2], 32, bb)
            k += 1
    ctx.sync()
    dt = (time.perf_counter() - t0) / k
    gbs = 2 * bb / dt / 1e9
    print(json.dumps({"kernel": label, "src_off": soff, "dst_off": doff, "bytes": bb,
                      "ms_per_launch_wall": round(dt * 1e3, 4), "GBps": round(gbs, 1), "frac": round(gbs / 8000, 4)}),
          flush=True)
ctx.close()
