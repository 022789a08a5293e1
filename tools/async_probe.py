#!/usr/bin/env python3
"""Host->host rate of vf_invert_frames_async at different submission depths, on pinned
buffers, with no distributor in the way (isolates the C pipeline from the Python plumbing).
Reports host time spent inside submit and inside wait, for a batch given as per-frame
pieces and as one contiguous segment.

    python tools/async_probe.py [--size 1080p] [--batch 16] [--batches 48]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-video-filter_amd"))

import numpy as np  # noqa: E402

from vfilter import Context  # noqa: E402
from vfilter.synthetic import SIZES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="1080p")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--batches", type=int, default=48)
    ap.add_argument("--ring", type=int, default=4, help="distinct pinned batch buffers")
    args = ap.parse_args()
    h, w = SIZES[args.size]
    fb = h * w * 3
    bb = fb * args.batch
    ctx = Context(0, max_frame_bytes=fb, max_batch=args.batch)
    ps = [ctx.alloc_host(bb) for _ in range(args.ring)]
    pd = [ctx.alloc_host(bb) for _ in range(args.ring)]
    for p in ps:
        np.ctypeslib.as_array((ctypes.c_uint8 * bb).from_address(p))[:] = 7
    for pieces in ("frames", "contiguous"):
        for depth in (1, 2, 4):
            for mode in ("async", "sync"):
                if mode == "sync" and depth > 1:
                    continue
                t_sub = t_wait = 0.0
                t0 = time.perf_counter()
                q = []
                for b in range(args.batches):
                    k = b % args.ring
                    if pieces == "frames":
                        srcs = [ps[k] + i * fb for i in range(args.batch)]
                        dsts = [pd[k] + i * fb for i in range(args.batch)]
                        sizes = [fb] * args.batch
                    else:
                        srcs, dsts, sizes = [ps[k]], [pd[k]], [bb]
                    a = time.perf_counter()
                    if mode == "sync":
                        ctx.invert_frames_host(srcs, dsts, sizes)
                        t_sub += time.perf_counter() - a
                        continue
                    q.append(ctx.invert_frames_async(srcs, dsts, sizes))
                    t_sub += time.perf_counter() - a
                    if len(q) >= depth:
                        a = time.perf_counter()
                        ctx.wait(q.pop(0))
                        t_wait += time.perf_counter() - a
                a = time.perf_counter()
                for t in q:
                    ctx.wait(t)
                t_wait += time.perf_counter() - a
                dt = time.perf_counter() - t0
                print(json.dumps({"mode": mode, "pieces": pieces, "depth": depth, "size": args.size,
                                  "fps": round(args.batches * args.batch / dt, 1),
                                  "GBps_each_way": round(args.batches * bb / dt / 1e9, 2),
                                  "submit_ms_per_batch": round(1e3 * t_sub / args.batches, 3),
                                  "wait_ms_per_batch": round(1e3 * t_wait / args.batches, 3)}), flush=True)
    for p in ps + pd:
        ctx.free_host(p)
    ctx.close()


if __name__ == "__main__":
    main()
