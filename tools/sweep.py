#!/usr/bin/env python3
"""Throughput sweep on one MI355X (run on the GPU box; writes JSON lines).

  kernel   HBM-resident invert rate per resolution (480p / 1080p / 4K) and, for 1080p,
           BASELINE.json configs[4]'s large-batch sweep (256 ... 4096 frames, 1.6-25.5 GB in):
           frames/s and algorithmic GB/s (2 bytes moved per byte) vs the 8 TB/s HBM peak.
  e2e      host->host rate through vf_invert_batch_host (pinned and pageable) per resolution,
           i.e. PCIe-inclusive; reported separately from the kernel rate.

    python tools/sweep.py [--out gpurun_out/sweep.jsonl] [--quick]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-video-filter_amd"))

import numpy as np  # noqa: E402

from vfilter import Context  # noqa: E402
from vfilter.synthetic import SIZES, synthetic_frame  # noqa: E402

PEAK = 8000.0


def kernel_point(ctx, tag, h, w, batch, ring_min_bytes=2.4e9, steps=40, warm=3, warm_ms=0.0, timed_ms=0.0):
    fb = h * w * 3
    bb = fb * batch
    nbuf = max(1, int(ring_min_bytes // (2 * bb)))
    if bb * 2 * nbuf < ring_min_bytes:
        nbuf = max(nbuf, 1)
    frame = synthetic_frame(1, h, w).reshape(-1)
    srcs, dsts = [], []
    for _ in range(nbuf):
        s, d = ctx.alloc_device(bb), ctx.alloc_device(bb)
        for f in range(batch):
            ctx.upload(s + f * fb, frame, fb)
        srcs.append(s)
        dsts.append(d)
    ctx.sync()
    steps = max(4, min(steps, int(40 * 4e8 / (2 * bb)) + 4))
    # warm for at least warm_ms of kernel time (clocks and the fabric settle after the
    # PCIe-bound upload phase), then time at least timed_ms
    done_ms, est = 0.0, None
    while True:
        ms_w, _ = ctx.bench_device_ring(srcs, dsts, bb, warm)
        done_ms += ms_w
        est = ms_w / warm
        if done_ms >= warm_ms:
            break
    steps = max(steps, int(timed_ms / est) + 1)
    region, _ = ctx.bench_device_ring(srcs, dsts, bb, steps)
    _, iso = ctx.bench_device_ring(srcs, dsts, bb, max(min(steps, 40), 10), per_launch=True)
    for s, d in zip(srcs, dsts):
        ctx.free_device(s)
        ctx.free_device(d)
    ms = region / steps
    gbs = 2 * bb / (ms * 1e-3) / 1e9
    return {"kind": "kernel", "size": tag, "frame": [h, w, 3], "batch": batch, "bytes_in": bb,
            "ring_buffers": nbuf, "steps": steps, "warm_ms": round(done_ms, 1), "ms_per_launch": round(ms, 4),
            "isolated_ms_median": round(float(np.median(iso)), 4),
            "isolated_ms_min_max": [round(float(np.min(iso)), 4), round(float(np.max(iso)), 4)],
            "frames_per_s": round(batch / (ms * 1e-3), 1), "GBps": round(gbs, 1), "frac_of_peak": round(gbs / PEAK, 4)}


def e2e_point(ctx, tag, h, w, batch, reps=4):
    fb = h * w * 3
    n = fb * batch
    host = np.empty(n, np.uint8)
    for f in range(batch):
        host[f * fb:(f + 1) * fb] = synthetic_frame(f, h, w).reshape(-1)
    out = np.empty_like(host)
    res = {"kind": "e2e", "size": tag, "frame": [h, w, 3], "batch": batch}
    ps, pd = ctx.alloc_host(n), ctx.alloc_host(n)
    try:
        src = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ps))
        dst = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pd))
        src[:] = host
        for label, (a, b) in (("pageable", (host, out)), ("pinned", (src, dst))):
            ctx.invert_batch_host(a, b, fb, batch)
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.invert_batch_host(a, b, fb, batch)
            dt = (time.perf_counter() - t0) / reps
            res[f"{label}_fps"] = round(batch / dt, 1)
            res[f"{label}_GBps_each_way"] = round(n / dt / 1e9, 2)
        assert np.array_equal(dst[:fb], np.bitwise_not(src[:fb]))  # sanity only
    finally:
        ctx.free_host(ps)
        ctx.free_host(pd)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.jsonl"))
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--e2e-only", action="store_true")
    ap.add_argument("--c5-only", action="store_true", help="only the configs[4] large-batch points")
    ap.add_argument("--c5-point", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--warm-ms", type=float, default=300.0, help="configs[4] points: min kernel ms of warmup")
    ap.add_argument("--timed-ms", type=float, default=200.0, help="configs[4] points: min kernel ms timed")
    args = ap.parse_args()
    if args.c5_point:
        c = Context(0)
        print(json.dumps(kernel_point(c, "1080p", 1080, 1920, args.c5_point, ring_min_bytes=0, steps=12,
                                      warm=5, warm_ms=args.warm_ms, timed_ms=args.timed_ms)))
        c.close()
        return
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    ctx = Context(0, max_frame_bytes=2160 * 3840 * 3, max_batch=4)
    points = [("480p", 32), ("480p", 256), ("1080p", 32), ("4k", 16), ("4k", 64)]
    if args.c5_only:
        points = []
    sweep = [256, 512, 1024] if args.quick else [256, 512, 1024, 2048, 4096]
    with open(args.out, "w") as f:
        def emit(r):
            f.write(json.dumps(r) + "\n")
            f.flush()
            print(json.dumps(r), flush=True)
        for tag, b in ([] if args.e2e_only else points):
            h, w = SIZES[tag]
            emit(kernel_point(ctx, tag, h, w, b))
        # configs[4]: one launch over the whole resident batch.  Each point runs in a fresh
        # process: after many alloc/free cycles a multi-GB hipMalloc measured up to 20 % slower
        # (profiles/r01_large_buffers.txt), which a worker that allocates once never sees.
        for b in ([] if args.e2e_only else sweep):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--c5-point", str(b),
                                "--warm-ms", str(args.warm_ms), "--timed-ms", str(args.timed_ms)],
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError(f"configs[4] point {b} failed: {r.stderr[-500:]}")
            emit(json.loads(r.stdout.strip().splitlines()[-1]))
        for tag, b in ((("480p", 32), ("1080p", 32), ("4k", 16)) if not args.c5_only else ()):
            h, w = SIZES[tag]
            emit(e2e_point(ctx, tag, h, w, b))
    ctx.close()


if __name__ == "__main__":
    main()
