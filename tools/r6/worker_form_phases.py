#!/usr/bin/env python3
"""Where the JPEG worker form's host time goes at the reference app's operating point (512 x 512,
batches of 64, three in flight on one thread, as bench.jpeg_mode's worker_form): per batch, the
Python-side time in invert_batch_submit and in invert_batch_result, and the library's own phase
split (VF_JPEG_TRACE: prep_dec / prep_enc / queue per submit; wait per result), against the
GPU-resident time of the same batch.  Prints one JSON line.
  VF_JPEG_TRACE=1 python tools/r6/worker_form_phases.py [512sq|480p] [batch]"""
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-video-filter_amd")]
from vfilter import Context  # noqa: E402
from vfilter.jpeg import TurboJPEG  # noqa: E402
from vfilter.synthetic import synthetic_scene  # noqa: E402

size = sys.argv[1] if len(sys.argv) > 1 else "512sq"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 64
h, w = {"512sq": (512, 512), "480p": (480, 640), "1080p": (1080, 1920)}[size]
ctx = Context(int(os.environ.get("VF_DEVICE", "0")))
tj = TurboJPEG(ctx=ctx)
enc = tj.encode_batch([synthetic_scene(s, h, w) for s in range(8)])
jpgs = [enc[i % 8] for i in range(batch)]
ctx.jpeg_bench_invert(jpgs, 85, 1, 0, iters=2)
ms, _ = ctx.jpeg_bench_invert(jpgs, 85, 1, 0, iters=20)
depth, reps = 3, 40
ts, tr = [], []
for warm in (True, False):
    q = []
    t0 = time.perf_counter()
    for i in range(reps if not warm else 6):
        a = time.perf_counter()
        q.append(tj.invert_batch_submit(jpgs))
        ts.append(time.perf_counter() - a)
        if len(q) == depth:
            a = time.perf_counter()
            tj.invert_batch_result(q.pop(0))
            tr.append(time.perf_counter() - a)
    for t in q:
        tj.invert_batch_result(t)
    wall = time.perf_counter() - t0
    if warm:
        ts.clear()
        tr.clear()
med = lambda x: sorted(x)[len(x) // 2] * 1e3  # noqa: E731
print(json.dumps({"size": size, "batch": batch, "gpu_resident_ms_per_batch": round(ms, 4),
                  "worker_ms_per_batch": round(wall / reps * 1e3, 4), "submit_ms_median": round(med(ts), 4),
                  "result_ms_median": round(med(tr), 4)}), flush=True)
ctx.close()
