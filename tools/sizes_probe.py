"""Wall clock vs hipEvent region of bench_device_ring, repeated (diagnoses the sizes leg)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-video-filter_amd")); sys.path.insert(0, ROOT)
import numpy as np
import torch
import bench
from vfilter import Context
torch.cuda.set_device(0)
ctx = Context(0, max_frame_bytes=bench.FRAME_BYTES, max_batch=32)
for hw, batch in (((1080, 1920), 32), ((2160, 3840), 16)):
    srcs, dsts, bb, _ = bench.make_ring(ctx, batch, 2.4, np, hw=hw, distinct=8)
    for steps in (10, 100, 100, 300, 100):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        region, _ = ctx.bench_device_ring(srcs, dsts, bb, steps)
        t1 = time.perf_counter()
        ctx.sync()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(hw, steps, f"call {1e3*(t1-t0):.2f} ms  region {region:.2f} ms  sync {1e3*(t2-t1):.2f} ms", flush=True)
    for s, d in zip(srcs, dsts):
        ctx.free_device(s); ctx.free_device(d)
