#!/usr/bin/env python3
"""Host->host JPEG invert (the worker's use_jpeg=True path) in the forms the worker could use,
one size per run, each in a fresh process so codec settings (read at codec creation) apply:
  1thread      one invert_batch call at a time
  2threads     two host threads, each call leasing its own codec (kernels ordered by the
               context's compute gate)
  2threads_nogate   the same with VF_JPEG_GATE=0 (kernels of the two codecs may overlap)
  async        ONE host thread keeping two batches in flight (invert_batch_submit / _result,
               vf_jpeg_invert_submit & co.): the InverterWorker's form
  async3       the same with three batches in flight
Prints one JSON line per mode.  VF_JPEG_TRACE=1 adds the library's per-call phase times.
  python tools/jpeg_modes.py 1080p [mode]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-video-filter_amd")]

SIZES = {"512sq": (512, 512), "480p": (480, 640), "1080p": (1080, 1920), "4k": (2160, 3840)}


def run(size, mode, batch=32, reps=24):
    from vfilter import Context
    from vfilter.jpeg import TurboJPEG
    from vfilter.synthetic import synthetic_scene
    h, w = SIZES[size]
    ctx = Context(0)
    tj = TurboJPEG(ctx=ctx)
    jpgs = tj.encode_batch([synthetic_scene(s, h, w) for s in range(8)])
    jpgs = [jpgs[i % 8] for i in range(batch)]
    if mode.startswith("async"):
        depth = int(mode[5:] or 2)  # batches in flight ("async" = 2, "async3" = 3)
        for _ in range(3):  # warm the codecs (the first use of a codec allocates its buffers)
            ts = [tj.invert_batch_submit(jpgs) for _ in range(depth)]
            for t in ts:
                tj.invert_batch_result(t)
        t0 = time.perf_counter()
        q = [tj.invert_batch_submit(jpgs) for _ in range(depth - 1)]
        for _ in range(reps - depth + 1):
            q.append(tj.invert_batch_submit(jpgs))
            out = tj.invert_batch_result(q.pop(0))
        for t in q[:-1]:
            tj.invert_batch_result(t)
        out = tj.invert_batch_result(q[-1])
        dt = time.perf_counter() - t0
        assert [bytes(o) for o in out] == tj.invert_batch(jpgs)
    elif mode == "1thread":
        for _ in range(3):
            tj.invert_batch(jpgs)
        t0 = time.perf_counter()
        for _ in range(reps):
            tj.invert_batch(jpgs)
        dt = time.perf_counter() - t0
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(2) as ex:
            list(ex.map(lambda _: tj.invert_batch(jpgs), range(4)))
            t0 = time.perf_counter()
            list(ex.map(lambda _: tj.invert_batch(jpgs), range(reps)))
            dt = time.perf_counter() - t0
    ms, stages = ctx.jpeg_bench_invert(jpgs, 85, 1, 0, iters=10)
    print(json.dumps({"size": size, "mode": mode, "batch": batch, "fps": round(reps * batch / dt, 1),
                      "ms_per_batch": round(dt / reps * 1e3, 3), "gpu_resident_ms": round(ms, 3)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    size = sys.argv[1] if len(sys.argv) > 1 else "1080p"
    if len(sys.argv) > 2:
        run(size, sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 32)
    else:
        for mode in ("1thread", "2threads", "async"):
            env = dict(os.environ)
            if mode == "2threads_nogate":
                env["VF_JPEG_GATE"] = "0"
            subprocess.run([sys.executable, __file__, size, mode], env=env, check=True, timeout=300)
