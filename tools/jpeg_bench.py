#!/usr/bin/env python3
"""JPEG-mode throughput: the reference's default per-frame path (use_jpeg=True)
decode -> bitwise_not -> encode (inverter.py:32 -> :41 -> :44) on one MI355X.

Frames are synthetic camera-like scenes (oracle.jpeg.synthetic_scene), encoded once with the
PyTurboJPEG defaults (q85, 4:2:2) as the app does (webcam_app.py:110).  Reported per size:
  gpu_resident   the fused GPU pass (vf_jpeg_bench_invert): inputs already in HBM; wall ms per
                 batch and per-stage ms (hipEvents), frames/s
  host_to_host   vfilter.jpeg.TurboJPEG.invert_batch from Python bytes to Python bytes, one
                 call at a time, and from 2 host threads (the JPEG worker's submit form)
  cpu_reference  libjpeg-turbo 2.1.2 (the codec under PyTurboJPEG; the image's libjpeg.so.8)
                 decode + np.bitwise_not + encode, 1 host core, per frame as the reference
  parity         GPU output == oracle.invert_jpeg for the first frame of each batch

  python tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 20 --out gpurun_out/jpeg.jsonl
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-video-filter_amd")]

import numpy as np  # noqa: E402

from oracle import jpeg as J  # noqa: E402

SIZES = {"512sq": (512, 512), "480p": (480, 640), "720p": (720, 1280), "1080p": (1080, 1920), "4k": (2160, 3840)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1080p")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--subsamp", type=int, default=J.TJSAMP_422)
    ap.add_argument("--content", default="scene", choices=("scene", "hard"),
                    help="scene: 8 camera-like scenes at q85; hard: 32 distinct noisy scenes at q95 "
                         "(vfilter.synthetic.synthetic_noisy_scene)")
    ap.add_argument("--seed0", type=int, default=0, help="first content seed (frames use seed0 .. seed0 + 31)")
    ap.add_argument("--out", default="")
    ap.add_argument("--resident-only", action="store_true",
                    help="only the GPU-resident batches (kernel profiles without the concurrent host forms)")
    args = ap.parse_args()
    from vfilter import Context
    from vfilter.jpeg import TurboJPEG
    ctx = Context(0)
    tj = TurboJPEG(ctx=ctx)
    for name in args.sizes.split(","):
        h, w = SIZES[name]
        if args.content == "hard":
            from vfilter.synthetic import synthetic_noisy_scene
            frames = [synthetic_noisy_scene(args.seed0 + s, h, w) for s in range(min(args.batch, 32))]
            jpgs = [J.encode(frames[i % len(frames)], 95, J.TJPF_BGR, args.subsamp) for i in range(args.batch)]
        else:
            frames = [J.synthetic_scene(args.seed0 + s, h, w) for s in range(min(args.batch, 8))]
            jpgs = [J.encode(frames[i % len(frames)], 85, J.TJPF_BGR, args.subsamp) for i in range(args.batch)]
        in_bytes = sum(len(j) for j in jpgs)
        ms, stages = ctx.jpeg_bench_invert(jpgs, 85, args.subsamp, 0, iters=2)  # warm
        ms, stages = ctx.jpeg_bench_invert(jpgs, 85, args.subsamp, 0, iters=args.iters)
        outs = tj.invert_batch(jpgs)
        parity = outs[0] == J.invert_jpeg(jpgs[0])
        if args.resident_only:
            rec = {"kind": "jpeg_invert", "size": name, "content": args.content, "batch": args.batch,
                   "gpu_resident_ms_per_batch": round(ms, 3), "gpu_resident_fps": round(args.batch / (ms / 1e3), 1),
                   "stages_ms": {k: round(v, 4) for k, v in stages.items()}, "parity_vs_oracle": parity}
            print(json.dumps(rec), flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")
            continue
        t0 = time.perf_counter()
        reps = max(1, args.iters // 4)
        for _ in range(reps):
            tj.invert_batch(jpgs)
        h2h = (time.perf_counter() - t0) / reps
        # the worker's form: batches handed to 2 host threads (InverterWorker.submit_batch),
        # one batch's host work overlapping the other's GPU work
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(2) as ex:
            list(ex.map(lambda _: tj.invert_batch(jpgs), range(2)))  # warm the second codec
            preps = max(4, args.iters // 2)
            t0 = time.perf_counter()
            list(ex.map(lambda _: tj.invert_batch(jpgs), range(preps)))
            h2h_pipe = (time.perf_counter() - t0) / preps
        # CPU reference: libjpeg-turbo per frame, 1 core
        ok, why = J.libjpeg_available()
        cpu = None
        if ok and args.cpu_seconds > 0:
            n = 0
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < args.cpu_seconds:
                j = jpgs[n % len(jpgs)]
                J.libjpeg_encode(np.bitwise_not(J.libjpeg_decode(j)), 85, J.TJPF_BGR, args.subsamp, False)
                n += 1
            dt = time.perf_counter() - t0
            cpu = {"fps": round(n / dt, 2), "cores": 1, "frames": n, "kind": "reference codec (libjpeg-turbo 2.1.2)"}
        rec = {"kind": "jpeg_invert", "size": name, "content": args.content, "frame": [h, w, 3], "batch": args.batch,
               "subsamp": args.subsamp, "quality": 85, "jpeg_bytes_in_mean": round(in_bytes / args.batch),
               "jpeg_bytes_out_mean": round(sum(len(o) for o in outs) / len(outs)),
               "gpu_resident_ms_per_batch": round(ms, 3), "gpu_resident_fps": round(args.batch / (ms / 1e3), 1),
               "stages_ms": {k: round(v, 4) for k, v in stages.items()},
               "host_to_host_ms_per_batch": round(h2h * 1e3, 3), "host_to_host_fps": round(args.batch / h2h, 1),
               "host_to_host_2threads_fps": round(args.batch / h2h_pipe, 1),
               "cpu_reference": cpu, "parity_vs_oracle": parity}
        print(json.dumps(rec), flush=True)
        if args.out:
            with open(args.out, "a") as f:
                f.write(json.dumps(rec) + "\n")
    ctx.close()


if __name__ == "__main__":
    main()
