#!/usr/bin/env python3
"""BASELINE.json configs[0]: synthetic 640x480 RGB frames through a distributor + 2 local CPU
worker processes (plumbing, no GPU) — the reference's pipeline and this build's, side by side
on the same host.  Build container only: the reference exists here, not on the GPU box.

  reference   distributor.py + worker.py (imported from <reference_dir>, run with
              /opt/conda/bin/python3.9 -B, the only interpreter here with pyzmq) with a
              plugin subclass of the reference Worker (its extension point, worker.py:78-80)
              doing what inverter.py:34,41,46 does for a 640x480 frame: frombuffer ->
              reshape -> bitwise_not -> tobytes (inverter.py hard-codes 480x480, so the
              reference InverterWorker itself rejects these frames).
  build       vfilter.distributor.Distributor + vfilter.worker.Worker subclasses with the
              same CPU plugin, (i) policy "latest" / display reassembly / wire v0 (the
              reference's semantics) and (ii) lossless "pull" / in-order reassembly / wire v1
              batches of 8.

The plugin is numpy on the CPU in both, because configs[0] is the no-GPU plumbing case; what
is measured is the distribution machinery.  The GPU worker's numbers are bench.py's.

Each run offers frames at a fixed rate (or as fast as the producer can, "max") for
--seconds and reports delivered frames/s (distinct frame indices collected) and the share of
offered frames delivered.

  python tools/config0_bench.py [--seconds 5] [--rates 30,300,1000,3000,max] [--out FILE]
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-video-filter_amd")
REF_PY = "/opt/conda/bin/python3.9"
H, W = 480, 640


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def frames(n):
    import numpy as np
    rng = np.random.default_rng(0)
    return [rng.integers(0, 256, (H, W, 3), dtype=np.uint8).tobytes() for _ in range(n)]


def offer(add, pool, rate, seconds):
    """Add frames at `rate` fps (0 = as fast as possible) for `seconds`; returns frames offered."""
    n = 0
    t0 = time.perf_counter()
    while True:
        now = time.perf_counter()
        if now - t0 >= seconds:
            return n
        if rate:
            due = t0 + n / rate
            if now < due:
                time.sleep(min(due - now, 0.002))
                continue
        add(pool[n % len(pool)])
        n += 1


# ---- reference side (runs under python3.9 with the reference on sys.path) -----------------

def _ref_worker(ref_dir, dport, cport):
    sys.path.insert(0, ref_dir)
    sys.stdout = open(os.devnull, "w")  # worker.py:54 prints one line per frame
    import numpy as np
    from worker import Worker

    class Plugin(Worker):  # inverter.py:29-46 raw path at 640x480
        def __call__(self, frame_bytes):
            f = np.frombuffer(frame_bytes, dtype=np.uint8).reshape(H, W, 3)
            return np.bitwise_not(f).tobytes()

    Plugin("localhost", dport, cport).start()


def run_reference(ref_dir, rates, seconds):
    sys.path.insert(0, ref_dir)
    from distributor import Distributor

    class Counting(Distributor):
        """Counts results as the reference's collect thread logs them (distributor.py:266)."""
        def __init__(self, *a, **k):
            self.seen = set()
            super().__init__(*a, **k)

        def log_frame_complete_timing(self, frame_index, *a, **k):
            self.seen.add(int(frame_index))

    pool = frames(16)
    out = []
    ctx = mp.get_context("spawn")
    for rate in rates:
        dport, cport = free_port(), free_port()
        d = Counting(dport, cport)
        d.start()
        ws = [ctx.Process(target=_ref_worker, args=(ref_dir, dport, cport), daemon=True) for _ in range(2)]
        for w in ws:
            w.start()
        time.sleep(2.0)  # workers connect and start polling
        devnull = open(os.devnull, "w")
        so, sys.stdout = sys.stdout, devnull  # add_frame_for_distribution prints on overflow
        try:
            t0 = time.perf_counter()
            n = offer(d.add_frame_for_distribution, pool, rate, seconds)
            el = time.perf_counter() - t0
            time.sleep(0.5)  # in-flight frames land (counted, not timed)
        finally:
            sys.stdout = so
        got = len(d.seen)
        d.running = False
        for w in ws:
            w.terminate()
            w.join(5)
        out.append({"side": "reference", "mode": "latest/display, wire v0 (zmq)", "offered_rate": rate or "max",
                    "offered": n, "delivered": got, "delivered_fps": round(got / el, 1),
                    "delivered_share": round(got / max(n, 1), 3)})
        time.sleep(0.5)
    return out


# ---- build side (this interpreter) --------------------------------------------------------

def _build_worker(dport, cport, protocol, batch):
    sys.path.insert(0, PKG)
    import numpy as np
    from vfilter.worker import Worker

    class Plugin(Worker):
        def __call__(self, frame_bytes):
            return np.bitwise_not(np.frombuffer(frame_bytes, dtype=np.uint8))

    Plugin("127.0.0.1", dport, cport, protocol=protocol, batch=batch, transport="tcp").start()


def run_build(rates, seconds):
    sys.path.insert(0, PKG)
    from vfilter.distributor import Distributor
    pool = frames(16)
    out = []
    ctx = mp.get_context("spawn")
    modes = (("latest/display, wire v0 (tcp)", dict(policy="latest", reassembly="display"), "v0", 1),
             ("pull/ordered lossless, wire v1 batch 8 (tcp)", dict(policy="pull", reassembly="ordered",
                                                                   queue_size=64), "v1", 8))
    for label, kw, protocol, batch in modes:
        for rate in rates:
            d = Distributor(0, 0, transport="tcp", host="127.0.0.1", verbose=False, **kw)
            d.start()
            ws = [ctx.Process(target=_build_worker, args=(d.distribute_port, d.collect_port, protocol, batch),
                              daemon=True) for _ in range(2)]
            for w in ws:
                w.start()
            t0 = time.time()
            while d.num_workers() < 2 and time.time() - t0 < 30:
                time.sleep(0.02)
            if protocol == "v0":
                time.sleep(1.0)
            got = [0]
            stop = threading.Event()
            lossless = kw["policy"] != "latest"

            def drain():  # the consumer of the in-order stream
                while not stop.is_set():
                    if d.get_next_frame(timeout=0.1) is not None:
                        got[0] += 1

            th = threading.Thread(target=drain, daemon=True)
            if lossless:
                th.start()
            t0 = time.perf_counter()
            n = offer(lambda f: d.add_frame_for_distribution(f, shape=[H, W, 3]), pool, rate, seconds)
            if lossless:
                while got[0] < n and time.perf_counter() - t0 < seconds + 30:
                    time.sleep(0.002)
            el = time.perf_counter() - t0
            if not lossless:
                time.sleep(0.5)  # in-flight frames land (counted, not timed)
            stop.set()
            delivered = got[0] if lossless else d.results_received
            for w in ws:
                w.terminate()
                w.join(5)
            d.cleanup()
            out.append({"side": "build", "mode": label, "offered_rate": rate or "max", "offered": n,
                        "delivered": delivered, "delivered_fps": round(delivered / el, 1),
                        "delivered_share": round(delivered / max(n, 1), 3)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--rates", default="30,300,1000,3000,max")
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--side", default="both", choices=("both", "reference", "build"))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rates = [0 if r == "max" else float(r) for r in a.rates.split(",")]
    rows = []
    if a.side == "reference":
        rows = run_reference(a.reference, rates, a.seconds)
    else:
        if a.side == "both":
            if not os.path.isdir(a.reference) or not os.path.exists(REF_PY):
                print("reference or python3.9 missing: build side only", file=sys.stderr)
            else:
                env = {k: v for k, v in os.environ.items() if k not in ("PYTHONHOME", "PYTHONPATH")}
                r = subprocess.run([REF_PY, "-B", os.path.abspath(__file__), "--side", "reference",
                                    "--seconds", str(a.seconds), "--rates", a.rates, "--reference", a.reference],
                                   env=env, capture_output=True, text=True, timeout=600)
                if r.returncode != 0:
                    raise SystemExit(f"reference side failed: {r.stderr[-2000:]}")
                rows += [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
        rows += run_build(rates, a.seconds)
    host = {"cpus": len(os.sched_getaffinity(0)), "config": "configs[0]: 640x480 RGB, 2 CPU workers",
            "seconds": a.seconds}
    for row in rows:
        row.update(host)
        print(json.dumps(row), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
