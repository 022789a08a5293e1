"""Helpers for the plumbing tests: worker processes with a test plugin.

``OracleWorker`` is a plugin (the reference's extension point, worker.py:78-80) whose
arithmetic is the CPU oracle — test infrastructure, so the plumbing (dispatch, sharding,
rings, reassembly) can be tested on a machine without a GPU.  ``GpuWorker`` runs the
product ``InverterWorker`` (libvfilter_hip.so) and is used only by ``-m gpu`` tests.
"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "distributed-video-filter_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from vfilter.worker import Worker  # noqa: E402


class OracleWorker(Worker):
    def __call__(self, frame):
        from oracle import oracle
        return oracle.invert_bytes(frame)


def _watch(stop_event, worker):
    stop_event.wait()
    worker.stop()


def run_worker(dport, cport, stop_event, protocol="v1", batch=4, transport="tcp", kind="oracle",
               delay=0.0, device=0, use_jpeg=False):
    if kind == "gpu":
        from vfilter.inverter import InverterWorker
        w = InverterWorker("127.0.0.1", dport, cport, delay, use_jpeg=use_jpeg, device=device,
                           install_signal_handlers=False, batch=batch, protocol=protocol,
                           transport=transport)
    else:
        w = OracleWorker("127.0.0.1", dport, cport, batch=batch, protocol=protocol, transport=transport)
    threading.Thread(target=_watch, args=(stop_event, w), daemon=True).start()
    try:
        w.start()
    finally:
        w.close()


def spawn_workers(n, dport, cport, **kw):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    stop = ctx.Event()
    procs = [ctx.Process(target=run_worker, args=(dport, cport, stop), kwargs=kw, daemon=True) for _ in range(n)]
    for p in procs:
        p.start()
    return stop, procs


def stop_workers(stop, procs, timeout=10.0):
    stop.set()
    for p in procs:
        p.join(timeout)
        if p.is_alive():
            p.terminate()
            p.join(2.0)
