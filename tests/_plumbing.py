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
    delay = 0.0        # per frame
    batch_delay = 0.0  # per batch: a fixed cost per call, like a GPU launch + host staging

    def process_batch(self, frames, metas, outs):
        if self.batch_delay > 0:
            import time
            time.sleep(self.batch_delay)
        return super().process_batch(frames, metas, outs)

    def __call__(self, frame):
        from oracle import oracle
        if self.delay > 0:
            import time
            time.sleep(self.delay)
        return oracle.invert_bytes(frame)


class ResizingWorker(OracleWorker):
    """A plugin whose result size differs from its input's, like a re-encoded JPEG: the
    inverted bytes plus a 7-byte trailer, or half of them for frames of 64 bytes or less."""

    def __call__(self, frame):
        from oracle import oracle
        x = oracle.invert_bytes(frame)
        return x[: len(x) // 2] if len(x) <= 64 else x + b"trailer"


class _RingMixin:
    """The worker's ring form (Worker.submit_ring_batch): the whole batch from its records,
    results landing in the slots' output halves (RingResults), as the GPU plugin's do."""

    def submit_ring_batch(self, ring, cols):
        from vfilter.worker import ring_results
        slots, nbs = cols["slot"].tolist(), cols["nbytes"].tolist()
        outs = [ring.out_view(s_, ring.slot_bytes) for s_ in slots]
        results = []
        for s_, n_ in zip(slots, nbs):
            try:
                results.append(self(ring.in_view(s_, n_)))
            except Exception as e:
                results.append(e)
        return ("ring", ring_results(results, outs))

    def poll_batch(self, handle, block):
        if handle[0] == "ring":
            return handle[1], []
        return super().poll_batch(handle, block)


class RingOracleWorker(_RingMixin, OracleWorker):
    pass


class RingResizingWorker(_RingMixin, ResizingWorker):
    pass


def _watch(stop_event, worker):
    stop_event.wait()
    worker.stop()


def run_worker(dport, cport, stop_event, protocol="v1", batch=4, transport="tcp", kind="oracle",
               delay=0.0, device=0, use_jpeg=False, batch_delay=0.0, inflight=1):
    if kind == "gpu":
        from vfilter.inverter import InverterWorker
        w = InverterWorker("127.0.0.1", dport, cport, delay, use_jpeg=use_jpeg, device=device,
                           install_signal_handlers=False, batch=batch, protocol=protocol,
                           transport=transport)
    else:
        cls = {"resizing": ResizingWorker, "ring": RingOracleWorker,
               "ring_resizing": RingResizingWorker}.get(kind, OracleWorker)
        w = cls("127.0.0.1", dport, cport, batch=batch, protocol=protocol, transport=transport, inflight=inflight)
        w.delay = delay
        w.batch_delay = batch_delay
    threading.Thread(target=_watch, args=(stop_event, w), daemon=True).start()
    try:
        w.start()
    finally:
        w.close()


class _Stops:
    """One stop event per worker process: setting an event a killed process was waiting on
    would block forever (multiprocessing's Condition waits for the sleeper to acknowledge)."""

    def __init__(self, events):
        self.events = events

    def set_for(self, procs):
        for ev, p in zip(self.events, procs):
            if p.is_alive():
                ev.set()


def spawn_workers(n, dport, cport, **kw):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    stops = _Stops([ctx.Event() for _ in range(n)])
    procs = [ctx.Process(target=run_worker, args=(dport, cport, ev), kwargs=kw, daemon=True)
             for ev in stops.events]
    for p in procs:
        p.start()
    return stops, procs


def stop_workers(stop, procs, timeout=10.0):
    stop.set_for(procs)
    for p in procs:
        p.join(timeout)
        if p.is_alive():
            p.terminate()
            p.join(2.0)
