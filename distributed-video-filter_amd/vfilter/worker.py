"""Worker runtime: the per-process frame loop (reference: worker.py:5-80).

Plugin API unchanged: subclass ``Worker`` and implement ``__call__(frame) -> bytes-like``
(worker.py:78-80).  The loop pulls frames from a distributor, calls the plugin, and pushes
results back.  Two protocols (``vfilter.wire``):

  v0  the reference loop, message for message (worker.py:35-76): send "READY" (NOBLOCK),
      poll 10 ms, receive [index, frame], call the plugin, send the 5-part result.  Use it
      against the reference's own distributor.py.
  v1  batched and pipelined: keep ``depth`` credit requests of ``batch`` frames in flight,
      hand each received batch to ``process_batch`` (default: the plugin per frame; a GPU
      plugin overrides it with one gathered device call), send one result message per
      batch.  Frames may arrive in a shared-memory ring (``vfilter.shm``); the worker then
      maps the ring, page-locks it once for the GPU and writes results in place.

Per-frame exceptions are caught, counted and reported (the reference prints and drops the
frame, worker.py:74-76; v1 additionally tells the distributor which index failed so an
in-order consumer does not wait for it).  One worker process owns one GPU.
"""
from __future__ import annotations

import collections
import os
import threading
import time
from typing import List, Optional, Sequence

import numpy as np

from . import transport as tp
from . import wire
from .shm import FrameRing


class WorkerFailed(RuntimeError):
    """Raised out of ``Worker.start`` after ``max_job_failures`` consecutive batches could not
    be collected (e.g. a sticky device error): the process should exit non-zero so that a
    supervisor starts a fresh one (the distributor re-queues the frames it never got back)."""


def _same_buffer(r, o) -> bool:
    """True when result ``r`` was written in place at the start of ring output view ``o``
    (the whole view, or, for a plugin whose results have their own size, a prefix of it)."""
    if o is None or not isinstance(r, np.ndarray):
        return False
    return r.nbytes <= o.nbytes and (r.nbytes == 0 or r.ctypes.data == o.ctypes.data)


class RingResults:
    """Results of a batch started from ring addresses (``Worker.submit_ring_batch``): every
    frame's result was written at the start of its slot's output half, ``nbytes`` long (an int64
    array), except the frames in ``errors`` ({position: message}) and in ``overflow``
    ({position: bytes-like}: results larger than the half, sent back as socket parts)."""
    __slots__ = ("nbytes", "errors", "overflow")

    def __init__(self, nbytes, errors=None, overflow=None):
        self.nbytes = np.asarray(nbytes, np.int64)
        self.errors = errors or {}
        self.overflow = overflow or {}


def ring_results(results: Sequence, outs: Sequence) -> RingResults:
    """``RingResults`` of per-frame results against their ring output views (a plugin's per-frame
    fallback inside a ring batch)."""
    nb = np.zeros(len(results), np.int64)
    errors, over = {}, {}
    for i, (r, o) in enumerate(zip(results, outs)):
        if isinstance(r, Exception):
            errors[i] = f"{type(r).__name__}: {r}"
        elif _same_buffer(r, o):
            nb[i] = r.nbytes
        else:
            rb = np.frombuffer(r, dtype=np.uint8)
            nb[i] = rb.nbytes
            if rb.nbytes <= o.nbytes:
                o[:rb.nbytes] = rb
            else:
                over[i] = r
    return RingResults(nb, errors, over)


class Worker:
    # True for a plugin whose results have their own size (a re-encoded JPEG): ring frames then
    # get their slot's whole output half to write into, and the result carries its length
    sized_results = False
    # consecutive batches whose collection raised before the loop gives up (WorkerFailed)
    max_job_failures = 8

    def __init__(self, host: str = "localhost", distribute_port: int = 5555, collect_port: int = 5556, *,
                 transport: str = "auto", protocol: str = "v1", batch: int = 1, depth: int = 0,
                 inflight: int = 1, verbose: bool = False):
        self.host = host
        self.distribute_port = distribute_port
        self.collect_port = collect_port
        self.running = False
        self.shutdown_requested = False
        self.process_id = os.getpid()                       # worker.py:14
        if protocol not in ("v0", "v1"):
            raise ValueError("protocol must be 'v0' (reference) or 'v1'")
        self.protocol = protocol
        self.batch = max(1, int(batch))
        # requests kept outstanding: one more than the batches that can be in processing
        self.depth = int(depth) if depth else max(1, int(inflight)) + 1
        self.verbose = verbose
        self.transport = tp.resolve(transport)
        self._zctx = tp.make_context(self.transport)
        self.dealer_socket = tp.DealerEnd(self.transport, host, distribute_port, self._zctx)   # worker.py:20-21
        self.collect_socket = tp.PushEnd(self.transport, host, collect_port, self._zctx)       # worker.py:24-25
        self.frames_processed = 0
        self.errors = 0
        self.inflight = max(1, int(inflight))  # batches in progress at once (protocol v1)
        self._tls = threading.local()
        self._ring_lock = threading.Lock()
        self._ring: Optional[FrameRing] = None
        self._ring_name: Optional[str] = None
        self.wid = f"{self.process_id}-{id(self):x}"  # ties results to this loop's requests
        if verbose:
            print(f"Worker started on ports {distribute_port} (request) and {collect_port} (send)")
            print(f"Process ID: {self.process_id}")

    # -- plugin API (worker.py:78-80) ----------------------------------------------------
    def __call__(self, frame):
        raise NotImplementedError("Subclasses must implement __call__ method")

    def process_batch(self, frames: Sequence, metas: Sequence[wire.FrameMeta], outs: Sequence) -> List:
        """Filter a batch.  ``outs[i]`` is a writable buffer of the input's size for frame i's
        result when the frame lives in the shared-memory ring, else None.  Returns, per frame,
        the result or an Exception instance for a frame that failed.  A result written in
        place is returned as ``outs[i]`` itself; any other bytes-like result (e.g. a JPEG,
        whose size differs from its input's) is copied into the slot's output half by the
        loop when it fits, else sent as a socket payload.  Default: the plugin, frame by frame."""
        results = []
        for f, o in zip(frames, outs):
            try:
                r = self(f)
                if o is not None and memoryview(r).nbytes == o.nbytes:
                    o[:] = np.frombuffer(r, dtype=np.uint8)
                    r = o  # in place; a result of another size goes back as its own buffer
                results.append(r)
            except Exception as e:  # worker.py:74-76
                results.append(e)
        return results

    def on_ring_attached(self, ring: FrameRing) -> None:
        """Hook: a GPU worker page-locks the ring here."""

    def numa_node(self) -> Optional[int]:
        """Hook: NUMA node the distributor should place this worker's ring slice on (a GPU
        worker returns its GPU's node)."""
        return None

    # -- loop --------------------------------------------------------------------------
    def start(self, max_frames: Optional[int] = None):
        """Run until ``running`` is cleared (signal) or ``max_frames`` results were sent."""
        self.running = True
        if self.verbose:
            print("Worker is running...")
        try:
            if self.protocol == "v0":
                self._loop_v0(max_frames)
            else:
                self._loop_v1(max_frames)
        finally:
            self.running = False

    def stop(self):
        self.running = False

    def close(self):
        self.running = False
        if self._ring is not None:
            self._ring.close()
            self._ring = None
        self.dealer_socket.close()
        self.collect_socket.close()
        if self._zctx is not None:
            self._zctx.term()

    def _loop_v0(self, max_frames):
        """worker.py:35-76, with the per-frame print gated by ``verbose``."""
        while self.running and (max_frames is None or self.frames_processed < max_frames):
            try:
                try:
                    self.dealer_socket.send(wire.encode_request(version=0))      # worker.py:39
                except BlockingIOError:
                    time.sleep(0.001)
                    continue
                except Exception as e:
                    if type(e).__name__ == "Again":
                        time.sleep(0.001)
                        continue
                    raise
                if self.dealer_socket.poll(10):                               # worker.py:46
                    start_time = time.time()                                  # worker.py:47
                    d = wire.decode_dispatch(self.dealer_socket.recv())       # worker.py:50-51
                    meta, frame = d.metas[0], d.payloads[0]
                    if self.verbose:
                        print(f"Processing frame {meta.index}")
                    try:
                        processed = self(frame)                               # worker.py:57
                    except Exception as e:                                    # worker.py:74-76
                        self.errors += 1
                        print(f"Error in worker: {e}")
                        continue
                    end_time = time.time()                                    # worker.py:59
                    self.collect_socket.send(wire.encode_result_v0(meta.index, self.process_id,
                                                                   start_time, end_time, processed))
                    self.frames_processed += 1
            except Exception as e:
                print(f"Error in worker: {e}")
                continue

    @property
    def last_spans(self) -> List[dict]:
        """GPU spans of the batch the calling thread processed last (set by process_batch)."""
        return getattr(self._tls, "spans", [])

    @last_spans.setter
    def last_spans(self, spans: List[dict]) -> None:
        self._tls.spans = spans

    def _attach_ring(self, name: str, slot_bytes: int) -> FrameRing:
        with self._ring_lock:
            if self._ring is None or self._ring_name != name:
                if self._ring is not None:
                    self._ring.close()
                self._ring = FrameRing(name=name, slot_bytes=slot_bytes)
                self._ring_name = name
                self.on_ring_attached(self._ring)
            return self._ring

    # -- asynchronous batch hooks (a GPU plugin overrides these) ----------------------------
    def request_credit(self) -> int:
        """Frames asked for by the next request (protocol v1): ``batch``; a plugin may adapt it
        to the frames it sees (InverterWorker with ``batch=0``)."""
        return self.batch

    def submit_ring_batch(self, ring: FrameRing, cols: np.ndarray):
        """Hook: start a v2 batch whose every frame is in ``ring`` from its records (``cols``:
        wire.COLS, slots and sizes as arrays) and return a handle whose ``poll_batch`` results
        are a ``RingResults`` -- no Python object per frame (a GPU plugin computes the slots'
        addresses from the ring's base).  None: use ``submit_batch`` on per-frame views."""
        return None

    def submit_batch(self, frames: Sequence, metas: Sequence[wire.FrameMeta], outs: Sequence):
        """Start a batch and return a handle for ``poll_batch``.  Default: run
        ``process_batch`` now (synchronously)."""
        self.last_spans = []
        try:
            results = self.process_batch(frames, metas, outs)
        except Exception as e:
            results = [e] * len(frames)
        return ("done", results, self.last_spans)

    def poll_batch(self, handle, block: bool):
        """(results, spans) once the batch behind ``handle`` is complete, else None (only
        when ``block`` is False)."""
        return handle[1], handle[2]

    def _start_job(self, d: wire.Dispatch, start_time: float):
        ring = None
        if d.ring is not None:
            ring = self._attach_ring(d.ring["name"], int(d.ring["slot_bytes"]))
        frames, outs = [], []
        if d.cols is not None and ring is not None and len(d.cols) and bool((d.cols["slot"] >= 0).all()):
            h = self.submit_ring_batch(ring, d.cols)
            if h is not None:  # the whole batch from addresses
                return d, start_time, h, ring, None
        if d.cols is not None:  # v2: slots and sizes straight from the records
            slots, nbs = d.cols["slot"].tolist(), d.cols["nbytes"].tolist()
            whole = ring.slot_bytes if (ring is not None and self.sized_results) else None
            for s, nb, p in zip(slots, nbs, d.payloads):
                if s >= 0:
                    frames.append(ring.in_view(s, nb))
                    outs.append(ring.out_view(s, whole or nb))
                else:
                    frames.append(p)
                    outs.append(None)
        else:
            for m, p in zip(d.metas, d.payloads):
                if m.slot is not None:
                    frames.append(ring.in_view(m.slot, m.nbytes))
                    # a plugin whose results have their own size (JPEG) gets the whole output half
                    outs.append(ring.out_view(m.slot, ring.slot_bytes if self.sized_results else m.nbytes))
                else:
                    frames.append(p)
                    outs.append(None)
        if self.verbose:
            print(f"Processing frames {[m.index for m in d.metas]}")
        return d, start_time, self.submit_batch(frames, d.metas, outs), ring, outs

    def _finish_job(self, job, block: bool) -> bool:
        d, start_time, handle, ring, outs = job
        got = self.poll_batch(handle, block)
        if got is None:
            return False
        results, spans = got
        end_time = time.time()
        if isinstance(results, RingResults):
            return self._finish_ring(d, start_time, end_time, results, spans)
        if d.cols is not None:
            return self._finish_v2(d, start_time, end_time, results, spans, ring, outs)
        metas, payloads = [], []
        for m, r, o in zip(d.metas, results, outs):
            om = wire.FrameMeta(index=m.index, nbytes=m.nbytes, shape=m.shape, slot=m.slot,
                                start=start_time, end=end_time)
            payload = None
            if isinstance(r, Exception):
                om.error = f"{type(r).__name__}: {r}"
                self.errors += 1
                print(f"Error in worker: frame {m.index}: {r}")
            elif m.slot is None:
                payload = r
            elif _same_buffer(r, o):
                if r.nbytes != m.nbytes:  # written in place, with its own length
                    om.nbytes = r.nbytes
                    om.shape = None
            else:
                # a result of its own size (JPEG): into the slot's output half when it fits,
                # else back over the socket; either way the result carries its length
                rb = np.frombuffer(r, dtype=np.uint8)
                om.nbytes = rb.nbytes
                om.shape = None
                if rb.nbytes <= ring.slot_bytes:
                    ring.out_view(m.slot, rb.nbytes)[:] = rb
                else:
                    om.slot = None
                    payload = r
            payloads.append(payload)
            metas.append(om)
        try:
            self.collect_socket.send(wire.encode_result(self.process_id, metas, payloads, spans, wid=self.wid))
        except Exception as e:  # the distributor re-queues frames whose result never arrives
            self.errors += 1
            print(f"Error in worker: could not send results {[m.index for m in metas]}: {e}")
            return True
        self.frames_processed += len(metas)
        return True

    def _finish_ring(self, d, start_time, end_time, res: RingResults, spans) -> bool:
        """``_finish_job`` for a batch started by ``submit_ring_batch``: the records as dispatched
        with each result's length, array operations only (plus the rare error / overflow)."""
        cols = d.cols.copy()
        changed = res.nbytes != cols["nbytes"]
        cols["nbytes"] = res.nbytes
        cols["ndim"][changed] = -1  # a result of its own size has no shape
        payloads = []
        for i in sorted(res.overflow):
            if i not in res.errors:
                cols["slot"][i] = -1
                payloads.append(res.overflow[i])
        for i, msg in res.errors.items():
            self.errors += 1
            print(f"Error in worker: frame {int(cols['index'][i])}: {msg}")
        try:
            self.collect_socket.send(wire.encode_result2(self.process_id, cols, payloads, start_time, end_time,
                                                         wid=self.wid, errors=res.errors, spans=spans))
        except Exception as e:  # the distributor re-queues frames whose result never arrives
            self.errors += 1
            print(f"Error in worker: could not send results {cols['index'].tolist()}: {e}")
            return True
        self.frames_processed += len(cols)
        return True

    def _finish_v2(self, d, start_time, end_time, results, spans, ring, outs) -> bool:
        """``_finish_job`` for a v2 dispatch: the result records are the dispatch's, with each
        result's own length (and slot -1 where it goes back as a part)."""
        cols = d.cols.copy()
        slots, nbs = cols["slot"].tolist(), cols["nbytes"].tolist()
        errors, payloads = {}, []
        for i, (r, o) in enumerate(zip(results, outs)):
            if r is o and o.nbytes == nbs[i]:  # written in place, the input's length
                continue
            if isinstance(r, Exception):
                errors[i] = f"{type(r).__name__}: {r}"
                self.errors += 1
                print(f"Error in worker: frame {int(cols['index'][i])}: {r}")
            elif slots[i] < 0:
                payloads.append(r)
                cols["nbytes"][i] = memoryview(r).nbytes
            elif _same_buffer(r, o):
                if r.nbytes != nbs[i]:  # written in place, with its own length
                    cols["nbytes"][i] = r.nbytes
                    cols["ndim"][i] = -1
            else:  # a result of its own size (JPEG): into the slot when it fits, else a part
                rb = np.frombuffer(r, dtype=np.uint8)
                cols["nbytes"][i] = rb.nbytes
                cols["ndim"][i] = -1
                if rb.nbytes <= ring.slot_bytes:
                    ring.out_view(slots[i], rb.nbytes)[:] = rb
                else:
                    cols["slot"][i] = -1
                    payloads.append(r)
        try:
            self.collect_socket.send(wire.encode_result2(self.process_id, cols, payloads, start_time, end_time,
                                                         wid=self.wid, errors=errors, spans=spans))
        except Exception as e:  # the distributor re-queues frames whose result never arrives
            self.errors += 1
            print(f"Error in worker: could not send results {cols['index'].tolist()}: {e}")
            return True
        self.frames_processed += len(cols)
        return True

    def _fail_job(self, job, exc: Exception) -> None:
        """A batch whose collection raised: report every frame of it as failed (so an in-order
        consumer does not wait for them) and drop the job."""
        d, start_time = job[0], job[1]
        if d.cols is not None:
            msg = f"{type(exc).__name__}: {exc}"
            self.errors += len(d.cols)
            print(f"Error in worker: batch {d.cols['index'].tolist()}: {msg}")
            try:
                self.collect_socket.send(wire.encode_result2(self.process_id, d.cols, [], start_time, time.time(),
                                                             wid=self.wid, errors={i: msg for i in range(len(d.cols))}))
            except Exception as e:  # the distributor re-queues frames whose result never arrives
                print(f"Error in worker: could not report the failed batch: {e}")
            return
        metas = [wire.FrameMeta(index=m.index, nbytes=m.nbytes, shape=m.shape, slot=m.slot,
                                start=start_time, end=time.time(), error=f"{type(exc).__name__}: {exc}")
                 for m in d.metas]
        self.errors += len(metas)
        print(f"Error in worker: batch {[m.index for m in d.metas]}: {type(exc).__name__}: {exc}")
        try:
            self.collect_socket.send(wire.encode_result(self.process_id, metas, [None] * len(metas), [],
                                                        wid=self.wid))
        except Exception as e:  # the distributor re-queues frames whose result never arrives
            print(f"Error in worker: could not report the failed batch: {e}")

    def _collect_jobs(self, jobs, block_when: int) -> None:
        """Finish jobs at the head of ``jobs`` in arrival order.  A job whose collection raises
        is popped and reported as failed (not retried); after ``max_job_failures`` in a row the
        loop raises WorkerFailed."""
        while jobs:
            try:
                if not self._finish_job(jobs[0], block=len(jobs) >= block_when):
                    return
                jobs.popleft()
                self._job_failures = 0
            except Exception as e:
                self._fail_job(jobs.popleft(), e)
                self._job_failures = getattr(self, "_job_failures", 0) + 1
                if self._job_failures >= self.max_job_failures:
                    raise WorkerFailed(f"{self._job_failures} batches in a row failed; last: "
                                       f"{type(e).__name__}: {e}") from e

    def _loop_v1(self, max_frames):
        """Credit loop: ``depth`` requests outstanding; up to ``inflight`` received batches
        in progress at once (a GPU plugin submits them asynchronously, so the device works
        on batch i while this loop receives and submits batch i+1); results go out in
        arrival order."""
        outstanding = 0
        jobs: "collections.deque" = collections.deque()
        numa = self.numa_node()
        while self.running and (max_frames is None or self.frames_processed < max_frames):
            try:
                while outstanding < self.depth:
                    self.dealer_socket.send(wire.encode_request(self.request_credit(), shm=True, wid=self.wid,
                                                                numa=numa, wire=wire.WIRE))
                    outstanding += 1
                self._collect_jobs(jobs, self.inflight)
                if len(jobs) >= self.inflight:
                    continue
                # with batches in flight, wake every 0.2 ms to collect the one that finished
                # (a 1 ms wait here delayed every result by up to a batch's GPU time)
                if not self.dealer_socket.poll(0.2 if jobs else 10):
                    continue
                parts = self.dealer_socket.recv()
                start_time = time.time()
                try:
                    d = wire.decode_dispatch(parts)
                except Exception as e:
                    print(f"Error in worker: bad dispatch message: {e}")
                    continue
                if d.version >= 1:
                    outstanding -= 1
                jobs.append(self._start_job(d, start_time))
            except WorkerFailed:
                raise
            except Exception as e:  # worker.py:74-76: report and keep serving
                self.errors += 1
                print(f"Error in worker: {type(e).__name__}: {e}")
                time.sleep(0.01)
        while jobs:  # finish what was accepted before stopping
            job = jobs.popleft()
            try:
                self._finish_job(job, block=True)
            except Exception as e:
                self._fail_job(job, e)
