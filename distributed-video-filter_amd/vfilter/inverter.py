"""InverterWorker: the reference's filter plugin on the MI355X (reference: inverter.py:9-64).

``InverterWorker.__call__(frame_bytes) -> bytes`` keeps the reference's contract
(inverter.py:29-46): decode (JPEG, or raw bytes), optional artificial ``delay``, invert,
re-encode.  The invert is ``vfilter.bitwise_not`` — hand-written gfx950 kernels via
libvfilter_hip.so — instead of ``cv2.bitwise_not`` (inverter.py:41).  ``process_batch``
inverts a whole dispatched batch with ONE gathered device call (H2D || kernel || D2H), and
when frames arrive in the shared-memory ring the ring is page-locked once so the GPU DMAs
straight from/to it.

Raw frames: the reference reshapes every raw frame to 480x480x3 (inverter.py:34) and drops
any other size with a ValueError (worker.py:74-76).  The invert needs no shape, so any size
is accepted here; the v1 wire format carries the shape when a producer provides it.

JPEG (the reference default, ``use_jpeg=True``, inverter.py:10): ``vfilter.jpeg.TurboJPEG``
(PyTurboJPEG's API on the gfx950 baseline-JPEG codec, bit-exact with libjpeg-turbo) replaces
``turbojpeg.TurboJPEG`` (inverter.py:7,13).  A batch runs decode -> invert -> encode as one
fused GPU pass; ``submit_batch`` stages and queues it (vf_jpeg_invert_submit) and returns, so
the worker loop receives and stages batch k+1 while batch k is on the GPU — one host thread,
two codecs (each in-flight batch holds its own codec, stream and buffers).
"""
from __future__ import annotations

import argparse
import os
import signal
import time
from typing import List, Optional, Sequence

import numpy as np

from . import wire
from ._lib import Context, default_device
from .jpeg import TurboJPEG
from .worker import RingResults, Worker, WorkerFailed, ring_results


# JPEG frames up to this many bytes on average are asked for in batches of SMALL_CREDIT: a
# batch's host work (parse, ~25 launches) is then spread over twice the frames (the reference
# app's 512 x 512 crops: +30-50 % through the system); larger frames in batches
# of CREDIT
SMALL_JPEG_BYTES = 64 * 1024
CREDIT, SMALL_CREDIT = 32, 64


def auto_credit(mean_jpeg_bytes: float) -> int:
    """The batch a JPEG worker started with ``batch=0`` asks for, from its frames' mean size."""
    return SMALL_CREDIT if 0 < mean_jpeg_bytes <= SMALL_JPEG_BYTES else CREDIT


class InverterWorker(Worker):
    def __init__(self, host: str = "localhost", distribute_port: int = 5555, collect_port: int = 5556,
                 delay: float = 0.0, use_jpeg: bool = True, *, device: Optional[int] = None,
                 max_frame_bytes: int = 3840 * 2160 * 3, install_signal_handlers: bool = True,
                 tj_version: int = 3, **worker_kw):
        # batches in progress at once: raw, batch i on the GPU while batch i+1 is received;
        # JPEG, three, since the kernels of batches on separate codecs overlap (1080p worker
        # form 24.6 k fps with 3 in flight vs 21.4 k with 2: profiles/r02_jpeg_depth.jsonl)
        if worker_kw.get("inflight") is None:
            worker_kw["inflight"] = 3 if use_jpeg else 2
        # batch=0: JPEG requests adapt to the frames (auto_credit); raw frames in batches of 32
        self.auto_credit = use_jpeg and worker_kw.get("batch") == 0
        if worker_kw.get("batch") == 0:
            worker_kw["batch"] = CREDIT
        self._jpeg_bytes = 0.0  # running mean of the JPEG frames submitted (auto_credit)
        super().__init__(host, distribute_port, collect_port, **worker_kw)
        self.delay = delay
        self.device = default_device() if device is None else device
        self.ctx = Context(self.device, max_frame_bytes=max_frame_bytes,
                           max_batch=max(1, SMALL_CREDIT if self.auto_credit else self.batch))
        # inverter.py:13 — TurboJPEG() with PyTurboJPEG's defaults, on this worker's GPU
        self.jpeg = TurboJPEG(ctx=self.ctx, tj_version=tj_version) if use_jpeg else None
        # re-encoded JPEGs written straight into their ring slots (VF_JPEG_SCATTER=0: copied by the loop)
        self.sized_results = self.jpeg is not None and os.environ.get("VF_JPEG_SCATTER", "1") != "0"
        self._registered: List[int] = []
        if self.jpeg is None:  # raw frames off the socket land in the pinned arena: read in place
            self.dealer_socket.recv_alloc = lambda n: self.ctx.pinned_empty((n,))
        if install_signal_handlers:                                  # inverter.py:16-18
            signal.signal(signal.SIGINT, self._signal_handler)
            signal.signal(signal.SIGTERM, self._signal_handler)
        if self.verbose:
            print("Inverter worker started")
            print(f"Processing delay: {self.delay} seconds")

    def _signal_handler(self, signum, frame):                        # inverter.py:22-27
        if not self.shutdown_requested:
            self.shutdown_requested = True
            print(f"\nReceived signal {signum}, shutting down...")
            self.running = False

    # -- one frame (inverter.py:29-46) ------------------------------------------------------
    def __call__(self, frame_bytes):
        if self.jpeg and self.delay <= 0:
            return self.jpeg.invert(frame_bytes)                    # inverter.py:32 -> :41 -> :44, fused
        if self.jpeg:
            frame = self.jpeg.decode(frame_bytes)                   # inverter.py:32
        else:
            frame = np.frombuffer(frame_bytes, dtype=np.uint8)      # inverter.py:34, any size
        if self.delay > 0:                                          # inverter.py:37-38
            time.sleep(self.delay)
        out = self.ctx.pinned_empty_like(frame)  # written directly over PCIe, recycled after the send
        if frame.nbytes:
            self.ctx.invert_host(frame, out, frame.nbytes)          # inverter.py:41
        if self.jpeg:
            return self.jpeg.encode(out)                            # inverter.py:44
        return out                                                   # inverter.py:46 (buffer, no copy)

    # -- a dispatched batch: one gathered device call ------------------------------------
    def process_batch(self, frames: Sequence, metas: Sequence[wire.FrameMeta], outs: Sequence) -> List:
        if self.jpeg and self.delay <= 0:
            # the whole batch in one fused GPU pass; results are JPEGs of their own size (the
            # loop puts ring frames' results into their slots, see Worker._finish_job)
            try:
                return self.jpeg.invert_batch(list(frames))
            except Exception:  # retry frame by frame so a bad frame fails alone (worker.py:74-76)
                return super().process_batch(frames, metas, outs)
        if self.jpeg:
            return super().process_batch(frames, metas, outs)
        if self.delay > 0:
            time.sleep(self.delay * len(frames))
        srcs, dsts, sizes, results = [], [], [], []
        for f, o in zip(frames, outs):
            src = f if isinstance(f, np.ndarray) else np.frombuffer(f, dtype=np.uint8)
            dst = o if o is not None else np.empty(src.nbytes, np.uint8)
            srcs.append(src)
            dsts.append(dst)
            sizes.append(src.nbytes)
            results.append(dst)
        t_call = time.time()
        try:
            self.ctx.invert_frames_host(srcs, dsts, sizes)
        except Exception as e:
            return [e] * len(frames)
        self.last_spans = gpu_spans(self.ctx.last_timeline(), t_call)
        return results

    # -- asynchronous submission ---------------------------------------------------------
    def submit_batch(self, frames: Sequence, metas: Sequence[wire.FrameMeta], outs: Sequence):
        """Queue the batch with vf_invert_frames_async and return to receiving at once: the
        context's engine thread streams consecutive batches through the GPU back to back.
        Ring frames (page-locked) are inverted in place (zero-copy); socket payloads are staged.
        JPEG batches are queued on a codec of their own (vf_jpeg_invert_submit: fused decode ->
        invert -> encode) and collected later, ring frames' results straight into their slots."""
        if self.jpeg:
            self._note_jpeg_bytes(float(sum(len(f) for f in frames)), len(frames))
        if self.jpeg and self.delay <= 0:
            try:  # staged and queued now; the loop receives the next batch while this one runs
                return ("jpeg", self.jpeg.invert_batch_submit(list(frames)), list(frames), list(outs))
            except Exception:  # a frame the host parser refuses: frame by frame (worker.py:74-76)
                return ("done", super().process_batch(frames, metas, outs), [])
        if self.jpeg or self.delay > 0:
            return super().submit_batch(frames, metas, outs)
        srcs, dsts = [], []
        for f, o in zip(frames, outs):
            src = f if isinstance(f, np.ndarray) else np.frombuffer(f, dtype=np.uint8)
            srcs.append(src)
            dsts.append(o if o is not None else np.empty(src.nbytes, np.uint8))
        try:
            ticket = self.ctx.invert_frames_async(srcs, dsts, [s.nbytes for s in srcs])
        except Exception as e:
            return ("done", [e] * len(frames), [])
        return ("gpu", ticket, srcs, dsts)  # srcs kept alive until the ticket completes

    def _note_jpeg_bytes(self, total: float, n: int) -> None:
        if n:
            m = total / n
            self._jpeg_bytes = m if not self._jpeg_bytes else 0.75 * self._jpeg_bytes + 0.25 * m

    def request_credit(self) -> int:
        return auto_credit(self._jpeg_bytes) if self.auto_credit else self.batch

    def submit_ring_batch(self, ring, cols):
        """The worker's ring form: every frame of the batch in this worker's page-locked ring
        slice, so the inputs and outputs are base + slot arithmetic -- one address array each,
        no ndarray per frame (at 512 x 512 JPEG, 60-80 k frames/s, the per-frame Python of the
        view path was the worker's bound).  Raw: one zero-copy launch over the slots; JPEG: one
        fused codec batch whose results are scattered into the slots' output halves."""
        if self.delay > 0:
            return None
        sb = ring.slot_bytes
        slots, nbs = cols["slot"], cols["nbytes"]
        if len(slots) and (int(slots.min()) < 0 or int(slots.max()) >= ring.nslots or int(nbs.min()) < 0
                           or int(nbs.max()) > sb):
            return None  # a record outside this ring slice: never a raw GPU address; the views path
        ina = np.uint64(ring.base_address) + cols["slot"].astype(np.uint64) * np.uint64(2 * sb)
        nb = cols["nbytes"]
        if self.jpeg:
            self._note_jpeg_bytes(float(nb.sum()), len(nb))
            try:
                t = self.jpeg.invert_batch_submit_addrs(ina, nb)
            except Exception:  # a frame the host parser refuses: the per-frame views path
                return None
            return ("jpeg_ring", t, ina + np.uint64(sb), sb, ring, cols)
        try:
            t = self.ctx.invert_frames_async_addrs(ina, ina + np.uint64(sb), nb)
        except Exception:
            return None
        return ("gpu_ring", t, nb, time.time())

    def poll_batch(self, handle, block: bool):
        if handle[0] == "jpeg_ring":
            _, ticket, outa, sb, ring, cols = handle
            if not block and not self.jpeg.invert_batch_ready(ticket):
                return None
            try:
                sizes, over = self.jpeg.invert_batch_result_into_addrs(ticket, outa, sb)
                return RingResults(sizes, {}, over), []
            except Exception:  # e.g. a truncated stream the GPU found: frame by frame
                slots, nbs = cols["slot"].tolist(), cols["nbytes"].tolist()
                frames = [ring.in_view(s_, n_) for s_, n_ in zip(slots, nbs)]
                outs = [ring.out_view(s_, sb) for s_ in slots]
                return ring_results(Worker.process_batch(self, frames, [None] * len(frames), outs), outs), []
        if handle[0] == "gpu_ring":
            _, ticket, nb, t_call = handle
            if not block and not self.ctx.query(ticket):
                return None
            try:
                ms = self.ctx.wait(ticket)
            except Exception as e:
                return RingResults(nb, {i: f"{type(e).__name__}: {e}" for i in range(len(nb))}), []
            t_end = time.time()
            spans = gpu_spans(self.ctx.last_timeline(), t_end - ms / 1e3) if ms >= 0 else []
            return RingResults(nb), spans
        if handle[0] == "jpeg":
            _, ticket, frames, outs = handle
            if not block and not self.jpeg.invert_batch_ready(ticket):
                return None
            try:
                if any(o is not None for o in outs):  # ring frames: straight into their slots
                    return self.jpeg.invert_batch_result_into(ticket, outs), []
                return self.jpeg.invert_batch_result(ticket), []
            except Exception:  # e.g. a truncated stream the GPU found: frame by frame
                return Worker.process_batch(self, frames, [None] * len(frames), [None] * len(frames)), []
        if handle[0] != "gpu":
            return super().poll_batch(handle, block)
        _, ticket, _srcs, dsts = handle
        if not block and not self.ctx.query(ticket):
            return None
        try:
            ms = self.ctx.wait(ticket)
        except Exception as e:
            return [e] * len(dsts), []
        t_end = time.time()
        spans = gpu_spans(self.ctx.last_timeline(), t_end - ms / 1e3) if ms >= 0 else []
        return dsts, spans

    def numa_node(self):
        from .numa import gpu_numa_node
        return gpu_numa_node(self.device)

    def on_ring_attached(self, ring) -> None:
        """Page-lock the ring (this worker's own slice, with the distributor's per-worker
        layout) once: the slot pipeline then DMAs straight from the input halves and into the
        output halves (no staging copy)."""
        try:
            self._registered.append(self.ctx.host_register(ring.buf, ring.nbytes))
        except Exception as e:  # still correct through staging, just slower
            print(f"Inverter worker: could not page-lock ring {ring.name}: {e}")

    def close(self):
        for a in self._registered:
            try:
                self.ctx.host_unregister(a)
            except Exception:
                pass
        self._registered.clear()
        super().close()
        self.ctx.close()


def gpu_spans(timeline, t_call: float) -> List[dict]:
    """Per-chunk {H2D, kernel, D2H} spans in wall-clock seconds: the call's start event is
    taken as ``t_call`` (the host time just before the call)."""
    spans = []
    for nbytes, h0, k0, k1, d1 in timeline:
        if min(h0, k0, k1, d1) < 0:
            continue
        spans.append({"name": "H2D", "begin": t_call + h0 / 1e3, "end": t_call + k0 / 1e3, "bytes": nbytes})
        spans.append({"name": "kernel", "begin": t_call + k0 / 1e3, "end": t_call + k1 / 1e3, "bytes": nbytes})
        spans.append({"name": "D2H", "begin": t_call + k1 / 1e3, "end": t_call + d1 / 1e3, "bytes": nbytes})
    return spans


def pin_to_gpu_node(device=None) -> bool:
    """Keep the worker process on the CPUs of its GPU's NUMA node (VF_WORKER_PIN=0: leave it).
    Done before the context exists, so the codec's and the copy pool's threads inherit it: the
    host half of a batch (parsing, staging, the ring slice the distributor bound to that node)
    then stays on one socket instead of wherever the scheduler last put the thread."""
    if os.environ.get("VF_WORKER_PIN", "1") == "0":
        return False
    from . import numa
    from ._lib import default_device
    cpus = numa.node_cpus(numa.gpu_numa_node(default_device() if device is None else device))
    if not cpus:
        return False
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        return False
    return True


def main(argv=None):
    """inverter.py:48-61 plus the GPU worker's knobs."""
    ap = argparse.ArgumentParser(description="Inverter worker for video processing (MI355X backend)")
    ap.add_argument("--distribute-port", type=int, default=5555,
                    help="Port to request frames from webcam app (default: 5555)")
    ap.add_argument("--collect-port", type=int, default=5556,
                    help="Port to send inverted frames to webcam app (default: 5556)")
    ap.add_argument("--delay", type=float, default=0.0,
                    help="Artificial processing delay in seconds (default: 0.0)")
    ap.add_argument("--host", default="localhost", help="distributor host (reference: hard-coded localhost)")
    ap.add_argument("--raw", action="store_true",
                    help="raw H x W x 3 frames (use_jpeg=False); default JPEG frames, as the reference CLI")
    ap.add_argument("--jpeg", action="store_true", help=argparse.SUPPRESS)  # the default; kept for old scripts
    ap.add_argument("--device", type=int, default=None, help="GPU ordinal (default: VF_DEVICE / LOCAL_RANK / 0)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per request (protocol v1); default 0: JPEG 64 while the frames average "
                         "<= 64 KB (the reference app's 512 x 512 crops), else 32 (inverter.auto_credit); "
                         "raw 32")
    ap.add_argument("--inflight", type=int, default=None,
                    help="batches in progress at once (protocol v1; default 3 for JPEG, 2 for raw)")
    ap.add_argument("--protocol", choices=("v0", "v1"), default="v1",
                    help="v0 = the reference wire protocol (use against the reference distributor.py)")
    ap.add_argument("--transport", choices=("auto", "zmq", "tcp"), default="auto")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args(argv)
    pin_to_gpu_node(args.device)
    worker = InverterWorker(args.host, args.distribute_port, args.collect_port, args.delay,
                            use_jpeg=not args.raw, device=args.device, batch=args.batch, inflight=args.inflight,
                            protocol=args.protocol, transport=args.transport, verbose=args.verbose)
    try:
        worker.start()
    except WorkerFailed as e:  # a fresh process, not a re-exec: let the supervisor restart it
        print(f"Inverter worker: giving up: {e}")
        raise SystemExit(3)
    finally:
        worker.close()


if __name__ == "__main__":
    main()
