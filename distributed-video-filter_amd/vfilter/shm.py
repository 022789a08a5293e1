"""Shared-memory frame ring: the same-node data plane between distributor and workers.

The reference moves every frame through ZeroMQ/TCP twice (dispatch and result,
distributor.py:236-238 / worker.py:63-67): two socket copies per direction, ~2-4.5 GB/s
per stream, far below what one MI355X takes in over PCIe (~50 GB/s per
direction).  Here the distributor writes each frame once into a slot of a ring in POSIX
shared memory and sends only the slot number; the worker page-locks the whole ring once
with ``hipHostRegister`` (``vf_host_register``), so the GPU DMA reads the input straight
out of the slot and writes the result straight into the slot's output half — no host copy
in the worker at all.

Layout: ``nslots`` slots of ``2 * slot_bytes`` each: [input | output], 4 KiB aligned.
"""
from __future__ import annotations

import threading
from multiprocessing import shared_memory
from typing import List, Optional

import numpy as np

PAGE = 4096


def _round_up(n: int, a: int = PAGE) -> int:
    return (n + a - 1) // a * a


class FrameRing:
    def __init__(self, nslots: int = 0, slot_bytes: int = 0, name: Optional[str] = None):
        if name is None:
            if nslots < 1 or slot_bytes < 1:
                raise ValueError("FrameRing: nslots and slot_bytes must be positive")
            self.slot_bytes = _round_up(slot_bytes)
            self.nslots = nslots
            size = self.nslots * 2 * self.slot_bytes
            free = shm_free_bytes()
            if free is not None and size > free:
                # a tmpfs segment larger than the free space maps fine and SIGBUSes on write
                raise MemoryError(f"FrameRing of {size} B exceeds free /dev/shm ({free} B)")
            self.shm = shared_memory.SharedMemory(create=True, size=size)
            self.owner = True
        else:
            self.shm = _attach(name)
            self.owner = False
            self.slot_bytes = slot_bytes
            self.nslots = self.shm.size // (2 * slot_bytes)
        self.name = self.shm.name
        self.buf = np.ndarray((self.shm.size,), dtype=np.uint8, buffer=self.shm.buf)
        self._free: List[int] = list(range(self.nslots - 1, -1, -1))
        self._cv = threading.Condition()

    # -- addressing -----------------------------------------------------------------------
    def in_view(self, slot: int, nbytes: int) -> np.ndarray:
        o = slot * 2 * self.slot_bytes
        return self.buf[o:o + nbytes]

    def out_view(self, slot: int, nbytes: int) -> np.ndarray:
        o = slot * 2 * self.slot_bytes + self.slot_bytes
        return self.buf[o:o + nbytes]

    @property
    def base_address(self) -> int:
        return self.buf.ctypes.data

    @property
    def nbytes(self) -> int:
        return self.shm.size

    # -- slot allocation (owner side) -----------------------------------------------------
    def acquire(self, timeout: Optional[float] = None) -> Optional[int]:
        with self._cv:
            if not self._cv.wait_for(lambda: bool(self._free), timeout=timeout):
                return None
            return self._free.pop()

    def try_acquire(self) -> Optional[int]:
        with self._cv:
            return self._free.pop() if self._free else None

    def release(self, slot: int) -> None:
        with self._cv:
            self._free.append(slot)
            self._cv.notify()

    def free_slots(self) -> int:
        with self._cv:
            return len(self._free)

    # -- lifetime -------------------------------------------------------------------------
    def close(self) -> None:
        self.buf = None
        try:
            self.shm.close()
        except BufferError:
            pass  # a view is still alive; the mapping goes with the process
        if self.owner:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass


_copy_pool = None
_COPY_SPLIT = 4 << 20  # frames from 4 MiB on are copied by several threads


def copy_into(dst: np.ndarray, src, threads: int = 4) -> None:
    """dst[:] = src for a frame going into a ring slot.  One core copies ~10-25 GB/s, well
    under one GPU's PCIe Gen5 x16 rate; large frames are split over ``threads`` threads with
    ``ctypes.memmove`` (which releases the GIL), so the producer does not cap a 4K stream.
    ``threads=1``: one memmove on the calling thread, still without the GIL (for producers
    that already copy from several threads at once)."""
    s = src if isinstance(src, np.ndarray) else np.frombuffer(src, dtype=np.uint8)
    s = s.reshape(-1).view(np.uint8)
    n = s.nbytes
    if n != dst.nbytes:
        raise ValueError(f"copy_into: {n} bytes into a view of {dst.nbytes}")
    if n < _COPY_SPLIT or not s.flags.c_contiguous or not dst.flags.c_contiguous:
        dst[:] = s
        return
    import ctypes
    d0, s0 = dst.ctypes.data, s.ctypes.data
    if threads <= 1:
        ctypes.memmove(d0, s0, n)
        return
    global _copy_pool
    if _copy_pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _copy_pool = ThreadPoolExecutor(max_workers=4, thread_name_prefix="vf-copy")
    parts = 4
    per = ((n + parts - 1) // parts + 4095) & ~4095

    def part(i):
        b = i * per
        e = min(n, b + per)
        if e > b:
            ctypes.memmove(d0 + b, s0 + b, e - b)

    list(_copy_pool.map(part, range(parts)))


def shm_free_bytes() -> Optional[int]:
    try:
        import os
        st = os.statvfs("/dev/shm")
        return st.f_bavail * st.f_frsize
    except (OSError, AttributeError):
        return None


_attach_lock = threading.Lock()


def _attach(name: str) -> shared_memory.SharedMemory:
    """Map the owner's segment without registering it with the resource tracker: CPython
    registers every attach and would unlink the owner's segment when this process exits
    (bpo-38119); unregistering afterwards instead removes the owner's own registration when
    the tracker is shared (multiprocessing "spawn" children share their parent's)."""
    import sys
    if sys.version_info >= (3, 13):
        return shared_memory.SharedMemory(name=name, track=False)
    from multiprocessing import resource_tracker
    skip = {name, "/" + name.lstrip("/")}
    with _attach_lock:
        reg = resource_tracker.register

        def register(rname, rtype):  # only this attach is skipped: another thread creating a
            if rtype == "shared_memory" and rname in skip:  # segment meanwhile still registers it
                return None
            return reg(rname, rtype)

        resource_tracker.register = register
        try:
            return shared_memory.SharedMemory(name=name)
        finally:
            resource_tracker.register = reg
