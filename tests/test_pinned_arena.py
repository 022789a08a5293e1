"""The context's pinned result arena (vfilter._lib._PinnedArena), host logic on the CPU.

``vfilter.bitwise_not(frame)`` returns its result in page-locked, device-mapped memory from
the context's arena so the invert kernel writes it directly over PCIe (the drop-in's own
shape, inverter.py:41).  Here a stand-in for the context's allocator checks the bookkeeping:
blocks are recycled by size once the last view of an array is gone, free blocks beyond the
keep limit are returned, a context closed while arrays are alive is destroyed only after the
last of them goes (their memory must outlive them) and then not from the garbage collector's
finalizer but at the next ``reap_closed_contexts()``; live results past the arena's cap, or a
failed page-locked allocation, make ``try_empty`` give None (the drop-in then returns an
ordinary array), and a closed context refuses calls."""
import gc
import types

import numpy as np

import pytest

from vfilter._lib import Context, VFilterError, _PinnedArena, _vp, reap_closed_contexts


class _FakeCtx:
    def __init__(self):
        self._closing = False
        self.live = {}
        self.freed = []
        self.closed = False
        self._arena = _PinnedArena(self, keep_bytes=64 << 10)

    def alloc_host(self, n):
        buf = np.zeros(n, np.uint8)
        self.live[buf.ctypes.data] = buf
        return buf.ctypes.data

    def _free_host_raw(self, p):
        self.freed.append(p)
        self.live.pop(p)

    def close(self):  # Context.close's rule
        self._closing = True
        for p in self._arena.drain():
            self._free_host_raw(p)
        if self._arena.outstanding == 0:
            self._destroy()

    def _destroy(self):
        self.closed = True


def test_arrays_are_recycled_by_size_after_the_last_view():
    ctx = _FakeCtx()
    a = ctx._arena.empty((8, 10, 3))
    assert a.shape == (8, 10, 3) and a.dtype == np.uint8 and a.flags.writeable
    a[:] = 7
    pa = a.ctypes.data
    view = a[2:]
    del a
    gc.collect()
    assert ctx._arena.outstanding == 1  # the view keeps the block
    del view
    gc.collect()
    assert ctx._arena.outstanding == 0
    b = ctx._arena.empty((240,))  # same 4 KiB class: the same block again
    assert b.ctypes.data == pa and len(ctx.live) == 1
    c = ctx._arena.empty((5000,))  # another class: a new allocation
    assert c.ctypes.data != pa and len(ctx.live) == 2


def test_free_blocks_beyond_the_keep_limit_are_returned():
    ctx = _FakeCtx()
    arrs = [ctx._arena.empty((32 << 10,)) for _ in range(4)]  # 4 x 32 KiB, keep 64 KiB
    del arrs
    gc.collect()
    assert len(ctx.freed) == 2 and len(ctx.live) == 2


def test_close_waits_for_live_arrays():
    ctx = _FakeCtx()
    a = ctx._arena.empty((100,))
    ctx.close()
    assert not ctx.closed  # an array of the arena is alive
    del a
    gc.collect()
    assert not ctx.closed  # the finalizer only queued it
    assert reap_closed_contexts() == 1 and ctx.closed and not ctx.live
    assert reap_closed_contexts() == 0


def test_try_empty_respects_the_cap_and_allocation_failures():
    ctx = _FakeCtx()
    ctx._arena.cap_bytes = 3 * 4096
    a = [ctx._arena.try_empty((4096,)) for _ in range(3)]
    assert all(x is not None for x in a) and ctx._arena.outstanding_bytes == 3 * 4096
    assert ctx._arena.try_empty((1,)) is None  # a fourth block would pass the cap
    del a
    gc.collect()
    keep = ctx._arena.try_empty((100,))
    assert keep is not None and ctx._arena.outstanding_bytes == 4096

    def refuse(n):
        raise VFilterError("hipHostMalloc failed")
    ctx._arena.cap_bytes = 1 << 30
    ctx.alloc_host = refuse
    assert ctx._arena.try_empty((1 << 20,)) is None and ctx._arena.outstanding == 1  # the live one above


def test_closed_context_refuses_calls():
    c = Context.__new__(Context)  # no library context behind it: only the guard is exercised
    c._closing, c._h = True, _vp(1)
    c._lib = types.SimpleNamespace(vf_invert_host=lambda *a: 0)
    with pytest.raises(VFilterError, match="closed"):
        c.invert_host(np.zeros(4, np.uint8), np.zeros(4, np.uint8))
    c._h = _vp()  # nothing to destroy
