"""The distributor's native control plane (libvfdist.so, include/vfdist.h) on the CPU: its C ABI,
engine selection, every wire form a worker may speak (v2 binary, v1 JSON per-frame, the
reference's v0), workers without the shared-memory ring, worker loss (deadline eviction,
re-queue, duplicates, shard re-take), malformed peers, and the grouped producer / consumer
calls.  The same Distributor API runs on the Python engine in test_plumbing.py /
test_worker_loss.py, several of them parametrised over both engines."""
import os
import re
import socket
import struct
import subprocess
import threading
import time

import numpy as np
import pytest

from _plumbing import spawn_workers, stop_workers
from oracle import oracle
from vfilter import native
from vfilter import transport as tp
from vfilter import wire
from vfilter.distributor import Distributor
from vfilter.shm import FrameRing

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vfdist.h")


def header_symbols():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(vfd_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_exactly_the_header():
    assert os.path.exists(native.library_path()), "run `make lib`"
    out = subprocess.run(["nm", "-D", "--defined-only", native.library_path()], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (vfd_[a-z0-9_]+)$", out, flags=re.M))
    assert exported == set(header_symbols())
    assert sorted(native.SIGNATURES) == header_symbols()
    assert native.load_library().vfd_abi_version() == native.ABI_VERSION
    assert native.FRAME.itemsize == 72


def test_engine_selection():
    kw = dict(transport="tcp", host="127.0.0.1", verbose=False)
    d = Distributor(0, 0, policy="pull", reassembly="ordered", ring_slots=4, ring_slot_bytes=4096, **kw)
    try:
        assert isinstance(d, native.NativeDistributor) and d.engine == "native"
    finally:
        d.cleanup()
    for extra in (dict(policy="latest"), dict(policy="pull"), dict(policy="pull", reassembly="ordered"),
                  dict(policy="pull", reassembly="ordered", ring_slots=4, ring_slot_bytes=64, ring_layout="shared"),
                  dict(policy="pull", reassembly="ordered", ring_slots=4, ring_slot_bytes=64, engine="python")):
        d = Distributor(0, 0, **kw, **extra)
        try:
            assert type(d) is Distributor and d.engine == "python"
        finally:
            d.cleanup()
    with pytest.raises(ValueError, match="native"):
        Distributor(0, 0, policy="latest", engine="native", **kw)


def test_auto_engine_falls_back_when_the_library_cannot_load(monkeypatch, capsys):
    """engine='auto' never fails for a missing libvfdist.so: the Python engine serves, with one
    notice; engine='native' still refuses loudly."""
    from vfilter import distributor as dmod
    monkeypatch.setattr(native, "available", lambda: False)
    monkeypatch.setattr(dmod, "_auto_notice_shown", False)
    kw = dict(transport="tcp", host="127.0.0.1", verbose=False, policy="pull", reassembly="ordered",
              ring_slots=4, ring_slot_bytes=4096)
    d = Distributor(0, 0, **kw)
    try:
        assert type(d) is Distributor and d.engine == "python"
    finally:
        d.cleanup()
    assert "uses the Python engine" in capsys.readouterr().err
    monkeypatch.setenv("VFDIST_LIB", "/nonexistent/libvfdist.so")
    monkeypatch.setattr(native, "_lib", None)
    with pytest.raises(native.NativeError, match="not found"):
        Distributor(0, 0, engine="native", **kw)


def _native(**kw):
    kw.setdefault("transport", "tcp")
    kw.setdefault("host", "127.0.0.1")
    kw.setdefault("verbose", False)
    kw.setdefault("reassembly", "ordered")
    d = Distributor(0, 0, engine="native", **kw)
    d.start()
    return d


def _wait(cond, timeout=10.0, what=""):
    t0 = time.monotonic()
    while not cond():
        assert time.monotonic() - t0 < timeout, f"timed out: {what}"
        time.sleep(0.01)


def _commit_all(d, frames):
    slots = d.reserve_frames(len(frames[0]), len(frames))
    assert len(slots) == len(frames)
    for s_, f in zip(slots, frames):
        d.frame_view(s_, len(f))[:] = np.frombuffer(f, np.uint8)
    return d.commit_frames(slots, [len(f) for f in frames])


class _Manual:
    """A worker end driven by the test, speaking a chosen wire form."""

    def __init__(self, d, wid, wire_version=2, shm=True):
        self.dealer = tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port)
        self.push = tp.PushEnd("tcp", "127.0.0.1", d.collect_port)
        self.wid, self.wire, self.shm = wid, wire_version, shm
        self.ring = None

    def request(self, credit=4):
        self.dealer.send(wire.encode_request(credit, shm=self.shm, wid=self.wid, wire=self.wire))

    def recv(self, timeout=5.0):
        if not self.dealer.poll(int(timeout * 1000)):
            return None
        return wire.decode_dispatch(self.dealer.recv())

    def answer(self, disp, fail=()):
        """Invert every frame (in its slot, or back as a part) in the form the dispatch came."""
        if disp.ring is not None and (self.ring is None or self.ring.name != disp.ring["name"]):
            self.ring = FrameRing(name=disp.ring["name"], slot_bytes=int(disp.ring["slot_bytes"]))
        metas, pays = [], []
        for m, p in zip(disp.metas, disp.payloads):
            om = wire.FrameMeta(m.index, m.nbytes, m.shape, m.slot, 1.0, 2.0)
            if m.index in fail:
                om.error = "ValueError: planned"
                pays.append(None)
            elif m.slot is not None:
                self.ring.out_view(m.slot, m.nbytes)[:] = np.bitwise_not(self.ring.in_view(m.slot, m.nbytes))
                pays.append(None)
            else:
                pays.append(oracle.invert_bytes(bytes(p)))
            metas.append(om)
        if disp.version == 2:
            cols = wire.columns(metas)
            errors = {i: m.error for i, m in enumerate(metas) if m.error}
            self.push.send(wire.encode_result2(os.getpid(), cols, [p for p in pays if p is not None], 1.0, 2.0,
                                               wid=self.wid, errors=errors))
        else:
            self.push.send(wire.encode_result(os.getpid(), metas, pays, wid=self.wid))

    def close(self):
        if self.ring is not None:
            self.ring.close()
        self.dealer.close()
        self.push.close()


@pytest.mark.timeout(60)
@pytest.mark.parametrize("wire_version,shm", [(2, True), (1, True), (2, False), (1, False)])
def test_each_wire_form_with_and_without_the_ring(wire_version, shm):
    """v2 or v1 (per-frame JSON, what a round-3/4 worker reads), reading the ring slice or taking
    frames as socket parts (a worker on another node): every frame once, in order, bit-exact,
    with its shape, and every slot back."""
    d = _native(policy="pull", queue_size=32, ring_slots=8, ring_slot_bytes=64 * 48 * 3, zero_copy=True)
    w = _Manual(d, "W", wire_version, shm)
    try:
        w.request(3)
        _wait(lambda: d.num_workers() == 1, what="register")
        frames = [oracle.synthetic_frame(i, *((48, 64) if i % 2 else (5, 7))) for i in range(20)]
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(f) for f in frames], daemon=True)
        th.start()
        got = 0
        while got < len(frames):
            disp = w.recv()
            assert disp is not None, d.ordering_stats()
            assert disp.version == (2 if wire_version == 2 else 1)
            assert all((m.slot is not None) == shm for m in disp.metas)
            w.answer(disp)
            w.request(3)
            while True:
                item = d.get_next_frame(timeout=0.05)
                if item is None:
                    break
                idx, view, info = item
                assert idx == got and bytes(view) == oracle.invert_bytes(frames[idx].tobytes())
                assert info["shape"] == list(frames[idx].shape) and info["process_id"] == str(os.getpid())
                d.release_frame(idx)
                got += 1
        th.join(5)
        st = d.ordering_stats()
        assert st["released"] == 20 and st["workers"][next(iter(st["workers"]))]["wire"] == wire_version
        _wait(lambda: d.free_slots() == d.total_slots(), what="slots back")
    finally:
        w.close()
        d.cleanup()


@pytest.mark.timeout(120)
def test_reference_v0_and_v1_workers_together():
    """Worker processes of this build (v2) and ones speaking the reference's own messages (v0:
    READY -> [index, frame] -> 5-part result, worker.py:35-76) on one native distributor."""
    d = _native(policy="pull", queue_size=24, ring_slots=8, ring_slot_bytes=96 * 64 * 3)
    stop, procs = spawn_workers(1, d.distribute_port, d.collect_port, protocol="v0")
    stop2, procs2 = spawn_workers(1, d.distribute_port, d.collect_port, protocol="v1", batch=3, delay=0.003)
    try:
        _wait(lambda: d.num_workers() == 2, 60, "register")
        frames = [oracle.synthetic_frame(i, 96, 64) for i in range(60)]
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(f) for f in frames], daemon=True)
        th.start()
        pids = set()
        for i in range(60):
            item = d.get_next_frame(timeout=20)
            assert item is not None, d.ordering_stats()
            assert item[0] == i and bytes(item[1]) == oracle.invert_bytes(frames[i].tobytes())
            pids.add(item[2]["process_id"])
        th.join(5)
        assert len(pids) == 2
        wires = sorted(w["wire"] for w in d.ordering_stats()["workers"].values())
        assert wires == [0, 2]
    finally:
        stop_workers(stop, procs)
        stop_workers(stop2, procs2)
        d.cleanup()


@pytest.mark.timeout(60)
def test_deadline_requeue_duplicates_and_shard_retake():
    """Shard policy, 2 workers.  A stops answering: past batch_timeout it is evicted, its frames
    are copied into B's slice and go to B, and B serves A's shard.  A's late answers are
    duplicates; A asks again, is taken back and re-takes its home shard."""
    d = _native(policy="shard", shard_workers=2, shard_chunk=2, queue_size=64, ring_slots=12, ring_slot_bytes=4096,
                batch_timeout=0.3, zero_copy=True)
    a, b = _Manual(d, "A"), _Manual(d, "B")
    try:
        a.request()
        _wait(lambda: d.num_workers() == 1)
        b.request()
        _wait(lambda: d.num_workers() == 2)
        frames = [bytes([i + 1]) * 64 for i in range(8)]
        _commit_all(d, frames)                                 # one commit: each worker gets a batch
        da, db = a.recv(), b.recv()
        assert [m.index for m in da.metas] == [0, 1, 4, 5]    # shard 0 = chunks 0, 2
        assert [m.index for m in db.metas] == [2, 3, 6, 7]
        b.answer(db)
        b.request()
        _wait(lambda: d.ordering_stats()["evictions"] == 1, 5, "A evicted")
        st = d.ordering_stats()
        assert st["frames_requeued"] == 4
        db2 = b.recv()
        assert [m.index for m in db2.metas] == [0, 1, 4, 5]   # A's frames, now in B's slice
        b.answer(db2)
        for i in range(8):
            item = d.get_next_frame(timeout=5)
            assert item is not None and item[0] == i and bytes(item[1]) == oracle.invert_bytes(frames[i])
            d.release_frame(i)
        a.answer(da)                                           # too late: duplicates
        a.request()
        _wait(lambda: d.ordering_stats()["duplicates"] == 4 and d.num_workers() == 2, 5, "A back")
        ws = {w["wid"]: w for w in d.ordering_stats()["workers"].values()}
        assert ws["A"]["shards"] == [0] and ws["B"]["shards"] == [1] and ws["A"]["alive"]
        d.add_frame_for_distribution(b"\x09" * 64)            # index 8, chunk 4 -> shard 0 -> A again
        da2 = a.recv()
        assert [m.index for m in da2.metas] == [8]
        _wait(lambda: d.free_slots() == d.total_slots() - 1, 5, "slots back")  # frame 8 in flight
    finally:
        a.close()
        b.close()
        d.cleanup()


@pytest.mark.timeout(60)
def test_errors_max_attempts_and_cancel():
    """A frame a worker reports failed is skipped by the in-order consumer; a frame whose every
    dispatch times out is counted lost after max_attempts; a cancelled reservation too."""
    d = _native(policy="pull", queue_size=16, ring_slots=8, ring_slot_bytes=4096, batch_timeout=0.2, max_attempts=2,
                zero_copy=True)
    a = _Manual(d, "A")
    try:
        a.request(2)
        _wait(lambda: d.num_workers() == 1)
        _commit_all(d, [b"\x01" * 16, b"\x02" * 16])
        disp = a.recv()
        assert [m.index for m in disp.metas] == [0, 1]
        a.answer(disp, fail={0})
        item = d.get_next_frame(timeout=5)
        assert item[0] == 1 and bytes(item[1]) == b"\xfd" * 16
        st = d.ordering_stats()
        assert st["result_errors"] == 1 and st["lost"] == 1
        d.add_frame_for_distribution(b"\x03" * 16)             # index 2: never answered
        for attempt in range(2):
            a.request(1)
            disp = a.recv()
            assert [m.index for m in disp.metas] == [2]
            _wait(lambda: d.ordering_stats()["evictions"] == attempt + 1, 5, "evicted")
        st = d.ordering_stats()
        assert st["frames_lost"] == 1 and st["lost"] == 2
        a.request(1)                                            # A asks again: taken back
        _wait(lambda: d.num_workers() == 1, 5, "A back")
        slot = d.reserve_frame(16)
        assert d.reserved_index(slot) == 3
        d.cancel_frame(slot)
        d.add_frame_for_distribution(b"\x05" * 16)             # index 4 passes the cancelled 3
        a.answer(a.recv())
        item = d.get_next_frame(timeout=5)
        assert item is not None and item[0] == 4 and d.ordering_stats()["lost"] == 3
        with pytest.raises(ValueError):
            d.reserve_frame(5000)                               # larger than a slot
    finally:
        a.close()
        d.cleanup()


@pytest.mark.timeout(60)
@pytest.mark.parametrize("bad", [1 << 63, 1 << 40])
def test_malformed_peer_is_dropped_alone(bad):
    d = _native(policy="pull", queue_size=16, ring_slots=4, ring_slot_bytes=4096, zero_copy=True)
    a = _Manual(d, "A")
    raw = socket.create_connection(("127.0.0.1", d.collect_port))
    try:
        a.request(1)
        _wait(lambda: d.num_workers() == 1)
        raw.sendall(struct.pack("<I", 2) + struct.pack("<Q", bad))
        raw.settimeout(5)
        assert raw.recv(1) == b""                               # the engine closed it
        d.add_frame_for_distribution(b"\x07" * 8)
        a.answer(a.recv())
        item = d.get_next_frame(timeout=5)
        assert item is not None and bytes(item[1]) == b"\xf8" * 8
    finally:
        raw.close()
        a.close()
        d.cleanup()


@pytest.mark.timeout(60)
@pytest.mark.parametrize("order", [[0, 0, 1], [1, 0, 1], [0, 1, 1, 0]])
def test_result_with_a_repeated_index(order):
    """A RESULT2 whose records repeat a frame index (a buggy or malicious worker) must not take
    the one-pass fast path (it would free that frame twice): each index is booked once, the
    repeat is dropped, and the engine keeps serving."""
    d = _native(policy="pull", queue_size=16, ring_slots=8, ring_slot_bytes=4096, zero_copy=True)
    a = _Manual(d, "A")
    try:
        a.request(2)
        _wait(lambda: d.num_workers() == 1)
        frames = [b"\x01" * 16, b"\x02" * 16]
        _commit_all(d, frames)
        disp = a.recv()
        assert [m.index for m in disp.metas] == [0, 1]
        if a.ring is None or a.ring.name != disp.ring["name"]:
            a.ring = FrameRing(name=disp.ring["name"], slot_bytes=int(disp.ring["slot_bytes"]))
        by_index = {m.index: m for m in disp.metas}
        for m in disp.metas:
            a.ring.out_view(m.slot, m.nbytes)[:] = np.bitwise_not(a.ring.in_view(m.slot, m.nbytes))
        metas = [wire.FrameMeta(i, by_index[i].nbytes, by_index[i].shape, by_index[i].slot, 1.0, 2.0) for i in order]
        a.push.send(wire.encode_result2(os.getpid(), wire.columns(metas), [], 1.0, 2.0, wid="A"))
        for i in range(2):
            item = d.get_next_frame(timeout=5)
            assert item is not None and item[0] == i and bytes(item[1]) == oracle.invert_bytes(frames[i])
            d.release_frame(i)
        d.add_frame_for_distribution(b"\x07" * 8)               # index 2: the engine still serves
        a.request(1)
        a.answer(a.recv())
        item = d.get_next_frame(timeout=5)
        assert item is not None and item[0] == 2 and bytes(item[1]) == b"\xf8" * 8
        d.release_frame(2)
        _wait(lambda: d.free_slots() == d.total_slots(), 5, "slots back")
    finally:
        a.close()
        d.cleanup()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("engine", ["native", "python"])
def test_fill_frames_columnar_copy(engine):
    """fill_frames (vfd_fill): every frame of a reservation group copied into its slot by one
    call, from an address column -- the producer form of the bench's small-JPEG legs.  Frames of
    several sizes, 2 worker processes, every result in order and bit-exact; an unreserved slot
    or an oversized frame is refused before anything is copied."""
    kw = dict(policy="pull", queue_size=64, ring_slots=24, ring_slot_bytes=32 * 32 * 3, zero_copy=True)
    if engine == "native":
        d = _native(**kw)
    else:
        d = Distributor(0, 0, engine="python", transport="tcp", host="127.0.0.1", verbose=False,
                        reassembly="ordered", **kw)
        d.start()
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=8)
    try:
        _wait(lambda: d.num_workers() == 2, 60, "register")
        kinds = [oracle.synthetic_frame(k, 32, 32).reshape(-1)[: 32 * 32 * 3 - 97 * k].copy() for k in range(5)]
        addr = np.array([k_.ctypes.data for k_ in kinds], np.uint64)
        nbk = np.array([k_.nbytes for k_ in kinds], np.int64)
        n = 400

        def produce():
            done = 0
            while done < n:
                slots, idx = d.reserve_frames_array(kinds[0].nbytes, min(16, n - done))
                d.fill_frames(slots, addr[idx % 5], nbk[idx % 5])
                assert d.commit_frames(slots, nbk[idx % 5]) == idx.tolist()
                done += len(slots)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        i = 0
        while i < n:
            b = d.get_next_batch(32, timeout=20)
            assert len(b), d.ordering_stats()
            assert b.index.tolist() == list(range(i, i + len(b)))
            for k in range(len(b)):
                assert bytes(b.view(k)) == oracle.invert_bytes(kinds[(i + k) % 5].tobytes())
            d.release_frames(b.index)
            i += len(b)
        th.join(5)
        slots, idx = d.reserve_frames_array(kinds[0].nbytes, 2)
        view = d.frame_view(int(slots[0]), 64)
        view[:] = 0x5A
        big = np.zeros(1 << 20, np.uint8)  # past the slot (ring_slot_bytes rounded up to pages)
        with pytest.raises((native.NativeError, ValueError), match="does not fit"):
            d.fill_frames(slots, [addr[0], big.ctypes.data], [int(nbk[0]), big.nbytes])
        with pytest.raises((native.NativeError, ValueError), match="not reserved"):
            d.fill_frames([int(slots[0]), 10 ** 6], [addr[0], addr[1]], [64, 64])
        assert (view == 0x5A).all()  # refused calls copied nothing
        for s_ in slots.tolist():
            d.cancel_frame(s_)
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(120)
def test_grouped_array_calls_and_batches():
    """reserve_frames_array / commit_frames / get_next_batch / release_frames: the consumer's
    columnar form, with 2 worker processes, every frame in order and bit-exact."""
    d = _native(policy="pull", queue_size=64, ring_slots=24, ring_slot_bytes=32 * 32 * 3, zero_copy=True)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=8)
    try:
        _wait(lambda: d.num_workers() == 2, 60, "register")
        kinds = [oracle.synthetic_frame(k, 32, 32).reshape(-1) for k in range(5)]
        n = 400

        def produce():
            done = 0
            while done < n:
                slots, idx = d.reserve_frames_array(kinds[0].nbytes, min(16, n - done))
                for s_, i in zip(slots.tolist(), idx.tolist()):
                    d.frame_view(s_, kinds[0].nbytes)[:] = kinds[i % 5]
                got = d.commit_frames(slots, [kinds[0].nbytes] * len(slots), [[32, 32, 3]] * len(slots))
                assert got == idx.tolist()
                done += len(slots)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        i = 0
        while i < n:
            b = d.get_next_batch(32, timeout=20)
            assert len(b), d.ordering_stats()
            assert b.index.tolist() == list(range(i, i + len(b)))
            for k in range(len(b)):
                assert bytes(b.view(k)) == oracle.invert_bytes(kinds[(i + k) % 5].tobytes())
            assert b.info(0)["shape"] == [32, 32, 3]
            d.release_frames(b.index)
            i += len(b)
        th.join(5)
        _wait(lambda: d.free_slots() == d.total_slots(), what="slots back")
    finally:
        stop_workers(stop, procs)
        d.cleanup()
