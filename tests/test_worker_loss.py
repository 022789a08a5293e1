"""Lossless fan-out survives losing workers (CPU, stdlib transport, oracle plugin).

The reference tolerates workers joining and leaving (pull/READY, distributor.py:224-241) and
drops a frame whose worker fails (worker.py:74-76).  The lossless policies here must neither
stall nor lose silently: a worker that dies (SIGKILL: its connection closes) or stops
answering (SIGSTOP: only the batch deadline notices) is evicted, its frames go to the other
workers, and every frame is released in index order — or counted lost after
``max_attempts`` dispatches — within a bound.
"""
import os
import signal
import threading
import time

import numpy as np
import pytest

from _plumbing import spawn_workers, stop_workers
from oracle import oracle
from vfilter import transport as tp
from vfilter import wire
from vfilter.distributor import Distributor


def _dist(**kw):
    kw.setdefault("transport", "tcp")
    kw.setdefault("host", "127.0.0.1")
    kw.setdefault("verbose", False)
    d = Distributor(0, 0, **kw)
    d.start()
    return d


def _wait_workers(d, n, timeout=60):
    t0 = time.time()
    while d.num_workers() < n:
        assert time.time() - t0 < timeout, "workers did not register"
        time.sleep(0.02)


def _drain(d, frames, bound_s):
    """Every frame in order (or counted lost) within ``bound_s`` seconds in total."""
    t_end = time.monotonic() + bound_s
    got, lost_before = [], 0
    expect = 0
    while expect < len(frames):
        item = d.get_next_frame(timeout=max(0.01, t_end - time.monotonic()))
        assert item is not None, f"stalled at frame {expect}: {d.ordering_stats()}"
        idx, data, info = item
        assert idx >= expect
        expect = idx + 1
        assert bytes(data) == oracle.invert_bytes(frames[idx].tobytes()), f"frame {idx} differs"
        got.append(idx)
    return got


@pytest.mark.timeout(120)
@pytest.mark.parametrize("policy", ["pull", "shard"])
@pytest.mark.parametrize("how", ["kill", "stop"])
@pytest.mark.parametrize("engine", ["python", "native"])
def test_losing_one_of_three_workers_mid_stream(policy, how, engine):
    frames = [oracle.synthetic_frame(i % 7, 48, 64) for i in range(150)]
    d = _dist(engine=engine, policy=policy, reassembly="ordered", queue_size=24, shard_workers=3, shard_chunk=4,
              ring_slots=12, ring_slot_bytes=48 * 64 * 3, batch_timeout=1.5)
    stop, procs = spawn_workers(3, d.distribute_port, d.collect_port, protocol="v1", batch=4, delay=0.004)
    try:
        _wait_workers(d, 3)
        victim = procs[1]
        released = []

        def produce():
            for f in frames:
                d.add_frame_for_distribution(f)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        t0 = time.monotonic()
        while len(released) < 30:
            idx, data, _ = d.get_next_frame(timeout=30)
            assert bytes(data) == oracle.invert_bytes(frames[idx].tobytes())
            released.append(idx)
        os.kill(victim.pid, signal.SIGKILL if how == "kill" else signal.SIGSTOP)
        try:
            rest = _drain_from(d, frames, released[-1] + 1, bound_s=60)
        finally:
            if how == "stop":
                os.kill(victim.pid, signal.SIGCONT)
        th.join(10)
        s = d.ordering_stats()
        released += rest
        assert released == list(range(len(frames))), "every frame, in order, exactly once"
        assert s["evictions"] >= 1 and s["frames_lost"] == 0
        assert time.monotonic() - t0 < 60
    finally:
        stop_workers(stop, procs)
        d.cleanup()


def _drain_from(d, frames, start, bound_s):
    t_end = time.monotonic() + bound_s
    out = []
    for i in range(start, len(frames)):
        item = d.get_next_frame(timeout=max(0.01, t_end - time.monotonic()))
        assert item is not None, f"stalled at frame {i}: {d.ordering_stats()}"
        idx, data, _ = item
        assert idx == i and bytes(data) == oracle.invert_bytes(frames[i].tobytes()), i
        out.append(idx)
    return out


class _ManualWorker:
    """A v1 worker end driven by the test: requests, receives, answers (or not)."""

    def __init__(self, d, wid):
        self.dealer = tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port)
        self.push = tp.PushEnd("tcp", "127.0.0.1", d.collect_port)
        self.wid = wid

    def request(self, credit=4):
        self.dealer.send(wire.encode_request(credit, shm=False, wid=self.wid))

    def recv(self, timeout=5.0):
        if not self.dealer.poll(int(timeout * 1000)):
            return None
        return wire.decode_dispatch(self.dealer.recv())

    def answer(self, disp):
        metas = [wire.FrameMeta(m.index, m.nbytes, start=1.0, end=2.0) for m in disp.metas]
        outs = [oracle.invert_bytes(p) for p in disp.payloads]
        self.push.send(wire.encode_result(os.getpid(), metas, outs, wid=self.wid))

    def close(self):
        self.dealer.close()
        self.push.close()


def _step_until(d, cond, timeout=5.0):
    t0 = time.monotonic()
    while not cond():
        d.dispatch_step(1)
        assert time.monotonic() - t0 < timeout


@pytest.mark.timeout(60)
def test_deadline_requeue_and_home_shard_retake():
    """Shard policy, 2 workers.  Worker A stops answering: after the deadline its shard and
    its in-flight frames move to B.  A asks again: it is taken back and re-takes its shard;
    its late answers are duplicates and are dropped."""
    d = Distributor(0, 0, policy="shard", reassembly="ordered", shard_workers=2, shard_chunk=2, queue_size=64,
                    transport="tcp", host="127.0.0.1", verbose=False, batch_timeout=0.3)
    d.running = True  # stepped by hand: no threads
    a, b = _ManualWorker(d, "A"), _ManualWorker(d, "B")
    coll = threading.Thread(target=d.check_inverter_output, daemon=True)
    coll.start()
    try:
        a.request()
        _step_until(d, lambda: d.num_workers() == 1)
        b.request()
        _step_until(d, lambda: d.num_workers() == 2)
        frames = [bytes([i]) * 8 for i in range(8)]
        for f in frames:
            d.add_frame_for_distribution(f)
        d.dispatch_step(0)
        da, db = a.recv(), b.recv()
        assert [m.index for m in da.metas] == [0, 1, 4, 5]   # shard 0 = chunks 0, 2
        assert [m.index for m in db.metas] == [2, 3, 6, 7]
        b.answer(db)
        time.sleep(0.35)
        d.dispatch_step(0)                                  # A is past its deadline
        st = d.ordering_stats()
        assert st["evictions"] == 1 and st["frames_requeued"] == 4
        b.request()
        _step_until(d, lambda: b.dealer.poll(0))
        db2 = b.recv()
        assert [m.index for m in db2.metas] == [0, 1, 4, 5]  # A's frames, now on B
        b.answer(db2)
        for i in range(8):
            item = d.get_next_frame(timeout=5)
            assert item is not None and item[0] == i and bytes(item[1]) == oracle.invert_bytes(frames[i])
        a.answer(da)                                        # too late: duplicates
        a.request()
        _step_until(d, lambda: d.ordering_stats()["duplicates"] == 4 and d.num_workers() == 2)
        ws = {w["home_shard"]: w for w in d.ordering_stats()["workers"].values()}
        assert ws[0]["alive"] and ws[0]["shards"] == [0] and ws[1]["shards"] == [1]
        d.add_frame_for_distribution(b"\x09" * 8)           # index 8, chunk 4 -> shard 0 -> A again
        d.dispatch_step(0)
        da2 = a.recv()
        assert [m.index for m in da2.metas] == [8]
    finally:
        d.running = False
        coll.join(2)
        a.close()
        b.close()
        d.cleanup()


@pytest.mark.timeout(60)
def test_frame_lost_after_max_attempts():
    """A frame whose every dispatch times out is counted lost after max_attempts, and the
    in-order consumer moves past it."""
    d = Distributor(0, 0, policy="pull", reassembly="ordered", queue_size=16, transport="tcp",
                    host="127.0.0.1", verbose=False, batch_timeout=0.2, max_attempts=2)
    d.running = True
    a = _ManualWorker(d, "A")
    coll = threading.Thread(target=d.check_inverter_output, daemon=True)
    coll.start()
    try:
        d.add_frame_for_distribution(b"\x01" * 4)
        d.add_frame_for_distribution(b"\x02" * 4)
        for attempt in range(2):
            a.request(credit=1)
            _step_until(d, lambda: a.dealer.poll(0))
            assert [m.index for m in a.recv().metas] == [0]  # frame 0 again and again
            time.sleep(0.25)
            d.dispatch_step(0)
        s = d.ordering_stats()
        assert s["frames_lost"] == 1 and s["lost"] == 1 and s["evictions"] == 2
        a.request(credit=1)
        _step_until(d, lambda: a.dealer.poll(0))
        d1 = a.recv()
        assert [m.index for m in d1.metas] == [1]
        a.answer(d1)
        item = d.get_next_frame(timeout=5)
        assert item is not None and item[0] == 1
    finally:
        d.running = False
        coll.join(2)
        a.close()
        d.cleanup()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("engine,kind", [("python", "resizing"), ("native", "resizing"), ("native", "ring_resizing")])
def test_ring_results_of_their_own_size(engine, kind):
    """A plugin whose result size differs from the input's (as a re-encoded JPEG does) through
    the shared-memory ring: smaller and larger results land in the slot's output half when
    they fit, otherwise travel back over the socket; the distributor reads each result's own
    length."""
    shapes = [(4, 4), (17, 33), (64, 64)]   # 48 B (halved), 1,683 B (+7 fits), 12,288 B (+7: no room)
    frames = [oracle.synthetic_frame(i, *shapes[i % 3]) for i in range(30)]
    d = _dist(engine=engine, policy="pull", reassembly="ordered", queue_size=16, ring_slots=8, ring_slot_bytes=64 * 64 * 3)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=3, kind=kind)
    try:
        _wait_workers(d, 2)
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(f) for f in frames], daemon=True)
        th.start()
        for i, f in enumerate(frames):
            item = d.get_next_frame(timeout=30)
            assert item is not None and item[0] == i, d.ordering_stats()
            x = oracle.invert_bytes(f.tobytes())
            want = x[: len(x) // 2] if len(x) <= 64 else x + b"trailer"
            assert bytes(item[1]) == want, i
        th.join(10)
        assert d.free_slots() == d.total_slots()
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(120)
def test_per_worker_slices_numa_bound():
    """ring_layout='per_worker': each worker maps only its own slice (ring bytes / N per
    worker); a worker that reports a NUMA node gets its slice bound there."""
    from vfilter import numa
    d = Distributor(0, 0, policy="shard", reassembly="ordered", shard_workers=2, shard_chunk=2, queue_size=16,
                    ring_slots=4, ring_slot_bytes=4096, transport="tcp", host="127.0.0.1", verbose=False,
                    engine="python")  # stepped by hand (dispatch_step): the Python engine's loop
    d.running = True
    socks = [tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port) for _ in range(2)]
    try:
        socks[0].send(wire.encode_request(2, shm=True, wid="w0", numa=0))
        socks[1].send(wire.encode_request(2, shm=True, wid="w1"))
        _step_until(d, lambda: d.num_workers() == 2)
        for i in range(4):
            d.add_frame_for_distribution(bytes([i]) * 100)
        d.dispatch_step(0)
        rings = []
        for s in socks:
            assert s.poll(5000)
            disp = wire.decode_dispatch(s.recv())
            assert all(m.slot is not None for m in disp.metas) and disp.payloads == [None, None]
            rings.append(disp.ring["name"])
        assert rings[0] != rings[1]
        # keyed by the node each worker reported (the two may register in either order)
        info = {w["slice"]["numa"]: w["slice"] for w in d.ordering_stats()["workers"].values()}
        assert set(info) == {0, None}
        assert info[0]["bytes"] == info[None]["bytes"] == 4 * 2 * 4096
        if numa.node_count() >= 1 and numa._syscalls() is not None:
            assert info[0]["numa_bound"] is True
        assert d.total_slots() == 8
    finally:
        d.running = False
        for s in socks:
            s.close()
        d.cleanup()


@pytest.mark.timeout(60)
def test_worker_that_stops_asking_is_evicted():
    """A worker that keeps its connection but stops asking (no disconnect notice: ZeroMQ
    gives none) while frames wait for it loses its shard after the timeout."""
    d = Distributor(0, 0, policy="shard", reassembly="ordered", shard_workers=2, shard_chunk=1, queue_size=64,
                    transport="tcp", host="127.0.0.1", verbose=False, batch_timeout=0.3)
    d.running = True
    a, b = _ManualWorker(d, "A"), _ManualWorker(d, "B")
    coll = threading.Thread(target=d.check_inverter_output, daemon=True)
    coll.start()
    try:
        a.request(credit=1)
        _step_until(d, lambda: d.num_workers() == 1)
        b.request(credit=1)
        _step_until(d, lambda: d.num_workers() == 2)
        d.add_frame_for_distribution(b"\\x00")          # index 0 -> shard 0 -> A
        d.dispatch_step(0)
        da = a.recv()
        a.answer(da)                                     # A's credit is used; it never asks again
        for i in range(1, 5):
            d.add_frame_for_distribution(bytes([i]))     # shard 0 (even) waits for A
        d.dispatch_step(0)
        db = b.recv()
        b.answer(db)
        t0 = time.monotonic()
        while d.ordering_stats()["evictions"] == 0:
            d.dispatch_step(1)
            assert time.monotonic() - t0 < 5
        got = [m.index for m in da.metas + db.metas]
        while len(got) < 5:
            b.request(credit=4)
            _step_until(d, lambda: b.dealer.poll(0))
            dd = b.recv()
            b.answer(dd)
            got += [m.index for m in dd.metas]
        assert sorted(got) == list(range(5))
        for i in range(5):
            item = d.get_next_frame(timeout=5)
            assert item is not None and item[0] == i
    finally:
        d.running = False
        coll.join(2)
        a.close()
        b.close()
        d.cleanup()


def _sticky_worker(dport, cport):
    from _plumbing import OracleWorker

    class W(OracleWorker):  # batches that can never be collected: a sticky device error
        def submit_batch(self, frames, metas, outs):
            return ("sticky", len(frames))

        def poll_batch(self, handle, block):
            raise RuntimeError("hipErrorIllegalAddress (sticky)")

    return W("127.0.0.1", dport, cport, batch=2, protocol="v1", transport="tcp", inflight=1)


@pytest.mark.timeout(60)
def test_uncollectable_batches_are_reported_then_the_worker_exits():
    """a batch whose collection raises is popped and reported as failed (every
    frame an error result, so the in-order consumer skips it) instead of being retried every
    10 ms forever; after max_job_failures in a row the loop raises WorkerFailed, which the
    worker CLI turns into a non-zero exit for a supervisor to restart."""
    from vfilter.worker import WorkerFailed
    d = _dist(policy="pull", reassembly="ordered", queue_size=64)
    w = _sticky_worker(d.distribute_port, d.collect_port)
    failed = []

    def run():
        try:
            w.start()
        except WorkerFailed as e:
            failed.append(e)

    th = threading.Thread(target=run, daemon=True)
    th.start()
    try:
        _wait_workers(d, 1)
        for i in range(40):
            d.add_frame_for_distribution(oracle.synthetic_frame(i, 4, 4))
        th.join(30)
        assert not th.is_alive() and failed, "the worker kept retrying"
        assert w.max_job_failures == 8
        # every frame of the 8 failed batches (1 or 2 frames each: the first request may be
        # served with the first frame) is reported as an error result
        assert 8 <= w.errors <= 16
        t0 = time.time()
        while d.result_errors < w.errors and time.time() - t0 < 10:
            time.sleep(0.02)
        assert d.result_errors == w.errors
    finally:
        w.close()
        d.cleanup()


@pytest.mark.timeout(60)
def test_evicted_workers_slots_come_back_after_the_grace_period():
    """ZeroMQ reports no disconnects, so a worker that hangs is evicted without
    ``gone`` and its in-flight frames' ring slots stay quarantined.  After one more
    ``batch_timeout`` they are freed (the ring does not shrink per eviction); a result that
    still arrives later is dropped."""
    d = Distributor(0, 0, policy="pull", reassembly="ordered", queue_size=16, transport="tcp",
                    host="127.0.0.1", verbose=False, batch_timeout=0.3, ring_slots=4, ring_slot_bytes=64,
                    engine="python")  # stepped by hand (dispatch_step): the Python engine's loop
    d.running = True
    a, b = _ManualWorker(d, "A"), _ManualWorker(d, "B")
    coll = threading.Thread(target=d.check_inverter_output, daemon=True)
    coll.start()
    try:
        a.request()
        _step_until(d, lambda: d.num_workers() == 1)
        frames = [bytes([i]) * 8 for i in range(4)]
        for f in frames:
            d.add_frame_for_distribution(f)
        d.dispatch_step(0)
        da = a.recv()
        assert [m.index for m in da.metas] == [0, 1, 2, 3]
        b.request()
        _step_until(d, lambda: d.num_workers() == 2)
        total = d.total_slots()
        time.sleep(0.35)
        d.dispatch_step(0)                                  # A evicted (hung), not gone
        assert d.ordering_stats()["evictions"] == 1
        b.request()
        _step_until(d, lambda: b.dealer.poll(0))
        db = b.recv()
        b.answer(db)
        for i in range(4):
            item = d.get_next_frame(timeout=5)
            assert item is not None and item[0] == i and bytes(item[1]) == oracle.invert_bytes(frames[i])
        assert d.free_slots() == total - 4                  # A's copies still quarantined
        time.sleep(0.35)
        _step_until(d, lambda: d.free_slots() == total)     # grace period over: slots back
        assert d.quarantine_expired == 4
        a.answer(da)                                        # far too late: dropped
        time.sleep(0.2)
        assert d.free_slots() == total and d.ordering_stats()["released"] == 4
    finally:
        d.running = False
        coll.join(2)
        a.close()
        b.close()
        d.cleanup()


@pytest.mark.timeout(60)
def test_shared_ring_slots_of_an_evicted_worker_wait_for_its_result():
    """a slot of the SHARED ring can be dispatched to any worker, so an evicted
    worker that was only slow could write its stale result over the slot's next owner's.  Such
    slots are not freed by the grace period; the late result (or a disconnect) frees them, and
    the late result itself is dropped.  (A per-worker slice's slots do come back after the grace
    period: only their own worker writes them, in dispatch order -- the test above.)"""
    d = Distributor(0, 0, policy="pull", reassembly="ordered", queue_size=16, transport="tcp",
                    host="127.0.0.1", verbose=False, batch_timeout=0.3, ring_slots=8, ring_slot_bytes=64,
                    ring_layout="shared")
    d.running = True
    a, b = _ManualWorker(d, "A"), _ManualWorker(d, "B")
    coll = threading.Thread(target=d.check_inverter_output, daemon=True)
    coll.start()
    try:
        a.request()
        _step_until(d, lambda: d.num_workers() == 1)
        frames = [bytes([i + 1]) * 8 for i in range(4)]
        for f in frames:
            d.add_frame_for_distribution(f)
        d.dispatch_step(0)
        da = a.recv()
        assert [m.index for m in da.metas] == [0, 1, 2, 3]
        b.request()
        _step_until(d, lambda: d.num_workers() == 2)
        total = d.total_slots()
        time.sleep(0.35)
        d.dispatch_step(0)                                  # A evicted (hung), not gone
        assert d.ordering_stats()["evictions"] == 1
        b.request()
        _step_until(d, lambda: b.dealer.poll(0))
        db = b.recv()
        b.answer(db)
        for i in range(4):
            item = d.get_next_frame(timeout=5)
            assert item is not None and item[0] == i and bytes(item[1]) == oracle.invert_bytes(frames[i])
            d.release_frame(item[0])
        held = total - d.free_slots()
        assert held == 4                                    # A's slots, quarantined
        time.sleep(0.7)
        for _ in range(5):
            d.dispatch_step(0)
        assert d.free_slots() == total - 4 and d.quarantine_expired == 0  # not freed by time alone
        a.answer(da)                                        # the late result frees them, and is dropped
        _step_until(d, lambda: d.free_slots() == total)
        assert d.ordering_stats()["released"] == 4
    finally:
        d.running = False
        coll.join(2)
        a.close()
        b.close()
        d.cleanup()


@pytest.mark.timeout(60)
def test_latest_policy_keeps_the_slot_frame_after_a_refused_send():
    """Reference policy (latest-wins, v0 READY): a dispatch the transport refuses (the worker
    is gone) does not consume the frame -- distributor.py:238-241 books last_frame_sent only
    after a successful send -- so the next READY still gets it."""
    d = _dist(engine="python")
    a = tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port)
    b = tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port)
    try:
        real_send = d.distribute_socket.send
        refused = []

        def send_once_refused(pid, parts):
            if not refused:
                refused.append(pid)
                return False
            return real_send(pid, parts)

        d.distribute_socket.send = send_once_refused
        d.add_frame_for_distribution(b"\x11" * 32)
        t0 = time.time()
        while d.current_frame_data is None:                 # in the latest-wins slot
            assert time.time() - t0 < 10
            time.sleep(0.01)
        a.send(wire.encode_request(version=0))              # served, but the send is refused
        t0 = time.time()
        while not refused:
            assert time.time() - t0 < 10, "no dispatch attempted"
            time.sleep(0.01)
        b.send(wire.encode_request(version=0))
        assert b.poll(5000), "the frame in the dispatch slot was dropped with the refused send"
        disp = wire.decode_dispatch(b.recv())
        assert [m.index for m in disp.metas] == [0] and bytes(disp.payloads[0]) == b"\x11" * 32
        assert d.frames_dropped == 0
    finally:
        a.close()
        b.close()
        d.cleanup()
