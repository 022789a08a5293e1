"""Transport and lock hygiene of the Python distributor engine (VERDICT r04 items 2 and 8,
ADVICE r04): no socket send under the distributor's lock, malformed frames drop only their
peer, the v2 wire form is negotiated, and a shared-ring slot of an evicted worker is not held
for ever where the transport reports no disconnects."""
import socket
import struct
import threading
import time

import numpy as np
import pytest

from oracle import oracle
from vfilter import transport as tp
from vfilter import wire
from vfilter.distributor import Distributor


@pytest.mark.timeout(120)
@pytest.mark.parametrize("reader", ["thread", "select"])
def test_single_threaded_worker_sending_large_results_while_dispatches_wait(monkeypatch, reader):
    """Frames as socket payloads (no ring): a single-threaded worker keeps two requests out and
    sends each batch's large results before it reads the next dispatch.  With a send under the
    distributor's lock, the blocked dispatch send held the lock the result reader needed while the
    worker was blocked sending those results (round 4's hang); now it completes in either reader."""
    monkeypatch.setattr(tp, "_READER", reader)
    d = Distributor(0, 0, policy="pull", reassembly="ordered", transport="tcp", host="127.0.0.1",
                    verbose=False, queue_size=64, batch_wait=0.0)
    d.start()
    nb = 6 << 20          # two 6 MiB frames per batch: far more than a loopback socket buffers
    nframes = 12
    frames = [np.full(nb, i + 1, np.uint8) for i in range(nframes)]
    dealer = tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port)
    push = tp.PushEnd("tcp", "127.0.0.1", d.collect_port)
    failed = []

    def worker():  # one thread: send results first, read the next dispatch after
        try:
            for _ in range(2):
                dealer.send(wire.encode_request(2, shm=False, wid="solo"))
            done = 0
            while done < nframes:
                assert dealer.poll(20000), "no dispatch"
                disp = wire.decode_dispatch(dealer.recv())
                metas = [wire.FrameMeta(m.index, m.nbytes, start=1.0, end=2.0) for m in disp.metas]
                push.send(wire.encode_result(7, metas, [oracle.invert_bytes(p) for p in disp.payloads], wid="solo"))
                done += len(metas)
                dealer.send(wire.encode_request(2, shm=False, wid="solo"))
        except Exception as e:  # reported by the main thread
            failed.append(e)

    th = threading.Thread(target=worker, daemon=True)
    th.start()
    try:
        for f in frames:
            d.add_frame_for_distribution(f)
        for i in range(nframes):
            item = d.get_next_frame(timeout=30)
            assert item is not None, f"stalled at frame {i}: {d.ordering_stats()}"
            idx, data, _ = item
            assert idx == i and bytes(data[:8]) == bytes([255 - (i + 1)]) * 8 and len(data) == nb
        th.join(10)
        assert not failed, failed
    finally:
        dealer.close()
        push.close()
        d.cleanup()


@pytest.mark.timeout(60)
@pytest.mark.parametrize("reader", ["thread", "select"])
@pytest.mark.parametrize("bad", ["len2^63", "len2^62", "parts"])
def test_malformed_frame_drops_only_that_peer(monkeypatch, reader, bad):
    """A peer announcing an absurd part length (2^62: MemoryError, 2^63: OverflowError in a
    bytearray) or part count is dropped before anything is allocated; the listener keeps
    serving its other peers, in either reader form."""
    monkeypatch.setattr(tp, "_READER", reader)
    router = tp.RouterEnd("tcp", "127.0.0.1", 0)
    good = tp.DealerEnd("tcp", "127.0.0.1", router.port)
    raw = socket.create_connection(("127.0.0.1", router.port))
    try:
        good.send([b"hello"])
        assert router.poll(5000)
        gpid, parts = router.recv()
        assert parts == [b"hello"]
        if bad == "parts":
            raw.sendall(struct.pack("<I", 1 << 30))
        else:
            raw.sendall(struct.pack("<I", 1) + struct.pack("<Q", 1 << (63 if bad == "len2^63" else 62)))
        # the bad peer is reported gone; the good one is still read
        gone = None
        t0 = time.time()
        while gone is None and time.time() - t0 < 5:
            if router.poll(200):
                p_, parts = router.recv()
                if parts is None:
                    gone = p_
        assert gone is not None and gone != gpid
        good.send([b"still", b"here"])
        assert router.poll(5000)
        assert router.recv() == (gpid, [b"still", b"here"])
        assert router.send(gpid, [b"ok"])
        assert good.poll(5000) and good.recv() == [b"ok"]
    finally:
        raw.close()
        good.close()
        router.close()


def test_wire_v2_roundtrip_and_negotiation():
    """v2 records carry every field (index, nbytes, slot or none, shape or none), results carry
    their own lengths, errors and per-frame times; v1 encoders write the per-frame form every
    build reads, while decoders still take round 4's columnar form."""
    ms = [wire.FrameMeta(10, 5, [1, 1, 5]), wire.FrameMeta(11, 9, None, slot=3), wire.FrameMeta(12, 2, [2], slot=0)]
    cols = wire.columns(ms)
    d = wire.decode_dispatch(wire.encode_dispatch2(cols, [b"aaaaa"], {"name": "r", "slot_bytes": 4096}))
    assert d.version == 2 and d.ring == {"name": "r", "slot_bytes": 4096}
    assert list(d.metas) == ms and d.payloads == [b"aaaaa", None, None]
    rc = cols.copy()
    rc["nbytes"][1] = 77
    rc["slot"][2] = -1
    r = wire.decode_result(wire.encode_result2(42, rc, [b"zz"], 1.0, 2.0, wid="w", errors={0: "boom"}))
    assert r.version == 2 and r.pid == "42" and r.wid == "w"
    assert [m.error for m in r.metas] == ["boom", None, None]
    assert r.metas[1].nbytes == 77 and r.metas[1].slot == 3 and r.metas[2].slot is None
    assert r.payloads == [None, None, b"zz"] and r.metas[0].start == 1.0 and r.metas[2].end == 2.0
    r = wire.decode_result(wire.encode_result2(1, rc, [b"a", b"zz"], 0, 0, starts=[1.0, 2.0, 3.0], ends=[4.0, 5.0, 6.0]))
    assert [m.start for m in r.metas] == [1.0, 2.0, 3.0] and [m.end for m in r.metas] == [4.0, 5.0, 6.0]
    assert not wire.v2_shape_ok([1, 2, 3, 4, 5]) and wire.v2_shape_ok(None) and wire.v2_shape_ok([480, 640, 3])
    with pytest.raises(ValueError):
        wire.decode_dispatch([wire.FRAMES_V2, b"{}", b"x" * 39])
    # negotiation: "wire" rides the v1 request; absent means 1
    assert wire.decode_request(wire.encode_request(4, wire=2)).wire == 2
    assert wire.decode_request(wire.encode_request(4)).wire == 1
    # v1 output is the per-frame form
    import json
    head = json.loads(wire.encode_dispatch(ms, [b"aaaaa", None, None])[1])
    assert "frames" in head and head["frames"][1] == {"index": 11, "nbytes": 9, "shape": None, "slot": 3}


def _manual(d, wid, wire_version):
    dealer = tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port)
    dealer.send(wire.encode_request(3, shm=True, wid=wid, wire=wire_version))
    return dealer


@pytest.mark.timeout(60)
def test_python_engine_speaks_each_peer_its_own_wire():
    """A worker that advertises "wire": 2 gets FRAMES2, one that does not gets per-frame FRAMES1
    (what a round-3 or round-4 worker reads)."""
    d = Distributor(0, 0, policy="pull", reassembly="ordered", transport="tcp", host="127.0.0.1", verbose=False,
                    queue_size=16, engine="python")
    d.running = True
    a, b = _manual(d, "A", 2), _manual(d, "B", 1)
    try:
        t0 = time.monotonic()
        while d.num_workers() < 2:
            d.dispatch_step(1)
            assert time.monotonic() - t0 < 5
        for i in range(6):
            d.add_frame_for_distribution(bytes([i]) * 10)
        d.dispatch_step(0)
        tags = set()
        for s in (a, b):
            assert s.poll(5000)
            parts = s.recv()
            tags.add((bytes(parts[0]), len(wire.decode_dispatch(parts).metas)))
        assert {t for t, _ in tags} == {wire.FRAMES_V2, wire.FRAMES_V1}
        assert sum(n for _, n in tags) == 6
    finally:
        d.running = False
        a.close()
        b.close()
        d.cleanup()


@pytest.mark.timeout(60)
def test_shared_ring_quarantine_is_bounded_without_disconnect_notices():
    """with ZeroMQ (no disconnect notices) a dead worker's shared-ring slots are
    freed after QUARANTINE_HOLD batch timeouts instead of never; with tcp they wait for the
    late result or the disconnect (test_worker_loss.py)."""
    d = Distributor(0, 0, policy="pull", reassembly="ordered", queue_size=16, transport="tcp", host="127.0.0.1",
                    verbose=False, batch_timeout=0.1, ring_slots=8, ring_slot_bytes=64, ring_layout="shared",
                    max_attempts=1, engine="python")
    d._disconnect_notices = False  # as under "zmq"
    d.running = True
    a = tp.DealerEnd("tcp", "127.0.0.1", d.distribute_port)
    try:
        a.send(wire.encode_request(4, shm=True, wid="A"))
        t0 = time.monotonic()
        while d.num_workers() < 1:
            d.dispatch_step(1)
            assert time.monotonic() - t0 < 5
        total = d.total_slots()
        for i in range(4):
            d.add_frame_for_distribution(bytes([i]) * 8)
        d.dispatch_step(0)
        assert a.poll(5000)
        time.sleep(0.15)
        d.dispatch_step(0)                       # evicted, never answers, no disconnect
        assert d.ordering_stats()["evictions"] == 1
        assert d.free_slots() < total
        time.sleep(0.2)
        d.dispatch_step(0)
        assert d.free_slots() < total            # not yet: within QUARANTINE_HOLD batch timeouts
        t0 = time.monotonic()
        while d.free_slots() < total:
            d.dispatch_step(1)
            assert time.monotonic() - t0 < 5
        assert d.quarantine_forced == 4
    finally:
        d.running = False
        a.close()
        d.cleanup()
