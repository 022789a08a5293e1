"""Distributor / worker plumbing on the CPU (BASELINE configs[0] and the ordering logic of
configs[2]/[3]), with the stdlib TCP transport and a test plugin whose arithmetic is the
oracle.  The GPU versions of these flows are in test_gpu_plumbing.py."""
import glob
import json
import os
import random
import threading
import time

import numpy as np
import pytest

from _plumbing import spawn_workers, stop_workers
from oracle import oracle
from vfilter import wire
from vfilter import transport as tp
from vfilter.distributor import Distributor
from vfilter.reorder import DisplayBuffer, OrderedBuffer

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ---- reassembly policies ----------------------------------------------------------------

@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "ref_display_*.json"))))
def test_display_buffer_matches_reference_trace(path):
    d = json.load(open(path))
    b = DisplayBuffer(d["frame_delay"], d["frame_buffer_size"])
    for i, (op, rec) in enumerate(zip(d["ops"], d["records"])):
        got = {"op": op}
        if op[0] == "recv":
            b.receive(op[1], oracle.payload_for(op[1]), "4242", 1.0 + op[1], 1.5 + op[1])
        elif op[0] == "update":
            got["ret"] = b.update_display_frame()
        else:
            fd = b.get_frame_to_display()
            got["ret"] = None if fd is None else oracle.payload_index(fd)
        got.update({"keys": sorted(b.received_frames), "current_display_frame": b.current_display_frame,
                    "latest_received_frame": b.latest_received_frame})
        assert got == rec, f"{os.path.basename(path)} op #{i}"
    e = d["stored_entry"]
    ent = b.received_frames[e["index"]]
    assert (ent["process_id"], ent["start_time"], ent["end_time"]) == (e["process_id"], e["start_time"], e["end_time"])


def test_display_buffer_matches_oracle_on_random_streams():
    rng = random.Random(3)
    for trial in range(30):
        fd, bs = rng.randint(0, 8), rng.randint(1, 60)
        ref = oracle.RefReorderBuffer(fd, bs)
        got = DisplayBuffer(fd, bs)
        for _ in range(400):
            r = rng.random()
            if r < 0.6:
                i = rng.randint(0, 300)
                ref.receive(i, i)
                got.receive(i, i, "p", 0.0, 0.0)
            elif r < 0.8:
                assert ref.update_display_frame() == got.update_display_frame()
            else:
                assert ref.get_frame_to_display() == got.get_frame_to_display()
            assert sorted(ref.received_frames) == sorted(got.received_frames)
            assert ref.current_display_frame == got.current_display_frame


def test_ordered_buffer_releases_each_index_once_in_order():
    rng = np.random.default_rng(0)
    n = 500
    order = np.argsort(np.arange(n) + rng.uniform(0, 25, n))
    lost = set(rng.choice(n, 10, replace=False).tolist())
    b = OrderedBuffer()
    out = []
    for k, i in enumerate(order):
        i = int(i)
        if i in lost:
            b.mark_lost(i)
        else:
            b.push(i, i * 7, now=float(k))
        out += [x[0] for x in b.pop_ready(now=float(k))]
    assert out == [i for i in range(n) if i not in lost]
    s = b.stats()
    assert s["released"] == n - len(lost) and s["lost"] == len(lost) and s["buffered"] == 0
    assert s["max_depth"] >= 1 and s["out_of_order"] > 0


# ---- wire -----------------------------------------------------------------------------------

def test_wire_v0_is_the_reference_layout():
    assert wire.encode_request(version=0) == [b"READY"]
    assert wire.encode_dispatch_v0(12, b"abc") == [b"12", b"abc"]
    parts = wire.encode_result_v0(12, 4242, 1.25, 2.5, b"xyz")
    assert parts[:4] == [b"12", b"4242", b"1.25", b"2.5"]
    r = wire.decode_result(parts)
    assert r.version == 0 and r.pid == "4242" and r.metas[0].index == 12 and r.payloads[0] == b"xyz"
    d = wire.decode_dispatch([b"7", b"frame"])
    assert d.version == 0 and d.metas[0].index == 7 and d.payloads == [b"frame"]


def test_wire_v1_roundtrip_with_ring_and_errors():
    metas = [wire.FrameMeta(0, 5, [1, 1, 5]), wire.FrameMeta(1, 9, None, slot=3), wire.FrameMeta(2, 2)]
    parts = wire.encode_dispatch(metas, [b"aaaaa", None, b"bb"], ring={"name": "r", "slot_bytes": 4096})
    d = wire.decode_dispatch(parts)
    assert [m.index for m in d.metas] == [0, 1, 2] and d.payloads == [b"aaaaa", None, b"bb"]
    assert d.ring == {"name": "r", "slot_bytes": 4096} and d.metas[0].shape == [1, 1, 5]
    rm = [wire.FrameMeta(0, 5, start=1.0, end=2.0), wire.FrameMeta(1, 9, slot=3), wire.FrameMeta(2, 2, error="boom")]
    r = wire.decode_result(wire.encode_result(99, rm, [b"zzzzz", None, None]))
    assert r.pid == "99" and r.payloads == [b"zzzzz", None, None] and r.metas[2].error == "boom"
    assert wire.decode_request(wire.encode_request(8, shm=True)) == wire.Request(1, 8, True)
    assert wire.decode_request([b"HELLO"]) is None


def test_wire_v1_columns_roundtrip_every_field():
    """The columnar v1 metadata: every FrameMeta field survives dispatch and result encoding
    for uniform and mixed shapes, slots present / absent / mixed, per-frame and uniform times,
    sparse errors; the earlier per-frame form ({"frames": [...]}) still decodes."""
    import json as _json
    rng = random.Random(5)
    for trial in range(40):
        n = rng.randint(1, 40)
        same_shape = trial % 3 == 0
        ms = []
        for i in range(n):
            shape = [4, 6, 3] if same_shape else rng.choice([None, [480, 640, 3], [2, 3, 3]])
            slot = None if trial % 4 == 1 else (rng.randrange(256) if trial % 4 else rng.choice([None, 7]))
            st = 1.5 if trial % 2 else rng.random()
            ms.append(wire.FrameMeta(1000 * trial + i, rng.randrange(1, 10 ** 7), shape, slot, st,
                                     st + (0.25 if trial % 2 else rng.random()),
                                     rng.choice([None, None, None, f"err {i}"])))
        pay = [None if m.slot is not None else bytes([i % 256]) * 3 for i, m in enumerate(ms)]
        d = wire.decode_dispatch(wire.encode_dispatch(ms, pay))
        for a, b in zip(ms, d.metas):
            assert (a.index, a.nbytes, a.shape, a.slot) == (b.index, b.nbytes, b.shape, b.slot)
        assert d.payloads == pay
        rpay = [p_ if m.error is None else None for p_, m in zip(pay, ms)]
        r = wire.decode_result(wire.encode_result(7, ms, rpay, wid="w"))
        assert r.metas == ms and r.wid == "w"
        assert r.payloads == [p_ if (m.slot is None and m.error is None) else None for p_, m in zip(pay, ms)]
    legacy = [wire.RESULT_V1, _json.dumps({"pid": "3", "frames": [m.to_json() for m in ms]}).encode()]
    legacy += [p_ for p_, m in zip(rpay, ms) if m.slot is None and m.error is None]
    assert wire.decode_result(legacy).metas == ms


# ---- transport -------------------------------------------------------------------------------

@pytest.mark.parametrize("reader", ["thread", "select"])
def test_tcp_transport_roles(monkeypatch, reader):
    """Both listener forms (VF_TCP_READER: a reader thread per peer, or one select loop per
    listener): multipart messages in both directions, a 3 MiB part, an empty part, several peers
    on one listener, and a peer's disconnect reported as (peer, None)."""
    monkeypatch.setattr(tp, "_READER", reader)
    router = tp.RouterEnd("tcp", "127.0.0.1", 0)
    pull = tp.PullEnd("tcp", "127.0.0.1", 0)
    dealer = tp.DealerEnd("tcp", "127.0.0.1", router.port)
    push = tp.PushEnd("tcp", "127.0.0.1", pull.port)
    big = np.random.default_rng(1).integers(0, 256, 3 << 20, dtype=np.uint8)
    try:
        dealer.send([b"READY"])
        assert router.poll(2000)
        peer, parts = router.recv()
        assert parts == [b"READY"] and len(peer) == 5
        assert router.send(peer, [b"1", big])
        assert dealer.poll(2000)
        got = dealer.recv()
        assert got[0] == b"1" and bytes(got[1]) == big.tobytes()
        push.send([b"a", b"", memoryview(big)[:10]])
        assert pull.poll(2000)
        assert [bytes(x) for x in pull.recv()] == [b"a", b"", big[:10].tobytes()]
        assert not router.send(b"\x00nope", [b"x"])  # unknown peer: dropped, like ROUTER
        # more peers on the same listeners, messages interleaved, then one disconnects
        pushes = [tp.PushEnd("tcp", "127.0.0.1", pull.port) for _ in range(3)]
        for r in range(5):
            for i, q in enumerate(pushes):
                q.send([b"m", bytes([i, r]), big[: 70000 + r].tobytes()])
        seen = []
        while len(seen) < 15:
            assert pull.poll(2000)
            got = pull.recv()
            assert got[0] == b"m" and bytes(got[2]) == big[: 70000 + got[1][1]].tobytes()
            seen.append(bytes(got[1]))
        assert sorted(seen) == sorted(bytes([i, r]) for i in range(3) for r in range(5))
        dealer.close()
        deadline = time.time() + 5
        gone = None
        while gone is None and time.time() < deadline:
            if router.poll(200):
                p_, parts = router.recv()
                if parts is None:
                    gone = p_
        assert gone == peer
        for q in pushes:
            q.close()
    finally:
        for s in (dealer, push, router, pull):
            s.close()


# ---- end-to-end plumbing with worker processes -------------------------------------------------

def _dist(**kw):
    kw.setdefault("transport", "tcp")
    kw.setdefault("host", "127.0.0.1")
    kw.setdefault("verbose", False)
    d = Distributor(0, 0, **kw)
    d.start()
    return d


def _frames(n, shapes):
    return [oracle.synthetic_frame(i, *shapes[i % len(shapes)]) for i in range(n)]


def _drain_ordered(d, frames, timeout=30.0):
    got = []
    for i in range(len(frames)):
        item = d.get_next_frame(timeout=timeout)
        assert item is not None, f"timed out waiting for frame {i}: {d.ordering_stats()}"
        idx, data, info = item
        assert idx == i
        assert bytes(data) == oracle.invert_bytes(frames[i].tobytes()), f"frame {i} differs"
        got.append(info)
    return got


@pytest.mark.timeout(120)
def test_configs0_latest_policy_two_v0_workers():
    """configs[0]: 640x480 frames through the distributor + 2 CPU workers speaking the
    reference protocol (v0); reference policy: latest-wins dispatch, lossy display."""
    d = _dist(policy="latest", reassembly="display", frame_delay=2)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v0")
    try:
        frames = _frames(40, [(480, 640)])
        sent = []
        for f in frames:
            sent.append(d.add_frame_for_distribution(f.tobytes()))
            time.sleep(0.02)  # 50 fps offered
        t0 = time.time()
        while time.time() - t0 < 10 and d.results_received < 20:
            time.sleep(0.05)
        assert d.results_received >= 20
        with d._lock:
            snap = {i: e for i, e in d.received_frames.items()}
        assert snap
        for i, e in snap.items():
            assert bytes(e["frame_data"]) == oracle.invert_bytes(frames[i].tobytes())
            assert e["start_time"] <= e["end_time"]
        assert d.update_display_frame() in (True, False)
        shown = d.get_frame_to_display()
        assert shown is not None and any(bytes(shown) == bytes(e["frame_data"]) for e in snap.values())
        st = d.get_frame_stats()
        assert st["total_frames_processed"] == 40 and st["frame_delay"] == 2
        pids = {e["process_id"] for e in snap.values()}
        assert len(pids) >= 1
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(120)
def test_lossless_pull_ordered_two_workers():
    d = _dist(policy="pull", reassembly="ordered", queue_size=32)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=4)
    try:
        t0 = time.time()
        while d.num_workers() < 2 and time.time() - t0 < 60:  # pull: a late worker could get nothing
            time.sleep(0.02)
        frames = _frames(80, [(120, 160), (97, 33), (480, 640)])
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(f) for f in frames])
        th.start()
        infos = _drain_ordered(d, frames)
        th.join()
        assert len({i["process_id"] for i in infos}) == 2  # both workers took part
        s = d.ordering_stats()
        assert s["released"] == 80 and s["lost"] == 0 and s["frames_dropped"] == 0
        assert infos[2]["shape"] == [480, 640, 3]
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(120)
def test_shard_policy_assigns_index_chunks_round_robin():
    d = _dist(policy="shard", reassembly="ordered", shard_workers=2, shard_chunk=4, queue_size=64)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=4)
    try:
        time.sleep(1.0)  # let both workers register before frames arrive
        frames = _frames(48, [(64, 64)])
        for f in frames:
            d.add_frame_for_distribution(f)
        infos = _drain_ordered(d, frames)
        owner = [infos[c * 4]["process_id"] for c in range(12)]
        for c in range(12):  # a chunk stays on one worker; chunks alternate
            assert {infos[c * 4 + k]["process_id"] for k in range(4)} == {owner[c]}
        assert len(set(owner)) == 2 and all(owner[c] == owner[c % 2] for c in range(12))
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("engine,kind", [("python", "oracle"), ("native", "oracle"), ("native", "ring")])
def test_shared_memory_ring_mixed_resolutions(engine, kind):
    """configs[3]-shaped stream (mixed sizes) through the shared-memory ring: only slot
    numbers cross the sockets; results are read from the ring's output halves."""
    shapes = [(480, 640), (720, 1280), (1080, 1920)]
    d = _dist(engine=engine, policy="pull", reassembly="ordered", queue_size=16, ring_slots=12,
              ring_slot_bytes=1080 * 1920 * 3)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=3, kind=kind)
    try:
        frames = _frames(30, shapes)
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(f) for f in frames])
        th.start()
        _drain_ordered(d, frames)
        th.join()
        assert d.free_slots() == d.total_slots()  # every slot returned
        s = d.ordering_stats()
        assert s["released"] == 30 and s["reorder_wait_max_ms"] >= 0.0
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(120)
def test_failed_frames_are_reported_and_skipped():
    """A worker that fails a frame reports it (v1 "error"); the in-order consumer skips it
    instead of waiting forever (the reference just loses it, worker.py:74-76)."""
    d = _dist(policy="pull", reassembly="ordered", queue_size=16)
    stop, procs = spawn_workers(1, d.distribute_port, d.collect_port, protocol="v1", batch=2)
    try:
        frames = _frames(6, [(8, 8)])
        for f in frames:
            d.add_frame_for_distribution(f)
        _drain_ordered(d, frames)
        # a result message that reports an error for index 6 (what a failing plugin sends)
        d._on_result(wire.Result("1", [wire.FrameMeta(6, 3, error="ValueError: bad")], [None]))
        d.add_frame_for_distribution(b"abc")  # index 6 is already accounted for as lost
        f7 = oracle.synthetic_frame(7, 8, 8)
        d.add_frame_for_distribution(f7)
        item = d.get_next_frame(timeout=20)
        assert item is not None and item[0] == 7 and bytes(item[1]) == oracle.invert_bytes(f7.tobytes())
        assert d.ordering_stats()["lost"] == 1 and d.result_errors == 1
    finally:
        stop_workers(stop, procs)
        d.cleanup()


def test_perfetto_trace_reference_schema_plus_gpu_spans(tmp_path, capsys):
    """export_perfetto_trace writes the reference's Chrome-trace schema
    (distributor.py:100-146): 'i' capture instants, 'X' worker spans keyed by worker pid; plus
    GPU spans on named tracks of the worker's pid."""
    d = Distributor(0, 0, 5, True, transport="tcp", host="127.0.0.1", verbose=False,
                    trace_file=str(tmp_path / "t.pftrace"))
    try:
        t0 = d.trace_start_time
        d.add_frame_for_distribution(b"abc", t0 + 0.5)
        res = wire.Result("4242", [wire.FrameMeta(0, 3, start=t0 + 1.0, end=t0 + 1.25)], [b"xyz"],
                          spans=[{"name": "H2D", "begin": t0 + 1.0, "end": t0 + 1.1, "bytes": 3},
                                 {"name": "kernel", "begin": t0 + 1.1, "end": t0 + 1.15, "bytes": 3},
                                 {"name": "D2H", "begin": t0 + 1.15, "end": t0 + 1.2, "bytes": 3}])
        d._on_result(res)
        d.export_perfetto_trace()
        ev = json.load(open(tmp_path / "t.pftrace"))["traceEvents"]
        inst = [e for e in ev if e["ph"] == "i"]
        assert inst[0]["name"] == "Frame 0 - frame_captured" and inst[0]["cat"] == "video_frames"
        assert inst[0]["ts"] == 500000 and inst[0]["args"]["absolute_timestamp"] == t0 + 0.5
        xs = [e for e in ev if e["ph"] == "X" and e.get("cat") != "gpu"]
        assert xs[0]["name"] == "Frame 0 - frame_inverted_received" and xs[0]["pid"] == 4242
        assert xs[0]["ts"] == 1000000 and xs[0]["dur"] == 250000
        assert abs(xs[0]["args"]["duration_ms"] - 250.0) < 1e-6
        gpu = [e for e in ev if e.get("cat") == "gpu"]
        assert [g["name"] for g in gpu] == ["GPU H2D", "GPU kernel", "GPU D2H"]
        assert [g["tid"] for g in gpu] == [1, 2, 3] and all(g["pid"] == 4242 for g in gpu)
        meta = [e for e in ev if e["ph"] == "M"]
        assert {m["args"]["name"] for m in meta} == {"GPU H2D", "GPU kernel", "GPU D2H"}
        # the reference's summary after an export (distributor.py:151-171), plus the GPU stages
        d.add_frame_for_distribution(b"def", t0 + 0.6)
        d.export_perfetto_trace()
        out = capsys.readouterr().out
        assert "Average frame capture interval: 100.00ms" in out and "Frame capture rate: 10.0 FPS" in out
        assert "Average processing duration: 250.00ms" in out and "Processing rate: 4.0 FPS" in out
        assert "Total frames processed: 1" in out and "GPU kernel: 1 spans" in out
        sm = d.trace_summary()
        assert abs(sm["gpu"]["H2D"]["GBps"] - 3 / 0.1 / 1e9) < 1e-12
    finally:
        d.cleanup()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("engine", ["python", "native"])
def test_zero_copy_reserve_commit_and_release(engine):
    """Ring mode without host copies in the distributor: the producer fills a reserved slot
    in place; the ordered consumer reads the result view and releases the slot."""
    d = _dist(engine=engine, policy="pull", reassembly="ordered", queue_size=8, ring_slots=6, ring_slot_bytes=64 * 64 * 3,
              zero_copy=True)
    stop, procs = spawn_workers(1, d.distribute_port, d.collect_port, protocol="v1", batch=2)
    try:
        frames = _frames(20, [(64, 64), (32, 16)])

        def produce():
            for f in frames:
                slot = d.reserve_frame(f.nbytes)
                d.frame_view(slot, f.nbytes)[:] = f.reshape(-1)
                d.commit_frame(slot, f.nbytes, shape=list(f.shape))

        th = threading.Thread(target=produce)
        th.start()
        for i, f in enumerate(frames):
            idx, view, info = d.get_next_frame(timeout=20)
            assert idx == i and isinstance(view, np.ndarray)
            assert view.tobytes() == oracle.invert_bytes(f.tobytes())
            d.release_frame(idx)
        th.join()
        assert d.free_slots() == d.total_slots()
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("engine", ["python", "native"])
def test_concurrent_producers_fill_the_frame_their_reservation_fixed(engine):
    """Several producer threads reserve, fill and commit at once (tools/pipeline_bench.py's
    producer): with per-worker slices the index is fixed at reservation
    (``reserved_index``), so each thread writes the content of that index; the in-order
    consumer sees every index once, with its own content, and every slot comes back."""
    d = _dist(engine=engine, policy="pull", reassembly="ordered", queue_size=12, ring_slots=6, ring_slot_bytes=48 * 40 * 3,
              zero_copy=True)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=3)
    try:
        while d.num_workers() < 2:
            time.sleep(0.05)
        kinds = _frames(5, [(48, 40), (16, 8), (33, 7)])
        n = 90
        counter = iter(range(n))
        lock = threading.Lock()

        def produce():
            while True:
                with lock:
                    if next(counter, None) is None:
                        return
                slot = d.reserve_frame(max(f.nbytes for f in kinds))
                idx = d.reserved_index(slot)
                assert idx is not None
                f = kinds[idx % len(kinds)]
                d.frame_view(slot, f.nbytes)[:] = f.reshape(-1)
                d.commit_frame(slot, f.nbytes, shape=list(f.shape))

        ths = [threading.Thread(target=produce) for _ in range(3)]
        for th in ths:
            th.start()
        for i in range(n):
            item = d.get_next_frame(timeout=30)
            assert item is not None, d.ordering_stats()
            idx, view, _ = item
            assert idx == i
            assert view.tobytes() == oracle.invert_bytes(kinds[i % len(kinds)].tobytes()), i
            d.release_frame(idx)
        for th in ths:
            th.join()
        assert d.free_slots() == d.total_slots()
    finally:
        stop_workers(stop, procs)
        d.cleanup()


def test_busy_worker_request_waits_to_be_filled():
    """Batch filling (the dispatch rule): while a worker has a batch in flight, its request for
    `credit` frames is held until that many are queued or the oldest has waited batch_wait;
    an idle worker, a v0 worker, a credit of 1 and batch_wait=0 are answered at once."""
    from vfilter.distributor import _Peer
    d = Distributor(0, 0, transport="tcp", host="127.0.0.1", verbose=False, policy="pull",
                    reassembly="ordered", batch_wait=0.5)
    try:
        p = _Peer(b"w", wire.Request(version=1, credit=8), 0)
        now = time.monotonic()
        d._pending.extend({"frame_index": i, "queued_at": now} for i in range(3))
        assert not d._fill_pending(p, 8)               # idle worker: serve what there is
        p.inflight[99] = {"frame_index": 99}
        assert d._fill_pending(p, 8)                   # busy: wait for 8 ...
        assert not d._fill_pending(p, 3)               # ... or serve a request that is full
        assert not d._fill_pending(p, 1)
        d._pending[0]["queued_at"] = now - 0.6         # ... or once the oldest waited batch_wait
        assert not d._fill_pending(p, 8)
        d._pending[0]["queued_at"] = now
        d.batch_wait = 0.0
        assert not d._fill_pending(p, 8)
        d.batch_wait = 0.5
        p.version = 0
        assert not d._fill_pending(p, 8)
    finally:
        d.cleanup()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("engine", ["python", "native"])
def test_grouped_reserve_commit_get_release(engine):
    """The grouped forms (reserve_frames / commit_frames / get_next_frames / release_frames)
    behave as their one-frame forms called in a row: every index once, in order, with its
    own content, and every slot back."""
    d = _dist(engine=engine, policy="pull", reassembly="ordered", queue_size=16, ring_slots=10, ring_slot_bytes=24 * 20 * 3,
              zero_copy=True)
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=4)
    try:
        while d.num_workers() < 2:
            time.sleep(0.05)
        kinds = _frames(4, [(24, 20), (5, 3)])
        n = 120

        def produce():
            done = 0
            while done < n:
                slots = d.reserve_frames(24 * 20 * 3, min(6, n - done))
                assert slots
                nbs, shs = [], []
                for s_ in slots:
                    f = kinds[d.reserved_index(s_) % len(kinds)]
                    d.frame_view(s_, f.nbytes)[:] = f.reshape(-1)
                    nbs.append(f.nbytes)
                    shs.append(list(f.shape))
                d.commit_frames(slots, nbs, shs)
                done += len(slots)

        th = threading.Thread(target=produce)
        th.start()
        i = 0
        while i < n:
            items = d.get_next_frames(5, timeout=30)
            assert items, d.ordering_stats()
            for idx, view, _ in items:
                assert idx == i
                assert view.tobytes() == oracle.invert_bytes(kinds[i % len(kinds)].tobytes()), i
                i += 1
            d.release_frames([it[0] for it in items])
        th.join()
        assert d.free_slots() == d.total_slots()
        assert d.get_next_frames(3, timeout=0.2) == []
    finally:
        stop_workers(stop, procs)
        d.cleanup()
