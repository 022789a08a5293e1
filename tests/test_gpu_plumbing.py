"""The product worker (InverterWorker on libvfilter_hip.so) behind the distributor, on the
GPU: BASELINE configs[2] (4K, batch 16, frame-index sharded, in-order reassembly) and
configs[3] (mixed 480p/1080p/4K) at small frame counts, bit-exact against the oracle.
Worker processes share the box's one GPU (2 processes <= the 16-process limit)."""
import os
import threading
import time

import numpy as np
import pytest

from _plumbing import spawn_workers, stop_workers
from oracle import oracle
from vfilter.distributor import Distributor

pytestmark = pytest.mark.gpu


def _run(d, frames, n_workers, batch, timeout=60):
    stop, procs = spawn_workers(n_workers, d.distribute_port, d.collect_port, protocol="v1", batch=batch,
                                kind="gpu")
    try:
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(f) for f in frames])
        th.start()
        infos = []
        for i in range(len(frames)):
            item = d.get_next_frame(timeout=timeout)
            assert item is not None, f"frame {i} never came back: {d.ordering_stats()}"
            idx, data, info = item
            assert idx == i
            assert np.array_equal(np.frombuffer(data, np.uint8), oracle.invert(frames[i]).reshape(-1)), i
            infos.append(info)
        th.join()
        return infos
    finally:
        stop_workers(stop, procs)


def _sharded_4k(nworkers, nframes, ring_slots):
    """configs[2]: 4K frames, batch 16, frame-index shards of 16 over ``nworkers`` GPU worker
    processes (all on this box's one GPU), each with its own ring slice; in-order release,
    bit-exact, chunk c served by the owner of shard c % nworkers, every slot returned."""
    d = Distributor(0, 0, policy="shard", reassembly="ordered", shard_workers=nworkers, shard_chunk=16,
                    queue_size=2 * 16 * nworkers, ring_slots=ring_slots, ring_slot_bytes=2160 * 3840 * 3,
                    transport="tcp", host="127.0.0.1", verbose=False)
    d.start()
    try:
        base = [oracle.synthetic_frame(s, 2160, 3840) for s in range(4)]
        want = [oracle.invert(b).reshape(-1) for b in base]
        stop, procs = spawn_workers(nworkers, d.distribute_port, d.collect_port, protocol="v1", batch=16,
                                    kind="gpu")
        try:
            t0 = time.time()
            while d.num_workers() < nworkers:  # every shard's home worker registered
                assert time.time() - t0 < 90, f"{d.num_workers()} of {nworkers} workers registered"
                assert all(p.is_alive() for p in procs), "a worker process died"
                time.sleep(0.05)
            th = threading.Thread(target=lambda: [d.add_frame_for_distribution(base[i % 4]) for i in range(nframes)])
            th.start()
            owners = []
            for i in range(nframes):
                item = d.get_next_frame(timeout=60)
                assert item is not None, d.ordering_stats()
                idx, data, info = item
                assert idx == i
                assert np.array_equal(np.frombuffer(data, np.uint8), want[i % 4]), i
                owners.append(info["process_id"])
            th.join()
        finally:
            stop_workers(stop, procs)
        nchunks = nframes // 16
        chunks = [set(owners[c * 16:(c + 1) * 16]) for c in range(nchunks)]
        assert all(len(c) == 1 for c in chunks)
        owner = [next(iter(c)) for c in chunks]
        assert len(set(owner[:nworkers])) == nworkers       # one shard per worker
        assert all(owner[c] == owner[c % nworkers] for c in range(nchunks))  # chunk_owner(i, 16, N)
        st = d.ordering_stats()
        assert st["released"] == nframes and st["lost"] == 0 and st["evictions"] == 0
        assert d.free_slots() == d.total_slots() == nworkers * ring_slots
        return st
    finally:
        d.cleanup()


@pytest.mark.timeout(180)
def test_configs2_4k_batch16_sharded_in_order_ring():
    _sharded_4k(2, 64, 24)


@pytest.mark.timeout(240)
def test_configs2_4k_batch16_eight_way_shard_one_card():
    """BASELINE configs[2]'s fan-out width: 8 worker processes (on the box's one GPU), 8
    frame-index shards, 160 frames (10 chunks of 16) through 8 per-worker ring slices."""
    st = _sharded_4k(8, 160, 16)
    assert len(st["workers"]) == 8


@pytest.mark.timeout(180)
@pytest.mark.parametrize("reader", ["thread", "select"])
def test_configs3_mixed_resolution_pull_tcp_payloads(monkeypatch, reader):
    """Frames as socket payloads (no ring) through the Python engine, in both reader forms: the
    select form hung here in round 4 (a handler's blocking dispatch send under the distributor's
    lock); dispatches are now sent outside it."""
    from vfilter import transport as tp
    monkeypatch.setattr(tp, "_READER", reader)
    shapes = [(480, 640), (1080, 1920), (2160, 3840)]
    frames = [oracle.synthetic_frame(i, *shapes[i % 3]) for i in range(24)]
    d = Distributor(0, 0, 5, True, policy="pull", reassembly="ordered", queue_size=16, transport="tcp",
                    host="127.0.0.1", verbose=False)
    d.start()
    try:
        infos = _run(d, frames, 2, batch=4)
        assert [i["shape"] for i in infos[:3]] == [list(s) + [3] for s in shapes]
        s = d.ordering_stats()
        assert s["released"] == 24 and s["lost"] == 0
        # GPU spans from the workers' slot events reach the trace (H2D -> kernel -> D2H)
        ev = [e for e in d.trace_events() if e.get("cat") == "gpu"]
        kern = [e for e in ev if e["name"] == "GPU kernel"]
        assert kern and all(e["tid"] == 2 and e["dur"] >= 0 for e in kern)
        assert sum(e["args"]["bytes"] for e in kern) == sum(f.nbytes for f in frames)
        assert {e["name"] for e in ev} == {"GPU H2D", "GPU kernel", "GPU D2H"}
    finally:
        d.cleanup()


@pytest.mark.timeout(120)
def test_inverter_worker_call_matches_captured_reference(golden_dir):
    """The product InverterWorker.__call__ (raw) against the reference's own __call__ outputs
    captured in tests/golden/ref_inverter_call.json (inverter.py:34 -> :41 -> :46); where the
    reference raises ValueError (sizes other than 480x480) the product inverts."""
    import hashlib
    import json
    from vfilter.inverter import InverterWorker
    d = json.load(open(os.path.join(golden_dir, "ref_inverter_call.json")))
    w = InverterWorker("127.0.0.1", 1, 1, 0.0, use_jpeg=False, install_signal_handlers=False, transport="tcp")
    try:
        for c in d["cases"]:
            x = oracle.synthetic_frame(c["seed"], *c["shape"][:2]).tobytes()
            assert hashlib.sha256(x).hexdigest() == c["input_sha256"]
            y = bytes(w(x))
            assert len(y) == c["output_len"] and hashlib.sha256(y).hexdigest() == c["output_sha256"]
        for e in d["other_sizes"]:
            x = oracle.synthetic_frame(1, *e["shape"][:2]).tobytes()
            assert bytes(w(x)) == oracle.invert_bytes(x)
    finally:
        w.close()


@pytest.mark.timeout(120)
def test_inverter_worker_call_matches_reference_raw_path():
    """InverterWorker.__call__ on a 480x480 raw frame == the reference's raw path output
    (inverter.py:34 -> :41 -> :46), and any other size works too (the reference drops it)."""
    from vfilter.inverter import InverterWorker
    w = InverterWorker("127.0.0.1", 1, 1, 0.0, use_jpeg=False, install_signal_handlers=False, transport="tcp")
    try:
        x = oracle.synthetic_frame(9, 480, 480).tobytes()
        assert bytes(w(x)) == oracle.reference_raw_call(x)
        y = oracle.synthetic_frame(9, 1080, 1920).tobytes()
        assert bytes(w(y)) == oracle.invert_bytes(y)
    finally:
        w.close()


@pytest.mark.timeout(120)
def test_inverter_worker_jpeg_mode_matches_reference_path():
    """use_jpeg=True (the reference default): __call__ = decode -> bitwise_not -> encode
    (inverter.py:32 -> :41 -> :44), bit-exact with the oracle's restatement of PyTurboJPEG /
    libjpeg-turbo; with --delay the unfused path gives the same bytes."""
    from oracle import jpeg as J
    from vfilter.inverter import InverterWorker
    jpg = J.encode(J.synthetic_scene(4, 480, 640))
    small = J.encode(J.synthetic_scene(5, 64, 48))
    w = InverterWorker("127.0.0.1", 1, 1, 0.0, use_jpeg=True, install_signal_handlers=False, transport="tcp")
    wd = InverterWorker("127.0.0.1", 1, 1, 0.001, use_jpeg=True, install_signal_handlers=False, transport="tcp")
    try:
        want = J.invert_jpeg(jpg)
        assert bytes(w(jpg)) == want
        assert bytes(wd(jpg)) == want
        res = w.process_batch([jpg, small], [None, None], [None, None])
        assert bytes(res[0]) == want and bytes(res[1]) == J.invert_jpeg(small)
        bad = w.process_batch([jpg, b"\xff\xd8garbage"], [None, None], [None, None])
        assert bytes(bad[0]) == want and isinstance(bad[1], Exception)  # a bad frame fails alone
        h = w.submit_batch([jpg, small], [None, None], [None, None])  # the worker loop's async form
        got, _ = w.poll_batch(h, block=True)
        assert [bytes(g) for g in got] == [want, J.invert_jpeg(small)]
    finally:
        w.close()
        wd.close()


@pytest.mark.timeout(180)
def test_jpeg_mode_through_ring_in_order():
    """JPEG frames (the reference default) through the shared-memory ring: each result is a
    JPEG of its own size, written into the slot's output half (or sent back over the socket
    when it does not fit) and read with its own length."""
    from oracle import jpeg as J
    jpgs = [J.encode(J.synthetic_scene(i, 480, 640) if i % 3 else
                     np.random.default_rng(i).integers(0, 256, (96, 128, 3), dtype=np.uint8), 85)
            for i in range(24)]
    slot = max(len(j) for j in jpgs)
    d = Distributor(0, 0, policy="pull", reassembly="ordered", queue_size=16, ring_slots=8, ring_slot_bytes=slot,
                    transport="tcp", host="127.0.0.1", verbose=False)
    d.start()
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=4, kind="gpu",
                                use_jpeg=True)
    try:
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(j) for j in jpgs])
        th.start()
        for i in range(len(jpgs)):
            item = d.get_next_frame(timeout=60)
            assert item is not None, d.ordering_stats()
            assert item[0] == i and bytes(item[1]) == J.invert_jpeg(jpgs[i]), i
        th.join()
        assert d.free_slots() == d.total_slots()
        assert d.ordering_stats()["result_errors"] == 0
    finally:
        stop_workers(stop, procs)
        d.cleanup()


@pytest.mark.timeout(180)
def test_jpeg_mode_through_distributor_in_order():
    """The reference's default deployment: JPEG frames (webcam_app.py:110) through the
    distributor to 2 GPU workers in JPEG mode and back in index order, bit-exact."""
    from oracle import jpeg as J
    jpgs = [J.encode(J.synthetic_scene(i, 480 if i % 2 else 1080, 640 if i % 2 else 1920)) for i in range(24)]
    d = Distributor(0, 0, 5, True, policy="pull", reassembly="ordered", queue_size=16, transport="tcp",
                    host="127.0.0.1", verbose=False)
    d.start()
    stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=4, kind="gpu",
                                use_jpeg=True)
    try:
        th = threading.Thread(target=lambda: [d.add_frame_for_distribution(j) for j in jpgs])
        th.start()
        for i in range(len(jpgs)):
            item = d.get_next_frame(timeout=60)
            assert item is not None, d.ordering_stats()
            idx, data, _ = item
            assert idx == i
            assert bytes(data) == J.invert_jpeg(jpgs[i]), i
        th.join()
    finally:
        stop_workers(stop, procs)
        d.cleanup()
