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


@pytest.mark.timeout(180)
def test_config3_4k_batch16_sharded_in_order_ring():
    d = Distributor(0, 0, policy="shard", reassembly="ordered", shard_workers=2, shard_chunk=16,
                    queue_size=64, ring_slots=24, ring_slot_bytes=2160 * 3840 * 3, transport="tcp",
                    host="127.0.0.1", verbose=False)
    d.start()
    try:
        frames = [oracle.synthetic_frame(i % 4, 2160, 3840) for i in range(64)]
        stop, procs = spawn_workers(2, d.distribute_port, d.collect_port, protocol="v1", batch=16, kind="gpu")
        try:
            time.sleep(3.0)  # both workers register (GPU context creation) before frames flow
            th = threading.Thread(target=lambda: [d.add_frame_for_distribution(f) for f in frames])
            th.start()
            owners = []
            for i in range(len(frames)):
                item = d.get_next_frame(timeout=60)
                assert item is not None, d.ordering_stats()
                idx, data, info = item
                assert idx == i
                assert np.array_equal(np.frombuffer(data, np.uint8), oracle.invert(frames[i]).reshape(-1))
                owners.append(info["process_id"])
            th.join()
        finally:
            stop_workers(stop, procs)
        chunks = [set(owners[c * 16:(c + 1) * 16]) for c in range(4)]
        assert all(len(c) == 1 for c in chunks) and chunks[0] != chunks[1] and chunks[0] == chunks[2]
        assert d.ring.free_slots() == 24
    finally:
        d.cleanup()


@pytest.mark.timeout(180)
def test_config4_mixed_resolution_pull_tcp_payloads():
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
