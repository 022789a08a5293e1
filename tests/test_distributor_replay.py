"""The PRODUCT distributor driven through the op sequences captured from the real reference
(tests/golden/ref_ingest.json, ref_dispatch.json; capture_reference.py), step for step — the
oracle is pinned to the same files in test_oracle_golden.py.  CPU only.

ingest   distributor.py:173-203   global frame_index counter, queue.Queue(maxsize=10),
                                  drop-oldest-and-retry when full
dispatch distributor.py:205-251   one queued frame moves into the latest-wins slot per loop
                                  iteration; a READY is answered [index, frame] only if the
                                  slot's index > last_frame_sent
The capture waited > 10 ms after each add, i.e. one dispatch iteration per frame; here each
iteration is one ``Distributor.dispatch_step`` and the worker end is a real v0 DEALER over the
stdlib transport, so the reply bytes are the wire bytes.
"""
import json
import os
import time

import pytest

from vfilter import transport as tp
from vfilter import wire
from vfilter.distributor import Distributor


def _load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


def _dist(**kw):
    return Distributor(0, 0, transport="tcp", host="127.0.0.1", verbose=False, **kw)


def test_product_ingest_queue_matches_reference(golden_dir):
    d = _load(golden_dir, "ref_ingest.json")
    for case in d["cases"]:
        dist = _dist(queue_size=d["queue_maxsize"])
        try:
            for i in range(case["n_added"]):
                assert dist.add_frame_for_distribution(b"x%d" % i, 1000.0 + i) == i
            kept = []
            while not dist.frame_queue.empty():
                it = dist.frame_queue.get_nowait()
                kept.append([it["frame_index"], bytes(it["frame"]).decode(), it["timestamp"]])
            assert kept == case["kept"], case["n_added"]
            assert dist.frame_index_counter == case["frame_index_counter"]
            assert dist.frames_dropped == max(0, case["n_added"] - d["queue_maxsize"])
        finally:
            dist.cleanup()


def _recv_reply(dealer, timeout_s):
    if dealer.poll(int(timeout_s * 1000)):
        return [bytes(x) for x in dealer.recv()]
    return None


def test_product_dispatch_slot_matches_reference(golden_dir):
    steps = {s["step"]: s for s in _load(golden_dir, "ref_dispatch.json")["steps"]}
    dist = _dist()
    dealer = tp.DealerEnd("tcp", "127.0.0.1", dist.distribute_port)
    try:
        def add(i):  # one add, then one loop iteration (the capture's > 10 ms wait)
            dist.add_frame_for_distribution(b"frame-%d" % i)
            dist.dispatch_step(0)

        def ready(step):
            dealer.send(wire.encode_request(version=0))           # worker.py:39
            t0 = time.monotonic()
            while not dist.distribute_socket.poll(10):
                assert time.monotonic() - t0 < 5, "READY never arrived"
            dist.dispatch_step(0)
            got = _recv_reply(dealer, 0.3 if steps[step]["reply"] is None else 5.0)
            want = steps[step]["reply"]
            if want is None:
                assert got is None, (step, got)
            else:
                assert got is not None and len(got) == steps[step]["n_parts"], (step, got)
                assert [got[0].decode(), got[1].decode()] == want, step

        ready("ready-before-any-frame")
        add(0)
        ready("ready-after-frame-0")
        ready("ready-again-no-new-frame")
        for i in (1, 2, 3):
            add(i)
        ready("ready-after-frames-1-2-3")
        add(4)
        add(5)
        ready("ready-after-frames-4-5")
        ready("ready-again-no-new-frame-2")
        assert dist.last_frame_sent == 5
        # frames 1, 2 and 4 were overwritten in the slot before any READY took them
        assert dist.frames_dropped == 3
    finally:
        dealer.close()
        dist.cleanup()


def test_ordered_latest_drops_are_marked_lost():
    """policy='latest' with reassembly='ordered': a frame the latest policy discards is
    counted lost at once, so the in-order consumer is never left waiting for it."""
    dist = _dist(policy="latest", reassembly="ordered", queue_size=2)
    try:
        for i in range(5):
            dist.add_frame_for_distribution(b"f%d" % i)
        # indices 0..2 were dropped from the full queue (3 and 4 are queued)
        assert dist.frames_dropped == 3
        assert dist.ordering_stats()["next_index"] == 3
    finally:
        dist.cleanup()


def test_nonblocking_reject_does_not_consume_an_index():
    dist = _dist(policy="pull", reassembly="ordered", queue_size=2)
    try:
        assert dist.add_frame_for_distribution(b"a", block=False) == 0
        assert dist.add_frame_for_distribution(b"b", block=False) == 1
        assert dist.add_frame_for_distribution(b"c", block=False) == -1   # queue full
        assert dist.frame_index_counter == 2
        dist._pending.popleft()   # a worker took frame 0
        assert dist.add_frame_for_distribution(b"d", block=False) == 2
    finally:
        dist.cleanup()
