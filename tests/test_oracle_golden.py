"""Pin the CPU oracle to the golden fixtures (CPU only).

The oracle is the checker for every GPU parity test, so it is checked first: against the
known-answer vectors (tests/golden/kat.json, seeded_digests.json) and against traces of
the real reference distributor.py / worker.py (tests/golden/ref_*.json, captured by
tests/golden/capture_reference.py).
"""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle


def _load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module", autouse=True)
def _built_oracle():
    if not os.path.exists(oracle.ORACLE_LIB):
        rc = os.system(f"make -s -C {os.path.dirname(oracle.ORACLE_LIB)}/..")
        assert rc == 0, "make -C oracle failed"


def test_kat_numpy_and_c(golden_dir):
    kats = _load(golden_dir, "kat.json")["kats"]
    assert {k["name"] for k in kats} >= {"all_values_16x16x3", "ragged_17x13x3", "tiny_1x1x3", "empty_0x0x3"}
    for k in kats:
        x = np.frombuffer(bytes.fromhex(k["input_hex"]), dtype=np.uint8).reshape(k["shape"])
        want = bytes.fromhex(k["expected_hex"])
        assert oracle.invert(x).tobytes() == want, k["name"]
        assert oracle.c_invert(x).tobytes() == want, k["name"]
        assert oracle.invert_bytes(x.tobytes()) == want, k["name"]


def test_all_byte_values_covered(golden_dir):
    k = [k for k in _load(golden_dir, "kat.json")["kats"] if k["name"] == "all_values_16x16x3"][0]
    x = bytes.fromhex(k["input_hex"])
    assert sorted(set(x)) == list(range(256))
    y = bytes.fromhex(k["expected_hex"])
    assert all(a + b == 255 for a, b in zip(x, y))


@pytest.mark.parametrize("size", ["480sq", "480p", "1080p"])
def test_seeded_digests(golden_dir, size):
    for rec in _load(golden_dir, "seeded_digests.json")["frames"]:
        if rec["size"] != size:
            continue
        h, w, _ = rec["shape"]
        x = oracle.synthetic_frame(rec["seed"], h, w)
        assert hashlib.sha256(x.tobytes()).hexdigest() == rec["input_sha256"], "rng stream drifted"
        assert hashlib.sha256(oracle.invert(x).tobytes()).hexdigest() == rec["expected_sha256"]


def test_reference_raw_framing():
    """inverter.py:34 accepts exactly 480x480x3; other sizes raise ValueError."""
    x = oracle.synthetic_frame(0, 480, 480)
    out = oracle.reference_raw_call(x.tobytes())
    assert out == (255 - x.astype(np.int16)).astype(np.uint8).tobytes()
    with pytest.raises(ValueError):
        oracle.reference_raw_call(oracle.synthetic_frame(0, 480, 640).tobytes())


def test_reference_worker_payloads(golden_dir):
    """The real worker.py loop (plugin = byte inversion) returned ~x for every frame, in the
    5-part layout worker.py:63-67, and the oracle agrees byte for byte."""
    d = _load(golden_dir, "ref_worker.json")
    assert len(d["frames"]) >= 4
    for f in d["frames"]:
        x = bytes.fromhex(f["input_hex"])
        assert oracle.invert_bytes(x) == bytes.fromhex(f["output_hex"])
        assert f["process_id_is_worker_pid"] and f["start_le_end"]


def test_ingest_queue_matches_reference(golden_dir):
    d = _load(golden_dir, "ref_ingest.json")
    for case in d["cases"]:
        q = oracle.RefIngestQueue(d["queue_maxsize"])
        for i in range(case["n_added"]):
            q.add(b"x%d" % i, 1000.0 + i)
        kept = []
        while True:
            it = q.get_nowait()
            if it is None:
                break
            kept.append([it["frame_index"], it["frame"].decode(), it["timestamp"]])
        assert kept == case["kept"], case["n_added"]
        assert q.frame_index_counter == case["frame_index_counter"]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "ref_display_*.json"))))
def test_display_policy_matches_reference(path):
    d = json.load(open(path))
    got = oracle.replay_display_ops(d["ops"], d["frame_delay"], d["frame_buffer_size"])
    assert len(got) == len(d["records"])
    for i, (g, r) in enumerate(zip(got, d["records"])):
        assert g == r, f"{os.path.basename(path)} op #{i} {r['op']}: oracle {g} != reference {r}"


def test_dispatch_slot_matches_reference(golden_dir):
    """Replay ref_dispatch.json's scenario through the latest-wins slot model."""
    steps = {s["step"]: s["reply"] for s in _load(golden_dir, "ref_dispatch.json")["steps"]}
    q, slot = oracle.RefIngestQueue(), oracle.RefDispatchSlot()

    def add(i):  # the capture waits > 10 ms after each add: one dispatch iteration each
        q.add(b"frame-%d" % i)
        slot.pull(q.get_nowait())

    def ready():
        it = slot.on_ready()
        return None if it is None else [str(it["frame_index"]), it["frame"].decode()]

    assert ready() == steps["ready-before-any-frame"]
    add(0)
    assert ready() == steps["ready-after-frame-0"]
    assert ready() == steps["ready-again-no-new-frame"]
    for i in (1, 2, 3):
        add(i)
    assert ready() == steps["ready-after-frames-1-2-3"]
    add(4)
    add(5)
    assert ready() == steps["ready-after-frames-4-5"]
    assert ready() == steps["ready-again-no-new-frame-2"]


def test_oracle_raw_call_matches_reference_inverter(golden_dir):
    """ref_inverter_call.json: the reference's own InverterWorker.__call__ (use_jpeg=False,
    inverter.py:29-46) on seeded 480x480 frames, captured by capture_inverter_call.py (cv2 is
    absent: its bitwise_not was numpy's, so this pins the raw framing, see the fixture)."""
    d = _load(golden_dir, "ref_inverter_call.json")
    assert len(d["cases"]) >= 4 and "cv2.bitwise_not" in d["stand_ins"]
    for c in d["cases"]:
        h, w, _ = c["shape"]
        x = oracle.synthetic_frame(c["seed"], h, w).tobytes()
        assert hashlib.sha256(x).hexdigest() == c["input_sha256"], "rng stream drifted"
        y = oracle.reference_raw_call(x)
        assert isinstance(y, bytes) and len(y) == c["output_len"]
        assert hashlib.sha256(y).hexdigest() == c["output_sha256"]
        assert y[:64].hex() == c["output_prefix_hex"]
    for e in d["other_sizes"]:
        with pytest.raises(ValueError) as ei:
            oracle.reference_raw_call(np.zeros(e["shape"], np.uint8).tobytes())
        assert e["error_type"] == "ValueError" and str(ei.value) == e["error"]
