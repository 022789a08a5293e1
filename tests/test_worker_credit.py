"""The JPEG worker's request size (vfilter/inverter.py auto_credit): with
``batch=0`` (the CLI default) it asks for 64 frames while its frames average at most 64 KB (the
reference app's 512 x 512 crops, webcam_app.py:17,97-111) and 32 otherwise.  CPU only: the
policy and the running mean, without a GPU context."""
from types import SimpleNamespace

from vfilter import inverter as I


def test_auto_credit_thresholds():
    assert I.auto_credit(0) == I.CREDIT == 32          # nothing seen yet
    assert I.auto_credit(30_516) == I.SMALL_CREDIT == 64  # 512 x 512 q85
    assert I.auto_credit(I.SMALL_JPEG_BYTES) == 64
    assert I.auto_credit(I.SMALL_JPEG_BYTES + 1) == 32
    assert I.auto_credit(181_876) == 32                # 1080p q85


def test_request_credit_follows_the_frames():
    w = SimpleNamespace(auto_credit=True, batch=32, _jpeg_bytes=0.0)
    note = lambda total, n: I.InverterWorker._note_jpeg_bytes(w, total, n)  # noqa: E731
    credit = lambda: I.InverterWorker.request_credit(w)  # noqa: E731
    assert credit() == 32
    note(32 * 30_000, 32)
    assert credit() == 64
    for _ in range(8):  # the stream moves to 1080p: the running mean follows within a few batches
        note(32 * 180_000, 32)
    assert credit() == 32
    note(0, 0)  # an empty batch changes nothing
    assert credit() == 32
    fixed = SimpleNamespace(auto_credit=False, batch=16, _jpeg_bytes=1000.0)
    assert I.InverterWorker.request_credit(fixed) == 16
