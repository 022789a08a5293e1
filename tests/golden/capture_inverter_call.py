"""Capture the reference's own ``InverterWorker.__call__`` in raw mode.

Run in the build container only (the reference is not on the GPU box):

    env -u PYTHONHOME -u PYTHONPATH /opt/conda/bin/python3.9 -B \
        tests/golden/capture_inverter_call.py /root/reference tests/golden

``inverter.py`` imports ``cv2`` and ``turbojpeg`` at module level; neither exists in any
interpreter of this image (an ordinary ModuleNotFoundError).  Two in-memory stand-in modules are
registered first, as SURVEY §8(c) describes: ``cv2.bitwise_not`` -> ``numpy.bitwise_not`` and
a ``turbojpeg.TurboJPEG`` that is never called in raw mode.  The capture therefore pins the
reference's RAW FRAMING and call path -- ``np.frombuffer(...).reshape(480, 480, 3)``
(inverter.py:34), the filter call on that view (:41), ``.tobytes()`` (:46), and the
ValueError any other size raises (:34) -- not OpenCV's arithmetic, which the definition and
the all-256-values KAT pin (kat.json).  The fixture says so in its "stand_ins" field.

Nothing of the reference is copied: it is imported and called; only inputs (as seeds +
digests) and outputs (digests, a prefix, the error text) are written to
tests/golden/ref_inverter_call.json.
"""
import hashlib
import json
import os
import sys
import types

import numpy as np


def main(ref_dir: str, out_dir: str) -> None:
    cv2 = types.ModuleType("cv2")
    cv2.bitwise_not = np.bitwise_not           # stand-in: OpenCV is not installed
    tj = types.ModuleType("turbojpeg")

    class TurboJPEG:                            # stand-in: raw mode never calls it
        def __init__(self, *a, **k):
            pass

    tj.TurboJPEG = TurboJPEG
    sys.modules["cv2"] = cv2
    sys.modules["turbojpeg"] = tj
    sys.path.insert(0, ref_dir)
    import inverter  # noqa: E402  (the reference's inverter.py)

    w = inverter.InverterWorker(distribute_port=1, collect_port=1, delay=0.0, use_jpeg=False)
    cases = []
    for seed in range(4):
        x = np.random.default_rng(seed).integers(0, 256, (480, 480, 3), dtype=np.uint8).tobytes()
        y = w(x)
        assert isinstance(y, bytes)
        cases.append({"seed": seed, "shape": [480, 480, 3],
                      "input_sha256": hashlib.sha256(x).hexdigest(),
                      "output_sha256": hashlib.sha256(y).hexdigest(),
                      "output_len": len(y), "output_type": type(y).__name__,
                      "output_prefix_hex": y[:64].hex()})
    errors = []
    for shape in ((480, 640, 3), (1080, 1920, 3), (16, 16, 3)):
        x = np.zeros(shape, np.uint8).tobytes()
        try:
            w(x)
            errors.append({"shape": list(shape), "error": None})
        except Exception as e:  # worker.py:74-76 would print this and drop the frame
            errors.append({"shape": list(shape), "error_type": type(e).__name__, "error": str(e)})
    out = {"source": "inverter.py:29-46 (use_jpeg=False), called on the reference's own InverterWorker",
           "stand_ins": {"cv2.bitwise_not": "numpy.bitwise_not (OpenCV absent)",
                         "turbojpeg.TurboJPEG": "inert class (raw mode never calls it)"},
           "pins": "raw framing: frombuffer -> reshape(480,480,3) -> filter -> tobytes; ValueError for other sizes",
           "numpy": np.__version__, "python": sys.version.split()[0],
           "cases": cases, "other_sizes": errors}
    with open(os.path.join(out_dir, "ref_inverter_call.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(cases)} cases, {len(errors)} size checks")
    os._exit(0)  # the reference Worker's zmq sockets are never closed (inverter.py has no close)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
