"""This build's worker and distributor against the REAL reference, over real ZeroMQ (CPU).

Either half of the reference can be swapped for this build's independently: wire v0 is the
reference's own message layout (worker.py:39,50-51,63-67 / distributor.py:226-238,260-264).
Needs /root/reference and /opt/conda/bin/python3.9 (pyzmq); both exist only in the build
container, so the test skips elsewhere (e.g. on the GPU box).
"""
import json
import os
import subprocess

import pytest

REF = "/root/reference"
PY39 = "/opt/conda/bin/python3.9"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(PY39)),
                                reason="reference or its pyzmq interpreter not present")


def _run(mode):
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONHOME", "PYTHONPATH")}
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    r = subprocess.run([PY39, "-B", os.path.join(ROOT, "tests", "_interop_ref.py"), REF, ROOT, mode],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(150)
def test_reference_distributor_drives_this_worker():
    out = _run("ref-distributor")
    assert len(out["frames"]) == 4
    for f in out["frames"]:
        assert f["ok"] and f["exact"] and f["pid_is_worker"] and f["start_le_end"], f


@pytest.mark.timeout(150)
def test_this_distributor_drives_reference_worker():
    out = _run("ref-worker")
    assert len(out["frames"]) == 4
    for f in out["frames"]:
        assert f["ok"] and f["exact"] and f["pid_is_worker"] and f["start_le_end"], f
    assert out["stats"]["total_frames_processed"] == 4 and out["stats"]["frame_delay"] == 0
