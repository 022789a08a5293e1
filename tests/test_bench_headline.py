"""bench.py's output contract: the LAST stdout line is a compact headline (<= 7,000 bytes)
that the driver parses from a bounded stdout tail; the full record goes to a detail file.
Fed with full records of earlier rounds (N=1 and an N=4 rehearsal), which were 21-22 KB."""
import io
import json
import os
import sys
from contextlib import redirect_stderr, redirect_stdout

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORDS = ["profiles/r05_bench_end.json", "profiles/r05_bench_n4_rehearsal_1card.json"]
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _record(rel):
    path = os.path.join(ROOT, rel)
    if not os.path.exists(path):
        pytest.skip(f"{rel} not in this tree")
    last = [ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1]
    return json.loads(last)


@pytest.mark.parametrize("rel", RECORDS)
def test_headline_fits_and_keeps_the_contract(rel, tmp_path):
    line = _record(rel)
    assert len(json.dumps(line)) > 2 * bench.HEADLINE_MAX_BYTES  # the shape that went unparsed
    out, err = io.StringIO(), io.StringIO()
    with redirect_stdout(out), redirect_stderr(err):
        bench.emit(dict(line), str(tmp_path / "bench_detail.json"))
    last = out.getvalue().splitlines()[-1]
    assert len(last.encode()) <= bench.HEADLINE_MAX_BYTES
    h = json.loads(last)
    for k in REQUIRED:
        assert k in h, k
    assert h["value"] == line["value"] and h["n_gpus"] == line["n_gpus"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in h["roofline"], k
    assert h["roofline"]["traffic"] == line["roofline"]["traffic"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in h["cpu_baseline"], k
    assert h["cpu_baseline"]["multi_process"]["value"] == line["cpu_baseline"]["multi_process"]["value"]
    # one-number summaries of every leg survive
    assert set(h["sizes"]) == {"480p", "1080p", "4k"}
    assert set(h["configs4_sweep"]) == {"256", "512", "1024", "2048", "4096"}
    assert h["jpeg_mode"]["gpu_resident_fps"] == line["jpeg_mode"]["gpu_resident_fps"]
    assert "huffman_sync_ms" in h["jpeg_mode"]["hard"]
    legs = {k for k in line["distributor"] if k != "note"}
    assert set(h["distributor"]) == legs
    for leg in legs:
        assert h["distributor"][leg]["fps"] == line["distributor"][leg]["fps"]
        assert h["distributor"][leg]["n_errors"] == 0
    # the detail file holds the whole record and the headline points at it
    detail = json.load(open(tmp_path / "bench_detail.json"))
    assert detail["jpeg_mode"] == line["jpeg_mode"] and detail["distributor"] == line["distributor"]
    assert h["detail"].endswith("bench_detail.json")
    assert "[bench] detail: " in err.getvalue()


def test_headline_overflow_drops_legs_not_the_contract(tmp_path):
    line = _record(RECORDS[0])
    line["distributor"] = {f"leg{i}": {"fps": i, "n_errors": 0, "control_plane": {"fps": 1.0}} for i in range(400)}
    out = io.StringIO()
    with redirect_stdout(out), redirect_stderr(io.StringIO()):
        bench.emit(line, str(tmp_path / "d.json"))
    last = out.getvalue().splitlines()[-1]
    assert len(last.encode()) <= bench.HEADLINE_MAX_BYTES
    h = json.loads(last)
    assert "distributor" not in h and all(k in h for k in REQUIRED)


def test_headline_with_failed_legs():
    line = _record(RECORDS[0])
    line["jpeg_mode"] = {"error": "rc=1: " + "x" * 5000}
    line["distributor"] = {"jpeg_512": {"error": "timed out after 150 s"}, "note": "n"}
    line["per_frame"] = {"error": "rc=1"}
    line["cpu_baseline"] = None
    h = bench.headline(line)
    s = json.dumps(h)
    assert len(s) <= bench.HEADLINE_MAX_BYTES
    assert h["distributor"]["jpeg_512"]["error"].startswith("timed out")
    assert h["cpu_baseline"] is None


R06_RUNS = [("profiles/r06_bench_detail_end.json", "profiles/r06_bench_end.json"),
            ("profiles/r06_bench_detail_prefetch.json", "profiles/r06_bench_prefetch.json"),
            ("profiles/r06_bench_detail_reps5.json", "profiles/r06_bench_reps5.json"),
            ("profiles/r06_bench_detail_confirm.json", "profiles/r06_bench_confirm.json"),
            ("profiles/r06_bench_n2_rehearsal_1card_detail.json", "profiles/r06_bench_n2_rehearsal_1card.json"),
            ("profiles/r06_bench_n4_rehearsal_1card_detail.json", "profiles/r06_bench_n4_rehearsal_1card.json")]


@pytest.mark.parametrize("detail,headline", R06_RUNS)
def test_round6_headlines_are_what_emit_makes_of_their_detail(detail, headline, tmp_path):
    """The committed round-6 GPU runs (N=1 end and confirmation, the N=2 and N=4 one-card
    rehearsals): emit() on each detail record gives back, key for key, the headline that run
    printed last -- so the evidence under profiles/ is one record seen two ways, and the
    headline stays under the driver's limit at every N rehearsed."""
    path = os.path.join(ROOT, detail)
    if not os.path.exists(path):
        pytest.skip(f"{detail} not in this tree")
    rec = json.load(open(path))
    out = io.StringIO()
    with redirect_stdout(out), redirect_stderr(io.StringIO()):
        bench.emit(dict(rec), str(tmp_path / "bench_detail.json"))
    last = out.getvalue().splitlines()[-1]
    assert len(last.encode()) <= bench.HEADLINE_MAX_BYTES
    got, want = json.loads(last), _record(headline)
    got.pop("detail"), want.pop("detail")
    assert got == want
    assert all(k in got for k in REQUIRED)
    assert got["n_gpus"] == rec["n_gpus"] and got["value"] == rec["value"]
