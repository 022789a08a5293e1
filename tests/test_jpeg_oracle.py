"""The JPEG oracle (oracle/vf_jpeg_oracle.c) pinned against libjpeg-turbo — CPU only.

The reference's default mode runs PyTurboJPEG (inverter.py:32,44), a wrapper of libturbojpeg
from libjpeg-turbo; neither is installed.  The image's own libjpeg-turbo 2.1.2 (libjpeg.so.8,
the codec libturbojpeg wraps) is driven as TurboJPEG drives it (oracle/jpeg_xcheck.c), and the
restatement must match it bit for bit: encoded bytes and decoded pixels.  The committed golden
vectors (tests/golden/jpeg/, made from libjpeg-turbo by make_jpeg_golden.py) pin the oracle
even where the library is absent.  Also covers the product's host-only JPEG entry points.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import jpeg as J

LIBJPEG, WHY = J.libjpeg_available()
needs_libjpeg = pytest.mark.skipif(not LIBJPEG, reason=f"libjpeg-turbo unavailable: {WHY}")

SIZES = [(1, 1), (1, 17), (17, 1), (7, 5), (8, 8), (16, 16), (17, 13), (33, 9), (64, 48), (130, 66)]


def _img(kind, seed, h, w):
    if kind == "noise":
        return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    if kind == "black":
        return np.zeros((h, w, 3), np.uint8)
    if kind == "white":
        return np.full((h, w, 3), 255, np.uint8)
    if kind == "checker":
        y, x = np.mgrid[:h, :w]
        return np.repeat((((x + y) & 1) * 255).astype(np.uint8)[..., None], 3, axis=2)
    return J.synthetic_scene(seed, h, w)


@needs_libjpeg
@pytest.mark.parametrize("subsamp", [0, 1, 2, 3, 4])
def test_oracle_encode_matches_libjpeg(subsamp):
    for i, (h, w) in enumerate(SIZES):
        for kind in ("scene", "noise", "black", "white", "checker"):
            img = _img(kind, i, h, w)
            for q in (1, 25, 50, 85, 96, 100):
                for fast in (False, True):
                    a = J.libjpeg_encode(img, q, J.TJPF_BGR, subsamp, fast)
                    b = J.encode(img, q, J.TJPF_BGR, subsamp, J.TJFLAG_FASTDCT if fast else 0)
                    assert a == b, (h, w, kind, subsamp, q, fast)


@needs_libjpeg
@pytest.mark.parametrize("subsamp", [0, 1, 2, 3, 4])
def test_oracle_decode_matches_libjpeg(subsamp):
    for i, (h, w) in enumerate(SIZES):
        for kind in ("scene", "noise", "checker"):
            jpg = J.libjpeg_encode(_img(kind, 50 + i, h, w), 80, J.TJPF_BGR, subsamp, False)
            for fu in (False, True):
                for pf in (J.TJPF_BGR, J.TJPF_RGB):
                    a = J.libjpeg_decode(jpg, pf, fu)
                    b = J.decode(jpg, pf, J.TJFLAG_FASTUPSAMPLE if fu else 0)
                    assert np.array_equal(a, b), (h, w, kind, subsamp, fu, pf)


@needs_libjpeg
def test_oracle_full_frames_match_libjpeg():
    for ss in (J.TJSAMP_422, J.TJSAMP_420):
        img = J.synthetic_scene(11, 1080, 1920)
        jpg = J.libjpeg_encode(img, 85, J.TJPF_BGR, ss, False)
        assert J.encode(img, 85, J.TJPF_BGR, ss) == jpg
        assert np.array_equal(J.decode(jpg), J.libjpeg_decode(jpg))


def test_tj_version_dct_choice():
    assert J.fast_dct(0, 85, tj_version=3) is False
    assert J.fast_dct(J.TJFLAG_FASTDCT, 85, tj_version=3) is True
    assert J.fast_dct(0, 85, tj_version=2) is True
    assert J.fast_dct(0, 96, tj_version=2) is False
    assert J.fast_dct(J.TJFLAG_ACCURATEDCT, 85, tj_version=2) is False


def _golden():
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "jpeg")
    with open(os.path.join(d, "manifest.json")) as f:
        return d, json.load(f)["cases"]


def test_oracle_against_golden_vectors():
    """Vectors produced by libjpeg-turbo itself (tests/golden/make_jpeg_golden.py)."""
    d, cases = _golden()
    assert len(cases) >= 8
    for c in cases:
        jpg = open(os.path.join(d, c["file"]), "rb").read()
        assert hashlib.sha256(jpg).hexdigest() == c["jpeg_sha256"]
        dec = J.decode(jpg)
        assert hashlib.sha256(dec.tobytes()).hexdigest() == c["decoded_sha256"], c["file"]
        assert hashlib.sha256(J.invert_jpeg(jpg)).hexdigest() == c["inverted_sha256"], c["file"]
        assert hashlib.sha256(J.encode(dec)).hexdigest() == c["reencoded_sha256"], c["file"]
        # the source frame regenerates bit-exactly (numpy RNG drift would show here)
        h, w, _ = c["shape"]
        if c["kind"] == "scene":
            src = J.synthetic_scene(c["seed"], h, w)
        elif c["kind"] == "noise":
            src = np.random.default_rng(c["seed"]).integers(0, 256, (h, w, 3), dtype=np.uint8)
        else:
            src = np.full((h, w, 3), 200, np.uint8)
        assert hashlib.sha256(src.tobytes()).hexdigest() == c["source_sha256"]
        if not c.get("libjpeg_options"):  # restart markers / optimised tables: not TurboJPEG's encoder
            assert J.encode(src, c["quality"], J.TJPF_BGR, c["subsamp"],
                            J.TJFLAG_FASTDCT if c["fastdct"] else 0) == jpg
        else:
            assert J.info(jpg)["restart_interval"] == c["libjpeg_options"].get("restart_interval", 0) or \
                c["libjpeg_options"].get("restart_rows")


def test_product_header_parser_matches_oracle():
    """vf_jpeg_header (host-only, no GPU) on every golden file."""
    from vfilter._lib import jpeg_header
    d, cases = _golden()
    for c in cases:
        jpg = open(os.path.join(d, c["file"]), "rb").read()
        w, h, ss, cs = jpeg_header(jpg)
        assert (h, w) == tuple(c["shape"][:2])
        assert ss == c["subsamp"]
        assert cs == (2 if c["subsamp"] == J.TJSAMP_GRAY else 1)


def test_product_header_rejects_bad_streams():
    from vfilter import VFilterError
    from vfilter._lib import jpeg_header
    for bad in (b"", b"\xff\xd8", b"GIF89a....", b"\xff\xd8\xff\xd9"):
        with pytest.raises(VFilterError):
            jpeg_header(bad)


def test_product_synthetic_scene_matches_oracle_generator():
    """bench.py makes its JPEG-mode frames with vfilter.synthetic (it may not import the oracle)."""
    from vfilter.synthetic import synthetic_scene
    for seed, (h, w) in enumerate([(17, 13), (480, 640)]):
        assert np.array_equal(synthetic_scene(seed, h, w), J.synthetic_scene(seed, h, w))


def test_bad_huffman_tables_rejected_like_libjpeg():
    """Malformed DHT tables (tests/_jpeg_craft.py) are refused by libjpeg-turbo 2.1.2's
    jdhuff.c (JERR_BAD_HUFF_TABLE) and by the oracle; re-inserting the stream's own tables
    (a legal redefinition) still decodes identically in both.  The GPU codec is held to the
    same cases in tests/test_gpu_jpeg.py."""
    from _jpeg_craft import bad_tables, tables_of, with_table
    good = J.encode(_img("scene", 3, 48, 64))
    want = J.decode(good)
    for seg in tables_of(good).values():
        same = with_table(good, seg)
        assert np.array_equal(J.decode(same), want)
        if LIBJPEG:
            assert np.array_equal(J.libjpeg_decode(same), want)
    for name, seg in bad_tables():
        bad = with_table(good, seg)
        with pytest.raises(ValueError):
            J.decode(bad)
        if LIBJPEG:
            with pytest.raises(RuntimeError):
                J.libjpeg_decode(bad)
