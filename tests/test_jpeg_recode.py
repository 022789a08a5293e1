"""The test-side Huffman re-coder (tests/jpeg_recode.py) keeps every coefficient: re-coded
frames decode to the same pixels in the oracle and in the image's libjpeg-turbo, and the
tables it makes have many more codes longer than the GPU decoder's 9-bit lookahead than the
Annex K tables TurboJPEG writes (tests/test_gpu_jpeg.py test_custom_tables_long_codes)."""
import numpy as np
import pytest

import jpeg_recode as R
from oracle import jpeg as J


def _srcs():
    rng = np.random.default_rng(7)
    return [J.encode(rng.integers(0, 256, (64, 96, 3), dtype=np.uint8), 90, J.TJPF_BGR, J.TJSAMP_422),
            J.encode(J.synthetic_scene(5, 120, 160), 85, J.TJPF_BGR, J.TJSAMP_420),
            J.encode(J.synthetic_scene(6, 40, 56), 85, J.TJPF_BGR, J.TJSAMP_GRAY)]


@pytest.mark.parametrize("kw", [{}, {"dc_long": 11, "ac_long": 10}, {"ac_long": 16, "share": True}, {"split": True}])
def test_recode_keeps_pixels(kw):
    have_lib = J.libjpeg_available()[0]
    for j in _srcs():
        if kw.get("split") and J.info(j)["ncomp"] != 3:
            continue  # three components only
        r = R.recode(j, **kw)
        assert r != j
        want = J.decode(j)
        assert np.array_equal(J.decode(r), want)
        if have_lib:
            assert np.array_equal(J.libjpeg_decode(r), want)


def test_recoded_tables_have_many_long_codes():
    r = R.recode(_srcs()[0], dc_long=11, ac_long=10)
    segs, _, _ = R._segments(r)
    need = sum(R.long_prefixes(bits) for bits, _ in R._dht_tables(segs).values())
    assert need > 12
    annex_k = R._dht_tables(R._segments(_srcs()[0])[0])
    assert sum(R.long_prefixes(bits) for bits, _ in annex_k.values()) == 11  # 5 + 5 + 1 + 0


def test_split_tables_give_three_distinct_pairs():
    """recode(split=True): components 0, 1, 2 on (DC, AC) table ids (0, 0), (1, 1), (1, 0) --
    the case the span sync's 4-table layout cannot hold (vf_jpeg_host.hip, DecFrame::tabs4)."""
    r = R.recode(_srcs()[0], split=True)
    segs, _, _ = R._segments(r)
    sos = next(pl for m, pl in segs if m == 0xDA)
    assert [(sos[2 + 2 * c] >> 4, sos[2 + 2 * c] & 15) for c in range(3)] == R.SPLIT_IDS
    assert set(R._dht_tables(segs)) == {(0, 0), (0, 1), (1, 0), (1, 1)}
