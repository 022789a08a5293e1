"""Malformed-JPEG builders for the error-path tests (test infrastructure).

Each case inserts one extra DHT segment just before SOS, redefining a table the scan uses
(a later DHT replaces an earlier one with the same class and id, jdmarker.c get_dht).  The
tables are ones libjpeg-turbo's jdhuff.c ``jpeg_make_d_derived_tbl`` rejects with
JERR_BAD_HUFF_TABLE: over-subscribed lengths, an all-ones code, DC symbols above 15.
"""
from typing import Dict, List, Tuple


def dht_segment(tc: int, th: int, counts: List[int], vals: bytes) -> bytes:
    """One DHT segment holding one table: class ``tc`` (0 DC, 1 AC), id ``th``,
    ``counts[l-1]`` codes of length l (16 entries), then the symbols."""
    assert len(counts) == 16 and all(0 <= c <= 255 for c in counts) and sum(counts) == len(vals)
    body = bytes([(tc << 4) | th]) + bytes(counts) + bytes(vals)
    n = len(body) + 2
    return b"\xff\xc4" + bytes([n >> 8, n & 255]) + body


def with_table(jpeg: bytes, seg: bytes) -> bytes:
    i = jpeg.find(b"\xff\xda")
    assert i > 0, "no SOS"
    return jpeg[:i] + seg + jpeg[i:]


def _counts(d: Dict[int, int]) -> List[int]:
    return [d.get(l, 0) for l in range(1, 17)]


def bad_tables() -> List[Tuple[str, bytes]]:
    """(name, DHT segment) for each malformed table, all for table id 0 (luma)."""
    return [
        # 255 codes of length 1: the second one (code 1) already fills its length; before the
        # fix the lookahead fill ran off the end of a 1 KiB table.
        ("ac_oversubscribed_255x1", dht_segment(1, 0, _counts({1: 255}), bytes(range(255)))),
        ("ac_oversubscribed_3x1", dht_segment(1, 0, _counts({1: 3}), b"\x00\x01\x02")),
        # lengths 1, 2, 2 -> codes 0, 10, 11: 11 is all ones
        ("ac_all_ones_code", dht_segment(1, 0, _counts({1: 1, 2: 2}), b"\x00\x01\x11")),
        # one code at each length 1..15, two at 16: the second 16-bit code is all ones
        ("ac_all_ones_16", dht_segment(1, 0, _counts({**{l: 1 for l in range(1, 16)}, 16: 2}), bytes(range(17)))),
        ("dc_symbol_16", dht_segment(0, 0, _counts({2: 3}), b"\x00\x05\x10")),
    ]


def tables_of(jpeg: bytes) -> Dict[Tuple[int, int], bytes]:
    """{(class, id): a one-table DHT segment} for every Huffman table the stream defines."""
    out = {}
    i = 2
    while i + 4 <= len(jpeg) and jpeg[i] == 0xFF:
        m, n = jpeg[i + 1], (jpeg[i + 2] << 8) | jpeg[i + 3]
        if m == 0xDA:
            break
        if m == 0xC4:
            j, end = i + 4, i + 2 + n
            while j < end:
                tc, th = jpeg[j] >> 4, jpeg[j] & 15
                counts = list(jpeg[j + 1:j + 17])
                vals = jpeg[j + 17:j + 17 + sum(counts)]
                out[(tc, th)] = dht_segment(tc, th, counts, vals)
                j += 17 + sum(counts)
        i += 2 + n
    return out
