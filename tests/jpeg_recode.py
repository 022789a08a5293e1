"""TEST INFRASTRUCTURE: re-code a baseline JPEG's entropy-coded data with other Huffman tables.

The codec under the reference (libjpeg-turbo via PyTurboJPEG, inverter.py:32) decodes any
valid DHT, but TurboJPEG-made frames always carry the Annex K tables.  To exercise the GPU
decoder on tables with many codes longer than its kLook-bit lookahead (the second-level
slots, and the slow path when they run out: vf_jpeg.h kSubSlots), this module decodes a
scan's Huffman symbols with the file's own tables (T.81 F.2.2, as jdhuff.c) and writes the
same symbols and extra bits with new canonical tables (T.81 C / K.2 code assignment).  The
coefficients, hence the decoded pixels, are unchanged; tests check that with the oracle.

Pure Python: small frames only.  No restart markers (the input comes from the oracle encoder).
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, List, Tuple


def _segments(b: bytes):
    """(marker, payload) up to and including SOS, then the entropy-coded bytes and the tail."""
    assert b[0] == 0xFF and b[1] == 0xD8
    p, segs = 2, []
    while True:
        assert b[p] == 0xFF
        m = b[p + 1]
        ln = (b[p + 2] << 8) | b[p + 3]
        segs.append((m, b[p + 4:p + 2 + ln]))
        p += 2 + ln
        if m == 0xDA:
            break
    q = p
    while not (b[q] == 0xFF and b[q + 1] not in (0x00,) and not (0xD0 <= b[q + 1] <= 0xD7)):
        q += 1
    return segs, b[p:q], b[q:]


def _dht_tables(segs) -> Dict[Tuple[int, int], Tuple[List[int], List[int]]]:
    t = {}
    for m, pl in segs:
        if m != 0xC4:
            continue
        i = 0
        while i < len(pl):
            tc, th = pl[i] >> 4, pl[i] & 15
            bits = list(pl[i + 1:i + 17])
            n = sum(bits)
            t[(tc, th)] = (bits, list(pl[i + 17:i + 17 + n]))
            i += 17 + n
    return t


def _codes(bits: List[int], vals: List[int]) -> Dict[int, Tuple[int, int]]:
    """symbol -> (code, length), canonical (T.81 C.2)."""
    out, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            out[vals[k]] = (code, ln)
            code += 1
            k += 1
        code <<= 1
    return out


class _Bits:
    def __init__(self, data: bytes):
        self.d = data.replace(b"\xff\x00", b"\xff")
        self.pos = 0

    def bit(self) -> int:
        i = self.pos >> 3
        v = (self.d[i] >> (7 - (self.pos & 7))) & 1 if i < len(self.d) else 0
        self.pos += 1
        return v

    def read(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bit()
        return v

    def sym(self, dec: Dict[Tuple[int, int], int]) -> int:
        code = 0
        for ln in range(1, 17):
            code = (code << 1) | self.bit()
            if (ln, code) in dec:
                return dec[(ln, code)]
        raise ValueError("bad Huffman code")


def tokens(jpeg: bytes, with_comp: bool = False):
    """The scan's symbols in order: (class, table id, symbol, extra value, extra bits), plus the
    component with ``with_comp``."""
    segs, ecs, _ = _segments(jpeg)
    tabs = _dht_tables(segs)
    sof = next(pl for m, pl in segs if m in (0xC0, 0xC1))
    sos = next(pl for m, pl in segs if m == 0xDA)
    h, w, nc = (sof[1] << 8) | sof[2], (sof[3] << 8) | sof[4], sof[5]
    hs = [sof[7 + 3 * c] >> 4 for c in range(nc)]
    vs = [sof[7 + 3 * c] & 15 for c in range(nc)]
    td = [sos[2 + 2 * c] >> 4 for c in range(nc)]
    ta = [sos[2 + 2 * c] & 15 for c in range(nc)]
    dec = {k: {(ln, c): s for s, (c, ln) in _codes(*v).items()} for k, v in tabs.items()}
    if nc == 1:
        order = [0] * (((w + 7) // 8) * ((h + 7) // 8))
    else:
        mh, mv = max(hs), max(vs)
        nmcu = -(-w // (8 * mh)) * -(-h // (8 * mv))
        per = [c for c in range(nc) for _ in range(hs[c] * vs[c])]
        order = per * nmcu
    br = _Bits(ecs)
    out = []
    for c in order:
        s = br.sym(dec[(0, td[c])])
        out.append((0, td[c], s, br.read(s), s) + ((c,) if with_comp else ()))
        k = 1
        while k < 64:
            rs = br.sym(dec[(1, ta[c])])
            r, s = rs >> 4, rs & 15
            out.append((1, ta[c], rs, br.read(s), s) + ((c,) if with_comp else ()))
            if s:
                k += r + 1
            elif r == 15:
                k += 16
            else:
                break
    return out


def long_tables(freq: Counter, short_len: int, nshort: int, long_len: int) -> Tuple[List[int], List[int]]:
    """Canonical table: the nshort most frequent symbols get short_len bits, the rest
    long_len (Kraft sum < 1, so no code is all ones)."""
    syms = [s for s, _ in sorted(freq.items(), key=lambda x: (-x[1], x[0]))]
    bits = [0] * 16
    vals_by_len: Dict[int, List[int]] = {}
    for i, s in enumerate(syms):
        ln = short_len if i < nshort else long_len
        bits[ln - 1] += 1
        vals_by_len.setdefault(ln, []).append(s)
    assert sum(n / (1 << (i + 1)) for i, n in enumerate(bits)) < 1
    return bits, [s for ln in sorted(vals_by_len) for s in vals_by_len[ln]]


# split=True: table ids per component (DC, AC) -- three distinct pairs, so the components share
# no slot of the span sync's 4-table layout (DecFrame::tabs4) and a batch with such a frame
# takes the 6-table form
SPLIT_IDS = [(0, 0), (1, 1), (1, 0)]


def recode(jpeg: bytes, dc_long: int = 10, ac_long: int = 12, share: bool = False, split: bool = False) -> bytes:
    """The same image with new tables: per table id, the 2 (DC) / 8 (AC) most frequent
    symbols get 2 / 4-bit codes, every other symbol dc_long / ac_long bits.  share=True puts
    every component on table 0 of each class; split=True gives components 0, 1, 2 the table ids
    SPLIT_IDS (three components only)."""
    segs, _, tail = _segments(jpeg)
    toks = tokens(jpeg, with_comp=split)
    if share:
        toks = [(cl, 0, s, v, n) for cl, _, s, v, n in toks]
    if split:
        toks = [(cl, SPLIT_IDS[c][cl], s, v, n) for cl, _, s, v, n, c in toks]
    freq: Dict[Tuple[int, int], Counter] = {}
    for cl, th, s, _, _ in toks:
        freq.setdefault((cl, th), Counter())[s] += 1
    new = {}
    for (cl, th), f in freq.items():
        new[(cl, th)] = long_tables(f, 2, 2, dc_long) if cl == 0 else long_tables(f, 4, 8, ac_long)
    codes = {k: _codes(*v) for k, v in new.items()}
    acc, nacc, out = 0, 0, bytearray()

    def put(v: int, n: int):
        nonlocal acc, nacc
        acc = (acc << n) | (v & ((1 << n) - 1))
        nacc += n
        while nacc >= 8:
            byte = (acc >> (nacc - 8)) & 0xFF
            out.append(byte)
            if byte == 0xFF:
                out.append(0)
            nacc -= 8
        acc &= (1 << nacc) - 1

    for cl, th, s, v, n in toks:
        c, ln = codes[(cl, th)][s]
        put(c, ln)
        if n:
            put(v, n)
    if nacc:
        put((1 << (8 - nacc)) - 1, 8 - nacc)
    dht = bytearray()
    for (cl, th), (bits, vals) in sorted(new.items()):
        dht += bytes([(cl << 4) | th]) + bytes(bits) + bytes(vals)
    hdr = bytearray(b"\xff\xd8")
    for m, pl in segs:
        if m == 0xC4:
            continue
        if m == 0xDA:
            hdr += b"\xff\xc4" + (len(dht) + 2).to_bytes(2, "big") + dht
            if share or split:
                pl = bytearray(pl)
                for c in range(pl[0]):
                    pl[2 + 2 * c] = (SPLIT_IDS[c][0] << 4) | SPLIT_IDS[c][1] if split else 0
                pl = bytes(pl)
        hdr += bytes([0xFF, m]) + (len(pl) + 2).to_bytes(2, "big") + pl
    return bytes(hdr) + bytes(out) + tail


def long_prefixes(bits: List[int], look: int = 9) -> int:
    """kLook-bit prefixes under which only codes longer than `look` bits start (the
    second-level slots a table asks for; canonical codes put them at the top of code space)."""
    space = sum(n << (16 - ln) for ln, n in enumerate(bits, 1) if ln > look)
    return -(-space // (1 << (16 - look)))


def requant16(jpeg: bytes, scale: int) -> bytes:
    """The same entropy-coded data under 16-bit quantisation tables (DQT Pq = 1): every entry
    times `scale`, capped at 65535.  The coefficients are unchanged, their dequantised values
    (hence the picture) are not: with a large scale they leave the range in which the decoder's
    IDCT column pass may use 24-bit multiplies (vf_jpeg_types.h idct_col24_ok), which puts that
    frame on the 32-bit path."""
    segs, ecs, tail = _segments(jpeg)
    hdr = bytearray(b"\xff\xd8")
    for m, pl in segs:
        if m == 0xDB:
            i, new = 0, bytearray()
            while i < len(pl):
                pq, tq = pl[i] >> 4, pl[i] & 15
                n = 128 if pq else 64
                vals = ([(pl[i + 1 + 2 * k] << 8) | pl[i + 2 + 2 * k] for k in range(64)] if pq
                        else list(pl[i + 1:i + 65]))
                new.append(0x10 | tq)
                for v in vals:
                    new += min(65535, v * scale).to_bytes(2, "big")
                i += 1 + n
            pl = bytes(new)
        hdr += bytes([0xFF, m]) + (len(pl) + 2).to_bytes(2, "big") + pl
    return bytes(hdr) + ecs + tail
