"""Vectorised CPU simulation of the pass-based Huffman sync (k_sync) on one frame (analysis tool).

Every thread decodes its span (G subsequences of 256 bits) from a guessed entry state; inside a
workgroup of T threads, a thread whose entry differs from its predecessor's exit re-decodes
from that exit, stopping where it rejoins its previous trajectory at a checkpoint (every 64
bits), until no entry changes.  Reports, for pass 0, the rounds per workgroup (the serial
chain) and the symbols decoded (the work), per (G, T).

    python tools/sync_sim.py [--content hard|scene] [--size 1080p] [--g 1,2,4,8] [--t 256,64]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "distributed-video-filter_amd")]
from sync_distance import lut, parse  # noqa: E402

SUB = 256
CK = 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--content", default="hard", choices=("hard", "scene"))
    ap.add_argument("--size", default="1080p")
    ap.add_argument("--g", default="1,2,4,8")
    ap.add_argument("--t", default="256,64")
    ap.add_argument("--warm", default="0",
                    help="bits decoded from a guessed state BEFORE each span's start, unrecorded, so the "
                         "entry is (likely) synchronised already (comma list; 0 = entry guessed at the start)")
    a = ap.parse_args()
    from oracle import jpeg as J
    from vfilter.synthetic import synthetic_noisy_scene
    h, w = {"480p": (480, 640), "1080p": (1080, 1920), "4k": (2160, 3840)}[a.size]
    img = synthetic_noisy_scene(0, h, w) if a.content == "hard" else J.synthetic_scene(0, h, w)
    jp = J.encode(img, 95 if a.content == "hard" else 85, J.TJPF_BGR, J.TJSAMP_422)
    comps, sel, tabs, raw = parse(jp)
    blkc = []
    for k, (hs, vs) in enumerate(comps):
        blkc += [k] * (hs * vs)
    blkc = np.array(blkc)
    bpm = len(blkc)
    dcl = np.stack([lut(*tabs[sel[k][0]]) for k in range(len(comps))])
    acl = np.stack([lut(*tabs[0x10 | sel[k][1]]) for k in range(len(comps))])
    bits = np.unpackbits(np.frombuffer(raw + b"\0" * 8, np.uint8))
    nbits = len(raw) * 8
    win = np.zeros(nbits + 32, np.int64)
    for b in range(16):
        win[:nbits + 32 - 16] = (win[:nbits + 32 - 16] << 1) | bits[b:b + nbits + 16]

    def step(pos, z, c):
        k = blkc[c]
        dc = z == 0
        e = np.where(dc, dcl[k, win[pos]], acl[k, win[pos]])
        ln, sym = e >> 8, e & 255
        ln = np.where(ln == 0, 16, ln)
        r, s = sym >> 4, sym & 15
        s = np.where(dc, np.minimum(sym, 16), s)
        zn = np.where(dc, 1, np.where(s > 0, z + r + 1, np.where(r == 15, z + 16, 64)))
        pos = pos + ln + s
        wrap = zn >= 64
        return pos, np.where(wrap, 0, zn), np.where(wrap, (c + 1) % bpm, c)

    nsub = (nbits + SUB - 1) // SUB
    print(f"{a.content} {a.size}: {len(raw)} B, {nsub} subsequences of {SUB} bits")
    for G, T, W in [(int(g), int(t), int(wm)) for g in a.g.split(",") for t in a.t.split(",")
                     for wm in a.warm.split(",")]:
        if True:
            nth = (nsub + G - 1) // G
            span = G * SUB
            base = np.arange(nth) * span
            end = np.minimum(base + span, nbits)
            nck = span // CK
            # checkpoint records per thread: state at first boundary >= base + CK * (m + 1)
            rec = np.full((nth, nck), -1, np.int64)

            def decode(idx, p0, z0, c0, stop_on_join):
                """Decode threads idx from (p0, z0, c0) to their span end; returns exit + symbols."""
                pos, z, c = p0.copy(), z0.copy(), c0.copy()
                m = np.zeros(len(idx), np.int64)
                m = np.maximum(m, (pos - base[idx]) // CK)  # marks already passed
                act = pos < end[idx]
                syms = 0
                while act.any():
                    ii = np.nonzero(act)[0]
                    pn, zn, cn = step(pos[ii], z[ii], c[ii])
                    syms += len(ii)
                    pos[ii], z[ii], c[ii] = pn, zn, cn
                    mk = base[idx[ii]] + CK * (m[ii] + 1)
                    hit = (m[ii] < nck - 1) & (pn >= mk)
                    if hit.any():
                        hi = ii[hit]
                        st = (pos[hi] << 16) | (z[hi] << 8) | c[hi]
                        joined = stop_on_join & (rec[idx[hi], m[hi]] == st)
                        rec[idx[hi][~joined], m[hi][~joined]] = st[~joined]
                        m[hi] += 1
                        act[hi[joined]] = False
                        pos[hi[joined]] = -1  # exit unchanged
                    act &= pos < end[idx]
                    act &= pos >= 0
                return pos, z, c, syms

            idx = np.arange(nth)
            p0 = base.copy()
            z0 = np.zeros(nth, np.int64)
            c0 = np.zeros(nth, np.int64)
            warm_syms = 0
            if W > 0:  # warm-up: from (base - W, 0, 0) to the first symbol boundary >= base
                wp = np.maximum(base - W, 0)
                wz, wc = z0.copy(), c0.copy()
                act = (wp < base) & (idx > 0)
                while act.any():
                    ii = np.nonzero(act)[0]
                    wp[ii], wz[ii], wc[ii] = step(wp[ii], wz[ii], wc[ii])
                    warm_syms += len(ii)
                    act &= wp < base
                p0[1:], z0[1:], c0[1:] = wp[1:], wz[1:], wc[1:]
            ex_p, ex_z, ex_c, work = decode(idx, p0, z0, c0, False)
            work += warm_syms
            work0 = work
            exits = (ex_p << 16) | (ex_z << 8) | ex_c
            entry = (p0 << 16) | (z0 << 8) | c0
            entry[0] = 0
            rounds = np.zeros((nth + T - 1) // T, np.int64)
            first = (idx % T) == 0
            while True:
                pred = np.roll(exits, 1)
                need = (~first) & (pred != entry)
                if not need.any():
                    break
                ii = np.nonzero(need)[0]
                entry[ii] = pred[ii]
                rounds[np.unique(ii // T)] += 1
                p, z, c, s = decode(ii, entry[ii] >> 16, (entry[ii] >> 8) & 255, entry[ii] & 255, True)
                work += s
                ch = p >= 0
                exits[ii[ch]] = (p[ch] << 16) | (z[ch] << 8) | c[ch]
            total_syms = work
            # a workgroup's first thread keeps its entry in pass 0; pass 1 re-decodes where it
            # differs from the previous workgroup's last exit
            miss = int(((np.roll(exits, 1) != entry) & first & (idx > 0)).sum())
            print(f"  G={G:2d} T={T:3d} warm={W:5d}: threads {nth:6d}  rounds/WG mean {rounds.mean():6.1f} max "
                  f"{rounds.max():4d}  symbols decoded {total_syms / 1e6:7.2f} M (x{total_syms / (work0 - warm_syms):.2f} "
                  f"of one decode)  WG entries wrong after pass 0: {miss} of {len(rounds) - 1}")


if __name__ == "__main__":
    main()
