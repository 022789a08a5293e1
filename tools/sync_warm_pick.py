"""Which warm-up guess lands on the true path? (CPU analysis tool for the span sync's pass 0.)

k_syncg warms each span's entry by decoding the W bits before it from a guessed state (z = 0,
c = 0).  On hard content ~22 % of entries are still off the true path after 2,048 bits: the
position resynchronises in ~16 bits, a wrong block-in-MCU c rarely does.  Here the warm-up is
decoded from each c0 = 0 .. bpm-1, and each decode counts the events a valid stream never has
(an AC run past coefficient 63, a code the table lacks, a DC / AC size past 11 / 10); the guess
with the fewest events -- ties to the one whose last event is earliest -- is picked.  Prints the
fraction of wrong entries for c0 = 0 alone, for the pick, and for 'any of the bpm' (the bound).

    python tools/sync_warm_pick.py [--content hard|scene] [--warm 1024,2048] [--spans 2000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "distributed-video-filter_amd")]
from sync_distance import lut, parse  # noqa: E402

SUB, G = 256, 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--content", default="hard", choices=("hard", "scene"))
    ap.add_argument("--warm", default="1024,2048")
    ap.add_argument("--spans", type=int, default=2000)
    a = ap.parse_args()
    from oracle import jpeg as J
    from vfilter.synthetic import synthetic_noisy_scene
    if a.content == "hard":
        jp = J.encode(synthetic_noisy_scene(0, 1080, 1920), 95, J.TJPF_BGR, J.TJSAMP_422)
    else:
        jp = J.encode(J.synthetic_scene(0, 1080, 1920), 85, J.TJPF_BGR, J.TJSAMP_422)
    comps, sel, tabs, raw = parse(jp)
    blkc = [k for k, (hs, vs) in enumerate(comps) for _ in range(hs * vs)]
    bpm = len(blkc)
    dcl = [lut(*tabs[sel[k][0]]).tolist() for k in range(len(comps))]
    acl = [lut(*tabs[0x10 | sel[k][1]]).tolist() for k in range(len(comps))]
    bits = np.unpackbits(np.frombuffer(raw + b"\0" * 8, np.uint8))
    nbits = len(raw) * 8
    win = np.zeros(nbits + 32, np.int64)
    for b in range(16):
        win[:nbits + 16] = (win[:nbits + 16] << 1) | bits[b:b + nbits + 16]
    win = win.tolist()

    def step(P, Z, C):
        """one symbol; returns the state and whether it is impossible in a valid stream"""
        k = blkc[C]
        if Z == 0:
            e = dcl[k][win[P]]
            ln, sym = e >> 8, e & 255
            bad = ln == 0 or sym > 11
            P += (ln or 16) + min(sym, 16)
            Z = 1
        else:
            e = acl[k][win[P]]
            ln, sym = e >> 8, e & 255
            r, sz = sym >> 4, sym & 15
            bad = ln == 0 or sz > 10 or (sz and Z + r > 63) or (not sz and r == 15 and Z + 16 > 63)
            P += (ln or 16) + sz
            Z = Z + r + 1 if sz else (Z + 16 if r == 15 else 64)
        if Z >= 64:
            Z, C = 0, (C + 1) % bpm
        return P, Z, C, bad

    nsub = (nbits + SUB - 1) // SUB
    truth = {}
    P = Z = C = 0
    s = 0
    while P < nbits:
        while s < nsub and s * SUB <= P:
            truth[s] = (P, Z, C)
            s += 1
        P, Z, C, _ = step(P, Z, C)
    span = G * SUB
    nth = (nsub + G - 1) // G
    rng = np.random.default_rng(0)
    ids = rng.choice(np.arange(8, nth), size=min(a.spans, nth - 8), replace=False)
    print(f"{a.content} 1080p: {len(raw)} B, bpm {bpm}, {len(ids)} spans of {span} bits")
    for W in [int(x) for x in a.warm.split(",")]:
        wrong0 = wrongp = wrong_any = 0
        for i in ids:
            b = int(i) * span
            t = truth[int(i) * G]
            res = []
            for c0 in range(bpm):
                P, Z, C = b - W, 0, c0
                nbad, last = 0, -1
                while P < b:
                    P, Z, C, bad = step(P, Z, C)
                    if bad:
                        nbad += 1
                        last = P
                res.append(((P, Z, C), nbad, last))
            ok = [r[0] == t for r in res]
            wrong0 += not ok[0]
            wrong_any += not any(ok)
            pick = min(range(bpm), key=lambda q: (res[q][1], res[q][2]))
            wrongp += not ok[pick]
        n = len(ids)
        print(f"  warm {W:5d}: entry off the true path  c0=0: {100 * wrong0 / n:5.1f} %   "
              f"pick of {bpm}: {100 * wrongp / n:5.1f} %   none of {bpm}: {100 * wrong_any / n:5.1f} %")


if __name__ == "__main__":
    main()
