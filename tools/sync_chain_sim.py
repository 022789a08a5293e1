"""Pass-0 chain analysis of the span sync on one hard 1080p frame (analysis tool, CPU only).

Builds the true decoder state at every 256-bit subsequence start by a sequential decode
(tools/sync_distance.py's tables), then for spans of G = 4 subsequences and a warm-up of W bits:
  * how many spans' entries (after the warm-up) and exits (after warm-up + span) are off the
    true path;
  * per workgroup of T = 256 threads, the pass-0 time in decoded bits under k_syncg's rounds
    (every round costs its longest re-decode) and under an event-driven schedule (a thread
    re-decodes the moment its predecessor's exit changes, no barrier).
Re-decodes stop where they rejoin the thread's recorded trajectory at a 64-bit mark, as in
k_syncg.  DESIGN.md §12 quotes its output.

    python tools/sync_chain_sim.py [--warm 1024,2048,4096] [--wgs 62]
"""
import argparse
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "distributed-video-filter_amd")]
from sync_distance import lut, parse  # noqa: E402

SUB, CK, G, T = 256, 64, 4, 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", default="1024,2048,4096")
    ap.add_argument("--wgs", type=int, default=0, help="workgroups to replay (0: all)")
    a = ap.parse_args()
    from oracle import jpeg as J
    from vfilter.synthetic import synthetic_noisy_scene
    jp = J.encode(synthetic_noisy_scene(0, 1080, 1920), 95, J.TJPF_BGR, J.TJSAMP_422)
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
        k = blkc[C]
        if Z == 0:
            e = dcl[k][win[P]]
            P += (e >> 8 or 16) + min(e & 255, 16)
            Z = 1
        else:
            e = acl[k][win[P]]
            sym = e & 255
            r, sz = sym >> 4, sym & 15
            P += (e >> 8 or 16) + sz
            Z = Z + r + 1 if sz else (Z + 16 if r == 15 else 64)
        if Z >= 64:
            Z, C = 0, (C + 1) % bpm
        return P, Z, C

    pack = lambda P, Z, C: (P << 16) | (Z << 8) | C  # noqa: E731
    nsub = (nbits + SUB - 1) // SUB
    truth = [0] * nsub
    P = Z = C = 0
    s = 0
    while P < nbits:
        while s < nsub and s * SUB <= P:
            truth[s] = pack(P, Z, C)
            s += 1
        P, Z, C = step(P, Z, C)
    span = G * SUB
    nth = (nsub + G - 1) // G

    def decode(i, st, rec, check):
        """thread i's span from state st: (exit or None when it rejoined rec, bits decoded)"""
        b, e = i * span, min(i * span + span, nbits)
        P, Z, C = st >> 16, (st >> 8) & 255, st & 255
        p0, m = P, max(0, (P - b) // CK)
        while P < e:
            P, Z, C = step(P, Z, C)
            mk = b + CK * (m + 1)
            if mk < e and P >= mk:
                x = pack(P, Z, C)
                if check and rec.get(m) == x:
                    return None, P - p0
                rec[m] = x
                m += 1
        return pack(P, Z, C), P - p0

    print(f"hard 1080p: {len(raw)} B, {nsub} subsequences, {nth} spans of {span} bits")
    for W in [int(x) for x in a.warm.split(",")]:
        ent, ex, recs, t0 = [0] * nth, [0] * nth, [None] * nth, [0] * nth
        for i in range(nth):
            b = i * span
            st, wl = 0, 0
            if i:
                P, Z, C = max(0, b - W), 0, 0
                while P < b:
                    P, Z, C = step(P, Z, C)
                st, wl = pack(P, Z, C), P - max(0, b - W)
            recs[i] = {}
            x, L = decode(i, st, recs[i], False)
            ent[i], ex[i], t0[i] = st, x, wl + L
        ew = np.mean([ent[i] != truth[i * G] for i in range(1, nth)])
        xw = np.mean([ex[i] != truth[(i + 1) * G] for i in range(nth - 1)])
        rt, at = [], []
        nwg = (nth + T - 1) // T
        for wg in range(nwg if not a.wgs else min(a.wgs, nwg)):
            ids = list(range(wg * T, min(nth, wg * T + T)))
            base = max(t0[i] for i in ids)
            E, X, R = {i: ent[i] for i in ids}, {i: ex[i] for i in ids}, {i: dict(recs[i]) for i in ids}
            tr = base
            while True:  # rounds
                need = [i for i in ids[1:] if X[i - 1] != E[i]]
                if not need:
                    break
                mx, upd = 0, {}
                for i in need:
                    E[i] = X[i - 1]
                    x, L = decode(i, E[i], R[i], True)
                    mx = max(mx, L)
                    if x is not None:
                        upd[i] = x
                X.update(upd)
                tr += mx
            E, X, R = {i: ent[i] for i in ids}, {i: ex[i] for i in ids}, {i: dict(recs[i]) for i in ids}
            busy = {i: t0[i] for i in ids}
            pq = [(t0[i], i) for i in ids]
            heapq.heapify(pq)
            done = base
            while pq:  # event-driven
                t, i = heapq.heappop(pq)
                j = i + 1
                if j in E and X[i] != E[j]:
                    start = max(t, busy[j])
                    E[j] = X[i]
                    x, L = decode(j, E[j], R[j], True)
                    busy[j] = start + L
                    done = max(done, start + L)
                    if x is not None and x != X[j]:
                        X[j] = x
                        heapq.heappush(pq, (start + L, j))
            rt.append(tr)
            at.append(done)
        print(f"  warm {W:5d}: entries off the true path {ew:.3f}, exits {xw:.3f}; per workgroup (bits): "
              f"rounds mean {np.mean(rt):.0f} max {max(rt)}, event-driven mean {np.mean(at):.0f} max {max(at)}")


if __name__ == "__main__":
    main()
