#!/usr/bin/env python3
"""Idle time of the GPU between the kernels of a JPEG run (rocprofv3 --kernel-trace
--memory-copy-trace csv directory): per gap above 20 us, what ran before and after it, and
the busy / idle totals over the last timed stretch.
  python tools/jpeg_gaps.py gpurun_out/prof_jg"""
import csv
import glob
import re
import sys

d = sys.argv[1]
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("::")[-1][:24]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + n, r.get("Queue_Id", r.get("Stream_Id", ""))))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kind = r.get("Direction", r.get("Operation", "copy"))
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + kind[:20] + " " + r.get("Size", ""), ""))
ev.sort()
# the last 60 % of the run (the timed loop; warm-up and the final resident bench excluded by
# taking kernels of k_spec as batch markers)
marks = [e for e in ev if "k_spec" in e[2] or "k_sync" in e[2]]
print(f"events {len(ev)} batches {len(marks)}")
if len(marks) > 8:
    t0, t1 = marks[len(marks) // 4][0], marks[-12][0]
    win = [e for e in ev if t0 <= e[0] < t1 and e[2].startswith("K")]
    busy, end, gaps = 0, win[0][0], []
    for s, e, n, q in win:
        if s > end:
            gaps.append((s - end, prev, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        prev = n
    span = t1 - t0
    nb = sum(1 for m in marks if t0 <= m[0] < t1)
    print(f"window {span / 1e3:.1f} us over {nb} batches: kernels busy {busy / 1e3:.1f} us "
          f"({100 * busy / span:.1f} %), idle {(span - busy) / 1e3:.1f} us, per batch {span / nb / 1e3:.1f} us")
    for g, a, b in sorted(gaps, reverse=True)[:25]:
        if g > 20000:
            print(f"gap {g / 1e3:8.1f} us after {a:26s} before {b}")
    # one batch's sequence in full
    i = marks.index(next(m for m in marks if m[0] >= t0))
    s0, s1 = marks[i][0], marks[i + 1][0]
    base = s0
    for s, e, n, q in ev:
        if s0 - 300000 <= s < s1:
            print(f"{(s - base) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3} {n}")
