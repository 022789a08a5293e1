"""One batch's kernel timeline (start, gap before, duration) from a rocprofv3 kernel trace:
python tools/r3/batch_timeline.py <kernel_trace.csv> [batch index from the end, default 2]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def nm(r):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).split("::")[-1]
    return re.sub(r"^void ", "", n)


back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if nm(r).startswith("k_unstuff_count")]
spans = []
for a, b in zip(idx[:-1], idx[1:]):
    spans.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
i0, i1 = idx[-1 - back], idx[-back]
t0 = int(rows[i0]["Start_Timestamp"])
prev = None
busy = 0.0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    busy += (e - s) / 1e3
    print(f"{(s - t0) / 1e3:8.1f} {gap:6.1f} {(e - s) / 1e3:7.1f}  {nm(r)[:50]}")
    prev = e
span = (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3
print(f"batch span {span:.1f} us, kernels busy {busy:.1f} us; spans of all batches: median {sorted(spans)[len(spans) // 2]:.1f} us")
