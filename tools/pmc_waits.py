#!/usr/bin/env python3
"""Wait / issue breakdown of the JPEG kernels from two per-dispatch rocprofv3 PMC passes
(tools/r4/gpu_jpeg_pmc_waits.sh; analysis tool).

Per kernel, summed over the dispatches of the last batch (from the last k_unstuff_count on), and
per dispatch for the span sync k_syncg (one dispatch per pass): waves, then per wave SQ_WAVE_CYCLES
(wave residency), SQ_WAIT_ANY (waiting on anything: s_waitcnt, barriers, dependencies),
SQ_WAIT_INST_ANY (ready but not issued), SQ_ACTIVE_INST_VALU / _LDS, SQ_INST_CYCLES_VMEM, and the
instruction counts.  The fractions divide by SQ_WAVE_CYCLES; the counters' units (quad-cycles for
the WAIT counters) follow counter_defs.yaml, so read the fractions against each other, not as
absolute shares.

    python tools/pmc_waits.py DIR_A DIR_B [DIR_STATS]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_issue import short  # noqa: E402


def dispatches(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    disp = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        x = disp[int(r["Dispatch_Id"])]
        x["_name"] = short(r["Kernel_Name"])
        x["_dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        x[r["Counter_Name"]] = x.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(disp)
    starts = [i for i in ids if disp[i]["_name"] == "k_unstuff_count"]
    first = starts[-1] if starts else ids[0]
    return [disp[i] for i in ids if i >= first]


def main():
    a, b = dispatches(sys.argv[1]), dispatches(sys.argv[2])
    if len(sys.argv) > 3:
        f = glob.glob(f"{sys.argv[3]}/**/*kernel_stats.csv", recursive=True)
        if f:
            for r in csv.DictReader(open(f[0])):
                print(f"stats {short(r['Name']):24s} calls {int(r['Calls']):5d} avg {float(r['AverageNs']) / 1e3:8.1f} us")
    # pair the two passes' dispatches by order (same workload, same dispatch sequence)
    rows = []
    for x, y in zip(a, b):
        if x["_name"] != y["_name"]:
            print("dispatch order differs between passes:", x["_name"], y["_name"])
            break
        m = dict(y)
        m.update(x)
        rows.append(m)
    per = defaultdict(lambda: defaultdict(float))
    sync_rows = []
    for m in rows:
        n = m["_name"]
        if n == "k_syncg":
            sync_rows.append(m)
        for k, v in m.items():
            if not k.startswith("_"):
                per[n][k] += v
        per[n]["_dur_ns"] += m["_dur_ns"]

    def show(tag, d):
        w = d.get("SQ_WAVES", 0.0)
        if w < 64:
            return
        wc = d.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        out = {"dur_us": round(d["_dur_ns"] / 1e3, 1), "waves": int(w),
               "wave_cycles_per_wave": round(wc / w, 0),
               "wait_any/wave_cyc": round(d.get("SQ_WAIT_ANY", 0) / wc, 3),
               "wait_inst_any/wave_cyc": round(d.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
               "active_valu/wave_cyc": round(d.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
               "active_lds/wave_cyc": round(d.get("SQ_ACTIVE_INST_LDS", 0) / wc, 3),
               "vmem_cyc/wave_cyc": round(d.get("SQ_INST_CYCLES_VMEM", 0) / wc, 3),
               "wait_inst_lds/wave_cyc": round(d.get("SQ_WAIT_INST_LDS", 0) / wc, 3),
               "valu/wave": round(d.get("SQ_INSTS_VALU", 0) / w, 1), "lds/wave": round(d.get("SQ_INSTS_LDS", 0) / w, 1),
               "salu/wave": round(d.get("SQ_INSTS_SALU", 0) / w, 1),
               "vmem_rd/wave": round(d.get("SQ_INSTS_VMEM_RD", 0) / w, 1),
               "vmem_wr/wave": round(d.get("SQ_INSTS_VMEM_WR", 0) / w, 1),
               "busy_cycles": d.get("SQ_BUSY_CYCLES", 0.0)}
        print(tag, json.dumps(out))

    for i, m in enumerate(sync_rows):
        show(f"k_syncg pass {i}", dict(m))
    for n, d in sorted(per.items(), key=lambda kv: -kv[1]["_dur_ns"]):
        show(f"{n:24s}", d)


if __name__ == "__main__":
    main()
