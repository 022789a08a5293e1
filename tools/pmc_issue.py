#!/usr/bin/env python3
"""Issue fractions of the JPEG kernels from a per-dispatch rocprofv3 PMC pass.

  rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS ... GRBM_GUI_ACTIVE GRBM_COUNT \\
      -d DIR -o pmc -- python3 tools/jpeg_bench.py --sizes 1080p --batch 32 --iters 3
  python tools/pmc_issue.py DIR/pmc_counter_collection.csv [--durations KERNEL_STATS.csv]

Per kernel, its dispatches in the LAST batch of the run (from the last k_unstuff_count on; a
kernel dispatched several times per batch -- the span sync's passes, the scans -- is summed) give:
  waves, VALU / LDS / SALU instructions per wave,
  clock_GHz       GRBM_GUI_ACTIVE / the dispatch's duration (the counter ticks the GPU clock
                  while the GUI is busy; rocprofv3 sums it over the XCDs, so it is divided by 8),
  valu_issue_frac SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction holds a SIMD-32 for two
                  cycles, MI355X_MICROARCH.md "Wave scheduling") / (1024 SIMDs x kernel cycles),
  lds_issue_frac  SQ_INSTS_LDS / (256 CUs x kernel cycles) (one LDS instruction per CU per cycle
                  at best; b64 / b128 accesses take 2-4 cycles each, so this is a lower bound).
Kernel cycles = duration x clock.  With --durations (a rocprofv3 --stats kernel_stats.csv of the
same workload run WITHOUT counters) the durations come from there: counter collection
serialises dispatches and can stretch them.  Prints one JSON object keyed by kernel name.
"""
import argparse
import csv
import json
import re
from collections import defaultdict

SIMDS, CUS, XCDS = 1024, 256, 8


def short(name):  # "k_fdct" for "void vf::jpeg::(anonymous namespace)::k_fdct<2, 1, false>(...)"
    return re.sub(r"<.*", "", re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).split("::")[-1])


def per_kernel(counters_csv, durations_csv="", min_waves=1000):
    """{kernel: counts and fractions} from a counter_collection.csv (see the module docstring);
    bench.py's jpeg leg uses it.  Short kernels' clock estimates are unreliable (the GRBM
    window is wider than the dispatch), so their fractions use the median clock of the kernels
    above 50 us."""
    disp = defaultdict(dict)
    for r in csv.DictReader(open(counters_csv)):
        d = disp[int(r["Dispatch_Id"])]
        d["_name"] = short(r["Kernel_Name"])
        d["_dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # the last batch: every dispatch from the last k_unstuff_count on (a batch's first kernel),
    # summed per kernel -- the span sync runs k_syncg once per pass, and the last pass of a
    # batch returns at once (converged), so "the last dispatch" would say nothing
    starts = [i for i in disp if disp[i]["_name"] == "k_unstuff_count"]
    first = max(starts) if starts else None
    last = {}
    for i in sorted(disp):
        d = disp[i]
        if first is None or i < first:
            last[d["_name"]] = d
            continue
        if i == first:
            last = {}
        a = last.setdefault(d["_name"], {"_name": d["_name"], "_dur_ns": 0, "_long_ns": 0, "_long": d})
        for k, v in d.items():
            if not k.startswith("_"):
                a[k] = a.get(k, 0.0) + v
        a["_dur_ns"] += d["_dur_ns"]
        if d["_dur_ns"] > a["_long_ns"]:
            a["_long_ns"], a["_long"] = d["_dur_ns"], d
    stats = {}
    if durations_csv:
        for r in csv.DictReader(open(durations_csv)):
            stats[short(r["Name"])] = float(r["AverageNs"])
    def clock(d):  # from the kernel's longest dispatch in the batch (or its only one)
        d = d.get("_long", d)
        return d.get("GRBM_GUI_ACTIVE", 0.0) / XCDS / d["_dur_ns"] if d["_dur_ns"] else 0.0
    clk_of = {n: clock(d) for n, d in last.items()}
    longs = sorted(c for n, c in clk_of.items() if last[n]["_dur_ns"] > 50_000 and c > 0)
    clk_med = longs[len(longs) // 2] if longs else 2.4
    out = {}
    for name, d in last.items():
        waves = d.get("SQ_WAVES", 0.0)
        if waves < min_waves:
            continue
        # --durations gives one dispatch's average; a kernel run several times per batch keeps
        # its summed in-batch time
        dur = stats.get(name, d["_dur_ns"]) if "_long" not in d else d["_dur_ns"]
        clk = clk_of[name] if d["_dur_ns"] > 50_000 else clk_med
        cyc = dur * clk
        r = {"waves": int(waves), "duration_us": round(dur / 1e3, 2), "clock_GHz": round(clk, 3),
             "valu_total": d.get("SQ_INSTS_VALU", 0.0), "lds_total": d.get("SQ_INSTS_LDS", 0.0),
             "valu_per_wave": round(d.get("SQ_INSTS_VALU", 0) / waves, 1),
             "lds_per_wave": round(d.get("SQ_INSTS_LDS", 0) / waves, 1),
             "salu_per_wave": round(d.get("SQ_INSTS_SALU", 0) / waves, 1)}
        if cyc > 0:
            r["valu_issue_frac"] = round(2.0 * d.get("SQ_INSTS_VALU", 0) / (SIMDS * cyc), 3)
            r["lds_issue_frac"] = round(d.get("SQ_INSTS_LDS", 0) / (CUS * cyc), 3)
        out[name] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("counters")
    ap.add_argument("--durations", default="")
    ap.add_argument("--min-waves", type=int, default=1000)
    a = ap.parse_args()
    out = per_kernel(a.counters, a.durations, a.min_waves)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
