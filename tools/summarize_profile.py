#!/usr/bin/env python3
"""Condense rocprofv3 CSV output into committed summaries under profiles/.

Usage: python tools/summarize_profile.py <trace_dir> <out_prefix> [<counter_dir> ...]

<trace_dir> holds run_kernel_stats.csv / run_kernel_trace.csv of a --kernel-trace --stats run;
each <counter_dir> one --pmc pass (FETCH_SIZE or WRITE_SIZE: their TCC slots do not fit one
pass).  Writes <out_prefix>_kernel_stats.csv, <out_prefix>_summary.md and, with counters,
<out_prefix>_traffic.json.

HBM bytes per launch (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts the L2's memory-side read
requests at 64 B each (Infinity-Cache/MALL hits included, not excluded); it reports exactly half
the bytes of a 16-B-per-lane streaming read, other access widths are uncalibrated.  None of this
engine's kernels streams 16 B per lane as its main read (node records are scalar loads, body
fields 8 B per lane), so the figure used is FETCH_SIZE + WRITE_SIZE as reported ("measured");
2 x FETCH_SIZE + WRITE_SIZE is kept as an upper bound, and a bound whose implied rate exceeds
the 8 TB/s peak over the kernel's traced duration is flagged as impossible.
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

HBM_PEAK = 8.0e12


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"ROCPRIM_[0-9]+_NS::", "", name)
    return name.split("(")[0][:70]


def main():
    trace, prefix = sys.argv[1], sys.argv[2]
    counter_dirs = sys.argv[3:]
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    stats = os.path.join(trace, "run_kernel_stats.csv")
    lines, avg_ns = [], {}
    if os.path.exists(stats):
        shutil.copy(stats, prefix + "_kernel_stats.csv")
        rows = list(csv.DictReader(open(stats)))
        lines.append("## rocprofv3 --kernel-trace --stats (top kernels)\n")
        lines.append("| kernel | calls | total ms | avg us | min us | max us | % |")
        lines.append("|---|---|---|---|---|---|---|")
        for r in rows:
            avg_ns.setdefault(short(r["Name"]), float(r["AverageNs"]))
        for r in rows[:25]:
            lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | "
                         f"{float(r['TotalDurationNs']) / 1e6:.3f} | "
                         f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | "
                         f"{float(r['MaxNs']) / 1e3:.2f} | {float(r['Percentage']):.2f} |")
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in counter_dirs:
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        per = collections.defaultdict(float)  # (kernel, dispatch, counter) summed over blocks
        for r in csv.DictReader(open(f)):
            per[(short(r["Kernel_Name"]), r["Dispatch_Id"], r["Counter_Name"])] += \
                float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            counters[k][c].append(v)
    traffic = {}
    for name, cs in counters.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
            ent = {"fetch_bytes": round(f), "write_bytes": round(w),
                   "dispatches": len(cs["FETCH_SIZE"]),
                   "hbm_bytes_per_launch": round(f + w),
                   "hbm_bytes_upper": round(2 * f + w)}
            ns = avg_ns.get(name)
            if ns:
                ent["avg_us"] = round(ns / 1e3, 2)
                ent["measured_gbs"] = round((f + w) / (ns * 1e-9) / 1e9, 1)
                ent["upper_gbs"] = round((2 * f + w) / (ns * 1e-9) / 1e9, 1)
                ent["upper_possible"] = (2 * f + w) / (ns * 1e-9) <= HBM_PEAK
            traffic[name] = ent
    if traffic:
        with open(prefix + "_traffic.json", "w") as fh:
            json.dump(traffic, fh, indent=1, sort_keys=True)
        lines.append("\n## HBM traffic per launch (FETCH_SIZE + WRITE_SIZE as reported; upper "
                     "bound 2 x FETCH_SIZE + WRITE_SIZE; MALL hits included)\n")
        lines.append("| kernel | avg us | measured MB | GB/s | upper MB | upper GB/s |")
        lines.append("|---|---|---|---|---|---|")
        for name, t in sorted(traffic.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:14]:
            up = f"{t.get('upper_gbs', '-')}" + ("" if t.get("upper_possible", True) else " (impossible)")
            lines.append(f"| `{name}` | {t.get('avg_us', '-')} | "
                         f"{t['hbm_bytes_per_launch'] / 1e6:.1f} | {t.get('measured_gbs', '-')} | "
                         f"{t['hbm_bytes_upper'] / 1e6:.1f} | {up} |")
    with open(prefix + "_summary.md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
