#!/usr/bin/env python3
"""Condense rocprofv3 CSV output (gpurun_out/prof*/...) into a committed summary under
profiles/.  Usage: python tools/summarize_profile.py <prof_dir> <out_prefix>

Writes <out_prefix>_kernel_stats.csv (copy of rocprofv3 --stats) and <out_prefix>_summary.md;
if counter passes are present, per-kernel averages per dispatch, and <out_prefix>_traffic.json
with HBM bytes per launch per kernel, corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE (KB) x 2 (gfx950 tallies a 128-B read request as 64 B) + WRITE_SIZE (KB).
"""
import collections
import csv
import json
import os
import re
import shutil
import sys


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"ROCPRIM_[0-9]+_NS::", "", name)
    return name.split("(")[0][:70]


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    lines = []
    if os.path.exists(stats):
        shutil.copy(stats, prefix + "_kernel_stats.csv")
        rows = list(csv.DictReader(open(stats)))
        lines.append("## rocprofv3 --kernel-trace --stats (top kernels)\n")
        lines.append("| kernel | calls | total ms | avg us | % |")
        lines.append("|---|---|---|---|---|")
        for r in rows[:25]:
            name = short(r["Name"])
            lines.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | "
                         f"{float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.2f} |")
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            name = short(r["Kernel_Name"])
            counters[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if counters:
        lines.append("\n## PMC counters (average per dispatch; FETCH/WRITE_SIZE in KB as reported)\n")
        for name in sorted(counters, key=lambda k: -sum(sum(v) for v in counters[k].values()))[:12]:
            cs = counters[name]
            vals = ", ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items()))
            lines.append(f"- `{name}`: {vals}")
    traffic = {}
    for name, cs in counters.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
            traffic[name] = {"fetch_kb": round(f, 1), "write_kb": round(w, 1),
                             "dispatches": len(cs["FETCH_SIZE"]),
                             "hbm_bytes_per_launch": round(2 * f * 1024 + w * 1024)}
    if traffic:
        with open(prefix + "_traffic.json", "w") as fh:
            json.dump(traffic, fh, indent=1, sort_keys=True)
        lines.append("\n## HBM traffic per launch (FETCH_SIZE x 2 + WRITE_SIZE)\n")
        for name, t in sorted(traffic.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:10]:
            lines.append(f"- `{name}`: {t['hbm_bytes_per_launch'] / 1e6:.1f} MB "
                         f"(fetch {t['fetch_kb'] / 1024:.1f} MB x 2, write {t['write_kb'] / 1024:.1f} MB)")
    with open(prefix + "_summary.md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
