#!/usr/bin/env python3
"""Condense rocprofv3 CSV output (gpurun_out/prof*/...) into a committed summary under
profiles/.  Usage: python tools/summarize_profile.py <prof_dir> <out_prefix>

Writes <out_prefix>_kernel_stats.csv (copy of rocprofv3 --stats), and, if counter passes are
present, <out_prefix>_counters.md with per-kernel averages per dispatch.
"""
import collections
import csv
import os
import shutil
import sys


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
            name = r["Name"].split("(")[0].replace("void ", "")[:70]
            lines.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | "
                         f"{float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.2f} |")
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in sorted(os.listdir(src)):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
            counters[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if counters:
        lines.append("\n## PMC counters (average per dispatch; FETCH/WRITE_SIZE in KB as reported)\n")
        for name in sorted(counters, key=lambda k: -sum(sum(v) for v in counters[k].values()))[:12]:
            cs = counters[name]
            vals = ", ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items()))
            lines.append(f"- `{name}`: {vals}")
    with open(prefix + "_summary.md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
