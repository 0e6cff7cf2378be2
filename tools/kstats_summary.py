#!/usr/bin/env python3
"""Per-kernel, per-stream average durations from a rocprofv3 --kernel-trace CSV directory.

Usage: python tools/kstats_summary.py <trace_dir> [kernel_substring ...]
"""
import collections
import csv
import glob
import re
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    acc = collections.defaultdict(list)
    for r in rows:
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        if want and not any(w in name for w in want):
            continue
        acc[(name, r["Stream_Id"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, st), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name:28s} stream {st:>2s} n={len(v):4d} avg {sum(v) / len(v):8.1f} us  "
              f"min {min(v):8.1f}  total {sum(v) / 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
