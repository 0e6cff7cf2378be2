#!/usr/bin/env python3
"""Record the measured HBM bytes per launch of a workload's dominant kernel for bench.py.

Usage: python tools/update_traffic.py <config> <kernel> <profiles/<prefix>_traffic.json>
Writes profiles/hbm_traffic.json[config][kernel] = {hbm_bytes_per_launch, source}.  The
per-kernel file comes from tools/summarize_profile.py on a rocprofv3 FETCH_SIZE / WRITE_SIZE run
(tools/profile.sh) of the same bench configuration.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    config, kernel, src = sys.argv[1:4]
    per_kernel = json.load(open(src))
    hit = [(k, v) for k, v in per_kernel.items() if k.split("::")[-1].split("<")[0] == kernel]
    if not hit:
        sys.exit(f"{kernel} not in {src}")
    # the non-counting instantiation is the one bench.py times (k_traverse<false, ...>)
    name, ent = sorted(hit, key=lambda kv: ("<true" in kv[0], kv[0]))[0]
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data.setdefault(config, {})[kernel] = {
        "hbm_bytes_per_launch": ent["hbm_bytes_per_launch"],
        "hbm_bytes_upper": ent.get("hbm_bytes_upper"),
        "kernel_symbol": name,
        "source": os.path.relpath(src, ROOT),
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes; FETCH_SIZE + "
                  "WRITE_SIZE as reported (MALL hits included; no 16-B/lane streaming reads, "
                  "so the guide's x2 is only an upper bound: hbm_bytes_upper)",
    }
    with open(path, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=True)
    print(config, kernel, ent["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
