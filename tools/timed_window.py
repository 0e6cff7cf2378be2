#!/usr/bin/env python3
"""Kernel statistics of bench.py's TIMED call only, from rocprofv3 output (measurement helper).

Usage: python tools/timed_window.py <trace_dir> <launches> <out_prefix> [<fetch_dir> <write_dir>
                                    <pmc_launches>]

bench.py's timed region is one bh_step(K) call; a one-GPU C3 step launches the traversal twice,
so the call is the window from the start of the <launches> = 2 K -th last `k_traverse` launch to
the end of the trace (run the bench with --no-drop-in --no-counters --no-cpu-baseline
--no-verify, so nothing follows the call).  Per kernel (and stream): launches, total, average,
min, max in the window; the traversal's average is what bench.py's HIP events measure
(roofline.kernel_ms.avg).  With counter passes (rocprofv3 --pmc FETCH_SIZE, resp. WRITE_SIZE,
each a bench run whose timed call makes <pmc_launches> traversal launches): the HBM bytes per
traversal launch of those calls' windows, FETCH_SIZE + WRITE_SIZE as reported.
Writes <out_prefix>_timed_summary.md and <out_prefix>_timed.json.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

TRAV = "k_traverse<false"


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"ROCPRIM_[0-9]+_NS::", "", name)
    return name.split("(")[0][:72]


def find(d, suffix):
    hits = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not hits:
        sys.exit(f"no *{suffix} under {d}")
    return hits[0]


def window(trace_csv, launches):
    rows = list(csv.DictReader(open(trace_csv)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 r.get("Stream_Id", "?")) for r in rows)
    starts = [k[0] for k in ks if TRAV in k[2]]
    if len(starts) < launches:
        sys.exit(f"only {len(starts)} traversal launches in the trace")
    t0 = starts[-launches]
    return [k for k in ks if k[0] >= t0], t0


def counters(d, launches):
    """(kernel -> [value per dispatch]) of the window's dispatches: the last `launches`
    traversal dispatches and everything dispatched after the first of them."""
    f = find(d, "counter_collection.csv")
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        did = int(r["Dispatch_Id"])
        per[(did, r["Counter_Name"])] += float(r["Counter_Value"])
        names[did] = short(r["Kernel_Name"])
    trav = sorted(did for did, n in names.items() if TRAV in n)
    if len(trav) < launches:
        sys.exit(f"{d}: only {len(trav)} traversal dispatches")
    first = trav[-launches]
    out = collections.defaultdict(list)
    for (did, c), v in per.items():
        if did >= first:
            out[(names[did], c)].append(v)
    return out


def main():
    trace_dir, launches, prefix = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    win, t0 = window(find(trace_dir, "kernel_trace.csv"), launches)
    t_end = max(k[1] for k in win)
    by = collections.defaultdict(list)
    for s, e, name, st in win:
        by[(name, st)].append((e - s) / 1e3)
    rows = sorted(by.items(), key=lambda kv: -sum(kv[1]))
    trav = [d for (n, _), ds in by.items() if TRAV in n for d in ds]
    res = {"launches_expected": launches, "window_ms": round((t_end - t0) / 1e6, 4),
           "traversal": {"launches": len(trav), "avg_ms": round(sum(trav) / len(trav) / 1e3, 5),
                         "min_ms": round(min(trav) / 1e3, 5), "max_ms": round(max(trav) / 1e3, 5)},
           "kernels": {f"{n} [s{st}]": {"launches": len(ds), "total_us": round(sum(ds), 1),
                                        "avg_us": round(sum(ds) / len(ds), 2)}
                       for (n, st), ds in rows}}
    for v in ("1>", "2>"):
        ds = [d for (n, _), dd in by.items() if TRAV in n and n.endswith(v) for d in dd]
        if ds:
            res["traversal"]["kick_drift" if v == "1>" else "kick_only"] = {
                "launches": len(ds), "avg_ms": round(sum(ds) / len(ds) / 1e3, 5)}
    lines = [f"# Timed call only: {launches} traversal launches, window "
             f"{res['window_ms']:.3f} ms (from the first traversal of the call to its last kernel)",
             "", f"traversal: {len(trav)} launches, avg {res['traversal']['avg_ms'] * 1e3:.1f} us, "
             f"min {res['traversal']['min_ms'] * 1e3:.1f}, max {res['traversal']['max_ms'] * 1e3:.1f}",
             "", "| kernel [stream] | launches | total us | avg us | min us | max us |",
             "|---|---|---|---|---|---|"]
    for (n, st), ds in rows[:30]:
        lines.append(f"| `{n}` [s{st}] | {len(ds)} | {sum(ds):.1f} | {sum(ds) / len(ds):.2f} | "
                     f"{min(ds):.2f} | {max(ds):.2f} |")
    if len(sys.argv) > 6:
        fetch_dir, write_dir, pmc_launches = sys.argv[4], sys.argv[5], int(sys.argv[6])
        cf, cw = counters(fetch_dir, pmc_launches), counters(write_dir, pmc_launches)
        tr = {}
        for (name, c), vals in list(cf.items()) + list(cw.items()):
            if TRAV in name and c in ("FETCH_SIZE", "WRITE_SIZE"):
                tr.setdefault(name, {})[c] = vals
        traffic = {}
        for name, cs in tr.items():
            if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
                w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
                traffic[name] = {"fetch_bytes": round(f), "write_bytes": round(w),
                                 "dispatches": len(cs["FETCH_SIZE"]),
                                 "hbm_bytes_per_launch": round(f + w),
                                 "hbm_bytes_upper": round(2 * f + w)}
        allf = [v for n, cs in tr.items() for v in cs.get("FETCH_SIZE", [])]
        allw = [v for n, cs in tr.items() for v in cs.get("WRITE_SIZE", [])]
        if allf and allw:
            f = sum(allf) / len(allf) * 1024
            w = sum(allw) / len(allw) * 1024
            res["traffic"] = {"per_variant": traffic, "hbm_bytes_per_launch": round(f + w),
                              "hbm_bytes_upper": round(2 * f + w),
                              "method": "FETCH_SIZE + WRITE_SIZE (x 1 KiB) as reported, "
                                        "separate --pmc passes, the timed call's traversal "
                                        "dispatches only"}
            lines += ["", f"HBM per traversal launch (timed call of the counter runs): "
                          f"{(f + w) / 1e6:.1f} MB as reported, {(2 * f + w) / 1e6:.1f} MB upper "
                          f"(2 x FETCH_SIZE + WRITE_SIZE); "
                          f"{(f + w) / (res['traversal']['avg_ms'] * 1e-3) / 1e9:.0f} GB/s at "
                          f"the window's average duration"]
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    with open(prefix + "_timed.json", "w") as fh:
        json.dump(res, fh, indent=1)
    with open(prefix + "_timed_summary.md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines[:4]))


if __name__ == "__main__":
    main()
