#!/usr/bin/env python3
"""Kernel timeline of one step from a rocprofv3 --kernel-trace CSV (measurement helper).

Usage: python tools/timeline.py <run_kernel_trace.csv> [step_from_end=2] [out.txt] [anchor]

A one-GPU C3 step launches two fused traversals (`k_traverse<false, true, 1, *>` = kick + drift,
`<..., 2>` = kick only).  The window is from the start of the n-th last kick+drift traversal to
the start of the next one (another anchor kernel: 4th argument, e.g. k_let_flags for one LET
evaluation); every kernel in it is printed with its start / end offsets in us,
its queue and stream, so the overlap of the pipelined build with the second traversal and the
exposed gaps can be read off.  The summary line adds the union of busy time and the idle gaps.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                   r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    ks.sort()
    anchor = sys.argv[4] if len(sys.argv) > 4 else "k_traverse<false, true, 1,"
    starts = [k[0] for k in ks if anchor in k[2]]
    if len(starts) < back + 1:
        sys.exit("not enough steps in the trace")
    t0, t1 = starts[-back - 1], starts[-back]
    win = [k for k in ks if t0 <= k[0] < t1]
    out = []
    for s, e, name, q, st in win:
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if len(short) > 70:
            short = short[:70]
        out.append(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q} s{st}  {short}")
    # busy union and gaps
    iv = sorted((s, e) for s, e, *_ in win)
    busy, gaps, cs, ce = 0, [], iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((ce - t0, s - ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    out.append(f"step {(t1 - t0) / 1e3:.1f} us, busy union {busy / 1e3:.1f} us, "
               f"{len(gaps)} gaps, total gap {sum(g for _, g in gaps) / 1e3:.1f} us")
    for at, g in gaps:
        if g > 2000:
            out.append(f"  gap of {g / 1e3:.1f} us at {at / 1e3:.1f}")
    text = "\n".join(out)
    print(text)
    if len(sys.argv) > 3 and sys.argv[3] != "-":
        open(sys.argv[3], "w").write(text + "\n")


if __name__ == "__main__":
    main()
