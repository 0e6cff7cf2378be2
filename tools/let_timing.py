"""Per-rank build cost of the multi-rank engine, sharded (LET) vs replicated, on ONE GPU.

Runs the north-star decomposition -- C4 (1e7-body cloud) on W in-process ranks (bh_create_local:
one host thread per rank, the exchanges as device-to-device copies) -- for one bh_step(K) call
after a warm-up call, with the build mode chosen by BH_LET (1 = locally essential trees, 0 = every
rank builds the full tree).  The W ranks share the GPU, so per-rank numbers come from kernel
time: run it under `rocprofv3 --kernel-trace --stats` and pass the stats CSV to --summarize,
which splits the kernel time into build / traversal / exchange+integration and divides by
W x builds.

    BH_LET=1 python tools/let_timing.py --world 8 --steps 5
    python tools/let_timing.py --summarize <kernel_stats.csv> --world 8 --builds 10
"""
import argparse
import csv
import json
import os
import sys
import threading
import time

BUILD_PREFIXES = ("k_morton", "k_bucket", "k_key_", "k_prep", "k_cells", "k_emit_com", "k_span",
                  "k_com_span", "k_let_", "rocprim", "k_hilbert", "k_lane")


def summarize(path, world, builds):
    tot = {"build": 0.0, "traverse": 0.0, "other": 0.0}
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Name") or row.get("KernelName") or ""
            ns = float(row.get("TotalDurationNs") or row.get("TotalDuration") or 0.0)
            if "k_traverse" in name:
                cat = "traverse"
            elif any(p in name for p in BUILD_PREFIXES) and "k_let_kick" not in name:
                cat = "build"
            else:
                cat = "other"
            tot[cat] += ns
            per[name[:60]] = per.get(name[:60], 0.0) + ns
    out = {k: v / 1e6 for k, v in tot.items()}
    out["build_ms_per_rank_build"] = tot["build"] / 1e6 / (world * builds)
    out["top_kernels_ms"] = {k: round(v / 1e6, 3) for k, v in
                             sorted(per.items(), key=lambda kv: -kv[1])[:14]}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--scene", default="c4")
    ap.add_argument("--summarize", default=None)
    ap.add_argument("--builds", type=int, default=0)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize, a.world, a.builds or 2 * (a.steps + 1))
        return
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "barnes-hut-n-body_amd"))
    import bh_amd
    from bh_amd import scenes
    arrs = scenes.config_scene(a.scene)
    group = bh_amd.LocalGroup(a.world)
    params = bh_amd.default_params(theta=0.5)
    engines = [bh_amd.Engine(params, device=0, rank=r, local_group=group) for r in range(a.world)]
    out, errors = [None] * a.world, []

    def run(r):
        try:
            e = engines[r]
            e.reset_bodies(*arrs)
            e.step(1)  # warm-up: allocations
            e.synchronize() if hasattr(e, "synchronize") else None
            t0 = time.perf_counter()
            e.step(a.steps)
            t1 = time.perf_counter()
            out[r] = {"wall_s": t1 - t0, **e.let_stats()}
        except Exception as exc:
            errors.append(repr(exc))

    th = [threading.Thread(target=run, args=(r,)) for r in range(a.world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in engines:
        e.close()
    group.close()
    if errors:
        raise SystemExit(errors)
    print(json.dumps({"BH_LET": os.environ.get("BH_LET", "1"), "world": a.world,
                      "steps": a.steps, "n": len(arrs[0]), "ranks": out}))


if __name__ == "__main__":
    main()
