"""One GPU's share of the multi-GPU step, measured alone (bh_create_solo).

Rank `rank` of a `world`-rank engine on one GPU: its locally essential tree builds (or, with
BH_LET=0, the replicated full builds), the traversal of its Hilbert pieces, the integration of
every body -- everything a rank does in bench.py --gpus <world> except the RCCL exchanges and
waiting for peers.  The peers' bodies get zero acceleration, so the scene is not the reference's
(timing only).  Prints one JSON line: per-rank ms per step and its phases.

    python tools/solo_rank.py --world 8 --rank 0 --steps 10 --warmup 2 [--config c4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "barnes-hut-n-body_amd"))
import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--theta", type=float, default=0.5)
    a = ap.parse_args()
    arrs = scenes.config_scene(a.config)
    eng = bh_amd.Engine(bh_amd.default_params(theta=a.theta), device=0, rank=a.rank,
                        world=a.world, solo=True)
    eng.reset_bodies(*arrs)
    eng.step(a.warmup)
    eng.set_profiling(True)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.step(a.steps)
    eng.synchronize()
    dt = time.perf_counter() - t0
    ph = eng.last_timings()
    trav_ms, launches = eng.traverse_kernel_ms()
    out = {"tool": "solo_rank", "config": a.config, "n": len(arrs[0]), "world": a.world,
           "rank": a.rank, "steps": a.steps, "BH_LET": os.environ.get("BH_LET", "1"),
           "ms_per_step": round(1e3 * dt / a.steps, 4),
           "phase_ms_per_step": {k: round(v / a.steps, 4) for k, v in ph.items()},
           "traverse_launch_ms": round(trav_ms, 4), "traverse_launches": launches,
           "let": eng.let_stats()}
    lib = bh_amd.load_library()
    if hasattr(lib, "bh_debug_sort_stats"):  # a -DBH_SORT_STATS build: bucket paths (all builds)
        st = (ctypes.c_ulonglong * 8)()
        if lib.bh_debug_sort_stats(st) == 0:
            out["sort_stats"] = dict(zip(("radix", "radix_el", "bitonic", "bitonic_el", "global",
                                          "global_el"), (int(v) for v in st[:6])))
        lg = (ctypes.c_ulonglong * (256 * 4))()
        if hasattr(lib, "bh_debug_sort_log") and lib.bh_debug_sort_log(lg) == 0:
            # per bucket-sort launch in order: largest bucket, LDS-bitonic / global buckets
            out["sort_log"] = [[int(v) for v in lg[4 * i:4 * i + 4]] for i in range(256)
                               if lg[4 * i]]
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
