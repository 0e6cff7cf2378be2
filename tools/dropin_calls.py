#!/usr/bin/env python3
"""The front-end's call pattern on C3 for a kernel / copy trace (measurement helper): reset,
warm-up, then CALLS x (bh_step(1) + bh_map_bodies) with the pinned mirror on (or, with
--get-bodies, bh_get_bodies into resident buffers).  Run under
`rocprofv3 --kernel-trace --memory-copy-trace -- python3 tools/dropin_calls.py` and summarise with
tools/timeline.py (anchor k_traverse<false, true, 1, *>: one per call)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "barnes-hut-n-body_amd")]

import numpy as np  # noqa: E402

import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--get-bodies", action="store_true")
    ap.add_argument("--before", default="",
                    help="calls made before the mirror is switched on, as bench.py's drop_in leg "
                         "does: 's' = 45 x step(1), 'g' = 45 x (step(1) + get_bodies), e.g. 'sg'")
    ap.add_argument("--torch", action="store_true",
                    help="initialise torch's GPU context first, as bench.py does")
    a = ap.parse_args()
    if a.torch:
        import torch
        torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5))
    eng.reset_bodies(*scenes.config_scene(a.config))
    bufs = [np.zeros(eng.num_bodies()) for _ in range(5)]
    for c in a.before:
        for _ in range(45):
            eng.step(1)
            if c == "g":
                eng.get_bodies(out=bufs)
        eng.synchronize()
    eng.set_mirror(not a.get_bodies)
    for _ in range(a.warmup):
        eng.step(1)
    eng.synchronize()
    t = []
    for _ in range(a.calls):
        t0 = time.perf_counter()
        eng.step(1)
        t1 = time.perf_counter()
        if a.get_bodies:
            eng.get_bodies(out=bufs)
        else:
            eng.map_bodies()
        t.append((t1 - t0, time.perf_counter() - t1))
    print({"step_ms": [round(1e3 * s, 3) for s, _ in t],
           "read_ms": [round(1e3 * r, 3) for _, r in t],
           "frame_ms_mean": round(1e3 * sum(s + r for s, r in t) / len(t), 3),
           "torch": a.torch, "get_bodies": a.get_bodies, "before": a.before})


if __name__ == "__main__":
    main()
