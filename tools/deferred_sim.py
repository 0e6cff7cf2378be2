#!/usr/bin/env python3
"""Analysis (CPU, oracle): how often the traversal's point-force block runs.

Waves of 64 Morton-consecutive bodies walk the oracle's tree exactly like the GPU's shared
cursor (traverse.hip).  Inline, the force block executes on every node some lane accepts;
with deferred forces each lane queues its accepted nodes in a FIFO of depth Q and the block
runs once per "flush" (a FIFO full, or >= T lanes with queued work, or the final drain).
Prints force-block executions per wave for each (Q, T).  Test infrastructure only.

    python tools/deferred_sim.py [config=c3] [theta=0.5]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "barnes-hut-n-body_amd"), os.path.join(ROOT, "tools")]

import oracle  # noqa: E402
from bh_amd import scenes  # noqa: E402
from morton import morton_order  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    theta = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    arrs = scenes.config_scene(cfg)
    ref = oracle.Oracle(*arrs, theta=theta, threads=1)
    order = morton_order(arrs[0], arrs[1])
    waves = (len(order) + 63) // 64
    t0 = time.time()
    it, lv = ref.group_union(order)
    fi, co = ref.union_force_stats()
    print(f"{cfg} theta={theta}: {len(order)} bodies, {waves} waves; per wave: iterations "
          f"{it / waves:.1f}, force iterations (inline) {fi / waves:.1f}; lane efficiency "
          f"{lv / 64 / it:.3f}; contributions per body {co / len(order):.1f} "
          f"[{time.time() - t0:.1f} s]", flush=True)
    for q in (1, 2, 3, 4, 6, 8):
        row = []
        for t in (32, 48, 56, 64, 65):
            fl = ref.deferred_flushes(order, q, t)
            row.append(f"T={t}: {fl / waves:6.1f} ({fl / fi:.3f})")
        print(f"Q={q}: " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
