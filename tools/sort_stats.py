#!/usr/bin/env python3
"""Which path the adaptive bucket sort's buckets take (diagnostic build with -DBH_SORT_STATS).

Usage (GPU box): BH_ENGINE_LIB=<lib built with EXTRA=-DBH_SORT_STATS> python tools/sort_stats.py [config] [steps]
Counts, over every build of `steps` steps: buckets sorted by the LDS bin radix, by the LDS bitonic
network (a bin above RADIX_MAXBIN), by the global-memory network (a bucket above SORT_CAP), and
the elements each path handled.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))
import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    eng.reset_bodies(*scenes.config_scene(cfg))
    eng.step(steps)
    eng.synchronize()
    out = (ctypes.c_ulonglong * 8)()
    assert bh_amd.load_library().bh_debug_sort_stats(out) == 0
    r, rs, b, bs, g, gs = (int(v) for v in out[:6])
    tot = max(r + b + g, 1)
    print(f"{cfg} x {steps} steps: buckets radix {r} ({100 * r / tot:.1f} %, {rs} elements), "
          f"bitonic {b} ({100 * b / tot:.1f} %, {bs} elements), global {g} ({gs} elements)")
    eng.close()


if __name__ == "__main__":
    main()
