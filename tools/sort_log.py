#!/usr/bin/env python3
"""Per-launch log of the adaptive bucket sort (diagnostic build with -DBH_SORT_STATS).

Usage (GPU box): BH_ENGINE_LIB=<lib built with EXTRA=-DBH_SORT_STATS> python tools/sort_log.py [config] [steps]
Prints, for the last launches (a ring of 256): the largest bucket, the buckets that left the LDS
bin radix (block radix sort / bitonic network), the buckets and elements of the global network.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))
import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    eng.reset_bodies(*scenes.config_scene(cfg))
    eng.step(steps)
    eng.synchronize()
    lib = bh_amd.load_library()
    out = (ctypes.c_ulonglong * (256 * 4))()
    assert lib.bh_debug_sort_log(out) == 0
    rows = [tuple(int(out[4 * i + q]) for q in range(4)) for i in range(256)]
    rows = [r for r in rows if any(r)]
    print(f"{cfg} x {steps} steps: {len(rows)} launches logged")
    print("largest_bucket non_bin_radix global_buckets global_elements")
    for r in rows:
        print(*r)
    eng.close()


if __name__ == "__main__":
    main()
