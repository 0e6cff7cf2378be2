#!/usr/bin/env python3
"""Phase stamps of k_small_front (diagnostic build with -DBH_SF_TIMING).

Usage (GPU box): BH_ENGINE_LIB=<lib built with EXTRA=-DBH_SF_TIMING> python tools/sf_timing.py [config] [steps]
Steps a small scene and prints the median duration (us, 100 MHz wall clock) of the small build
front's phases over its last launches: keys load, bitonic sort, sorted outputs + key gather,
fixup + cell starts, prep, base scan.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))
import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c1_baseline"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    eng.reset_bodies(*scenes.config_scene(cfg))
    eng.step(steps)
    eng.synchronize()
    buf = np.zeros(64 * 8, dtype=np.uint64)
    assert bh_amd.load_library().bh_debug_sf_times(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    t = buf.reshape(64, 8).astype(np.int64)
    t = t[t[:, 6] > t[:, 0]]
    names = ["keys", "sort", "outputs + key gather", "fixup + cells", "prep", "scan"]
    d = np.diff(t[:, :7], axis=1) / 100.0
    print(f"{cfg}: {len(t)} launches; total median {np.median((t[:, 6] - t[:, 0]) / 100.0):.2f} us")
    for k, nm in enumerate(names):
        print(f"  {nm:22s} median {np.median(d[:, k]):6.2f} us")


if __name__ == "__main__":
    main()
