#!/usr/bin/env python3
"""Phase timeline of the breadth-first walk (diagnostic build with -DBH_BFS_TIMING).

Usage (GPU box): BH_ENGINE_LIB=<lib built with EXTRA=-DBH_BFS_TIMING> python tools/bfs_timing.py c1_code
Steps the scene a few times, evaluates once more and prints, over the launch's waves (one body
each): the median / p90 time of the bitmap clear + root, each level, the bitmap scan and the
terms + ordered sum (us at the 100 MHz wall clock), the number of levels and accepted nodes.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))
import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402

REC = 24


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c1_code"
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    eng.reset_bodies(*scenes.config_scene(cfg))
    eng.step(3)
    eng.compute_accelerations()
    lib = bh_amd.load_library()
    lib.bh_debug_bfs_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = min(eng.num_bodies(), 16384)
    buf = np.zeros(REC * n, dtype=np.uint64)
    assert lib.bh_debug_bfs_times(buf.ctypes.data, n) == 0
    t = buf.reshape(n, REC).astype(np.int64)
    ok = t[:, 19] > t[:, 0]
    t = t[ok]
    us = lambda a: np.asarray(a, dtype=np.float64) / 100.0  # 100 MHz ticks -> us
    levels = t[:, 20]
    print(f"{cfg}: {ok.sum()} of {n} waves stamped; levels median {np.median(levels):.0f} "
          f"max {levels.max()}, accepted median {np.median(t[:, 21]):.0f} max {t[:, 21].max()}")
    tot = us(t[:, 19] - t[:, 0])
    print(f"  whole walk: median {np.median(tot):.2f} us, p90 {np.percentile(tot, 90):.2f}")
    print(f"  clear + root: median {np.median(us(t[:, 1] - t[:, 0])):.2f}")
    prev = t[:, 1]
    for L in range(1, 16):
        has = levels >= L
        if not has.any():
            break
        d = us(t[has, 2 + L] - prev[has])
        print(f"  level {L:2d}: median {np.median(d):.2f} us ({has.sum()} waves)")
        prev = np.where(has, t[:, 2 + L], prev)
    last = np.where(levels > 15, t[:, 17], prev)
    print(f"  scan: median {np.median(us(t[:, 18] - last)):.2f}")
    print(f"  terms + sum: median {np.median(us(t[:, 19] - t[:, 18])):.2f}")
    span = us(t[:, 19].max() - t[:, 0].min())
    print(f"  launch span (first start -> last end): {span:.1f} us")


if __name__ == "__main__":
    main()
