#!/usr/bin/env python3
"""Per-wave timeline of the traversal (diagnostic build with -DBH_TRAV_TIMING).

Usage (GPU box): BH_ENGINE_LIB=<lib built with EXTRA=-DBH_TRAV_TIMING> python tools/trav_timing.py
Runs C3 a few steps, then one counting evaluation (per-wave iterations / force blocks) and one
production evaluation of the same state, and prints: the kernel span, wave duration
distribution, start-time spread, the tail (time from the 90th-percentile wave end to the last),
per-XCD spans and how wave duration follows the wave's iteration count.
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    eng.reset_bodies(*scenes.config_scene(cfg))
    eng.step(5)
    state = eng.get_bodies()
    probe = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    probe.reset_bodies(*state)
    lib = bh_amd.load_library()
    lib.bh_debug_trav_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = len(state[0])
    waves = (n + 63) // 64
    # counting walk on the probe: per-wave iterations (timing of the counting kernel is ignored)
    probe.compute_accelerations(visits=True)
    c = probe.traversal_counters()
    eng.set_profiling(True)
    eng.compute_accelerations()  # production walk (no kick), same state
    ms = eng.traverse_kernel_samples()
    buf = np.zeros(4 * waves, dtype=np.uint64)
    lib.bh_debug_trav_times(buf.ctypes.data, waves)
    t = buf.reshape(waves, 4)
    t0, t1 = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # us (100 MHz wall clock)
    d = e - s
    xcc = t[:, 3] & 0xF
    hw = t[:, 2]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    print(f"{cfg}: {waves} waves, kernel event {ms[0]*1e3:.1f} us, span {e.max():.1f} us")
    print("wave duration us: p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f" % tuple(np.percentile(d, [10, 50, 90, 99, 100])))
    print("wave start us: p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(s, [50, 90, 100])))
    print("wave end us: p50 %.1f p90 %.1f p99 %.1f max %.1f" % tuple(np.percentile(e, [50, 90, 99, 100])))
    busy = d.sum() / (1024 * 8)  # ideal: all wave-time packed onto 1024 SIMDs x 8 slots
    print(f"sum of wave durations / (1024 SIMDs x 8 slots) = {busy:.1f} us")
    for x in range(8):
        m = xcc == x
        print(f"  XCD {x}: waves {m.sum()} span {e[m].max():.1f} us mean dur {d[m].mean():.1f}")
    order = np.argsort(-d)[:10]
    print("slowest waves (index, dur, start, end):", [(int(i), round(float(d[i]), 1), round(float(s[i]), 1), round(float(e[i]), 1)) for i in order])
    print("counters:", c)
    per = np.zeros(waves)
    # ends per 10 us bucket: how many SIMD slots are still busy over time
    hist = np.histogram(e, bins=np.arange(0, e.max() + 10, 10))[0]
    print("waves ending per 10 us:", hist.tolist())
    starts = np.histogram(s, bins=np.arange(0, e.max() + 10, 10))[0]
    print("waves starting per 10 us:", starts.tolist())
    _ = per, cu, se


if __name__ == "__main__":
    main()
