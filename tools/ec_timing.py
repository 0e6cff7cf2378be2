#!/usr/bin/env python3
"""Per-workgroup timeline of k_emit_com (diagnostic build with -DBH_EC_TIMING).

Usage (GPU box): BH_ENGINE_LIB=<lib built with EXTRA=-DBH_EC_TIMING> python tools/ec_timing.py [config]
Runs a few steps of the scene, then reads the last build's per-workgroup wall-clock start/end
(100 MHz), slot counts and level counts, and prints the duration distribution, the kernel span,
the busiest CU and how the slow workgroups differ from the rest.
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
    arrs = scenes.config_scene(cfg)
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    eng.reset_bodies(*arrs)
    eng.step(3)
    eng.synchronize()
    n = eng.num_bodies()
    nwg = (n + 1023) // 1024
    lib = bh_amd.load_library()
    buf = (ctypes.c_uint64 * (8 * nwg))()
    rc = lib.bh_debug_ec_times(buf, nwg)
    assert rc == 0, rc
    a = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 8).astype(np.int64)
    ph, lv = a[:, 0:7], a[:, 7]
    t0, t1 = ph[:, 0], ph[:, 6]
    cnt, levels, cu = lv & 0xFFFF, (lv >> 16) & 0xFFFF, lv >> 32
    dur = (t1 - t0) * 10.0  # 100 MHz wall clock -> ns
    span = (t1.max() - t0.min()) * 10.0
    print(f"{cfg}: n={n} workgroups={nwg} kernel span {span / 1e3:.1f} us")
    q = np.percentile(dur, [0, 10, 50, 90, 99, 100]) / 1e3
    print("WG duration us  min/p10/p50/p90/p99/max:", " ".join(f"{x:.1f}" for x in q))
    print(f"sum of WG durations / (span x 256 CUs) = {dur.sum() / (span * 256):.2f} WGs resident")
    start_rel = (t0 - t0.min()) * 10.0 / 1e3
    print("WG start offsets us p50/p90/max:",
          " ".join(f"{x:.1f}" for x in np.percentile(start_rel, [50, 90, 100])))
    names = ["init loads", "skeleton+leaves", "jitter", "child lists", "COM levels", "final write"]
    for q_, nm in enumerate(names):
        d = (ph[:, q_ + 1] - ph[:, q_]) * 10.0 / 1e3
        print(f"  phase {nm:16s} us mean {d.mean():6.2f} p50 {np.median(d):6.2f} "
              f"p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
    slow = dur > np.percentile(dur, 90)
    print(f"slow 10%: slots mean {cnt[slow].mean():.0f} vs {cnt[~slow].mean():.0f}, "
          f"levels mean {levels[slow].mean():.1f} vs {levels[~slow].mean():.1f}")
    for lvl in sorted(set(levels.tolist())):
        sel = levels == lvl
        d_sk = (ph[sel, 2] - ph[sel, 1]) * 10.0 / 1e3
        d_com = (ph[sel, 5] - ph[sel, 4]) * 10.0 / 1e3
        print(f"  levels {lvl:2d}: {sel.sum():5d} WGs, mean {dur[sel].mean() / 1e3:.1f} us "
              f"(skeleton {d_sk.mean():.1f}, COM levels {d_com.mean():.1f})")
    print("distinct hw ids:", len(set(cu.tolist())))
    eng.close()


if __name__ == "__main__":
    main()
