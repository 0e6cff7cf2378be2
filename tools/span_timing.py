#!/usr/bin/env python3
"""Per-level timeline of k_com_span (diagnostic build with -DBH_SPAN_TIMING).

Usage (GPU box): BH_ENGINE_LIB=<lib built with EXTRA=-DBH_SPAN_TIMING> python tools/span_timing.py [config]
Runs a few steps, then reads group 0's wall-clock stamps (100 MHz) of the last launches: kernel
start, the span_list column read (own mask), each level J..0 (load wait + LDS level + barrier) and
the drain of the stores; prints them per launch, the even / odd launches apart (one GPU: the
critical-path build and the overlapped one alternate).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))
import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402

REC, W = 64, 32


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), device=0)
    eng.reset_bodies(*scenes.config_scene(cfg))
    eng.step(12)
    eng.synchronize()
    lib = bh_amd.load_library()
    buf = (ctypes.c_uint64 * (REC * W))()
    launches = ctypes.c_uint32(0)
    assert lib.bh_debug_span_times(buf, ctypes.byref(launches)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(REC, W).astype(np.int64)
    nl = launches.value
    order = [(nl - 1 - q) % REC for q in range(min(nl, 16))][::-1]
    print(f"{cfg}: {nl} launches; last {len(order)} (oldest first), us")
    rows = []
    for rec in order:
        t_n = int(a[rec, W - 1])
        st = a[rec, :t_n]
        d = np.diff(st) * 10.0 / 1e3
        rows.append(d)
        print(f"  total {(st[-1] - st[0]) * 10.0 / 1e3:6.1f}  own-mask {d[0]:5.2f}  levels "
              + " ".join(f"{x:.2f}" for x in d[1:-1]) + f"  drain {d[-1]:.2f}")
    for par in (0, 1):
        sel = [r for q, r in enumerate(rows) if q % 2 == par]
        if sel:
            m = np.mean(np.stack(sel), axis=0)
            print(f"mean of launches {par}::2: total {m.sum():.1f}  own-mask {m[0]:.2f}  "
                  f"levels sum {m[1:-1].sum():.1f} (max {m[1:-1].max():.2f})  drain {m[-1]:.2f}")
    eng.close()


if __name__ == "__main__":
    main()
