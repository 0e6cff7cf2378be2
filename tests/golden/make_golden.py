#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (committed; re-run only on purpose).

Each fixture holds the initial SoA arrays of a seeded scene, the parameters, and the state
after K reference steps (BarnesHutAlg.kt:405-439) computed by the C restatement
(oracle/bh_oracle.c) — and, for every fixture, cross-checked bit for bit against the
independent pure-Python restatement (oracle/py_oracle.py) before it is written.

PARITY UNPINNED: the reference itself (Kotlin/JVM) cannot run here and ships no vectors,
so these fixtures pin the two restatements against each other and against regressions;
they are not reference outputs.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))

import oracle  # noqa: E402
from oracle import py_oracle  # noqa: E402
from bh_amd import scenes  # noqa: E402

FIELDS = ("x", "y", "vx", "vy", "m")


def jitter_scene():
    base = [a.copy() for a in scenes.uniform(300, 1.0, seed=21)]
    ex = np.array([base[0][3], base[0][7] + 2e-4, 777.0, 777.0, 777.0, 1500.25])
    ey = np.array([base[1][3], base[1][7] - 1e-4, 222.0, 222.0, 222.0 + 3e-4, 100.5])
    arrs = [np.concatenate([base[0], ex]), np.concatenate([base[1], ey]),
            np.concatenate([base[2], np.zeros(6)]), np.concatenate([base[3], np.zeros(6)]),
            np.concatenate([base[4], np.full(6, 2.0)])]
    perm = np.random.default_rng(5).permutation(len(arrs[0]))
    return tuple(a[perm] for a in arrs)


def merge_scene():
    bx = [1000.0, 1007.9, 1008.1, 1000.0, 1003.0, 1500.0, 1504.0]
    by = [400.0, 400.0, 400.0, 406.0, 403.0, 300.0, 300.0]
    bm = [5000.0, 1.0, 1.0, 2.0, 4500.0, 10.0, 9000.0]
    f = scenes.uniform(120, 0.5, seed=9)
    return (np.concatenate([bx, f[0]]), np.concatenate([by, f[1]]), np.concatenate([np.zeros(7), f[2]]),
            np.concatenate([np.zeros(7), f[3]]), np.concatenate([bm, f[4]]))


def outside_scene():
    f = scenes.uniform(150, 1.0, seed=12)
    return (np.concatenate([f[0], [-3.0, 2402.0, 600.0]]), np.concatenate([f[1], [400.0, 10.0, -802.5]]),
            np.concatenate([f[2], [0.0, 0.0, 5.0]]), np.concatenate([f[3], [0.0, 0.0, 0.0]]),
            np.concatenate([f[4], [2.0, 2.0, 2.0]]))


CASES = [
    # name, scene, params, K list, python cross-check K
    ("c1_baseline_theta05", lambda: scenes.config_scene("c1_baseline"), dict(theta=0.5), [1, 10, 100], [1]),
    ("two_disks_600_theta03", lambda: scenes.two_disks(450, 150), dict(theta=0.3), [1, 20], [1, 20]),
    ("two_disks_600_theta0", lambda: scenes.two_disks(450, 150), dict(theta=0.0), [2], [2]),
    ("jitter_306", jitter_scene, dict(theta=0.5, merge_min_dist=0.0), [1, 5], [1, 5]),
    ("merge_127", merge_scene, dict(theta=0.5), [1, 30], [1, 30]),
    ("outside_153", outside_scene, dict(theta=0.7), [1, 10], [1, 10]),
    ("screen_1920x1080", lambda: scenes.two_disks(300, 100), dict(theta=0.5, width_px=1920, height_px=1080), [5], [5]),
]


def cfg_of(p):
    return dict(G=p.G, dt=p.dt, theta=p.theta, soft2=p.soft2, width_px=p.width_px,
                height_px=p.height_px, merge_max_mass=p.merge_max_mass, merge_min_dist=p.merge_min_dist)


def main():
    for name, make, over, ks, py_ks in CASES:
        arrs = make()
        p = oracle.params(**over)
        out = {f"init_{f}": np.asarray(a, dtype=np.float64) for f, a in zip(FIELDS, arrs)}
        out["params"] = np.array([p.G, p.dt, p.theta, p.soft2, p.width_px, p.height_px,
                                  p.merge_max_mass, p.merge_min_dist], dtype=np.float64)
        ref = oracle.Oracle(*arrs, p=p)
        pe = py_oracle.make_engine(*arrs, cfg_of(p))
        done = 0
        for k in ks:
            ref.step(k - done)
            state = ref.get_bodies()
            if k in py_ks:
                for _ in range(k - done):
                    pe.step()
                pst = py_oracle.state(pe)
                for f, a, b in zip(FIELDS, state, pst):
                    b = np.asarray(b, dtype=np.float64)
                    assert a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64)), \
                        f"{name} K={k}: C and Python restatements disagree on {f}"
                done_py = True
            else:
                pe = None  # python restatement not advanced past this point
            for f, a in zip(FIELDS, state):
                out[f"k{k}_{f}"] = a
            done = k
            if pe is None:
                py_ks = []
        out["ks"] = np.array(ks, dtype=np.int64)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        print(f"wrote {path} ({os.path.getsize(path)} B), K = {ks}")


if __name__ == "__main__":
    main()
