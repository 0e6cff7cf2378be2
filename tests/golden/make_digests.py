#!/usr/bin/env python3
"""Full-state digests at the SURVEY §8d parity horizons of the large configurations
(committed as tests/golden/digests.json; re-run only on purpose: ~30 min on 8 cores for the
10-step cases, ~3.5 h more for the 100-step ones).

For each case the C restatement (oracle/bh_oracle.c) runs the reference step (BHA:405-439)
K times from the seeded scene and the SHA-256 of every final SoA field (little-endian fp64,
caller order) is recorded, together with N.  The GPU tests recompute the same digests from the
engine's state, so the full 1e7-body state is compared bit for bit without shipping it or
running the oracle on the GPU box.  C5 records one theta = 0 evaluation: the digests of all
262 144 accelerations.

PARITY UNPINNED: these are the restatement's outputs, not the reference's (no JVM here).

    python tests/golden/make_digests.py [case ...]
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "barnes-hut-n-body_amd")]

import oracle  # noqa: E402
from bh_amd import scenes  # noqa: E402

FIELDS = ("x", "y", "vx", "vy", "m")
OUT = os.path.join(HERE, "digests.json")

# name: (scene, theta, steps K; 0 = one evaluation of the accelerations)
CASES = {
    "c3_k10": ("c3", 0.5, 10),
    "c3_k100": ("c3", 0.5, 100),   # the north star's 100-step horizon at the headline size
    "c4_k100": ("c4", 0.5, 100),   # ... and at the north-star size (~3 h on 8 cores)
    "c4_k10": ("c4", 0.5, 10),
    "c3x8_k2": ("c3x8", 0.5, 2),
    "c5_eval": ("c5", 0.0, 0),
}


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def run(name):
    scene, theta, k = CASES[name]
    arrs = scenes.config_scene(scene)
    ref = oracle.Oracle(*arrs, theta=theta, threads=os.cpu_count() or 8)
    t0 = time.time()
    if k == 0:
        ax, ay = ref.accelerations()
        ent = {"n": len(ax), "ax": sha(ax), "ay": sha(ay)}
    else:
        ref.step(k)
        st = ref.get_bodies()
        ent = {"n": len(st[0])}
        ent.update({f: sha(a) for f, a in zip(FIELDS, st)})
    ref.close()
    ent.update(scene=scene, theta=theta, steps=k, seconds=round(time.time() - t0, 1))
    return ent


def main():
    names = sys.argv[1:] or list(CASES)
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        db[name] = run(name)
        print(name, db[name], flush=True)
        with open(OUT, "w") as fh:
            json.dump(db, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
