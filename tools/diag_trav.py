#!/usr/bin/env python3
"""Diagnosis of the traversal's launch-to-launch spread: runs C3 in chunks of steps and prints
every traversal launch time in order; then evaluates the final state both in the long-running
engine and in a fresh engine holding a copy of it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "barnes-hut-n-body_amd")]
import numpy as np  # noqa: E402

import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402

chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
per = int(sys.argv[2]) if len(sys.argv) > 2 else 20
params = bh_amd.default_params(theta=0.5)
arrs = scenes.config_scene("c3")
eng = bh_amd.Engine(params)
eng.reset_bodies(*arrs)
eng.step(5)
eng.set_profiling(True)
for c in range(chunks):
    t0 = time.perf_counter()
    eng.step(per)
    dt = time.perf_counter() - t0
    s = eng.traverse_kernel_samples()
    print(f"chunk {c}: {1e3 * dt / per:.3f} ms/step n={eng.num_bodies()} trav " +
          " ".join(f"{v:.2f}" for v in s), flush=True)


def evals(e, tag, k=3):
    e.set_profiling(True)
    out = []
    for _ in range(k):
        e.compute_accelerations()
        out.append(e.traverse_kernel_samples()[0])
    print(tag, " ".join(f"{v:.3f}" for v in out), flush=True)


evals(eng, "main engine, eval of its state:")
state = eng.get_bodies()
fresh = bh_amd.Engine(params)
fresh.reset_bodies(*state)
evals(fresh, "fresh engine, eval of a copy:")
fresh.set_profiling(True)
fresh.step(per)
print("fresh engine, steps:", " ".join(f"{v:.2f}" for v in fresh.traverse_kernel_samples()))
_, _, vis = fresh.compute_accelerations(visits=True)
print("fresh counters", fresh.traversal_counters(), "vbar", float(np.mean(vis)))
_, _, vis = eng.compute_accelerations(visits=True)
print("main counters", eng.traversal_counters(), "vbar", float(np.mean(vis)))
