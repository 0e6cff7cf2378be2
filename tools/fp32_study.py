#!/usr/bin/env python3
"""C5 fp32-vs-fp64 study: on the C5 scene (uniform cloud, N = 262 144,
theta = 0) compare the fp32 all-pairs accelerations (GPU.kt physics, bh_nbody3d, z = 0)
with the exact fp64 theta = 0 engine, and time both kernels.  Also times the fp32 3-D step
on a GPU.kt-shaped sphere.  Writes profiles/<tag>_c5_fp32_study.json.

Usage (GPU box): python tools/fp32_study.py [tag]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))

import numpy as np  # noqa: E402

import bh_amd  # noqa: E402
from bh_amd import scenes  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    arrs = scenes.config_scene("c5")
    n = len(arrs[0])
    exact = bh_amd.Engine(bh_amd.default_params(theta=0.0), device=0)
    exact.reset_bodies(*arrs)
    exact.compute_accelerations()  # warm-up (allocations)
    exact.reset_bodies(*arrs)
    exact.set_profiling(True)
    t0 = time.perf_counter()
    ax, ay = exact.compute_accelerations()
    t64 = time.perf_counter() - t0
    x, y, vx, vy, m = exact.get_bodies()
    eng = bh_amd.NBody3D(device=0)
    eng.set(x, y, np.zeros_like(x), vx, vy, np.zeros_like(x), m)
    eng.accelerations()
    fx, fy, _ = eng.accelerations()
    k32 = eng.last_ms()
    g = np.stack([fx.astype(np.float64), fy.astype(np.float64)])
    w = np.stack([ax, ay])
    err = np.linalg.norm(g - w, axis=0) / np.linalg.norm(w, axis=0)
    # 3-D step throughput on a GPU.kt-shaped sphere of the same size
    from oracle import py_gpu3d
    sph = py_gpu3d.sphere(n - 1)
    eng.set(*sph)
    eng.step(1)
    eng.step(10)
    step_ms = eng.last_ms() / 10
    inter = float(n) * (n - 1)
    out = {
        "scene": f"c5 uniform cloud N={n}, theta=0, z=0 for the fp32 engine",
        "fp64_exact": {"eval_wall_ms": round(1e3 * t64, 3),
                       "note": "tree build + leaf list + k_direct, bit-identical to the oracle"},
        "fp32_allpairs": {"kernel_ms": round(k32, 3),
                          "interactions_per_s": round(inter / (k32 * 1e-3)),
                          "tflops_20flop": round(20 * inter / (k32 * 1e-3) / 1e12, 2)},
        "rel_err_per_body": {p: float(np.percentile(err, q)) for p, q in
                             (("p50", 50), ("p90", 90), ("p99", 99), ("p99.9", 99.9), ("max", 100))},
        "fp32_3d_step_sphere": {"n": n, "ms_per_step": round(step_ms, 3),
                                "body_steps_per_s": round(n / (step_ms * 1e-3))},
    }
    path = os.path.join(ROOT, "gpurun_out", f"{tag}_c5_fp32_study.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
