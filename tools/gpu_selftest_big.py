"""Exactness sweep of the in-range sqrt / seeded-reciprocal sequences (fastmath.hpp) against
IEEE sqrt, 1/sqrt and 1/x on the GPU: 2^30 generated operands per seed (bh_selftest_fast_math).
    python tools/gpu_selftest_big.py [n_seeds=4]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "barnes-hut-n-body_amd")]
import bh_amd  # noqa: E402

seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for s in range(seeds):
    t0 = time.time()
    bad = bh_amd.selftest_fast_math(1 << 30, seed=0x5EED0000 + s)
    print(f"seed {s}: 2^30 operands, mismatches {bad} ({time.time() - t0:.1f} s)", flush=True)
    if bad:
        sys.exit(1)
