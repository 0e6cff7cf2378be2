"""The C-ABI boundary (include/bh_engine.h) on CPU: the library loads, exports every
declared symbol, and fails loudly (no CPU fallback) when no GPU is visible."""
import os
import re
import subprocess

import numpy as np
import pytest

import bh_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bh_engine.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bh_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("bh_create", "bh_step", "bh_reset_bodies", "bh_get_bodies", "bh_get_quads",
                 "bh_compute_accelerations", "bh_destroy", "bh_last_error", "bh_create_dist"):
        assert must in names


def test_library_exports_every_declared_symbol(engine_lib):
    for name in declared_functions():
        assert hasattr(engine_lib, name), f"{name} declared in bh_engine.h but not exported"
    out = subprocess.run(["nm", "-D", "--defined-only", bh_amd.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (bh_[a-z0-9_]+)\b", out))
    assert set(declared_functions()) <= exported
    assert set(bh_amd.EXPORTED_SYMBOLS) <= exported


def test_default_params_match_config_kt():
    p = bh_amd.default_params()
    assert (p.G, p.dt, p.theta, p.soft2) == (80.0, 0.005, 0.30, 1.0)      # CFG:11,14,23,20
    assert (p.width_px, p.height_px) == (2400, 800)                      # CFG:5,8
    assert (p.merge_max_mass, p.merge_min_dist) == (4000.0, 8.0)         # BHA:315,321


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (7, 2), (1000, 3), (1_000_003, 8), (5, 8)])
def test_shard_ranges_partition_the_bodies(n, world):
    """Pieces (rank r, round k) tile [0, n) in the order r-major, k-minor -- every rank owns one
    contiguous range of lanes -- each a whole number of wavefronts except the last non-empty
    one; in the exchange buffer the pieces of round k are adjacent (in-place all-gather) and
    the slots are a permutation of the lanes."""
    pieces = []
    for r in range(world):
        for k in range(bh_amd.SHARD_ROUNDS):
            lo, hi = bh_amd.shard_range(n, r, world, k)
            assert 0 <= lo <= hi <= n
            pieces.append((r, k, lo, hi))
    assert pieces[0][2] == 0 and pieces[-1][3] == n
    assert all(pieces[i][3] == pieces[i + 1][2] for i in range(len(pieces) - 1))
    sub = pieces[0][3] - pieces[0][2]
    assert sub % 64 == 0 or n <= 64
    assert all(hi - lo in (sub, 0) or hi == n for _, _, lo, hi in pieces)
    if n <= 5000:
        slots = [bh_amd.gather_slot(n, world, q) for q in range(n)]
        assert len(set(slots)) == n
        for r, k, lo, hi in pieces:
            if hi > lo:
                assert bh_amd.gather_slot(n, world, lo) == (k * world + r) * sub
                assert slots[lo:hi] == list(range(slots[lo], slots[lo] + hi - lo))


def test_shard_range_rejects_bad_arguments():
    with pytest.raises(bh_amd.BhError):
        bh_amd.shard_range(10, 3, 2)
    with pytest.raises(bh_amd.BhError):
        bh_amd.shard_range(10, 0, 2, bh_amd.SHARD_ROUNDS)


def _gpu_visible():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU failure mode")
def test_engine_fails_loudly_without_a_gpu():
    with pytest.raises(bh_amd.BhError):
        bh_amd.Engine(bh_amd.default_params())


def test_scene_entry_points_validate_arguments(engine_lib):
    import ctypes
    D = ctypes.POINTER(ctypes.c_double)
    rc = engine_lib.bh_scene_uniform(10, 1.0, 1, 2400, 800, D(), D(), D(), D(), D())
    assert rc == bh_amd.BH_E_INVALID
    assert len(bh_amd.scenes.uniform(0, 1.0)[0]) == 0  # BF:165 n <= 0 -> empty list
    x = bh_amd.scenes.uniform(5, 1.0, seed=1)[0]
    assert np.all((x >= 0) & (x < 2400))
