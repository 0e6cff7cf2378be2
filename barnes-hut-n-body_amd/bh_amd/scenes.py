"""Seeded scene generators (BodyFactory.kt = BF) via the engine library's host-side C++
restatement (csrc/scenes.cpp).  Returns SoA float64 arrays (x, y, vx, vy, m).

Named configurations:
  c1_baseline  'R' scene per BASELINE.json: two galaxy disks, 2 x 1000 bodies
  c1_code      the code's defaultBodies() (NBodyPanel.kt:83-100): 10 000 + 2 500 bodies
  c2           Kepler disk, N = 1e5 (BF:11-61), seed 3
  c3           two colliding galaxy disks, 8e5 (r=300) + 2e5 (y=160, vx=-50, r=100,
               M_c=5e3, M_sat=500), seeds 1/2
  c4           uniform cloud over [0,2400) x [0,800), m = 0.5 (BF:160-177), seed 4
"""
from __future__ import annotations

import ctypes

import numpy as np

W_DEFAULT, H_DEFAULT = 2400, 800  # CFG:5,8
G_DEFAULT = 80.0                  # CFG:11


def _lib():
    from . import load_library
    return load_library()


def _out(n):
    return [np.zeros(n, dtype=np.float64) for _ in range(5)]


def _ptrs(arrs):
    return [a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) for a in arrs]


def galaxy_disk(n_total, eps_m2=0.03, phi0=0.0, bar_taper_r=None, radial_scale=None,
                speed_jitter=0.01, radial_jitter=0.0, clockwise=True, seed=1, vx=0.0, vy=0.0,
                x=W_DEFAULT * 0.5, y=H_DEFAULT * 0.5, r=200.0, min_r=8.0, central_mass=50_000.0,
                total_satellite_mass=5_000.0, G=G_DEFAULT):
    """BodyFactory.makeGalaxyDisk (BF:63-150) with rng = Random(seed)."""
    out = _out(n_total)
    rc = _lib().bh_scene_galaxy_disk(
        int(n_total), eps_m2, phi0, bar_taper_r if bar_taper_r else -1.0,
        radial_scale if radial_scale else -1.0, speed_jitter, radial_jitter, 1 if clockwise else 0,
        int(seed), vx, vy, x, y, r, min_r, central_mass, total_satellite_mass, G, *_ptrs(out))
    if rc != 0:
        raise ValueError(f"bh_scene_galaxy_disk rc={rc}")
    return tuple(out)


def kepler_disk(n_total, clockwise=True, radial_jitter=0.03, speed_jitter=0.01, seed=3, vx=0.0,
                vy=0.0, x=W_DEFAULT * 0.5, y=H_DEFAULT * 0.5, r=min(W_DEFAULT, H_DEFAULT) * 0.38,
                G=G_DEFAULT):
    """BodyFactory.makeKeplerDisk (BF:11-61), default rng Random(3)."""
    out = _out(n_total)
    rc = _lib().bh_scene_kepler_disk(int(n_total), 1 if clockwise else 0, radial_jitter,
                                     speed_jitter, int(seed), vx, vy, x, y, r, G, *_ptrs(out))
    if rc != 0:
        raise ValueError(f"bh_scene_kepler_disk rc={rc}")
    return tuple(out)


def uniform(n, m, seed=4, width_px=W_DEFAULT, height_px=H_DEFAULT):
    """BodyFactory.makeUniformRandom (BF:160-177) with rng = Random(seed)."""
    if n <= 0 or m <= 0.0:
        return tuple(np.zeros(0, dtype=np.float64) for _ in range(5))
    out = _out(n)
    rc = _lib().bh_scene_uniform(int(n), m, int(seed), int(width_px), int(height_px), *_ptrs(out))
    if rc != 0:
        raise ValueError(f"bh_scene_uniform rc={rc}")
    return tuple(out)


def concat(*scenes):
    return tuple(np.concatenate([s[k] for s in scenes]) for k in range(5))


def two_disks(n1, n2, seed1=1, seed2=2, G=G_DEFAULT, height_px=H_DEFAULT):
    """defaultBodies() (NBodyPanel.kt:83-100) with explicit seeds and body counts."""
    d1 = galaxy_disk(n1, r=300.0, central_mass=50_000.0, total_satellite_mass=5_000.0, seed=seed1,
                     G=G)
    d2 = galaxy_disk(n2, y=height_px * 0.2, vx=-50.0, r=100.0, central_mass=5_000.0,
                     total_satellite_mass=500.0, seed=seed2, G=G)
    return concat(d1, d2)


def config_scene(name: str):
    """Initial arrays of a named configuration (see module docstring)."""
    if name == "c1_baseline":
        return two_disks(1000, 1000)
    if name == "c1_code":
        return two_disks(10_000, 2_500)
    if name == "c2":
        return kepler_disk(100_000, seed=3)
    if name == "c3":
        return two_disks(800_000, 200_000)
    if name == "c4":
        return uniform(10_000_000, 0.5, seed=4)
    if name == "c5":  # theta = 0 direct-sum configuration
        return uniform(262_144, 0.5, seed=5)
    if name.startswith("c3x"):  # weak-scaling family: c3x<k> = k copies' worth of bodies
        k = int(name[3:])
        return two_disks(800_000 * k, 200_000 * k)
    raise KeyError(name)
