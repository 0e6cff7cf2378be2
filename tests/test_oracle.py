"""CPU tests of the oracle (test infrastructure) — no GPU needed.

The reference (Kotlin/JVM) has no tests and cannot run here, so parity is UNPINNED by the
reference; the oracle is pinned instead by (1) bit-for-bit agreement of two independent
restatements (oracle/bh_oracle.c vs oracle/py_oracle.py), (2) hand-computed known answers,
(3) physics invariants, (4) committed golden fixtures (tests/golden/, make_golden.py).
"""
import glob
import math
import os

import numpy as np
import pytest

import oracle
from bh_amd import scenes
from conftest import bits_equal
from oracle import py_oracle

FIELDS = ("x", "y", "vx", "vy", "m")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _cfg(**kw):
    c = dict(G=80.0, dt=0.005, theta=0.5, soft2=1.0, width_px=2400, height_px=800,
             merge_max_mass=4000.0, merge_min_dist=8.0)
    c.update(kw)
    return c


def _both(arrs, **kw):
    c = _cfg(**kw)
    return oracle.Oracle(*arrs, **c), py_oracle.make_engine(*arrs, c)


def _assert_same(ref, pe):
    a = ref.get_bodies()
    b = py_oracle.state(pe)
    for f, u, v in zip(FIELDS, a, b):
        assert bits_equal(u, v), f"{f} differs between the C and Python restatements"


# ---------------------------------------------------------------- known answers
def test_two_body_known_answer():
    """(100,100) m=1 and (103,104) m=2, G=80, eps^2=1: a1 = 80*2*(3,4)/26^1.5 (BHA:250-259)."""
    arrs = (np.array([100.0, 103.0]), np.array([100.0, 104.0]), np.zeros(2), np.zeros(2),
            np.array([1.0, 2.0]))
    ref = oracle.Oracle(*arrs, **_cfg(merge_min_dist=0.0))
    ax, ay = ref.accelerations()
    # the reference's own expression order: f = G*b.m*m*invR2; fx = f*dx*invR; a = fx/b.m
    r2 = 3.0 * 3.0 + 4.0 * 4.0 + 1.0
    inv_r = 1.0 / math.sqrt(r2)
    inv_r2 = 1.0 / r2
    f = 80.0 * 1.0 * 2.0 * inv_r2
    assert ax[0] == (f * 3.0 * inv_r) / 1.0 and ay[0] == (f * 4.0 * inv_r) / 1.0
    f = 80.0 * 2.0 * 1.0 * inv_r2
    assert ax[1] == (f * -3.0 * inv_r) / 2.0 and ay[1] == (f * -4.0 * inv_r) / 2.0
    k = 80.0 / 26.0 ** 1.5
    np.testing.assert_allclose(ax, [6 * k, -3 * k], rtol=1e-15)


def test_far_body_sees_root_centre_of_mass():
    """Four bodies in one corner cell, one far body: at theta 1.0 the far body accepts the
    internal node holding the four (BHA:228) and feels their centre of mass, which is the
    children-in-order weighted sum of BHA:189-200."""
    bx = np.array([100.0, 101.0, 100.0, 101.0, 2000.0])
    by = np.array([100.0, 100.0, 101.0, 101.0, 700.0])
    bm = np.array([1.0, 2.0, 3.0, 4.0, 1.0])
    ref = oracle.Oracle(bx, by, np.zeros(5), np.zeros(5), bm, **_cfg(theta=1.0, merge_min_dist=0.0))
    ax, ay, vis = ref.accelerations(visits=True)
    m_sum, cx, cy = 0.0, 0.0, 0.0
    for i in range(4):  # children order 0..3 == (x<,y<), (x>=,y<), (x<,y>=), (x>=,y>=)
        m_sum += bm[i]
        cx += bx[i] * bm[i]
        cy += by[i] * bm[i]
    comx, comy = cx / m_sum, cy / m_sum
    dx, dy = comx - 2000.0, comy - 700.0
    r2 = dx * dx + dy * dy + 1.0
    f = 80.0 * 1.0 * m_sum * (1.0 / r2)
    assert ax[4] == f * dx * (1.0 / math.sqrt(r2)) / 1.0
    assert ay[4] == f * dy * (1.0 / math.sqrt(r2)) / 1.0
    assert vis[4] < 8  # did not descend to the four leaves


def test_theta0_is_direct_sum():
    """theta = 0 never accepts an internal node (s2 < 0 is false): the traversal is the exact
    direct sum, in tree (Morton) order; compare with an index-order direct sum."""
    arrs = scenes.two_disks(300, 100)
    ref = oracle.Oracle(*arrs, **_cfg(theta=0.0, merge_min_dist=0.0))
    ax, ay = ref.accelerations()
    x, y, _, _, m = ref.get_bodies()
    dx = x[None, :] - x[:, None]
    dy = y[None, :] - y[:, None]
    r2 = dx * dx + dy * dy + 1.0
    f = 80.0 * m[:, None] * m[None, :] / r2
    np.fill_diagonal(f, 0.0)
    ex = (f * dx / np.sqrt(r2)).sum(axis=1) / m
    ey = (f * dy / np.sqrt(r2)).sum(axis=1) / m
    np.testing.assert_allclose(ax, ex, rtol=1e-9, atol=1e-9 * np.abs(ex).max())
    np.testing.assert_allclose(ay, ey, rtol=1e-9, atol=1e-9 * np.abs(ey).max())


def test_jitter_mutates_and_drops():
    """Two coincident bodies: subdividing below h < 1e-3 shifts each by +-1e-3 per the parity
    of its mantissa LSB (BHA:146-151) and the shifted bodies fall out of the tree."""
    arrs = (np.array([500.25, 500.25, 900.0]), np.array([300.5, 300.5, 200.0]), np.zeros(3),
            np.zeros(3), np.array([1.0, 1.0, 1.0]))
    ref, pe = _both(arrs, merge_min_dist=0.0)
    ax, ay, vis = ref.accelerations(visits=True)
    x, y, *_ = ref.get_bodies()
    assert x[0] != 500.25 and y[0] != 300.5  # mutated (permanently)
    assert abs(abs(x[0] - 500.25) - 1e-3) < 1e-12
    # both coincident bodies were dropped: the third body sees neither
    assert ax[2] == 0.0 and ay[2] == 0.0
    pe.compute_accelerations(pe.build_tree())
    _assert_same(ref, pe)


def test_outside_root_not_inserted_but_feels_force():
    arrs = (np.array([-3.0, 100.0]), np.array([400.0, 400.0]), np.zeros(2), np.zeros(2),
            np.array([5.0, 5.0]))
    ref = oracle.Oracle(*arrs, **_cfg(merge_min_dist=0.0))
    ax, ay = ref.accelerations()
    assert ax[0] > 0.0  # pulled toward the in-root body
    assert ax[1] == 0.0  # the outside body exerts nothing (BHA:126)


def test_merge_threshold_and_order():
    """m > 4000 absorbs bodies with d^2 < 64 (7.9 yes, 8.1 no), masses added in descending
    index order, list order preserved (BHA:463-532)."""
    arrs = (np.array([10.0, 17.9, 18.1, 10.0]), np.array([10.0, 10.0, 10.0, 15.0]), np.zeros(4),
            np.zeros(4), np.array([5000.0, 1.5, 2.5, 0.25]))
    ref, pe = _both(arrs, dt=0.0)
    ref.step(1)
    pe.step()
    x, y, vx, vy, m = ref.get_bodies()
    assert len(x) == 2 and x[1] == 18.1
    assert m[0] == (5000.0 + 0.25) + 1.5
    _assert_same(ref, pe)


# ---------------------------------------------------------------- restatement cross-checks
CROSS = [
    ("two_disks", lambda: scenes.two_disks(220, 80), dict(theta=0.5), 4),
    ("two_disks_theta03", lambda: scenes.two_disks(220, 80), dict(theta=0.3), 3),
    ("two_disks_theta12", lambda: scenes.two_disks(220, 80), dict(theta=1.2), 3),
    ("kepler", lambda: scenes.kepler_disk(250, seed=3), dict(theta=0.5), 3),
    ("uniform", lambda: scenes.uniform(300, 0.7, seed=4), dict(theta=0.5), 3),
    ("screen_1920", lambda: scenes.two_disks(200, 60), dict(theta=0.5, width_px=1920, height_px=1080), 3),
    ("negative_cells", lambda: _negative_cells(), dict(theta=0.5), 3),
    ("negative_cells_theta0", lambda: _negative_cells(), dict(theta=0.0), 2),
]


def _negative_cells():
    """A cloud with clusters of negative-mass bodies: their cells get mass 0 (only children of
    mass > 0 count, BHA:189-192) and are never entered (BHA:216)."""
    x, y, vx, vy, m = (a.copy() for a in scenes.uniform(300, 0.5, seed=9))
    for cx, cy, half in ((600.0, 300.0, 160.0), (1800.0, 500.0, 90.0), (1200.0, 100.0, 40.0)):
        inside = (np.abs(x - cx) < half) & (np.abs(y - cy) < half)
        m[inside] = -0.3
    return x, y, vx, vy, m


@pytest.mark.parametrize("name,make,over,k", CROSS, ids=[c[0] for c in CROSS])
def test_c_and_python_restatements_agree(name, make, over, k):
    ref, pe = _both(make(), **over)
    for _ in range(k):
        ref.step(1)
        pe.step()
    _assert_same(ref, pe)


def test_restatements_agree_on_visits_and_quads():
    arrs = scenes.two_disks(150, 50)
    ref, pe = _both(arrs, merge_min_dist=0.0)
    ax, ay, vis = ref.accelerations(visits=True)
    root = pe.build_tree()
    pax, pay = pe.compute_accelerations(root)
    assert bits_equal(ax, pax) and bits_equal(ay, pay)
    assert list(vis) == pe.visits
    quads = []
    root.visit_quads(lambda q: quads.append((q.cx, q.cy, q.h)))
    cx, cy, h = ref.quads()
    assert np.array_equal(np.array(quads), np.stack([cx, cy, h], axis=1))


# ---------------------------------------------------------------- golden fixtures
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_golden_fixture_replay(path):
    d = np.load(path, allow_pickle=False)
    G, dt, theta, soft2, W, H, mm, md = d["params"]
    p = oracle.params(G=G, dt=dt, theta=theta, soft2=soft2, width_px=int(W), height_px=int(H),
                      merge_max_mass=mm, merge_min_dist=md)
    ref = oracle.Oracle(*[d[f"init_{f}"] for f in FIELDS], p=p)
    done = 0
    for k in d["ks"]:
        ref.step(int(k) - done)
        done = int(k)
        for f, a in zip(FIELDS, ref.get_bodies()):
            assert bits_equal(a, d[f"k{k}_{f}"]), f"{os.path.basename(path)} K={k} {f}"


def test_scene_generators_are_deterministic_and_shaped():
    a = scenes.galaxy_disk(500, seed=7, r=300.0)
    b = scenes.galaxy_disk(500, seed=7, r=300.0)
    c = scenes.galaxy_disk(500, seed=8, r=300.0)
    for u, v in zip(a, b):
        assert bits_equal(u, v)
    assert not np.array_equal(a[0], c[0])
    x, y, vx, vy, m = a
    assert m[0] == 50_000.0 and x[0] == 1200.0 and y[0] == 400.0
    r = np.hypot(x[1:] - 1200.0, y[1:] - 400.0)
    assert r.min() >= 8.0 * (1 - 0.03) and r.max() <= 300.0 * 1.03
    assert np.allclose(m[1:], 5000.0 / 499)
    # clockwise circular velocity: v . r == 0
    assert np.abs(vx[1:] * (x[1:] - 1200.0) + vy[1:] * (y[1:] - 400.0)).max() < 1e-6 * r.max() * 100
    u = scenes.uniform(1000, 0.5, seed=4)
    assert u[0].min() >= 0.0 and u[0].max() < 2400.0 and u[1].max() < 800.0
    k = scenes.kepler_disk(300, seed=3)
    assert k[4][0] == 50_000.0


def test_state_file_round_trip(tmp_path):
    """The checkpoint format (csrc/state_io.cpp) written and read back by the host-side
    reader / writer: header fields and every fp64 word survive, N = 0 included."""
    from bh_amd import state_file
    rng = np.random.default_rng(3)
    params = dict(G=80.0, dt=0.005, theta=0.5, soft2=1.0, width_px=1920, height_px=1080,
                  merge_max_mass=4000.0, merge_min_dist=8.0)
    for n in (0, 1, 777):
        arrs = [rng.standard_normal(n) for _ in range(5)]
        p = tmp_path / f"s{n}.bhstate"
        state_file.write(p, params, *arrs)
        assert p.stat().st_size == 80 + 40 * n
        got_p, got = state_file.read(p)
        assert got_p == params
        for a, b in zip(arrs, got):
            assert np.array_equal(a.view(np.int64), b.view(np.int64))
    raw = bytearray((tmp_path / "s1.bhstate").read_bytes())
    raw[0] = ord("X")
    (tmp_path / "bad.bhstate").write_bytes(bytes(raw))
    with pytest.raises(ValueError):
        state_file.read(tmp_path / "bad.bhstate")
