"""CPU checks of the locally-essential-tree rule of the multi-rank build (csrc/let.hip).

A rank builds the full subtree only of the depth-8 cells within `gap2` of its own cells; every
other cell is kept as one childless record.  That is exact only if every body of an own cell
ACCEPTS every such cell as a whole under the reference's criterion (BarnesHutAlg.kt:222-228:
dist2 = dx*dx + dy*dy + SOFT2; s2 = (h*2)^2; accept iff s2 < theta2 * dist2) -- with the body
anywhere in its cell and the cell's centre of mass anywhere in the remote cell, both widened by
the jitter's reach (2e-3 per axis, BHA:146-151).  The rule is restated from let_include_gap2 and
checked on random and adversarial (closest-corner) placements in float64.
"""
import math

import numpy as np
import pytest

LET_P = 8
JITTER = 2e-3 * 1.0001


def geometry(width=2400, height=800):
    root_h = max(width, height) / 2.0 + 2.0  # BHA:360-361
    h = root_h
    for _ in range(LET_P):
        h = h / 2.0  # BHA:74
    s = h * 2.0
    return 2.0 * h, s * s  # cell width, s2 at depth 8


def include_gap2(theta2, soft2, w, s2):
    """let_include_gap2 (csrc/let.hip): cells with gx^2 + gy^2 <= gap2 are built locally."""
    m = 0.01
    q = s2 * (1.0 + 1e-6) / theta2 - soft2
    r = (m + math.sqrt(q if q > 0.0 else 0.0)) / w
    return r * r


def accepts(theta2, soft2, s2, bx, by, cx, cy):
    dx = cx - bx  # BHA:223-225, evaluated as written
    dy = cy - by
    dist2 = dx * dx + dy * dy + soft2
    return s2 < theta2 * dist2  # BHA:228


@pytest.mark.parametrize("theta", [0.3, 0.5, 0.7, 1.0, 1.6])
@pytest.mark.parametrize("soft2", [0.0, 1.0, 25.0])
def test_cells_beyond_the_halo_are_accepted_by_every_own_body(theta, soft2):
    w, s2 = geometry()
    theta2 = theta * theta
    g2 = include_gap2(theta2, soft2, w, s2)
    rng = np.random.default_rng(int(theta * 100 + soft2))
    kmax = int(math.floor(math.sqrt(max(g2, 0.0)))) + 3
    checked = 0
    for gx in range(0, kmax + 1):
        for gy in range(0, kmax + 1):
            if gx * gx + gy * gy <= g2:
                continue  # built locally: nothing to prove
            # own cell [0, w)^2, remote cell separated by gx / gy whole cells
            ox, oy = (gx + 1) * w, (gy + 1) * w
            # adversarial: the closest corners, pushed together by the jitter reach
            bx = np.array([w + JITTER, w - 1e-9, w])
            by = np.array([w + JITTER, w, w - 1e-9])
            cx = np.array([ox - JITTER, ox, ox])
            cy = np.array([oy - JITTER, oy, oy])
            # random placements inside both (widened) cells
            bx = np.concatenate([bx, rng.uniform(-JITTER, w + JITTER, 2000)])
            by = np.concatenate([by, rng.uniform(-JITTER, w + JITTER, 2000)])
            cx = np.concatenate([cx, ox + rng.uniform(-JITTER, w + JITTER, 2000)])
            cy = np.concatenate([cy, oy + rng.uniform(-JITTER, w + JITTER, 2000)])
            for i in range(len(bx)):
                assert accepts(theta2, soft2, s2, bx[i], by[i], cx[i], cy[i]), \
                    (theta, soft2, gx, gy, bx[i], by[i], cx[i], cy[i])
            checked += 1
    assert checked > 0


@pytest.mark.parametrize("theta", [0.5, 1.0])
def test_the_halo_is_not_wider_than_one_ring_beyond_need(theta):
    """Tightness: some cell at the largest included gap is opened by a body of the own cell
    (the halo holds cells that matter), so the rule costs at most the rounding to whole cells."""
    w, s2 = geometry()
    theta2, soft2 = theta * theta, 1.0
    g2 = include_gap2(theta2, soft2, w, s2)
    best = max((gx, gy) for gx in range(0, 20) for gy in range(0, 20) if gx * gx + gy * gy <= g2)
    gx, gy = best
    if gx == 0 and gy == 0:
        return
    # nearest corners of the own cell and the remote cell at that gap
    bx, by = w, w
    cx, cy = (gx + 1) * w, (gy + 1) * w
    d = math.hypot(cx - bx, cy - by)
    # one cell closer than the included gap is always opened
    assert not accepts(theta2, soft2, s2, bx, by, bx + max(d - w, 0.0), by)
