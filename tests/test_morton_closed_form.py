"""The build's Morton cell index (tree_build.hip k_morton) is the closed form of the reference's
descent (BHA:145-156: digit = p >= cell centre at every depth).  This checks the closed form --
rounded quotient, then two exact compares against the depth-J grid lines -- against the descent
itself in IEEE binary64 (numpy), on random points and on points at and next to grid lines, over
several screen geometries (Main.kt 640x480 .. 7680x4320 and odd sizes)."""
import numpy as np
import pytest


def geometry(W, H):
    root_cx, root_h = W / 2.0, max(W, H) / 2.0 + 2.0
    h = [root_h]
    while h[-1] >= 1e-3:
        h.append(h[-1] / 2.0)
    return root_cx, root_h, h, len(h) - 1  # J: first depth with h < 1e-3


def descent(p, root_cx, h, J):
    c = np.full_like(p, root_cx)
    idx = np.zeros(p.shape, dtype=np.int64)
    for d in range(J):
        bit = p >= c
        c = np.where(bit, c + h[d + 1], c - h[d + 1])
        idx = (idx << 1) | bit.astype(np.int64)
    return idx


def closed_form(p, root_cx, root_h, h, J):
    w = 2.0 * h[J]
    o = root_cx - root_h
    top = (1 << J) - 1
    c = np.clip(np.trunc((p - o) * (1.0 / w)).astype(np.int64), 0, top)
    lo = o + c.astype(np.float64) * w
    c = np.where(p < lo, c - 1, c)
    hi = o + (c + 1).astype(np.float64) * w
    c = np.where((c < top) & (p >= hi), c + 1, c)
    return c


@pytest.mark.parametrize("W,H", [(2400, 800), (640, 480), (1921, 1079), (7680, 4320), (100001, 3)])
def test_closed_form_equals_descent(W, H):
    root_cx, root_h, h, J = geometry(W, H)
    rng = np.random.default_rng(W)
    w = 2.0 * h[J]
    o = root_cx - root_h
    k = rng.integers(0, 1 << J, 60000).astype(np.float64)
    lines = o + k * w
    p = np.concatenate([
        o + rng.random(60000) * 2.0 * root_h,
        lines, np.nextafter(lines, -np.inf), np.nextafter(lines, np.inf),
        [o, np.nextafter(root_cx + root_h, -np.inf)],
    ])
    p = p[(p >= root_cx - root_h) & (p < root_cx + root_h)]  # Quad.contains (BHA:61-62)
    np.testing.assert_array_equal(closed_form(p, root_cx, root_h, h, J), descent(p, root_cx, h, J))
