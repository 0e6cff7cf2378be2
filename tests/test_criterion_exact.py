"""CPU check of the traversal's fast opening criterion (csrc/traverse.hip, walk<FAST>).

The reference opens a node unless s2 < theta2 * dist2 (BarnesHutAlg.kt:226-228), with
s2 = (h_d * 2)^2 and h_d = h_0 / 2^d, so s2 = s2_0 * 4^-d exactly.  The fast path forms s2 by
subtracting 2d from the exponent field of s2_0 (an integer operation on the scalar unit) and
compares it with RN(theta2 * dist2); the general path compares s2_0 with
ldexp(RN(theta2 * dist2), 2d).  Both must take the same decision as the reference's own
s2 computed by repeated halving -- checked here in float64 for every depth the node record can
carry (2d <= 255) and s2_0 down to the fast path's bound (fast_s2_ok: s2_0 >= 2^-760).
"""
import numpy as np
import pytest


def s2_by_exponent(s2root, two_d):
    bits = np.float64(s2root).view(np.uint64) - (np.uint64(two_d) << np.uint64(52))
    return bits.view(np.float64)


@pytest.mark.parametrize("s2root", [2.0 ** 22 * 1.3779, 5.779e6, 1.0, 2.0 ** -700, 2.0 ** -760])
def test_exponent_subtraction_is_the_exact_scaling(s2root):
    for two_d in range(0, 256, 2):
        got = s2_by_exponent(s2root, two_d)
        want = np.ldexp(np.float64(s2root), -two_d)
        assert got == want and np.isfinite(got) and got > 0.0, (s2root, two_d)


def test_matches_the_reference_s2_by_halving():
    # root half-widths of the reference's geometries (BHA:360-361: max(W, H) / 2 + 2)
    for h0 in [1202.0, 322.0, 3842.0, 642.0]:
        s2root = (h0 * 2.0) * (h0 * 2.0)
        h = h0
        for d in range(0, 100):
            s2_ref = (h * 2.0) * (h * 2.0)
            assert s2_by_exponent(s2root, 2 * d) == s2_ref, (h0, d)
            h = h / 2.0


def test_fast_and_general_criteria_agree():
    rng = np.random.default_rng(7)
    s2root = (1202.0 * 2.0) ** 2
    for theta in [0.3, 0.5, 1.0, 1.7]:
        theta2 = theta * theta
        for two_d in range(0, 120, 2):
            s2 = s2_by_exponent(s2root, two_d)
            # dist2 around the decision boundary s2 / theta2, including exact ties
            base = s2 / theta2
            d2 = base * (1.0 + rng.uniform(-1e-9, 1e-9, 400))
            d2 = np.concatenate([d2, [base, np.nextafter(base, 0), np.nextafter(base, np.inf)]])
            p = theta2 * d2  # RN(theta2 * dist2)
            fast = s2 < p
            general = s2root < np.ldexp(p, two_d)
            assert np.array_equal(fast, general), (theta, two_d)
