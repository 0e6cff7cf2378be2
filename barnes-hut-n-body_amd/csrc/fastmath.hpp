// Exact reduced-range sequences for the force kernels (traverse.hip, direct.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace bh {

// ---- exact fast paths for RN(sqrt(x)) and RN(1/x) ------------------------------------
// These are the instruction sequences the compiler emits for IEEE sqrt(double) and
// 1.0 / double on gfx950, with the operand-range scaling (v_cmp + v_ldexp / v_div_scale /
// v_div_fmas scaling) and the special-value fix-ups (v_cmp_class / v_div_fixup) removed.
// For a finite normal operand in [2^-600, 2^600] those removed steps are identities (no
// scaling is triggered, no special value occurs), so the results are bit-identical to the
// full sequences; a wave takes this path only when lane_fast_ok() holds for all its lanes.
__device__ __forceinline__ double sqrt_rn_inrange(double x) {
    double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return g;
}

// Same sqrt sequence, also returning its refined half-reciprocal h ~= 0.5 / sqrt(x)
// (relative error ~2^-45), the seed of the reciprocal below.
__device__ __forceinline__ double sqrt_rn_inrange_h(double x, double &hout) {
    double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    hout = h;
    return g;
}

// RN(1/b) from a seed y0 with relative error <= 2^-44: one Newton step brings y within
// 0.5 ulp + 2^-88 of 1/b -- the accuracy the compiler's sequence reaches after v_rcp_f64 and
// two steps -- and the final residual correction is that sequence's last two operations.
// The seeds: 2h for 1/sqrt(d2) (from the sqrt above), invR*invR for 1/d2 (rel. err 2^-51).
// bh_selftest_fast_math checks these against the IEEE operations on random operands.
__device__ __forceinline__ double rcp_rn_seeded(double b, double y0) {
    const double e = __builtin_fma(-b, y0, 1.0);
    const double y = __builtin_fma(y0, e, y0);
    const double r = __builtin_fma(-b, y, 1.0);
    return __builtin_fma(r, y, y);
}

__device__ __forceinline__ double rcp_rn_inrange(double b) {
    double y = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    double r = __builtin_fma(-b, y, 1.0);  // q = 1.0 * y = y exactly
    return __builtin_fma(r, y, y);
}

// Wave-uniform precondition for the exact fast paths: every tree node's centre of mass lies
// within the root cell or 2e-3 of it (a convex combination of inserted bodies; a jittered
// leaf body moved by at most 2 x 1e-3), so |comX|, |comY| < 2^31 always.  If the lane's own
// body is finite with |x|, |y| < 2^250 and soft2 is in [2^-600, 2^500], every dist2 of the
// traversal is in [soft2, 2^503] and both sqrt and the reciprocals stay in the range where
// sqrt_rn_inrange / rcp_rn_inrange equal the full IEEE sequences.
// Self term.  In the fast path a body's own leaf is not excluded: its dx = dy = +0.0 exactly
// (the leaf holds the body's own position), so the term is f * (+-0) * invR = +-0 with f and
// invR finite, and adding +-0 leaves the running sum unchanged (the sum starts at +0.0 and can
// never become -0.0) -- the reference's identity skip (BHA:219) without a compare or select.
// lane_self_ok() bounds |G m_b * m_b / soft2| < 2^1000 so that f is finite for that term.
__device__ __forceinline__ bool lane_self_ok(double Gm, double bm) {
    return __builtin_fabs(Gm * bm) < 0x1p400;
}

// The fast criterion forms s2 = s2_0 * 2^-2d by an exponent-field subtraction (traverse.hip):
// exact while the result stays normal, i.e. for every 2d <= 255 (NODE_DEPTH2_MASK) when
// s2_0 >= 2^-760; finite s2_0 only.
__device__ __forceinline__ bool fast_s2_ok(double s2root) {
    return s2root >= 0x1p-760 && s2root <= 0x1p1000;
}

__device__ __forceinline__ bool lane_fast_ok(double bx, double by, double soft2) {
    return __builtin_fabs(bx) < 0x1p250 && __builtin_fabs(by) < 0x1p250 && soft2 >= 0x1p-600 &&
           soft2 <= 0x1p500;
}

}  // namespace bh
