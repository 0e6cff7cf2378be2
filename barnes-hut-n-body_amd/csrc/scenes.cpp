// Scene generators: restatement of BodyFactory.kt (BF) with a deterministic seed.
//
// The reference seeds makeGalaxyDisk / makeUniformRandom with Random(Random.nextLong())
// (BF:74,163), i.e. unseeded; we take the seed as an argument and reproduce Kotlin's
// kotlin.random.Random(seed: Long) = XorWowRandom(seed.toInt(), (seed shr 32).toInt())
// (kotlin-stdlib 2.2.20, not vendored in the reference).  libm's
// cos/sin/exp/log/hypot may differ from the JVM by an ulp, so parity never depends on a
// scene being "Kotlin-generated": tests compare engines on identical arrays.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

#include "bh_engine.h"

namespace {

// kotlin.random.XorWowRandom
struct XorWow {
    int32_t x, y, z, w, v, addend;
    XorWow(int32_t seed1, int32_t seed2) {
        x = seed1;
        y = seed2;
        z = 0;
        w = 0;
        v = ~seed1;
        addend = (int32_t)(((uint32_t)seed1 << 10) ^ ((uint32_t)seed2 >> 4));
        for (int i = 0; i < 64; ++i) nextInt();
    }
    static XorWow fromLong(int64_t seed) { return XorWow((int32_t)seed, (int32_t)(seed >> 32)); }
    int32_t nextInt() {
        uint32_t t = (uint32_t)x;
        t = t ^ (t >> 2);
        x = y;
        y = z;
        z = w;
        uint32_t v0 = (uint32_t)v;
        w = (int32_t)v0;
        t = (t ^ (t << 1)) ^ v0 ^ (v0 << 4);
        v = (int32_t)t;
        addend = (int32_t)((uint32_t)addend + 362437u);
        return (int32_t)(t + (uint32_t)addend);
    }
    int32_t nextBits(int bits) {  // takeUpperBits
        return (int32_t)(((uint32_t)nextInt() >> (32 - bits)) & (uint32_t)(-(int32_t)(bits != 0)));
    }
    double nextDouble() {  // doubleFromParts(nextBits(26), nextBits(27))
        int64_t hi = nextBits(26);
        int64_t lo = nextBits(27);
        return (double)((hi << 27) + lo) / (double)(1LL << 53);
    }
};

constexpr double kPI = 3.141592653589793;  // Math.PI

// BF:43-47 / BF:118-123: stable sort by radius, cumulative enclosed mass.
std::vector<double> enclosed_mass(const double* x, const double* y, const double* m, int n, double cx,
                                  double cy) {
    std::vector<double> r(n);
    for (int i = 0; i < n; ++i) r[i] = std::hypot(x[i] - cx, y[i] - cy);
    std::vector<int> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return r[a] < r[b]; });
    std::vector<double> menc(n);
    double acc = 0.0;
    for (int i : idx) {
        acc += m[i];
        menc[i] = acc;
    }
    return menc;
}

}  // namespace

extern "C" {

// BF:63-150 makeGalaxyDisk.  bar_taper_r / radial_scale <= 0 (or NaN) mean the Kotlin
// defaults (null -> rMax*0.6, rMax/3.0).
int bh_scene_galaxy_disk(int32_t nTotal, double epsM2, double phi0, double barTaperR,
                         double radialScale, double speedJitter, double radialJitter,
                         int32_t clockwise, int64_t seed, double vx, double vy, double x, double y,
                         double r, double minR, double centralMass, double totalSatelliteMass,
                         double G, double* ox, double* oy, double* ovx, double* ovy, double* om) {
    if (nTotal < 1 || !ox || !oy || !ovx || !ovy || !om) return BH_E_INVALID;
    XorWow rng = XorWow::fromLong(seed);
    const double cx = x, cy = y, rMax = r;
    const int sats = std::max(nTotal - 1, 0);
    int n = 0;
    ox[n] = cx; oy[n] = cy; ovx[n] = vx; ovy[n] = vy; om[n] = centralMass; ++n;  // BF:90
    const double mSat = sats > 0 ? totalSatelliteMass / sats : 0.0;
    const double Rd = (radialScale > 0.0) ? radialScale : (rMax / 3.0);
    const double taperR = (barTaperR > 0.0) ? barTaperR : (rMax * 0.6);
    for (int s = 0; s < sats; ++s) {  // BF:105-116
        double u = rng.nextDouble();   // sampleExpRadius BF:97-102
        double A = std::exp(-(rMax - minR) / Rd);
        double t = 1 - u * (1 - A);
        double R = minR - Rd * std::log(t);
        double theta = rng.nextDouble() * 2.0 * kPI;
        double taper = std::exp(-(R / taperR) * (R / taperR));
        double R2 = R * (1.0 + epsM2 * std::cos(2.0 * (theta - phi0)) * taper);
        ox[n] = cx + R2 * std::cos(theta);
        oy[n] = cy + R2 * std::sin(theta);
        ovx[n] = 0.0; ovy[n] = 0.0; om[n] = mSat;
        ++n;
    }
    std::vector<double> Menc = enclosed_mass(ox, oy, om, n, cx, cy);
    for (int i = 1; i < n; ++i) {  // BF:126-147
        double dx = ox[i] - cx, dy = oy[i] - cy;
        double R = std::max(1e-6, std::hypot(dx, dy));
        double vCirc = std::sqrt(G * Menc[i] / R);
        double v = vCirc * (1.0 + (rng.nextDouble() - 0.5) * 2.0 * speedJitter);
        double tx, ty;
        if (clockwise) { tx = dy / R; ty = -dx / R; } else { tx = -dy / R; ty = dx / R; }
        double vx0 = tx * v, vy0 = ty * v;
        if (radialJitter > 0.0) {
            double vr = (rng.nextDouble() - 0.5) * 2.0 * radialJitter * vCirc;
            vx0 += (dx / R) * vr;
            vy0 += (dy / R) * vr;
        }
        ovx[i] = vx0 + vx;
        ovy[i] = vy0 + vy;
    }
    return BH_OK;
}

// BF:11-61 makeKeplerDisk (reference default rng = Random(3), BF:16).
int bh_scene_kepler_disk(int32_t nTotal, int32_t clockwise, double radialJitter, double speedJitter,
                         int64_t seed, double vx, double vy, double x, double y, double r, double G,
                         double* ox, double* oy, double* ovx, double* ovy, double* om) {
    if (nTotal < 1 || !ox || !oy || !ovx || !ovy || !om) return BH_E_INVALID;
    // Random(seed: Int) = XorWowRandom(seed, seed shr 31)
    XorWow rng((int32_t)seed, (int32_t)seed >> 31);
    const double CENTRAL_MASS = 50000.0, MIN_R = 8.0, TOTAL_SATELLITE_MASS = 5000.0;  // CFG:32-38
    const double cx = x, cy = y, rMax = r;
    const int sats = std::max(nTotal - 1, 0);
    int n = 0;
    ox[n] = cx; oy[n] = cy; ovx[n] = vx; ovy[n] = vy; om[n] = CENTRAL_MASS; ++n;
    const double mSat = sats > 0 ? TOTAL_SATELLITE_MASS / sats : 0.0;
    for (int s = 0; s < sats; ++s) {  // BF:33-41
        double u = rng.nextDouble();
        double rr = std::sqrt(u * (rMax * rMax - MIN_R * MIN_R) + MIN_R * MIN_R);
        double rJ = rr * (1.0 + (rng.nextDouble() - 0.5) * 2.0 * radialJitter);
        double ang = rng.nextDouble() * 2.0 * kPI;
        ox[n] = cx + rJ * std::cos(ang);
        oy[n] = cy + rJ * std::sin(ang);
        ovx[n] = 0.0; ovy[n] = 0.0; om[n] = mSat;
        ++n;
    }
    std::vector<double> Menc = enclosed_mass(ox, oy, om, n, cx, cy);
    for (int i = 1; i < n; ++i) {  // BF:49-59
        double dx = ox[i] - cx, dy = oy[i] - cy;
        double rr = std::max(1e-6, std::hypot(dx, dy));
        double vCirc = std::sqrt(G * Menc[i] / rr);
        double v = vCirc * (1.0 + (rng.nextDouble() - 0.5) * 2.0 * speedJitter);
        double tx, ty;
        if (clockwise) { tx = dy / rr; ty = -dx / rr; } else { tx = -dy / rr; ty = dx / rr; }
        ovx[i] = tx * v + vx;
        ovy[i] = ty * v + vy;
    }
    return BH_OK;
}

// BF:160-177 makeUniformRandom over [0, W) x [0, H).
int bh_scene_uniform(int32_t n, double m, int64_t seed, int32_t width_px, int32_t height_px,
                     double* ox, double* oy, double* ovx, double* ovy, double* om) {
    if (n <= 0 || m <= 0.0) return BH_OK;  // BF:165 empty list
    if (!ox || !oy || !ovx || !ovy || !om) return BH_E_INVALID;
    XorWow rng = XorWow::fromLong(seed);
    const double w = (double)width_px, h = (double)height_px;
    for (int i = 0; i < n; ++i) {
        double px = rng.nextDouble() * w;
        double py = rng.nextDouble() * h;
        ox[i] = px; oy[i] = py; ovx[i] = 0.0; ovy[i] = 0.0; om[i] = m;
    }
    return BH_OK;
}

}  // extern "C"
