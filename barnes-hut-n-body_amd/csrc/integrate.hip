// Kick-drift-kick integration (BHA:410-432) and the device side of the merge rule
// (BHA:463-532).  All elementwise, coalesced, in caller (list) order.
#include <hipcub/hipcub.hpp>

#include "bh_device.hpp"

namespace bh {
namespace {

constexpr int TB = 256;
inline unsigned grid_for(int64_t n) { return (unsigned)((n + TB - 1) / TB); }

// BHA:412-422 fused: v += a * dtHalf; x += v * DT.  The reference runs the kick loop over
// all bodies and then the drift loop; per body the operations are identical.
__global__ __launch_bounds__(TB) void k_kick_drift(int64_t n, const double *__restrict__ ax,
                                                   const double *__restrict__ ay,
                                                   double *__restrict__ x, double *__restrict__ y,
                                                   double *__restrict__ vx,
                                                   double *__restrict__ vy, double dtHalf,
                                                   double dt) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    double vxi = vx[i] + ax[i] * dtHalf;
    double vyi = vy[i] + ay[i] * dtHalf;
    vx[i] = vxi;
    vy[i] = vyi;
    x[i] = x[i] + vxi * dt;
    y[i] = y[i] + vyi * dt;
}

// BHA:429-432
__global__ __launch_bounds__(TB) void k_kick(int64_t n, const double *__restrict__ ax,
                                             const double *__restrict__ ay,
                                             double *__restrict__ vx, double *__restrict__ vy,
                                             double dtHalf) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    vx[i] = vx[i] + ax[i] * dtHalf;
    vy[i] = vy[i] + ay[i] * dtHalf;
}

struct HeavyPred {
    const double *m;
    double thr;
    __host__ __device__ bool operator()(const uint32_t &i) const { return m[i] > thr; }
};

// BHA:493-501: for every heavy body k (list order) and every body j != heavy[k]:
// dx*dx + dy*dy < minD2 (dx = bj.x - bi.x).  Candidates are appended in arbitrary order;
// the host sorts and replays them in the reference's sequential order.
__global__ __launch_bounds__(TB) void k_merge_candidates(int64_t n, const double *__restrict__ x,
                                                         const double *__restrict__ y,
                                                         const double *__restrict__ m,
                                                         const uint32_t *__restrict__ heavy,
                                                         uint32_t H, double minD2,
                                                         MergePair *__restrict__ pairs,
                                                         uint32_t cap, uint32_t *d_count) {
    int64_t j = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (j >= n) return;
    double xj = x[j], yj = y[j];
    for (uint32_t k = 0; k < H; ++k) {
        uint32_t hi = heavy[k];
        if ((int64_t)hi == j) continue;
        double dx = xj - x[hi];
        double dy = yj - y[hi];
        if (dx * dx + dy * dy < minD2) {
            uint32_t slot = atomicAdd(d_count, 1u);
            if (slot < cap) pairs[slot] = MergePair{k, (uint32_t)j, m[j]};
        }
    }
}

__global__ __launch_bounds__(TB) void k_compact_scatter(int64_t n, const uint32_t *__restrict__ keep,
                                                        const uint32_t *__restrict__ pos,
                                                        const double *s0, const double *s1,
                                                        const double *s2, const double *s3,
                                                        const double *s4, double *d0, double *d1,
                                                        double *d2, double *d3, double *d4) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n || !keep[i]) return;
    uint32_t o = pos[i];
    d0[o] = s0[i];
    d1[o] = s1[i];
    d2[o] = s2[i];
    d3[o] = s3[i];
    d4[o] = s4[i];
}

__global__ __launch_bounds__(TB) void k_apply_merge(uint32_t n_dead, const uint32_t *__restrict__ dead,
                                                    uint32_t n_upd, const uint32_t *__restrict__ upd_idx,
                                                    const double *__restrict__ upd_mass,
                                                    uint32_t *__restrict__ keep, double *__restrict__ m) {
    uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i < n_dead) keep[dead[i]] = 0u;
    if (i < n_upd) m[upd_idx[i]] = upd_mass[i];
}

__global__ __launch_bounds__(TB) void k_gather(const uint32_t *__restrict__ idx, uint32_t cnt,
                                               const double *__restrict__ src, double *__restrict__ dst) {
    uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i < cnt) dst[i] = src[idx[i]];
}

}  // namespace

void apply_merge(uint32_t n_dead, const uint32_t *dead, uint32_t n_upd, const uint32_t *upd_idx,
                 const double *upd_mass, uint32_t *keep, double *m, hipStream_t s) {
    uint32_t c = n_dead > n_upd ? n_dead : n_upd;
    if (c) k_apply_merge<<<(c + TB - 1) / TB, TB, 0, s>>>(n_dead, dead, n_upd, upd_idx, upd_mass, keep, m);
}

void gather_doubles(const uint32_t *idx, uint32_t cnt, const double *src, double *dst, hipStream_t s) {
    if (cnt) k_gather<<<(cnt + TB - 1) / TB, TB, 0, s>>>(idx, cnt, src, dst);
}

void kick_drift(int64_t n, const double *ax, const double *ay, double *x, double *y, double *vx,
                double *vy, double dtHalf, double dt, hipStream_t s) {
    if (n > 0) k_kick_drift<<<grid_for(n), TB, 0, s>>>(n, ax, ay, x, y, vx, vy, dtHalf, dt);
}

void kick(int64_t n, const double *ax, const double *ay, double *vx, double *vy, double dtHalf,
          hipStream_t s) {
    if (n > 0) k_kick<<<grid_for(n), TB, 0, s>>>(n, ax, ay, vx, vy, dtHalf);
}

size_t merge_cub_bytes(int64_t n) {
    size_t a = 0, b = 0;
    hipcub::CountingInputIterator<uint32_t> it(0);
    (void)hipcub::DeviceSelect::If(nullptr, a, it, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n,
                             HeavyPred{nullptr, 0.0});
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n);
    return a > b ? a : b;
}

hipError_t heavy_list(const double *m, int64_t n, double thr, uint32_t *heavy, uint32_t *d_count,
                      void *tmp, size_t tmp_bytes, hipStream_t s) {
    hipcub::CountingInputIterator<uint32_t> it(0);
    return hipcub::DeviceSelect::If(tmp, tmp_bytes, it, heavy, d_count, (int)n, HeavyPred{m, thr}, s);
}

void merge_candidates(int64_t n, const double *x, const double *y, const double *m,
                      const uint32_t *heavy, uint32_t H, double minD2, MergePair *pairs,
                      uint32_t cap, uint32_t *d_count, hipStream_t s) {
    (void)hipMemsetAsync(d_count, 0, sizeof(uint32_t), s);
    if (n > 0 && H > 0)
        k_merge_candidates<<<grid_for(n), TB, 0, s>>>(n, x, y, m, heavy, H, minD2, pairs, cap,
                                                      d_count);
}

hipError_t compact_bodies(int64_t n, const uint32_t *keep, const double *const src[5],
                          double *const dst[5], uint32_t *pos, uint32_t *d_count, void *tmp,
                          size_t tmp_bytes, hipStream_t s) {
    (void)d_count;
    hipError_t st = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, keep, pos, (int)n, s);
    if (st != hipSuccess) return st;
    k_compact_scatter<<<grid_for(n), TB, 0, s>>>(n, keep, pos, src[0], src[1], src[2], src[3],
                                                 src[4], dst[0], dst[1], dst[2], dst[3], dst[4]);
    return hipGetLastError();
}

}  // namespace bh
