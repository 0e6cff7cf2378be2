// θ = 0 force evaluation as a direct all-pairs sum.
//
// At θ = 0 the reference's criterion `s2 < 0 * dist2` (BHA:226-228) never accepts, so
// accumulateForce (BHA:215-239) recurses to every leaf: each body's force is the point force
// of every non-empty (mass != 0, BHA:216) leaf except its own (BHA:219), summed in the tree's
// depth-first pre-order.  Here that leaf sequence is extracted once per build (a stable
// compaction of the pre-order node array) and the O(N^2) sum runs as an LDS-tiled kernel:
// a workgroup stages 1024 leaves (x, y, m, slot) in LDS with coalesced loads, every lane (one
// body) reads them as broadcasts in sequence order — the reference's order, so the result is
// bit-identical to the tree walk — with no criterion, cursor or ballot in the loop.  Bound by
// fp64 VALU issue (one v_rsq_f64 and ~35 fp64 ops per interaction).
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "bh_device.hpp"
#include "fastmath.hpp"

namespace bh {
namespace {

constexpr int TB = 256;
typedef double double4_t __attribute__((ext_vector_type(4)));
#ifndef BH_DIRECT_TILE
#define BH_DIRECT_TILE 1024
#endif
constexpr int TILE = BH_DIRECT_TILE;

// The subtree [i + 1, next) of every mass-0 internal node (NODE_SKIP with descendants): the
// reference returns at that node (BHA:216) and never reaches its leaves -- which can hold
// negative masses -- so they must not enter the leaf sequence.  +1 / -1 at the range ends, then
// a prefix sum counts the covering mass-0 ancestors of every node.
__global__ __launch_bounds__(TB) void k_leaf_cover(const Node *__restrict__ nodes,
                                                   const uint32_t *__restrict__ d_T,
                                                   int32_t *__restrict__ cover, int64_t cap) {
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= cap || i >= (int64_t)*d_T) return;
    const Node nd = nodes[i];
    if ((nd.meta & NODE_SKIP) && (int64_t)nd.next > i + 1) {
        atomicAdd(cover + i + 1, 1);
        atomicAdd(cover + min((int64_t)nd.next, cap), -1);
    }
}

__global__ __launch_bounds__(TB) void k_leaf_flags(const Node *__restrict__ nodes,
                                                   const uint32_t *__restrict__ d_T,
                                                   const int32_t *__restrict__ covered,
                                                   uint8_t *__restrict__ flags, int64_t cap) {
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= cap) return;
    const uint32_t T = *d_T;
    uint8_t f = 0;
    if (i < (int64_t)T) {
        const uint32_t meta = nodes[i].meta;
        // BHA:216: mass == 0 never visited, nor is anything below a massless node
        f = (meta & NODE_LEAF) && !(meta & NODE_SKIP) && covered[i] == 0;
    }
    flags[i] = f;
}

__global__ __launch_bounds__(TB) void k_leaf_gather(const Node *__restrict__ nodes,
                                                    const uint32_t *__restrict__ sel,
                                                    const uint32_t *__restrict__ d_count,
                                                    LeafList L) {
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i >= *d_count) return;
    const Node nd = nodes[sel[i]];
    double4_t r;  // leaf: the body's own x, y, m (BHA:176-178)
    r.x = nd.comX;
    r.y = nd.comY;
    r.z = nd.mass;
    r.w = __longlong_as_double((long long)(nd.meta & NODE_BODY_MASK));
    reinterpret_cast<double4_t *>(L.rec)[i] = r;
}

typedef double double2_t __attribute__((ext_vector_type(2)));

template <bool FAST>
__device__ __forceinline__ void pair_force(double px, double py, double pm, double bx, double by,
                                           double Gm, double soft2, double &fx, double &fy) {
    const double dx = px - bx;  // BHA:251-258, expression order as written
    const double dy = py - by;
    const double r2 = dx * dx + dy * dy + soft2;
    double invR, invR2;
    if (FAST) {
        double h;
        const double r = sqrt_rn_inrange_h(r2, h);
        invR = rcp_rn_seeded(r, h + h);
        invR2 = rcp_rn_seeded(r2, invR * invR);
    } else {
        invR = 1.0 / sqrt(r2);
        invR2 = 1.0 / r2;
    }
    const double f = Gm * pm * invR2;
    fx += f * dx * invR;
    fy += f * dy * invR;
}

// One staged leaf: (x, y, m, slot bits).  NB bodies per lane (BH_DIRECT_NB): each broadcast
// record serves NB independent interaction chains.
#ifndef BH_DIRECT_NB
#define BH_DIRECT_NB 2  // C5: 77.1 -> 75.6 ms per evaluation (profiles/r03_let_fold_c5_nb_ab.txt)
#endif
constexpr int NB = BH_DIRECT_NB;

template <bool FAST>
__device__ __forceinline__ void leaf_terms(const double4_t &r, const double (&bx)[NB],
                                           const double (&by)[NB], const double (&Gm)[NB],
                                           double soft2, const uint32_t (&self)[NB],
                                           double (&fx)[NB], double (&fy)[NB]) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const bool other = (uint32_t)__double_as_longlong(r.w) != self[b];  // BHA:219
        if (FAST) {
            // no self-skip at all: the own leaf has dx = dy = +0.0, so its term is an exact
            // +-0.0 and fx, fy (never -0.0) are unchanged -- valid because the fast path
            // guarantees a finite f for it (fastmath.hpp, lane_self_ok) and r2 >= soft2 > 0
            (void)other;
            pair_force<true>(r.x, r.y, r.z, bx[b], by[b], Gm[b], soft2, fx[b], fy[b]);
        } else if (other) {
            pair_force<false>(r.x, r.y, r.z, bx[b], by[b], Gm[b], soft2, fx[b], fy[b]);
        }
    }
}

template <bool FAST>
__device__ __forceinline__ void sum_tile(const double4_t *s_rec, int cnt, const double (&bx)[NB],
                                         const double (&by)[NB], const double (&Gm)[NB],
                                         double soft2, const uint32_t (&self)[NB],
                                         double (&fx)[NB], double (&fy)[NB]) {
#ifndef BH_DIRECT_U
#define BH_DIRECT_U 4
#endif
    constexpr int U = BH_DIRECT_U;
    int j = 0;
    for (; j + U <= cnt; j += U) {
        double4_t r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = s_rec[j + u];  // broadcast reads, issued together
#pragma unroll
        for (int u = 0; u < U; ++u) leaf_terms<FAST>(r[u], bx, by, Gm, soft2, self, fx, fy);
    }
    for (; j < cnt; ++j) leaf_terms<FAST>(s_rec[j], bx, by, Gm, soft2, self, fx, fy);
}

__global__ __launch_bounds__(TB) void k_direct(LeafList L, const uint32_t *__restrict__ d_count,
                                               const double *__restrict__ x,
                                               const double *__restrict__ y,
                                               const double *__restrict__ m, int64_t lo,
                                               int64_t hi, double G, double soft2,
                                               double *__restrict__ a2) {
    __shared__ double4_t s_rec[TILE];
    int64_t p[NB];
    bool valid[NB];
    double bx[NB], by[NB], bm[NB], Gm[NB], fx[NB], fy[NB];
    uint32_t self[NB];
    bool slow = false;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        p[b] = lo + ((int64_t)blockIdx.x * NB + b) * TB + threadIdx.x;
        valid[b] = p[b] < hi;
        bx[b] = valid[b] ? x[p[b]] : 0.0;
        by[b] = valid[b] ? y[p[b]] : 0.0;
        bm[b] = valid[b] ? m[p[b]] : 1.0;
        Gm[b] = G * bm[b];  // (Config.G * b.m) first (BHA:256)
        self[b] = valid[b] ? (uint32_t)p[b] : 0xFFFFFFFFu;
        slow |= valid[b] && !(lane_fast_ok(bx[b], by[b], soft2) && lane_self_ok(Gm[b], bm[b]));
        fx[b] = 0.0;
        fy[b] = 0.0;
    }
    const bool fast = __ballot(slow) == 0ull;
    const uint32_t nl = *d_count;
    for (uint32_t t0 = 0; t0 < nl; t0 += TILE) {
        const int cnt = (int)min((uint32_t)TILE, nl - t0);
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += TB)
            s_rec[i] = reinterpret_cast<const double4_t *>(L.rec)[t0 + i];
        __syncthreads();
        if (fast)
            sum_tile<true>(s_rec, cnt, bx, by, Gm, soft2, self, fx, fy);
        else
            sum_tile<false>(s_rec, cnt, bx, by, Gm, soft2, self, fx, fy);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (!valid[b]) continue;
        double2_t acc;
        acc.x = fx[b] / bm[b];  // BHA:390-391
        acc.y = fy[b] / bm[b];
        *reinterpret_cast<double2_t *>(a2 + 2 * p[b]) = acc;
    }
}

}  // namespace

size_t leaf_select_bytes(int64_t node_cap) {
    size_t b = 0, c = 0;
    (void)rocprim::select(nullptr, b, rocprim::counting_iterator<uint32_t>(0),
                          (const uint8_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                          (size_t)node_cap);
    (void)rocprim::inclusive_scan(nullptr, c, (const int32_t *)nullptr, (int32_t *)nullptr,
                                  (size_t)node_cap, rocprim::plus<int32_t>());
    return b > c ? b : c;
}

hipError_t leaf_list_build(const Node *nodes, const uint32_t *d_T, int64_t node_cap,
                           uint8_t *flags, uint32_t *sel, uint32_t *d_count, const LeafList &L,
                           int64_t n, int32_t *cover, void *tmp, size_t tmp_bytes, hipStream_t s) {
    if (node_cap <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((node_cap + TB - 1) / TB);
    int32_t *covered = cover + node_cap + 1;
    hipError_t st = hipMemsetAsync(cover, 0, sizeof(int32_t) * (size_t)(node_cap + 1), s);
    if (st != hipSuccess) return st;
    k_leaf_cover<<<grid, TB, 0, s>>>(nodes, d_T, cover, node_cap);
    st = rocprim::inclusive_scan(tmp, tmp_bytes, cover, covered, (size_t)node_cap,
                                 rocprim::plus<int32_t>(), s);
    if (st != hipSuccess) return st;
    k_leaf_flags<<<grid, TB, 0, s>>>(nodes, d_T, covered, flags, node_cap);
    st = rocprim::select(tmp, tmp_bytes, rocprim::counting_iterator<uint32_t>(0),
                         flags, sel, d_count, (size_t)node_cap, s);
    if (st != hipSuccess) return st;
    if (n > 0) k_leaf_gather<<<(unsigned)((n + TB - 1) / TB), TB, 0, s>>>(nodes, sel, d_count, L);
    return hipGetLastError();
}

void direct_forces(const LeafList &L, const uint32_t *d_count, const double *x, const double *y,
                   const double *m, int64_t lo, int64_t hi, double G, double soft2, double *a2,
                   hipStream_t s) {
    if (hi <= lo) return;
    k_direct<<<(unsigned)((hi - lo + TB * NB - 1) / (TB * NB)), TB, 0, s>>>(L, d_count, x, y, m, lo,
                                                                          hi, G, soft2, a2);
}

}  // namespace bh
