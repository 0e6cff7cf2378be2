// Engine host code and the C-ABI (include/bh_engine.h).
//
// Replaces PhysicsEngine (BHA:287-532).  The engine owns SoA fp64 body arrays in HBM in the
// caller's list order, a Morton-ordered workspace for the tree, and one HIP stream.  A step
// is the reference's step() (BHA:405-439) as a fixed sequence of kernels on that stream;
// the only host round trips are the merge rule's (BHA:463-532) candidate count when heavy
// bodies exist, and the copy-in / copy-out calls.
//
// Multi-GPU (bh_create_dist): every rank holds the full replicated state and builds the
// same tree (deterministically, so the jitter mutates every replica identically); force
// evaluation is sharded by contiguous Morton ranges and the accelerations are all-gathered
// with RCCL over xGMI, after which every rank integrates the full set.  The merge rule is
// replicated (identical inputs, identical outcome) and needs no exchange.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <iterator>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "bh_device.hpp"
#include "bh_engine.h"

using namespace bh;

namespace {

constexpr int kPhases = 5;  // build, traverse, integrate, merge, allgather

struct DevArray {
    void *p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct bh_engine {
    bh_params p{};
    Geometry geo{};
    int device = 0;
    hipStream_t stream = nullptr;
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;

    int64_t n = 0;    // live bodies
    int64_t cap = 0;  // allocated bodies
    int J_alloc = -1; // J the node array was sized for

    double *x = nullptr, *y = nullptr, *vx = nullptr, *vy = nullptr, *m = nullptr;
    double *alt[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // compaction targets
    double *ax = nullptr, *ay = nullptr;
    double *a_sorted = nullptr;

    uint64_t *keys = nullptr, *keys_s = nullptr;
    uint32_t *idx = nullptr, *perm = nullptr;
    double *sx = nullptr, *sy = nullptr, *sm = nullptr;
    int8_t *cpl = nullptr;
    uint32_t *cnt = nullptr, *base = nullptr;
    Node *nodes = nullptr;
    size_t node_cap = 0;
    uint32_t *span_cnt = nullptr, *span_list = nullptr;
    uint4 *span_children = nullptr;
    uint32_t *scalars = nullptr;  // [0] unused, [1] error flags, [2] heavy count, [3] pair count
    uint32_t *visits32 = nullptr;
    uint32_t *wave_iters = nullptr;  // per-wave union of visited nodes (diagnostics)
    int64_t stat_lane_visits = 0, stat_wave_iters = 0, stat_waves = 0;

    // merge
    uint32_t *heavy = nullptr;
    uint32_t *keep = nullptr, *pos = nullptr;
    MergePair *pairs = nullptr;
    uint32_t pair_cap = 0;
    uint32_t *mdead = nullptr, *mupd = nullptr;
    double *mupd_mass = nullptr, *hmass = nullptr;
    uint32_t mcap = 0;
    int64_t heavy_count = -1;  // -1: unknown (recompute)
    std::vector<std::vector<uint32_t>> step_dead;  // per-step removals of the last bh_step
    std::vector<uint32_t> h_heavy;  // host copy of the ordered heavy list
    std::vector<double> h_hmass;    // and of the heavy bodies' masses
    void *pin = nullptr;            // pinned staging for the merge mailbox / uploads
    size_t pin_bytes = 0;

    void *cub_tmp = nullptr;
    size_t cub_bytes = 0;

    bool tree_valid = false;  // lastTree (BHA:304)

    // profiling
    bool profiling = false;
    std::vector<hipEvent_t> ev;  // pairs (start, stop) per phase interval
    std::vector<int> ev_phase;
    size_t ev_used = 0;
    double phase_ms[kPhases] = {0, 0, 0, 0, 0};
    double trav_ms_sum = 0.0;
    int64_t trav_launches = 0;
    bool timings_pending = false;

    std::string err;
};

namespace {

#define HIPCHK(e, expr)                                                                  \
    do {                                                                                 \
        hipError_t _st = (expr);                                                         \
        if (_st != hipSuccess) {                                                         \
            (e)->err = std::string(#expr) + ": " + hipGetErrorString(_st);              \
            return BH_E_DEVICE;                                                          \
        }                                                                                \
    } while (0)

#define NCCLCHK(e, expr)                                                                 \
    do {                                                                                 \
        ncclResult_t _st = (expr);                                                       \
        if (_st != ncclSuccess) {                                                        \
            (e)->err = std::string(#expr) + ": " + ncclGetErrorString(_st);              \
            return BH_E_COMM;                                                            \
        }                                                                                \
    } while (0)

#define TRY(expr)                      \
    do {                               \
        int _rc = (expr);              \
        if (_rc != BH_OK) return _rc;  \
    } while (0)

// Root cell (BHA:360-361) and the exact per-depth half-sizes (BHA:74).
int make_geometry(const bh_params &p, Geometry &g, std::string &err) {
    if (p.width_px <= 0 || p.height_px <= 0) {
        err = "width_px and height_px must be positive";
        return BH_E_INVALID;
    }
    std::memset(&g, 0, sizeof(g));
    const int W = p.width_px, H = p.height_px;
    g.root_cx = (double)W / 2.0;
    g.root_cy = (double)H / 2.0;
    g.root_h = (double)std::max(W, H) / 2.0 + 2.0;
    g.h[0] = g.root_h;
    for (int d = 1; d < MAX_DEPTH_TAB; ++d) g.h[d] = g.h[d - 1] / 2.0;
    int J = -1;
    for (int d = 0; d < MAX_DEPTH_TAB; ++d)
        if (g.h[d] < 1e-3) {
            J = d;
            break;
        }
    if (J < 1 || J > 30 || J + 3 > MAX_DEPTH_TAB) {
        err = "root cell too large for 64-bit Morton keys (jitter depth > 30)";
        return BH_E_INVALID;
    }
    g.J = J;
    for (int d = 0; d < MAX_DEPTH_TAB; ++d) {
        double s = g.h[d] * 2.0;  // BHA:226
        g.s2[d] = s * s;
    }
    return BH_OK;
}

template <typename T>
int dev_alloc(bh_engine *e, T *&ptr, size_t count) {
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
    }
    if (count == 0) count = 1;
    HIPCHK(e, hipMalloc((void **)&ptr, count * sizeof(T)));
    return BH_OK;
}

size_t node_capacity(int64_t n, int J) {
    // T = sum_a (1 + max(0, c(a) - c(a-1))) <= n + (J+1) * (n/2 + 2)
    return (size_t)n + (size_t)(J + 1) * ((size_t)n / 2 + 2) + 16;
}

int ensure_capacity(bh_engine *e, int64_t n) {
    const int J = e->geo.J;
    if (n <= e->cap && J == e->J_alloc) return BH_OK;
    int64_t cap = std::max<int64_t>(n, std::max<int64_t>(e->cap, 1));
    if (n > e->cap) {
        // keep the live state across a growth
        std::vector<double> keep5[5];
        if (e->n > 0 && e->x) {
            double *src[5] = {e->x, e->y, e->vx, e->vy, e->m};
            for (int k = 0; k < 5; ++k) {
                keep5[k].resize((size_t)e->n);
                HIPCHK(e, hipMemcpy(keep5[k].data(), src[k], sizeof(double) * e->n,
                                    hipMemcpyDeviceToHost));
            }
        }
        TRY(dev_alloc(e, e->x, cap));
        TRY(dev_alloc(e, e->y, cap));
        TRY(dev_alloc(e, e->vx, cap));
        TRY(dev_alloc(e, e->vy, cap));
        TRY(dev_alloc(e, e->m, cap));
        for (int k = 0; k < 5; ++k) TRY(dev_alloc(e, e->alt[k], cap));
        TRY(dev_alloc(e, e->ax, cap));
        TRY(dev_alloc(e, e->ay, cap));
        int64_t chunk = (cap + e->world - 1) / e->world;
        TRY(dev_alloc(e, e->a_sorted, 2 * chunk * e->world));
        TRY(dev_alloc(e, e->keys, cap));
        TRY(dev_alloc(e, e->keys_s, cap));
        TRY(dev_alloc(e, e->idx, cap));
        TRY(dev_alloc(e, e->perm, cap));
        TRY(dev_alloc(e, e->sx, cap));
        TRY(dev_alloc(e, e->sy, cap));
        TRY(dev_alloc(e, e->sm, cap));
        TRY(dev_alloc(e, e->cpl, cap + 32));  // slack for word-wise scans
        TRY(dev_alloc(e, e->cnt, cap + 1));
        TRY(dev_alloc(e, e->base, cap + 1));
        TRY(dev_alloc(e, e->visits32, cap));
        TRY(dev_alloc(e, e->wave_iters, cap / 64 + 2));
        TRY(dev_alloc(e, e->heavy, cap));
        TRY(dev_alloc(e, e->keep, cap));
        TRY(dev_alloc(e, e->pos, cap));
        if (e->n > 0 && !keep5[0].empty()) {
            double *dst[5] = {e->x, e->y, e->vx, e->vy, e->m};
            for (int k = 0; k < 5; ++k)
                HIPCHK(e, hipMemcpy(dst[k], keep5[k].data(), sizeof(double) * e->n,
                                    hipMemcpyHostToDevice));
        }
        e->cap = cap;
    }
    size_t ncap = node_capacity(e->cap, J);
    if (ncap > e->node_cap || J != e->J_alloc) {
        TRY(dev_alloc(e, e->nodes, ncap));
        TRY(dev_alloc(e, e->span_cnt, (size_t)J + 2));
        TRY(dev_alloc(e, e->span_list, (size_t)(J + 2) * span_stride_for(e->cap)));
        TRY(dev_alloc(e, e->span_children, (size_t)(J + 2) * span_stride_for(e->cap)));
        e->node_cap = ncap;
        e->J_alloc = J;
    }
    size_t cb = std::max(tree_cub_bytes(e->cap, J), merge_cub_bytes(e->cap));
    if (cb > e->cub_bytes) {
        if (e->cub_tmp) (void)hipFree(e->cub_tmp);
        e->cub_tmp = nullptr;
        HIPCHK(e, hipMalloc(&e->cub_tmp, cb));
        e->cub_bytes = cb;
    }
    return BH_OK;
}

TreeBuffers tree_buffers(bh_engine *e) {
    TreeBuffers b;
    b.x = e->x;
    b.y = e->y;
    b.m = e->m;
    b.keys = e->keys;
    b.keys_s = e->keys_s;
    b.idx = e->idx;
    b.perm = e->perm;
    b.sx = e->sx;
    b.sy = e->sy;
    b.sm = e->sm;
    b.cpl = e->cpl;
    b.cnt = e->cnt;
    b.base = e->base;
    b.nodes = e->nodes;
    b.scalars = e->scalars;
    b.span_cnt = e->span_cnt;
    b.span_list = e->span_list;
    b.span_stride = span_stride_for(e->cap);
    b.span_children = e->span_children;
    b.cub_tmp = e->cub_tmp;
    b.cub_bytes = e->cub_bytes;
    return b;
}

// ---- profiling events ----------------------------------------------------------------
int mark(bh_engine *e, int phase) {  // close the interval of `phase` that began at the last mark
    if (!e->profiling) return BH_OK;
    if (e->ev_used + 1 > e->ev.size()) {
        hipEvent_t ev;
        HIPCHK(e, hipEventCreate(&ev));
        e->ev.push_back(ev);
        e->ev_phase.push_back(-1);
    }
    HIPCHK(e, hipEventRecord(e->ev[e->ev_used], e->stream));
    e->ev_phase[e->ev_used] = phase;  // phase of the interval ending here (-1: start marker)
    ++e->ev_used;
    e->timings_pending = true;
    return BH_OK;
}

int collect_timings(bh_engine *e) {
    if (!e->timings_pending) return BH_OK;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (int k = 0; k < kPhases; ++k) e->phase_ms[k] = 0.0;
    e->trav_ms_sum = 0.0;
    e->trav_launches = 0;
    for (size_t i = 1; i < e->ev_used; ++i) {
        int ph = e->ev_phase[i];
        if (ph < 0) continue;
        float ms = 0.f;
        HIPCHK(e, hipEventElapsedTime(&ms, e->ev[i - 1], e->ev[i]));
        e->phase_ms[ph] += ms;
        if (ph == 1) {
            e->trav_ms_sum += ms;
            e->trav_launches += 1;
        }
    }
    e->timings_pending = false;
    return BH_OK;
}

// ---- one force evaluation: buildTree() + computeAccelerations() (BHA:359-395) -------------
int evaluate(bh_engine *e, uint32_t *visits) {
    const int64_t n = e->n;
    TRY(mark(e, -1));
    HIPCHK(e, tree_build(tree_buffers(e), n, e->geo, e->stream));
    TRY(mark(e, 0));
    ForceParams fp{e->p.G, e->p.soft2, e->p.theta * e->p.theta};  // BHA:378
    const uint32_t *d_T = e->base + n;
    if (e->world == 1 || visits) {
        traverse(e->nodes, d_T, e->sx, e->sy, e->sm, e->perm, 0, n, e->geo, fp, e->ax, e->ay,
                 nullptr, visits, e->wave_iters, e->stream);
        HIPCHK(e, hipGetLastError());
        TRY(mark(e, 1));
    } else {
        int64_t chunk = (n + e->world - 1) / e->world;
        int64_t lo = 0, hi = 0;
        bh_shard_range(n, e->rank, e->world, &lo, &hi);
        traverse(e->nodes, d_T, e->sx, e->sy, e->sm, e->perm, lo, hi, e->geo, fp, e->ax, e->ay,
                 e->a_sorted, nullptr, nullptr, e->stream);
        HIPCHK(e, hipGetLastError());
        TRY(mark(e, 1));
        NCCLCHK(e, ncclAllGather(e->a_sorted + 2 * e->rank * chunk, e->a_sorted, (size_t)(2 * chunk),
                                 ncclDouble, e->comm, e->stream));
        scatter_sorted_acc(e->a_sorted, e->perm, n, e->ax, e->ay, e->stream);
        HIPCHK(e, hipGetLastError());
        TRY(mark(e, 4));
    }
    return BH_OK;
}

int check_tree_flags(bh_engine *e) {
    uint32_t flags = 0;
    HIPCHK(e, hipMemcpyAsync(&flags, e->scalars + 1, sizeof(uint32_t), hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (flags) {
        e->err = "jitter replay reached an unsupported geometry (body stayed inside a depth J+1 cell)";
        return BH_E_STATE;
    }
    return BH_OK;
}

// ---- merge rule (BHA:463-532) ---------------------------------------------------------
// Heavy bodies (m > mergeMaxMass) only ever gain mass and are few, so the host keeps their
// ordered index list and masses; the device finds candidate pairs (d^2 < minD^2) with one
// kernel and posts them to a small mailbox that is copied back with ONE async copy into
// pinned memory — one host round trip per step.  The host replays the reference's
// sequential rule exactly over those pairs and the device applies removals by compaction.
constexpr uint32_t kMailboxPairs = 2048;

int pinned_reserve(bh_engine *e, size_t bytes) {
    if (bytes <= e->pin_bytes) return BH_OK;
    if (e->pin) (void)hipHostFree(e->pin);
    e->pin = nullptr;
    size_t nb = std::max<size_t>(bytes, 1 << 16);
    HIPCHK(e, hipHostMalloc(&e->pin, nb, hipHostMallocDefault));
    e->pin_bytes = nb;
    return BH_OK;
}

int merge_bufs(bh_engine *e, uint32_t need) {  // dead / update / mass staging on the device
    if (need <= e->mcap && e->mdead) return BH_OK;
    e->mcap = std::max<uint32_t>(need, 64) * 2;
    TRY(dev_alloc(e, e->mdead, e->mcap));
    TRY(dev_alloc(e, e->mupd, e->mcap));
    TRY(dev_alloc(e, e->mupd_mass, e->mcap));
    TRY(dev_alloc(e, e->hmass, e->mcap));
    return BH_OK;
}

int refresh_heavy_list(bh_engine *e) {  // ordered list of m > mergeMaxMass (BHA:474)
    const int64_t n = e->n;
    HIPCHK(e, heavy_list(e->m, n, e->p.merge_max_mass, e->heavy, e->scalars + 2, e->cub_tmp,
                         e->cub_bytes, e->stream));
    uint32_t hc = 0;
    HIPCHK(e, hipMemcpyAsync(&hc, e->scalars + 2, sizeof(uint32_t), hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->h_heavy.resize(hc);
    e->h_hmass.resize(hc);
    if (hc > 0) {
        TRY(merge_bufs(e, hc));
        gather_doubles(e->heavy, hc, e->m, e->hmass, e->stream);
        HIPCHK(e, hipMemcpyAsync(e->h_heavy.data(), e->heavy, sizeof(uint32_t) * hc,
                                 hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->h_hmass.data(), e->hmass, sizeof(double) * hc,
                                 hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
    }
    e->heavy_count = hc;
    return BH_OK;
}

int merge(bh_engine *e) {
    if (e->p.merge_min_dist <= 0.0 || e->n <= 1) return BH_OK;  // BHA:465
    TRY(mark(e, -1));
    const int64_t n = e->n;
    if (e->heavy_count < 0) TRY(refresh_heavy_list(e));
    const uint32_t H = (uint32_t)e->heavy_count;
    if (H == 0) {
        TRY(mark(e, 3));
        return BH_OK;
    }
    const double minD2 = e->p.merge_min_dist * e->p.merge_min_dist;  // BHA:468
    if (e->pair_cap == 0) {
        e->pair_cap = 1u << 16;
        TRY(dev_alloc(e, e->pairs, e->pair_cap + 1));
    }
    // mailbox = pairs[0] (count in .k) followed by up to pair_cap pairs
    MergePair *box = e->pairs;
    const size_t fast_bytes = sizeof(MergePair) * (1 + kMailboxPairs);
    TRY(pinned_reserve(e, std::max(fast_bytes, sizeof(MergePair) * (1 + (size_t)e->pair_cap))));
    uint32_t count = 0;
    for (;;) {
        merge_candidates(n, e->x, e->y, e->m, e->heavy, H, minD2, box + 1, e->pair_cap,
                         &box->k, e->stream);
        HIPCHK(e, hipGetLastError());
        HIPCHK(e, hipMemcpyAsync(e->pin, box, fast_bytes, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));  // the one round trip of the step
        count = reinterpret_cast<MergePair *>(e->pin)->k;
        if (count <= e->pair_cap) break;
        e->pair_cap = count + (count >> 1);
        TRY(dev_alloc(e, e->pairs, e->pair_cap + 1));
        box = e->pairs;
        TRY(pinned_reserve(e, sizeof(MergePair) * (1 + (size_t)e->pair_cap)));
    }
    if (count == 0) {
        TRY(mark(e, 3));
        return BH_OK;
    }
    if (count > kMailboxPairs) {
        HIPCHK(e, hipMemcpyAsync(e->pin, box, sizeof(MergePair) * (1 + (size_t)count),
                                 hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
    }
    const MergePair *pp = reinterpret_cast<const MergePair *>(e->pin) + 1;
    std::vector<MergePair> pr(pp, pp + count);
    std::sort(pr.begin(), pr.end(), [](const MergePair &a, const MergePair &b) {
        return a.k != b.k ? a.k < b.k : a.j < b.j;
    });
    // Sequential replay of BHA:470-531.  Heavy bodies are visited in list order; a heavy body
    // eaten earlier is skipped; victims are absorbed in descending index order (BHA:514-519).
    const std::vector<uint32_t> &hv = e->h_heavy;
    std::unordered_map<uint32_t, uint32_t> heavy_pos;
    for (uint32_t k = 0; k < H; ++k) heavy_pos[hv[k]] = k;
    std::vector<double> cur = e->h_hmass;
    std::vector<char> heavy_dead(H, 0);
    std::unordered_set<uint32_t> dead;
    std::vector<uint32_t> dead_list;
    size_t pi = 0;
    for (uint32_t k = 0; k < H; ++k) {
        size_t pe = pi;
        while (pe < pr.size() && pr[pe].k == k) ++pe;
        if (!heavy_dead[k]) {  // bi still in the list; its mass only grew: still heavy
            double mi = cur[k];
            for (size_t q = pe; q > pi; --q) {
                const MergePair &c = pr[q - 1];
                if (dead.count(c.j)) continue;
                auto it = heavy_pos.find(c.j);
                double mj = c.mj;
                if (it != heavy_pos.end()) {  // a heavy victim carries its grown mass
                    mj = cur[it->second];
                    heavy_dead[it->second] = 1;
                }
                mi += mj;  // BHA:518
                dead.insert(c.j);
                dead_list.push_back(c.j);
            }
            cur[k] = mi;
        }
        pi = pe;
    }
    if (dead_list.empty()) {
        TRY(mark(e, 3));
        return BH_OK;
    }
    std::sort(dead_list.begin(), dead_list.end());
    // upload: dead list | updated heavy (index, mass) | new heavy list, from pinned memory
    std::vector<uint32_t> upd;
    std::vector<double> upd_mass;
    std::vector<uint32_t> new_heavy;
    std::vector<double> new_hmass;
    for (uint32_t k = 0; k < H; ++k) {
        if (heavy_dead[k]) continue;
        const uint32_t hi = hv[k];
        if (std::memcmp(&cur[k], &e->h_hmass[k], sizeof(double)) != 0) {
            upd.push_back(hi);
            upd_mass.push_back(cur[k]);
        }
        // index after removal of every dead body before it (list order is preserved)
        uint32_t shift = (uint32_t)(std::lower_bound(dead_list.begin(), dead_list.end(), hi) -
                                    dead_list.begin());
        new_heavy.push_back(hi - shift);
        new_hmass.push_back(cur[k]);
    }
    const uint32_t nd = (uint32_t)dead_list.size(), nu = (uint32_t)upd.size(),
                   nh = (uint32_t)new_heavy.size();
    TRY(merge_bufs(e, std::max<uint32_t>(std::max(nd, nu), nh)));
    size_t up_bytes = 4 * (size_t)nd + 4 * (size_t)nu + 8 * (size_t)nu + 4 * (size_t)nh + 64;
    TRY(pinned_reserve(e, up_bytes + sizeof(MergePair) * (1 + (size_t)count)));
    char *u = static_cast<char *>(e->pin);
    uint32_t *u_dead = reinterpret_cast<uint32_t *>(u);
    uint32_t *u_upd = u_dead + nd;
    uint32_t *u_heavy = u_upd + nu;
    double *u_mass = reinterpret_cast<double *>(
        u + (((4 * (size_t)(nd + nu + nh)) + 7) & ~(size_t)7));
    std::memcpy(u_dead, dead_list.data(), 4 * (size_t)nd);
    std::memcpy(u_upd, upd.data(), 4 * (size_t)nu);
    std::memcpy(u_heavy, new_heavy.data(), 4 * (size_t)nh);
    std::memcpy(u_mass, upd_mass.data(), 8 * (size_t)nu);
    HIPCHK(e, hipMemcpyAsync(e->mdead, u_dead, 4 * (size_t)nd, hipMemcpyHostToDevice, e->stream));
    if (nu) {
        HIPCHK(e, hipMemcpyAsync(e->mupd, u_upd, 4 * (size_t)nu, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->mupd_mass, u_mass, 8 * (size_t)nu, hipMemcpyHostToDevice,
                                 e->stream));
    }
    HIPCHK(e, hipMemsetD32Async((hipDeviceptr_t)e->keep, 1, (size_t)n, e->stream));
    apply_merge(nd, e->mdead, nu, e->mupd, e->mupd_mass, e->keep, e->m, e->stream);
    const double *src[5] = {e->x, e->y, e->vx, e->vy, e->m};
    double *dst[5] = {e->alt[0], e->alt[1], e->alt[2], e->alt[3], e->alt[4]};
    HIPCHK(e, compact_bodies(n, e->keep, src, dst, e->pos, nullptr, e->cub_tmp, e->cub_bytes,
                             e->stream));
    if (nh) HIPCHK(e, hipMemcpyAsync(e->heavy, u_heavy, 4 * (size_t)nh, hipMemcpyHostToDevice,
                                     e->stream));
    std::swap(e->x, e->alt[0]);
    std::swap(e->y, e->alt[1]);
    std::swap(e->vx, e->alt[2]);
    std::swap(e->vy, e->alt[3]);
    std::swap(e->m, e->alt[4]);
    e->n = n - (int64_t)nd;
    e->step_dead.push_back(dead_list);
    e->h_heavy = std::move(new_heavy);
    e->h_hmass = std::move(new_hmass);
    e->heavy_count = nh;
    e->tree_valid = false;  // BHA:526
    TRY(mark(e, 3));
    return BH_OK;
}

// ---- one PhysicsEngine.step() (BHA:405-439) ------------------------------------------
int step_once(bh_engine *e) {
    const int64_t n = e->n;
    const double dtHalf = e->p.dt * 0.5;  // BHA:412
    if (n > 0) {
        TRY(evaluate(e, nullptr));  // a(t)
        TRY(mark(e, -1));
        kick_drift(n, e->ax, e->ay, e->x, e->y, e->vx, e->vy, dtHalf, e->p.dt, e->stream);
        HIPCHK(e, hipGetLastError());
        TRY(mark(e, 2));
        TRY(evaluate(e, nullptr));  // a(t+dt)
        TRY(mark(e, -1));
        kick(n, e->ax, e->ay, e->vx, e->vy, dtHalf, e->stream);
        HIPCHK(e, hipGetLastError());
        TRY(mark(e, 2));
        e->tree_valid = true;  // lastTree = root (BHA:435)
    }
    return merge(e);  // BHA:438
}

// ---- getTreeForDebug().visitQuads (BHA:265-274) from the Morton structure ------------
struct QuadWalker {
    const Geometry &g;
    const std::vector<uint64_t> &keys;
    const std::vector<int8_t> &cpl;
    const std::vector<uint32_t> &base;
    bh_engine *e;
    double *cx, *cy, *h;
    int64_t cap, k = 0;
    int rc = BH_OK;

    void emit(double qx, double qy, double qh) {
        if (k < cap) {
            cx[k] = qx;
            cy[k] = qy;
            h[k] = qh;
        }
        ++k;
    }
    static void child(double qx, double qy, double qh, int which, double &ox, double &oy,
                      double &oh) {  // BHA:73-81
        double hh = qh / 2.0;
        ox = (which & 1) ? qx + hh : qx - hh;
        oy = (which & 2) ? qy + hh : qy - hh;
        oh = hh;
    }
    void leaf_children(double qx, double qy, double qh) {
        for (int q = 0; q < 4; ++q) {
            double ox, oy, oh;
            child(qx, qy, qh, q, ox, oy, oh);
            emit(ox, oy, oh);
        }
    }
    void rec(int L, int64_t lo, int64_t hi, double qx, double qy, double qh) {
        emit(qx, qy, qh);
        if (hi - lo < 2) return;  // empty or single-body leaf
        if (L == g.J) {           // jitter cell: children from the replay
            int cp = lo > 0 ? (int)cpl[lo - 1] : -1;
            uint32_t ni = base[lo] + (uint32_t)(L - cp - 1);
            Node nd;
            if (hipMemcpy(&nd, e->nodes + ni, sizeof(Node), hipMemcpyDeviceToHost) != hipSuccess) {
                rc = BH_E_DEVICE;
                return;
            }
            uint32_t jmask = (nd.meta >> NODE_JMASK_SHIFT) & 0xFu;
            for (int q = 0; q < 4; ++q) {
                double ox, oy, oh;
                child(qx, qy, qh, q, ox, oy, oh);
                emit(ox, oy, oh);
                if (jmask & (1u << q)) leaf_children(ox, oy, oh);
            }
            return;
        }
        const int shift = 2 * (g.J - 1 - L);
        int64_t s = lo;
        for (int q = 0; q < 4; ++q) {
            int64_t e2 = s;
            while (e2 < hi && (int)((keys[e2] >> shift) & 3u) == q) ++e2;
            double ox, oy, oh;
            child(qx, qy, qh, q, ox, oy, oh);
            rec(L + 1, s, e2, ox, oy, oh);
            s = e2;
        }
    }
};

void set_defaults(bh_params *p) {
    p->G = 80.0;               // CFG:11
    p->dt = 0.005;             // CFG:14
    p->theta = 0.30;           // CFG:23
    p->soft2 = 1.0 * 1.0;      // CFG:17,20
    p->width_px = 2400;        // CFG:5
    p->height_px = 800;        // CFG:8
    p->merge_max_mass = 4000.0;  // BHA:315
    p->merge_min_dist = 8.0;     // BHA:321 = Config.MIN_R (CFG:35)
}

int engine_init(bh_engine *e, const bh_params *p, int device) {
    if (!p) {
        e->err = "params is NULL";
        return BH_E_INVALID;
    }
    e->p = *p;
    TRY(make_geometry(e->p, e->geo, e->err));
    e->device = device;
    HIPCHK(e, hipSetDevice(device));
    HIPCHK(e, hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    TRY(dev_alloc(e, e->scalars, 16));
    HIPCHK(e, hipMemset(e->scalars, 0, 16 * sizeof(uint32_t)));
    TRY(ensure_capacity(e, 1));
    return BH_OK;
}

}  // namespace

// =========================================================================================
extern "C" {

void bh_default_params(bh_params *p) {
    if (p) set_defaults(p);
}

int bh_create(const bh_params *p, int device, bh_engine **out) {
    if (!out) return BH_E_INVALID;
    *out = nullptr;
    bh_engine *e = new bh_engine();
    int rc = engine_init(e, p, device);
    if (rc != BH_OK) {
        std::fprintf(stderr, "bh_create: %s\n", e->err.c_str());
        bh_destroy(e);
        return rc;
    }
    *out = e;
    return BH_OK;
}

int bh_comm_unique_id(void *out128) {
    if (!out128) return BH_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return BH_E_COMM;
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id must be 128 bytes");
    std::memcpy(out128, &id, sizeof(id));
    return BH_OK;
}

int bh_create_dist(const bh_params *p, int device, int rank, int world, const void *unique_id,
                   bh_engine **out) {
    if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !unique_id))
        return BH_E_INVALID;
    *out = nullptr;
    bh_engine *e = new bh_engine();
    e->rank = rank;
    e->world = world;
    int rc = engine_init(e, p, device);
    if (rc == BH_OK && world > 1) {
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        ncclResult_t nr = ncclCommInitRank(&e->comm, world, id, rank);
        if (nr != ncclSuccess) {
            e->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(nr);
            rc = BH_E_COMM;
        }
    }
    if (rc != BH_OK) {
        std::fprintf(stderr, "bh_create_dist: %s\n", e->err.c_str());
        bh_destroy(e);
        return rc;
    }
    *out = e;
    return BH_OK;
}

void bh_destroy(bh_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->comm) (void)ncclCommDestroy(e->comm);
    void *ptrs[] = {e->x, e->y, e->vx, e->vy, e->m, e->alt[0], e->alt[1], e->alt[2], e->alt[3],
                    e->alt[4], e->ax, e->ay, e->a_sorted, e->keys, e->keys_s, e->idx, e->perm,
                    e->sx, e->sy, e->sm, e->cpl, e->cnt, e->base, e->nodes, e->scalars,
                    e->span_cnt, e->span_list, e->span_children,
                    e->visits32, e->wave_iters, e->heavy, e->keep, e->pos, e->pairs, e->mdead, e->mupd,
                    e->mupd_mass, e->hmass, e->cub_tmp};
    for (void *q : ptrs)
        if (q) (void)hipFree(q);
    for (hipEvent_t ev : e->ev) (void)hipEventDestroy(ev);
    if (e->pin) (void)hipHostFree(e->pin);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

const char *bh_last_error(const bh_engine *e) { return e ? e->err.c_str() : "null engine"; }

int bh_set_params(bh_engine *e, const bh_params *p) {
    if (!e || !p) return BH_E_INVALID;
    Geometry g;
    TRY(make_geometry(*p, g, e->err));
    HIPCHK(e, hipSetDevice(e->device));
    bool geo_changed = std::memcmp(&g, &e->geo, sizeof(g)) != 0;
    if (p->merge_max_mass != e->p.merge_max_mass) e->heavy_count = -1;
    e->p = *p;
    e->geo = g;
    if (geo_changed) {
        e->tree_valid = false;
        TRY(ensure_capacity(e, e->n));
    }
    return BH_OK;
}

int bh_get_params(const bh_engine *e, bh_params *p) {
    if (!e || !p) return BH_E_INVALID;
    *p = e->p;
    return BH_OK;
}

int bh_reset_bodies(bh_engine *e, int64_t n, const double *x, const double *y, const double *vx,
                    const double *vy, const double *m) {
    if (!e || n < 0 || (n > 0 && (!x || !y || !vx || !vy || !m))) return BH_E_INVALID;
    if (n >= (int64_t)NODE_BODY_MASK) {
        e->err = "too many bodies";
        return BH_E_INVALID;
    }
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->n = 0;  // old state is replaced, do not preserve it across a growth
    TRY(ensure_capacity(e, n));
    if (n > 0) {
        HIPCHK(e, hipMemcpyAsync(e->x, x, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->y, y, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->vx, vx, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->vy, vy, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->m, m, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->n = n;
    e->heavy_count = -1;
    e->tree_valid = false;  // BHA:348
    return BH_OK;
}

int bh_step(bh_engine *e, int32_t k) {
    if (!e || k < 0) return BH_E_INVALID;
    HIPCHK(e, hipSetDevice(e->device));
    e->ev_used = 0;
    e->timings_pending = false;
    HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, sizeof(uint32_t), e->stream));
    e->step_dead.clear();
    for (int32_t s = 0; s < k; ++s) TRY(step_once(e));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->n > 0 && k > 0) TRY(check_tree_flags(e));
    if (e->profiling) TRY(collect_timings(e));
    return BH_OK;
}

int64_t bh_num_bodies(const bh_engine *e) { return e ? e->n : -1; }

int bh_get_bodies(bh_engine *e, double *x, double *y, double *vx, double *vy, double *m,
                  int64_t cap, int64_t *n_out) {
    if (!e) return BH_E_INVALID;
    if (n_out) *n_out = e->n;
    if (cap < e->n) return BH_E_CAPACITY;
    HIPCHK(e, hipSetDevice(e->device));
    double *dst[5] = {x, y, vx, vy, m};
    double *src[5] = {e->x, e->y, e->vx, e->vy, e->m};
    for (int k = 0; k < 5; ++k)
        if (dst[k] && e->n > 0)
            HIPCHK(e, hipMemcpyAsync(dst[k], src[k], sizeof(double) * e->n, hipMemcpyDeviceToHost,
                                     e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return BH_OK;
}

int bh_compute_accelerations(bh_engine *e, double *ax, double *ay, int64_t *visits) {
    if (!e) return BH_E_INVALID;
    HIPCHK(e, hipSetDevice(e->device));
    const int64_t n = e->n;
    e->ev_used = 0;
    e->timings_pending = false;
    HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, sizeof(uint32_t), e->stream));
    if (n > 0) {
        TRY(evaluate(e, visits ? e->visits32 : nullptr));
        e->tree_valid = true;
        HIPCHK(e, hipStreamSynchronize(e->stream));
        TRY(check_tree_flags(e));
        if (ax) HIPCHK(e, hipMemcpy(ax, e->ax, sizeof(double) * n, hipMemcpyDeviceToHost));
        if (ay) HIPCHK(e, hipMemcpy(ay, e->ay, sizeof(double) * n, hipMemcpyDeviceToHost));
        if (visits) {
            std::vector<uint32_t> v((size_t)n);
            HIPCHK(e, hipMemcpy(v.data(), e->visits32, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
            int64_t lane_sum = 0;
            for (int64_t i = 0; i < n; ++i) {
                visits[i] = v[(size_t)i];
                lane_sum += v[(size_t)i];
            }
            const int64_t waves = (n + 63) / 64;
            std::vector<uint32_t> wi((size_t)waves);
            HIPCHK(e, hipMemcpy(wi.data(), e->wave_iters, sizeof(uint32_t) * waves,
                                hipMemcpyDeviceToHost));
            int64_t wsum = 0;
            for (uint32_t c : wi) wsum += c;
            e->stat_lane_visits = lane_sum;
            e->stat_wave_iters = wsum;
            e->stat_waves = waves;
        }
    }
    if (e->profiling) TRY(collect_timings(e));
    return BH_OK;
}

int bh_get_quads(bh_engine *e, double *cx, double *cy, double *h, int64_t cap, int64_t *n_out) {
    if (!e || cap < 0 || (cap > 0 && (!cx || !cy || !h))) return BH_E_INVALID;
    HIPCHK(e, hipSetDevice(e->device));
    const int64_t n = e->n;
    if (!e->tree_valid) {  // getTreeForDebug builds a fresh tree (BHA:329-332)
        if (n > 0) {
            HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, sizeof(uint32_t), e->stream));
            HIPCHK(e, tree_build(tree_buffers(e), n, e->geo, e->stream));
            TRY(check_tree_flags(e));
        }
        e->tree_valid = true;
    }
    std::vector<uint64_t> keys((size_t)n);
    std::vector<int8_t> cpl((size_t)n);
    std::vector<uint32_t> base((size_t)n + 1);
    if (n > 0) {
        HIPCHK(e, hipMemcpy(keys.data(), e->keys_s, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(cpl.data(), e->cpl, n, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(base.data(), e->base, sizeof(uint32_t) * (n + 1), hipMemcpyDeviceToHost));
    }
    int64_t M = 0;
    const uint64_t SENT = sentinel_key(e->geo.J);
    while (M < n && keys[(size_t)M] != SENT) ++M;
    QuadWalker w{e->geo, keys, cpl, base, e, cx, cy, h, cap};
    w.rec(0, 0, M, e->geo.root_cx, e->geo.root_cy, e->geo.root_h);
    if (w.rc != BH_OK) return w.rc;
    if (n_out) *n_out = w.k;
    return w.k > cap ? BH_E_CAPACITY : BH_OK;
}

int bh_last_removed(const bh_engine *e, int64_t *idx, int64_t cap, int64_t *n_out) {
    if (!e || cap < 0 || (cap > 0 && !idx)) return BH_E_INVALID;
    // compose the per-step removal lists into indices of the list before the call
    std::vector<int64_t> orig;  // sorted
    for (const auto &dl : e->step_dead) {
        std::vector<int64_t> add;
        size_t r = 0;
        int64_t shift = 0;
        for (uint32_t d : dl) {  // d ascending: index among the survivors so far
            int64_t o = (int64_t)d + shift;
            while (r < orig.size() && orig[r] <= o) {
                ++r;
                ++shift;
                o = (int64_t)d + shift;
            }
            add.push_back(o);
        }
        std::vector<int64_t> merged;
        std::merge(orig.begin(), orig.end(), add.begin(), add.end(), std::back_inserter(merged));
        orig.swap(merged);
    }
    if (n_out) *n_out = (int64_t)orig.size();
    if ((int64_t)orig.size() > cap) return BH_E_CAPACITY;
    for (size_t i = 0; i < orig.size(); ++i) idx[i] = orig[i];
    return BH_OK;
}

int bh_last_timings(const bh_engine *e, double *out5) {
    if (!e || !out5) return BH_E_INVALID;
    for (int k = 0; k < kPhases; ++k) out5[k] = e->phase_ms[k];
    return BH_OK;
}

int64_t bh_last_tree_nodes(const bh_engine *e) {
    if (!e || e->n <= 0) return 0;
    uint32_t T = 0;
    if (hipMemcpy(&T, e->base + e->n, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return T;
}

int bh_traverse_kernel_ms(const bh_engine *e, double *avg_ms, int64_t *launches) {
    if (!e || !avg_ms) return BH_E_INVALID;
    *avg_ms = e->trav_launches ? e->trav_ms_sum / (double)e->trav_launches : 0.0;
    if (launches) *launches = e->trav_launches;
    return BH_OK;
}

int bh_traversal_stats(const bh_engine *e, int64_t *lane_visits, int64_t *wave_iters,
                       int64_t *waves) {
    if (!e || !lane_visits || !wave_iters || !waves) return BH_E_INVALID;
    *lane_visits = e->stat_lane_visits;
    *wave_iters = e->stat_wave_iters;
    *waves = e->stat_waves;
    return BH_OK;
}

int bh_set_profiling(bh_engine *e, int enabled) {
    if (!e) return BH_E_INVALID;
    e->profiling = enabled != 0;
    return BH_OK;
}

int bh_shard_range(int64_t n, int rank, int world, int64_t *lo, int64_t *hi) {
    if (n < 0 || world < 1 || rank < 0 || rank >= world || !lo || !hi) return BH_E_INVALID;
    const int64_t chunk = (n + world - 1) / world;
    *lo = std::min<int64_t>(n, (int64_t)rank * chunk);
    *hi = std::min<int64_t>(n, *lo + chunk);
    return BH_OK;
}

int bh_synchronize(bh_engine *e) {
    if (!e) return BH_E_INVALID;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return BH_OK;
}

}  // extern "C"
