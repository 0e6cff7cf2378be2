// Kick-drift-kick integration (BHA:410-432), caller-order copies, and the device side of the
// merge rule (BHA:463-532).  All elementwise and coalesced over the slot (Morton) order.
#include <rocprim/device/device_scan.hpp>

#include "bh_device.hpp"

namespace bh {
namespace {

constexpr int TB = 256;
inline unsigned grid_for(int64_t n) { return (unsigned)((n + TB - 1) / TB); }

typedef double double2_t __attribute__((ext_vector_type(2)));

// BHA:412-422 fused: v += a * dtHalf; x += v * DT.  The reference runs the kick loop over
// all bodies and then the drift loop; per body the operations are identical.
// a2 is indexed by the traversal's lane when `lanes` is given (lane i holds body lanes[i]).
__global__ __launch_bounds__(TB) void k_kick_drift(int64_t n, const double *__restrict__ a2,
                                                   double *__restrict__ x, double *__restrict__ y,
                                                   double *__restrict__ vx,
                                                   double *__restrict__ vy, double dtHalf,
                                                   double dt, const uint32_t *__restrict__ lanes,
                                                   GatherLayout gl,
                                                   unsigned long long *__restrict__ vmax) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    double vxi = 0.0, vyi = 0.0;
    if (i < n) {
        const double2_t a = *reinterpret_cast<const double2_t *>(a2 + 2 * gather_slot(gl, i));
        const int64_t p = lanes ? (int64_t)lanes[i] : i;
        vxi = vx[p] + a.x * dtHalf;
        vyi = vy[p] + a.y * dtHalf;
        vx[p] = vxi;
        vy[p] = vyi;
        x[p] = x[p] + vxi * dt;
        y[p] = y[p] + vyi * dt;
    }
    if (vmax) wave_vmax(vmax, vxi, vyi);  // (multi-rank: the LET selection's displacement bound)
}

// The same kick + drift by lane of the traversal's lane map, after an evaluation that was made
// ahead (the deep pipeline, engine.cpp evaluate_pipelined), with the next build's first two passes
// (k_morton, k_bucket_count) for the moved body -- what the drifting traversal's epilogue does
// (traverse.hip trav_wave), operation for operation.
__global__ __launch_bounds__(TB) void k_kick_drift_keys(int64_t n, const double *__restrict__ a2,
                                                        double *__restrict__ x,
                                                        double *__restrict__ y,
                                                        double *__restrict__ vx,
                                                        double *__restrict__ vy,
                                                        const uint32_t *__restrict__ cidx,
                                                        double dtHalf, double dt,
                                                        const uint32_t *__restrict__ lanes,
                                                        Geometry g, MortonFuse mf) {
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const double2_t a = *reinterpret_cast<const double2_t *>(a2 + 2 * i);
    const int64_t p = lanes ? (int64_t)lanes[i] : i;
    const double vxi = vx[p] + a.x * dtHalf;
    const double vyi = vy[p] + a.y * dtHalf;
    vx[p] = vxi;
    vy[p] = vyi;
    const double nx = x[p] + vxi * dt, ny = y[p] + vyi * dt;
    x[p] = nx;
    y[p] = ny;
    if (mf.keys) {
        const uint64_t key = morton_key(g, nx, ny, (cidx[p] & CIDX_DEAD) != 0u);
        const uint32_t k32 = (uint32_t)(key >> key32_shift(g.J));
        mf.keys[p] = key;
        mf.keys32[p] = k32;
        const uint32_t b = find_bucket(mf.spl, mf.spl_nb, ((uint64_t)k32 << 32) | (uint64_t)p,
                                       (uint32_t)(p / SORT_B));
        mf.bkt[p] = b;
        mf.off[p] = bucket_offset(b, mf.counts);
    }
}

// BHA:429-432
__global__ __launch_bounds__(TB) void k_kick(int64_t n, const double *__restrict__ a2,
                                             double *__restrict__ vx, double *__restrict__ vy,
                                             double dtHalf, const uint32_t *__restrict__ lanes,
                                             GatherLayout gl) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const double2_t a = *reinterpret_cast<const double2_t *>(a2 + 2 * gather_slot(gl, i));
    const int64_t p = lanes ? (int64_t)lanes[i] : i;
    vx[p] = vx[p] + a.x * dtHalf;
    vy[p] = vy[p] + a.y * dtHalf;
}

// The pipelined step's copies of what the overlapped merge rule and build overwrite while the
// second traversal reads it (masses, flags, lane map, node count): one launch instead of four
// device copies.
__global__ __launch_bounds__(TB) void k_trav_inputs(int64_t n, const double *__restrict__ m,
                                                    double *__restrict__ m_t,
                                                    const uint32_t *__restrict__ cidx,
                                                    uint32_t *__restrict__ cidx_t,
                                                    const uint32_t *__restrict__ lanes,
                                                    uint32_t *__restrict__ lanes_t,
                                                    const uint32_t *__restrict__ T,
                                                    uint32_t *__restrict__ T_t,
                                                    uint32_t *__restrict__ box_header) {
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i == 0) *T_t = *T;
    if (box_header && i < (int64_t)(sizeof(MergeHeader) / sizeof(uint32_t))) box_header[i] = 0u;
    if (i >= n) return;
    m_t[i] = m[i];
    cidx_t[i] = cidx[i];
    if (lanes) lanes_t[i] = lanes[i];
}

__global__ __launch_bounds__(TB) void k_iota(uint32_t *__restrict__ p, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

struct Ptrs5 {
    const double *src[5];
    double *dst[5];
};

__global__ __launch_bounds__(TB) void k_scatter_caller(int64_t n, const uint32_t *__restrict__ cidx,
                                                       int k, Ptrs5 p) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const uint32_t o = cidx[i];
    if (o & CIDX_DEAD) return;  // a tombstone has no caller slot
    for (int j = 0; j < k; ++j) p.dst[j][o] = p.src[j][i];
}

// Caller-order mirror (engine.cpp bh_map_bodies): at the end of a bh_step call, before its
// compaction, the state holds every caller index of the list the call started from exactly once
// (tombstones keep theirs), so keep[c] = "c survives" over caller indices, its exclusive scan
// pos[c] = c's index in the list after the removals (BHA:519), and the live bodies scatter there.
// These kernels run next to the last traversal (wave priority, like the overlapped build).
__global__ __launch_bounds__(TB) void k_mirror_keep(int64_t n, const uint32_t *__restrict__ cidx,
                                                    uint32_t *__restrict__ keep) {
    chain_prio();
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = cidx[i];
    keep[c & ~CIDX_DEAD] = (c & CIDX_DEAD) ? 0u : 1u;
}

__global__ __launch_bounds__(TB) void k_mirror_survivors(int64_t n, const uint32_t *__restrict__ keep,
                                                         const uint32_t *__restrict__ pos,
                                                         const uint32_t *__restrict__ hdr_src,
                                                         uint32_t *__restrict__ out) {
    chain_prio();
    const int64_t c = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (c < MIRROR_HDR) out[c] = c < 4 ? hdr_src[c] : 0u;
    if (c < n && keep[c]) out[MIRROR_HDR + pos[c]] = (uint32_t)c;
}

__global__ void k_copy_u32(uint32_t *dst, const uint32_t *src) {
    chain_prio();
    *dst = *src;
}

__global__ __launch_bounds__(TB) void k_mirror_scatter(int64_t n, const uint32_t *__restrict__ cidx,
                                                       const uint32_t *__restrict__ pos, int k,
                                                       Ptrs5 p) {
    chain_prio();
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = cidx[i];
    if (c & CIDX_DEAD) return;
    const uint32_t o = pos[c];
    for (int j = 0; j < k; ++j) p.dst[j][o] = p.src[j][i];
}

__global__ __launch_bounds__(TB) void k_scatter_acc(int64_t n, const uint32_t *__restrict__ cidx,
                                                    const double *__restrict__ a2,
                                                    double *__restrict__ ax,
                                                    double *__restrict__ ay,
                                                    const uint32_t *__restrict__ lanes,
                                                    GatherLayout gl) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const uint32_t o = cidx[lanes ? (int64_t)lanes[i] : i];
    if (o & CIDX_DEAD) return;  // a tombstone has no caller slot
    const int64_t g = gather_slot(gl, i);
    ax[o] = a2[2 * g];
    ay[o] = a2[2 * g + 1];
}

// heavy bodies: m > mergeMaxMass (BHA:474), live ones only; appended in any order (the
// replay below orders them by caller index)
__global__ __launch_bounds__(TB) void k_heavy(int64_t n, const double *__restrict__ m,
                                              const uint32_t *__restrict__ cidx, double thr,
                                              uint32_t *__restrict__ heavy, MergeHeader *hdr) {
    chain_prio();
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    if (m[i] > thr && !(cidx[i] & CIDX_DEAD)) heavy[atomicAdd(&hdr->heavies, 1u)] = (uint32_t)i;
}

// BHA:493-501: for every heavy body h and every live body j != h: dx*dx + dy*dy < minD2 with
// dx = bj.x - bi.x.  Pairs are appended in any order; the replay sorts them.
// heavy_count (nullable): the heavy list was made by the build (k_prep); its count is copied to
// the header, which the host reads (finish_merges: no heavy body left -> the rule is skipped)
__global__ __launch_bounds__(TB) void k_candidates(int64_t n, const double *__restrict__ x,
                                                   const double *__restrict__ y,
                                                   const double *__restrict__ m,
                                                   const uint32_t *__restrict__ cidx,
                                                   const uint32_t *__restrict__ heavy,
                                                   double minD2, MergePair *box, uint32_t cap,
                                                   const uint32_t *__restrict__ heavy_count) {
    chain_prio();
    int64_t j = (int64_t)blockIdx.x * TB + threadIdx.x;
    MergeHeader *hdr = reinterpret_cast<MergeHeader *>(box);
    const uint32_t H = __builtin_amdgcn_readfirstlane(
        heavy_count ? *heavy_count
                    : __hip_atomic_load(&hdr->heavies, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (heavy_count && j == 0) hdr->heavies = H;
    if (j >= n || H == 0) return;
    const uint32_t cj = cidx[j];
    if (cj & CIDX_DEAD) return;
    const double xj = x[j], yj = y[j];
    for (uint32_t k = 0; k < H; ++k) {
        const uint32_t hs = heavy[k];
        if ((int64_t)hs == j) continue;
        const double dx = xj - x[hs];
        const double dy = yj - y[hs];
        if (dx * dx + dy * dy < minD2) {
            const uint32_t slot = atomicAdd(&hdr->pairs, 1u);
            if (slot < cap) box[1 + slot] = MergePair{cidx[hs], cj, hs, (uint32_t)j, m[hs], m[j]};
        }
    }
}

// Sequential replay of BHA:470-531 over candidate pairs sorted by (heavy, victim) caller
// index: heavy bodies in list order, one already absorbed is skipped; victims absorbed in
// descending list index (BHA:514-519), a heavy victim carrying the mass it has grown to;
// m[h] += m[v] in that order (BHA:518).  Removal = tombstone (CIDX_DEAD; the body leaves the
// tree, the candidate search and the output) plus an entry in the removal log; the host
// compacts once per bh_step call.
template <class K, class I>
__device__ void replay_sorted(const MergePair *pairs, uint32_t count, K key, I idx, double *m,
                              uint32_t *cidx, uint32_t *dlog, uint32_t &nd) {
    for (uint32_t q = 0; q < count;) {
        const uint32_t h = (uint32_t)(key(q) >> 32);
        uint32_t qe = q;
        while (qe < count && (uint32_t)(key(qe) >> 32) == h) ++qe;
        const uint32_t hs = pairs[idx(q)].h_slot;
        if (!(cidx[hs] & CIDX_DEAD)) {
            double mi = m[hs];
            bool any = false;
            for (uint32_t r = qe; r > q; --r) {
                const uint32_t vs = pairs[idx(r - 1)].v_slot;
                const uint32_t cv = cidx[vs];
                if (cv & CIDX_DEAD) continue;
                mi += m[vs];  // BHA:518
                dlog[nd++] = cv;
                cidx[vs] = cv | CIDX_DEAD;
                any = true;
            }
            if (any) m[hs] = mi;
        }
        q = qe;
    }
}

constexpr int REPLAY_TB = 256;
constexpr int REPLAY_LDS = 2048;   // pairs sorted in LDS
constexpr int REPLAY_FAST = 1024;  // pairs replayed entirely in LDS
constexpr int REPLAY_HASH = 4096;  // >= 2 * REPLAY_FAST involved bodies, power of two

__device__ __forceinline__ uint64_t pair_key(const MergePair &p) {
    return ((uint64_t)p.h_cidx << 32) | p.v_cidx;
}

constexpr int LARGE_HMAX = 256;       // distinct heavy bodies the bitmap replay handles
constexpr int LARGE_HTAB = 512;       // LDS hash table for them (power of two)
constexpr uint32_t KILLED = 1u << 31;  // vslot flag: removed by the running heavy

// Sequential rule (BHA:470-531) for long candidate lists, same semantics as replay_sorted:
// heavy bodies in caller order (LDS hash set of the pairs' heavies, sorted by one thread);
// for each live one, its victims in DESCENDING caller index come from a bitmap over caller
// indices (set in parallel, enumerated by a block scan), their state is gathered into LDS in
// chunks in parallel, and one thread adds the masses in order from LDS; tombstones are written
// back in parallel.  Returns false, having done nothing, if the pairs name more than
// LARGE_HMAX heavy bodies.
__device__ bool replay_large(const MergePair *__restrict__ pairs, uint32_t count, double *m,
                             uint32_t *cidx, uint32_t *dlog, uint32_t *scal, uint32_t *bits,
                             uint32_t *slot_of, uint32_t *vlist, uint32_t *s_tab,
                             uint32_t *s_hc, uint32_t *s_hs, uint32_t *s_scan, double *vm,
                             uint32_t *vslot, uint32_t *vcid, int chunk) {
    __shared__ uint32_t s_nh, s_maxc, s_total;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < LARGE_HTAB; i += REPLAY_TB) s_tab[i] = 0xFFFFFFFFu;
    if (tid == 0) {
        s_nh = 0;
        s_maxc = 0;
    }
    __syncthreads();
    uint32_t maxc = 0;
    for (uint32_t q = tid; q < count; q += REPLAY_TB) {  // distinct heavies (by slot)
        const uint32_t hs = pairs[q].h_slot;
        maxc = max(maxc, pairs[q].v_cidx);
        uint32_t h = (hs * 2654435761u) & (LARGE_HTAB - 1);
        for (uint32_t probe = 0; probe < LARGE_HTAB; ++probe) {
            const uint32_t prev = atomicCAS(&s_tab[h], 0xFFFFFFFFu, hs);
            if (prev == 0xFFFFFFFFu || prev == hs) break;
            h = (h + 1) & (LARGE_HTAB - 1);
        }
    }
    atomicMax(&s_maxc, maxc);
    __syncthreads();
    if (tid == 0) {  // compact, then order by caller index (insertion sort, <= LARGE_HMAX)
        uint32_t nh = 0;
        for (uint32_t i = 0; i < LARGE_HTAB; ++i) {
            const uint32_t hs = s_tab[i];
            if (hs == 0xFFFFFFFFu) continue;
            if (nh == LARGE_HMAX) {
                nh = LARGE_HMAX + 1;
                break;
            }
            s_hs[nh] = hs;
            s_hc[nh] = cidx[hs] & ~CIDX_DEAD;
            ++nh;
        }
        if (nh <= LARGE_HMAX)
            for (uint32_t i = 1; i < nh; ++i)
                for (uint32_t j = i; j > 0 && s_hc[j - 1] > s_hc[j]; --j) {
                    const uint32_t tc = s_hc[j], ts = s_hs[j];
                    s_hc[j] = s_hc[j - 1];
                    s_hs[j] = s_hs[j - 1];
                    s_hc[j - 1] = tc;
                    s_hs[j - 1] = ts;
                }
        s_nh = nh;
    }
    __syncthreads();
    const uint32_t nh = s_nh;
    if (nh > LARGE_HMAX) return false;
    const uint32_t nwords = (s_maxc >> 5) + 1;
    const uint32_t per = (nwords + REPLAY_TB - 1) / REPLAY_TB;
    // thread t owns words [w0, w1), thread 0 the highest: enumeration order = descending index
    const int64_t w1 = max((int64_t)nwords - (int64_t)tid * per, (int64_t)0);
    const int64_t w0 = max(w1 - (int64_t)per, (int64_t)0);
    uint32_t nd = scal[2];  // meaningful in thread 0
    for (uint32_t hi = 0; hi < nh; ++hi) {
        const uint32_t hs = s_hs[hi];
        if (cidx[hs] & CIDX_DEAD) continue;  // absorbed earlier in this replay (uniform)
        for (uint32_t w = tid; w < nwords; w += REPLAY_TB) bits[w] = 0u;
        __syncthreads();
        for (uint32_t q = tid; q < count; q += REPLAY_TB) {
            const MergePair pr = pairs[q];
            if (pr.h_slot != hs) continue;
            atomicOr(&bits[pr.v_cidx >> 5], 1u << (pr.v_cidx & 31));
            slot_of[pr.v_cidx] = pr.v_slot;
        }
        __syncthreads();
        uint32_t c = 0;
        for (int64_t w = w0; w < w1; ++w) c += __popc(bits[w]);
        s_scan[tid] = c;
        __syncthreads();
        if (tid == 0) {
            uint32_t acc = 0;
            for (uint32_t t = 0; t < REPLAY_TB; ++t) {
                const uint32_t v = s_scan[t];
                s_scan[t] = acc;
                acc += v;
            }
            s_total = acc;
        }
        __syncthreads();
        uint32_t off = s_scan[tid];
        for (int64_t w = w1 - 1; w >= w0; --w) {
            uint32_t b = bits[w];
            while (b) {
                const int k = 31 - __clz(b);
                vlist[off++] = ((uint32_t)w << 5) | (uint32_t)k;
                b &= ~(1u << k);
            }
        }
        __syncthreads();
        const uint32_t nv = s_total;
        double mi = tid == 0 ? m[hs] : 0.0;
        bool any = false;
        for (uint32_t c0 = 0; c0 < nv; c0 += (uint32_t)chunk) {
            const uint32_t cn = min((uint32_t)chunk, nv - c0);
            for (uint32_t k = tid; k < cn; k += REPLAY_TB) {
                const uint32_t vs = slot_of[vlist[c0 + k]];
                vslot[k] = vs;
                vm[k] = m[vs];
                vcid[k] = cidx[vs];
            }
            __syncthreads();
            if (tid == 0) {
                for (uint32_t k = 0; k < cn; ++k) {
                    const uint32_t cv = vcid[k];
                    if (cv & CIDX_DEAD) continue;
                    mi += vm[k];  // BHA:518
                    dlog[nd++] = cv;
                    vcid[k] = cv | CIDX_DEAD;
                    vslot[k] |= KILLED;
                    any = true;
                }
            }
            __syncthreads();
            for (uint32_t k = tid; k < cn; k += REPLAY_TB)
                if (vslot[k] & KILLED) cidx[vslot[k] & ~KILLED] = vcid[k];
            __syncthreads();
        }
        if (tid == 0 && any) m[hs] = mi;
        __syncthreads();
    }
    if (tid == 0) scal[2] = nd;
    return true;
}

__global__ __launch_bounds__(REPLAY_TB) void k_merge_replay(const MergePair *__restrict__ box,
                                                            uint32_t cap, double *m,
                                                            uint32_t *cidx, uint32_t *scal,
                                                            uint32_t *dlog, uint64_t *skeys,
                                                            uint32_t *sidx, uint32_t *bits,
                                                            uint32_t *slot_of, int key_bits,
                                                            uint32_t *heavy_count) {
    chain_prio();
    // (k_candidates, before this kernel on the stream, has read the build's heavy-list count)
    if (heavy_count && threadIdx.x == 0) *heavy_count = 0u;
    __shared__ uint64_t lk[REPLAY_LDS];
    __shared__ uint32_t li[REPLAY_LDS];
    __shared__ uint32_t hkey[REPLAY_HASH], hcidx[REPLAY_HASH];
    __shared__ double hmass[REPLAY_HASH];
    __shared__ uint8_t hflag[REPLAY_HASH];
    __shared__ uint16_t hh[REPLAY_FAST], hv[REPLAY_FAST];
    const MergeHeader *hdr = reinterpret_cast<const MergeHeader *>(box);
    const uint32_t count = hdr->pairs;
    if (count == 0) return;
    const MergePair *pairs = box + 1;
    if (count > cap) {  // pairs were dropped: cannot replay exactly
        if (threadIdx.x == 0) scal[3] = count;
        return;
    }
    uint32_t nd = scal[2];
    if (count > REPLAY_FAST) {  // long lists: bitmap-ordered replay (LDS reused as scratch)
        static_assert(REPLAY_LDS >= REPLAY_TB && REPLAY_HASH >= 2 * LARGE_HTAB, "LDS reuse");
        if (replay_large(pairs, count, m, cidx, dlog, scal, bits, slot_of, sidx, hkey,
                         hcidx, hcidx + LARGE_HMAX, li, hmass, reinterpret_cast<uint32_t *>(lk),
                         reinterpret_cast<uint32_t *>(lk) + REPLAY_LDS, REPLAY_LDS))
            return;
    }
    if (count <= REPLAY_LDS) {  // bitonic sort of (key, index) in LDS
        uint32_t P = 1;
        while (P < count) P <<= 1;
        for (uint32_t i = threadIdx.x; i < P; i += REPLAY_TB) {
            lk[i] = i < count ? pair_key(pairs[i]) : ~0ull;
            li[i] = i;
        }
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = threadIdx.x; i < P; i += REPLAY_TB) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const bool up = (i & k) == 0;
                        if ((lk[i] > lk[l]) == up) {
                            const uint64_t tk = lk[i];
                            lk[i] = lk[l];
                            lk[l] = tk;
                            const uint32_t ti = li[i];
                            li[i] = li[l];
                            li[l] = ti;
                        }
                    }
                }
                __syncthreads();
            }
        }
        if (count > REPLAY_FAST) {
            if (threadIdx.x == 0) {
                replay_sorted(
                    pairs, count, [&](uint32_t q) { return lk[q]; },
                    [&](uint32_t q) { return li[q]; }, m, cidx, dlog, nd);
                scal[2] = nd;
            }
            return;
        }
        // Fast path: every involved body gets an LDS entry (open-addressing table keyed by
        // slot, filled in parallel with its mass and caller index), so the sequential replay
        // below touches LDS only; changed masses / tombstones are written back in parallel.
        for (uint32_t i = threadIdx.x; i < REPLAY_HASH; i += REPLAY_TB) {
            hkey[i] = 0xFFFFFFFFu;
            hflag[i] = 0;
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < 2 * count; q += REPLAY_TB) {
            const MergePair &pr = pairs[li[q >> 1]];
            const uint32_t slot = (q & 1) ? pr.v_slot : pr.h_slot;
            uint32_t h = (slot * 2654435761u) & (REPLAY_HASH - 1);
            for (;;) {
                const uint32_t prev = atomicCAS(&hkey[h], 0xFFFFFFFFu, slot);
                if (prev == 0xFFFFFFFFu) {  // new entry: this thread loads the body's state
                    hmass[h] = m[slot];
                    hcidx[h] = cidx[slot];
                    break;
                }
                if (prev == slot) break;
                h = (h + 1) & (REPLAY_HASH - 1);
            }
            if (q & 1) hv[q >> 1] = (uint16_t)h; else hh[q >> 1] = (uint16_t)h;
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // BHA:470-531 in list order, on LDS
            for (uint32_t q = 0; q < count;) {
                const uint32_t h = (uint32_t)(lk[q] >> 32);
                uint32_t qe = q;
                while (qe < count && (uint32_t)(lk[qe] >> 32) == h) ++qe;
                const uint32_t eh = hh[q];
                if (!(hcidx[eh] & CIDX_DEAD)) {
                    double mi = hmass[eh];
                    bool any = false;
                    for (uint32_t r = qe; r > q; --r) {
                        const uint32_t ev = hv[r - 1];
                        const uint32_t cv = hcidx[ev];
                        if (cv & CIDX_DEAD) continue;
                        mi += hmass[ev];  // BHA:518
                        dlog[nd++] = cv;
                        hcidx[ev] = cv | CIDX_DEAD;
                        hflag[ev] |= 2;
                        any = true;
                    }
                    if (any) {
                        hmass[eh] = mi;
                        hflag[eh] |= 1;
                    }
                }
                q = qe;
            }
            scal[2] = nd;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < REPLAY_HASH; i += REPLAY_TB) {
            const uint32_t f = hflag[i];
            if (f & 1) m[hkey[i]] = hmass[i];
            if (f & 2) cidx[hkey[i]] = hcidx[i];
        }
        return;
    }
    // Long lists naming more heavies than the bitmap replay takes (rare): stable LSD radix sort
    // of (key, index) by the whole workgroup in global scratch (skeys / sidx hold 2 x cap),
    // 4-bit digits over the caller-index bits of the victim, then of the heavy.
    uint64_t *ka = skeys, *kb = skeys + cap;
    uint32_t *ia = sidx, *ib = sidx + cap;
    for (uint32_t i = threadIdx.x; i < count; i += REPLAY_TB) {
        ka[i] = pair_key(pairs[i]);
        ia[i] = i;
    }
    uint32_t *cnt = reinterpret_cast<uint32_t *>(lk);  // 16 digits x REPLAY_TB threads
    static_assert(sizeof(lk) >= 16 * REPLAY_TB * sizeof(uint32_t), "radix counters in LDS");
    const uint32_t per = (count + REPLAY_TB - 1) / REPLAY_TB;
    const uint32_t b0 = min(threadIdx.x * per, count), b1 = min(b0 + per, count);
    for (int pass = 0; pass < 2 * ((key_bits + 3) / 4); ++pass) {
        const int half = pass / ((key_bits + 3) / 4);  // 0: victim bits, 1: heavy bits
        const int shift = 32 * half + 4 * (pass % ((key_bits + 3) / 4));
        __syncthreads();
        uint32_t c[16];
        for (int d = 0; d < 16; ++d) c[d] = 0;
        for (uint32_t i = b0; i < b1; ++i) ++c[(ka[i] >> shift) & 15u];
        for (int d = 0; d < 16; ++d) cnt[d * REPLAY_TB + threadIdx.x] = c[d];
        __syncthreads();
        if (threadIdx.x == 0) {  // exclusive scan, digit-major: stable across threads
            uint32_t acc = 0;
            for (int i = 0; i < 16 * REPLAY_TB; ++i) {
                const uint32_t v = cnt[i];
                cnt[i] = acc;
                acc += v;
            }
        }
        __syncthreads();
        for (int d = 0; d < 16; ++d) c[d] = cnt[d * REPLAY_TB + threadIdx.x];
        for (uint32_t i = b0; i < b1; ++i) {
            const uint64_t k = ka[i];
            const uint32_t o = c[(k >> shift) & 15u]++;
            kb[o] = k;
            ib[o] = ia[i];
        }
        __threadfence_block();
        uint64_t *tk = ka;
        ka = kb;
        kb = tk;
        uint32_t *ti = ia;
        ia = ib;
        ib = ti;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    replay_sorted(
        pairs, count, [&](uint32_t q) { return ka[q]; }, [&](uint32_t q) { return ia[q]; },
        m, cidx, dlog, nd);
    scal[2] = nd;
}

__global__ __launch_bounds__(TB) void k_keep(int64_t n, const uint32_t *__restrict__ cidx,
                                             uint32_t *__restrict__ keep) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i < n) keep[i] = (cidx[i] & CIDX_DEAD) ? 0u : 1u;
}

// compaction (BHA:519 removeAt), order preserved; list indices shift past removed ones
// The same compaction for two extra arrays (the lazy lastTree's position snapshot).
__global__ __launch_bounds__(TB) void k_compact_pair(int64_t n, const uint32_t *__restrict__ keep,
                                                     const uint32_t *__restrict__ pos,
                                                     const double *__restrict__ sx,
                                                     const double *__restrict__ sy,
                                                     double *__restrict__ dx,
                                                     double *__restrict__ dy) {
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n || !keep[i]) return;
    dx[pos[i]] = sx[i];
    dy[pos[i]] = sy[i];
}
__global__ __launch_bounds__(TB) void k_compact(int64_t n, const uint32_t *__restrict__ keep,
                                                const uint32_t *__restrict__ pos, BodyState src,
                                                BodyState dst, const uint32_t *__restrict__ dead_cidx,
                                                uint32_t n_dead) {
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n || !keep[i]) return;
    const uint32_t o = pos[i];
    dst.x[o] = src.x[i];
    dst.y[o] = src.y[i];
    dst.vx[o] = src.vx[i];
    dst.vy[o] = src.vy[i];
    dst.m[o] = src.m[i];
    const uint32_t c = src.cidx[i];
    uint32_t lo = 0, hi = n_dead;  // number of removed list indices below c
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (dead_cidx[mid] < c) lo = mid + 1; else hi = mid;
    }
    dst.cidx[o] = c - lo;
}

// Lane map through a compaction: keep the lanes whose body survives (lane order preserved),
// renumbered to the bodies' new slots.
__global__ __launch_bounds__(TB) void k_lane_keep(int64_t n, const uint32_t *__restrict__ lanes,
                                                  const uint32_t *__restrict__ keep,
                                                  uint32_t *__restrict__ flag) {
    int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (q < n) flag[q] = keep[lanes[q]];
}

__global__ __launch_bounds__(TB) void k_lane_compact(int64_t n, const uint32_t *__restrict__ lanes,
                                                     const uint32_t *__restrict__ flag,
                                                     const uint32_t *__restrict__ qpos,
                                                     const uint32_t *__restrict__ pos,
                                                     uint32_t *__restrict__ out) {
    int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (q < n && flag[q]) out[qpos[q]] = pos[lanes[q]];
}

// The deep pipeline's forces (by lane) through the same lane compaction: out[qpos[q]] = a2[q].
__global__ __launch_bounds__(TB) void k_lane_pairs(int64_t n, const uint32_t *__restrict__ flag,
                                                   const uint32_t *__restrict__ qpos,
                                                   const double *__restrict__ a2,
                                                   double *__restrict__ out) {
    int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (q < n && flag[q])
        *reinterpret_cast<double2_t *>(out + 2 * (int64_t)qpos[q]) =
            *reinterpret_cast<const double2_t *>(a2 + 2 * q);
}

}  // namespace

void compact_lane_pairs(int64_t n, const uint32_t *flag, const uint32_t *qpos, const double *a2,
                        double *out, hipStream_t s) {
    if (n > 0) k_lane_pairs<<<grid_for(n), TB, 0, s>>>(n, flag, qpos, a2, out);
}

hipError_t compact_lanes(int64_t n, const uint32_t *lanes, const uint32_t *keep,
                         const uint32_t *pos, uint32_t *flag, uint32_t *qpos, uint32_t *out,
                         void *tmp, size_t tmp_bytes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_lane_keep<<<grid_for(n), TB, 0, s>>>(n, lanes, keep, flag);
    hipError_t st = rocprim::exclusive_scan(tmp, tmp_bytes, flag, qpos, 0u, (size_t)n,
                                            rocprim::plus<uint32_t>(), s);
    if (st != hipSuccess) return st;
    k_lane_compact<<<grid_for(n), TB, 0, s>>>(n, lanes, flag, qpos, pos, out);
    return hipGetLastError();
}

void kick_drift(int64_t n, const double *a2, double *x, double *y, double *vx, double *vy,
                double dtHalf, double dt, hipStream_t s, const uint32_t *lanes, GatherLayout gl,
                unsigned long long *vmax) {
    if (n > 0)
        k_kick_drift<<<grid_for(n), TB, 0, s>>>(n, a2, x, y, vx, vy, dtHalf, dt, lanes, gl, vmax);
}

void kick_drift_keys(int64_t n, const double *a2, double *x, double *y, double *vx, double *vy,
                     const uint32_t *cidx, double dtHalf, double dt, const uint32_t *lanes,
                     const Geometry &g, const MortonFuse &mf, hipStream_t s) {
    if (n > 0)
        k_kick_drift_keys<<<grid_for(n), TB, 0, s>>>(n, a2, x, y, vx, vy, cidx, dtHalf, dt, lanes,
                                                     g, mf);
}

void copy_trav_inputs(int64_t n, const double *m, double *m_t, const uint32_t *cidx,
                      uint32_t *cidx_t, const uint32_t *lanes, uint32_t *lanes_t,
                      const uint32_t *T, uint32_t *T_t, hipStream_t s, MergePair *box) {
    k_trav_inputs<<<grid_for(n > 0 ? n : 1), TB, 0, s>>>(n, m, m_t, cidx, cidx_t, lanes, lanes_t,
                                                          T, T_t,
                                                          reinterpret_cast<uint32_t *>(box));
}

void kick(int64_t n, const double *a2, double *vx, double *vy, double dtHalf, hipStream_t s,
          const uint32_t *lanes, GatherLayout gl) {
    if (n > 0) k_kick<<<grid_for(n), TB, 0, s>>>(n, a2, vx, vy, dtHalf, lanes, gl);
}

void iota_u32(uint32_t *p, int64_t n, hipStream_t s) {
    if (n > 0) k_iota<<<grid_for(n), TB, 0, s>>>(p, n);
}

void scatter_to_caller(int64_t n, const uint32_t *cidx, int k, const double *const *src,
                       double *const *dst, hipStream_t s) {
    if (n <= 0) return;
    Ptrs5 p{};
    for (int j = 0; j < k && j < 5; ++j) {
        p.src[j] = src[j];
        p.dst[j] = dst[j];
    }
    k_scatter_caller<<<grid_for(n), TB, 0, s>>>(n, cidx, k < 5 ? k : 5, p);
}

hipError_t mirror_index(int64_t n, const uint32_t *cidx, uint32_t *keep, uint32_t *pos, void *tmp,
                        size_t tmp_bytes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_mirror_keep<<<grid_for(n), TB, 0, s>>>(n, cidx, keep);
    hipError_t st = rocprim::exclusive_scan(tmp, tmp_bytes, keep, pos, 0u, (size_t)n,
                                            rocprim::plus<uint32_t>(), s);
    if (st != hipSuccess) return st;
    return hipGetLastError();
}

void mirror_survivors(int64_t n, const uint32_t *keep, const uint32_t *pos, const uint32_t *scalars,
                      uint32_t *out, hipStream_t s) {
    k_mirror_survivors<<<grid_for(n > MIRROR_HDR ? n : (int64_t)MIRROR_HDR), TB, 0, s>>>(
        n, keep, pos, scalars, out);
}

void copy_u32(uint32_t *dst, const uint32_t *src, hipStream_t s) {
    k_copy_u32<<<1, 1, 0, s>>>(dst, src);
}

__global__ void k_take_u32(uint32_t *dst, uint32_t *src, uint32_t set) {
    *dst |= *src | set;
    *src = 0u;
}

void take_u32(uint32_t *dst, uint32_t *src, hipStream_t s, uint32_t set) {
    k_take_u32<<<1, 1, 0, s>>>(dst, src, set);
}

__global__ __launch_bounds__(TB) void k_pack_readback(const uint32_t *__restrict__ scal,
                                                      const uint32_t *__restrict__ hdr,
                                                      const uint32_t *__restrict__ dlog,
                                                      uint32_t ahead, uint32_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    if (i >= 16u + ahead) return;
    uint32_t v = 0u;
    if (i < 4u) v = scal[i];
    else if (i < 12u) v = hdr[i - 4u];
    else if (i == 12u) v = scal[8];
    else if (i >= 16u) v = dlog[i - 16u];
    out[i] = v;
}

void pack_readback(const uint32_t *scal, const MergePair *box, const uint32_t *dlog, uint32_t ahead,
                   uint32_t *out, hipStream_t s) {
    static_assert(sizeof(MergeHeader) == 8 * sizeof(uint32_t), "header words");
    k_pack_readback<<<grid_for(16 + (int64_t)ahead), TB, 0, s>>>(
        scal, reinterpret_cast<const uint32_t *>(box), dlog, ahead, out);
}

void mirror_scatter(int64_t n, const uint32_t *cidx, const uint32_t *pos, int k,
                    const double *const *src, double *const *dst, hipStream_t s) {
    if (n <= 0) return;
    Ptrs5 p{};
    for (int j = 0; j < k && j < 5; ++j) {
        p.src[j] = src[j];
        p.dst[j] = dst[j];
    }
    k_mirror_scatter<<<grid_for(n), TB, 0, s>>>(n, cidx, pos, k < 5 ? k : 5, p);
}

void scatter_acc_to_caller(int64_t n, const uint32_t *cidx, const double *a2, double *ax,
                           double *ay, hipStream_t s, const uint32_t *lanes, GatherLayout gl) {
    if (n > 0) k_scatter_acc<<<grid_for(n), TB, 0, s>>>(n, cidx, a2, ax, ay, lanes, gl);
}

void merge_candidates(int64_t n, const double *x, const double *y, const double *m,
                      const uint32_t *cidx, double thr, double minD2, uint32_t *heavy,
                      MergePair *box, uint32_t cap, hipStream_t s, bool header_zeroed,
                      const uint32_t *heavy_count) {
    if (!header_zeroed) (void)hipMemsetAsync(box, 0, sizeof(MergeHeader), s);
    if (n <= 0) return;
    MergeHeader *hdr = reinterpret_cast<MergeHeader *>(box);
    if (!heavy_count) k_heavy<<<grid_for(n), TB, 0, s>>>(n, m, cidx, thr, heavy, hdr);
    k_candidates<<<grid_for(n), TB, 0, s>>>(n, x, y, m, cidx, heavy, minD2, box, cap,
                                            heavy_count);
}

void merge_replay(const MergePair *box, uint32_t cap, double *m, uint32_t *cidx, uint32_t *scal,
                  uint32_t *dlog, uint64_t *skeys, uint32_t *sidx, uint32_t *bits,
                  uint32_t *slot_of, int64_t n, hipStream_t s, uint32_t *heavy_count) {
    int key_bits = 1;  // caller indices are < n
    while (key_bits < 32 && (int64_t(1) << key_bits) < n) ++key_bits;
    k_merge_replay<<<1, REPLAY_TB, 0, s>>>(box, cap, m, cidx, scal, dlog, skeys, sidx, bits,
                                           slot_of, key_bits, heavy_count);
}

size_t compact_scratch_bytes(int64_t n) {
    size_t b = 0;
    (void)rocprim::exclusive_scan(nullptr, b, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u,
                                  (size_t)n, rocprim::plus<uint32_t>());
    return b;
}

void compact_pair(int64_t n, const uint32_t *keep, const uint32_t *pos, const double *sx,
                  const double *sy, double *dx, double *dy, hipStream_t s) {
    if (n > 0) k_compact_pair<<<grid_for(n), TB, 0, s>>>(n, keep, pos, sx, sy, dx, dy);
}

hipError_t compact_state(int64_t n, uint32_t *keep, const BodyState &src, const BodyState &dst,
                         const uint32_t *dead_cidx, uint32_t n_dead, uint32_t *pos, void *tmp,
                         size_t tmp_bytes, hipStream_t s) {
    k_keep<<<grid_for(n), TB, 0, s>>>(n, src.cidx, keep);
    hipError_t st = rocprim::exclusive_scan(tmp, tmp_bytes, keep, pos, 0u, (size_t)n,
                                            rocprim::plus<uint32_t>(), s);
    if (st != hipSuccess) return st;
    k_compact<<<grid_for(n), TB, 0, s>>>(n, keep, pos, src, dst, dead_cidx, n_dead);
    return hipGetLastError();
}

}  // namespace bh
