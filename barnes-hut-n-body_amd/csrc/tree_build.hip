// Quadtree build on the GPU — replaces BHTree.insert/insertIntoChild/subdivide/computeMass
// and PhysicsEngine.buildTree (BHA:125-202, BHA:359-366).
//
// Why a sort reproduces the reference's serial insertion: a PR-quadtree with <= 1 body per
// leaf is a pure function of the point set — a cell is subdivided iff >= 2 bodies reach it,
// and the child a body goes to is chosen by `x < cx`, `y < cy` against exact cell centres
// (BHA:153-154).  So every body's root-to-leaf path is its Morton key, computed here by the
// same exact comparisons (never by a rounding division).  The one order-dependent part of
// the reference — the deterministic jitter applied when a cell with h < 1e-3 is subdivided
// (BHA:146-151), which mutates positions and can drop bodies — is confined to the cells at
// the first depth J with h < 1e-3 that hold >= 2 bodies.  Those "jitter cells" are replayed
// exactly, in caller-list order, by one thread each (jitter_run).
//
// Pipeline (all on one stream, no host synchronisation):
//   k_morton     keys (2 bits per level, J levels) + slot payload
//   sort         (stable; bucket sort from the previous order) -> keys_s, perm
//   k_prep       state permuted into the new Morton order; c(a) = common digit count of
//                neighbours; node slot counts
//   exclusive scan                            -> base (pre-order slot of each body's nodes)
//   k_cells      first sorted body of every depth-D0 cell
//   k_emit_com   per 1024-body chunk, in LDS: internal node skeletons (depth, next) + leaf
//                records, replay of BHA:125-156 inside each jitter cell, centre of mass
//                bottom-up (children 0..3 in order, BHA:184-200) of the chunk-local nodes
//   k_span_*     the chunk-spanning nodes, levels J..0
#include <cstdlib>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/block/block_radix_sort.hpp>

#include "bh_device.hpp"

namespace bh {
namespace {

constexpr int TB = 256;

__device__ __forceinline__ int common_digits(uint64_t k1, uint64_t k2, int J) {
    uint64_t d = k1 ^ k2;
    if (d == 0) return J;
    return (__clzll((long long)d) - (64 - 2 * J)) >> 1;
}

// BHA:61-62 evaluated exactly as written.
__device__ __forceinline__ bool quad_contains(double cx, double cy, double h, double x, double y) {
    return x >= cx - h && x < cx + h && y >= cy - h && y < cy + h;
}

// Cell centre at depth L along the digits of `key` (BHA:73-81 applied L times).
__device__ void cell_centre(const Geometry &g, uint64_t key, int L, double &cx, double &cy) {
    cx = g.root_cx;
    cy = g.root_cy;
    for (int d = 0; d < L; ++d) {
        int digit = (int)((key >> (2 * (g.J - 1 - d))) & 3u);
        double hh = g.h[d + 1];
        cx = (digit & 1) ? cx + hh : cx - hh;
        cy = (digit & 2) ? cy + hh : cy - hh;
    }
}

__global__ __launch_bounds__(TB) void k_morton(int64_t n, const double *__restrict__ x,
                                               const double *__restrict__ y,
                                               const uint32_t *__restrict__ cidx, Geometry g,
                                               uint64_t *__restrict__ keys,
                                               uint32_t *__restrict__ keys32,
                                               uint32_t *__restrict__ idx) {
    chain_prio();
    int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = morton_key(g, x[i], y[i], (cidx[i] & CIDX_DEAD) != 0u);
    keys[i] = key;
    keys32[i] = (uint32_t)(key >> key32_shift(g.J));  // the sort key: top 32 of 2J+1 bits
    if (idx) idx[i] = (uint32_t)i;  // rocprim path only (the bucket sort uses the slot itself)
}

// ---- adaptive bucket sort of the 32-bit key prefixes -----------------------------------
// The state is kept in the Morton order of the previous build, so this build's keys arrive
// nearly sorted: bodies drift a few depth-16 cells per step, a few cross a high-level cell
// boundary and jump far in the order.  The previous build's sorted order supplies splitters:
// spl[t] = (key32 << 32 | slot) of its sorted position t * SORT_B, a sorted sequence of
// composites.  Sorting by the composite (key32, slot) IS the stable sort of key32 (ties in
// slot order), so buckets [spl[t], spl[t+1]) partition it exactly whatever the bucket sizes
// are, and each bucket is sorted on its own:
//   k_morton_count    key and bucket of every element (galloping from its old position's
//                     bucket), wave-aggregated atomic count -> offset inside the bucket
//   exclusive scan    bucket starts
//   k_bucket_scatter  composites to their bucket's range (any order inside it)
//   k_bucket_sort     one workgroup per bucket: bitonic sort in LDS (global memory for a
//                     bucket above SORT_CAP -- correct, slow, never seen in smooth evolution),
//                     then keys32_s, perm and the full keys keys_s = keys[perm]
// Splitters are (re)written by k_prep of every build; the first build after a reset uses
// rocprim (the splitters would describe other bodies).
constexpr int SORT_TB = 256;
#ifndef BH_SORT_CAP
#define BH_SORT_CAP 2048
#endif
constexpr int SORT_CAP = BH_SORT_CAP;  // LDS bucket capacity (16 KB of composites; 4 x SORT_B)

// k_morton and k_bucket_count in one launch (a build whose keys the drifting traversal did not
// compute: the overlapped next tree, a build after a reset with splitters): the same index space
// (TB == SORT_TB), the key kept in a register between the two.
__global__ __launch_bounds__(SORT_TB) void k_morton_count(int64_t n, const double *__restrict__ x,
                                                          const double *__restrict__ y,
                                                          const uint32_t *__restrict__ cidx,
                                                          Geometry g, uint64_t *__restrict__ keys,
                                                          uint32_t *__restrict__ keys32,
                                                          const uint64_t *__restrict__ spl,
                                                          uint32_t nb, uint32_t *__restrict__ bkt,
                                                          uint32_t *__restrict__ off,
                                                          uint32_t *__restrict__ counts) {
    chain_prio();
    const int64_t i = (int64_t)blockIdx.x * SORT_TB + threadIdx.x;
    const bool valid = i < n;
    uint32_t k32 = 0;
    if (valid) {
        const uint64_t key = morton_key(g, x[i], y[i], (cidx[i] & CIDX_DEAD) != 0u);
        k32 = (uint32_t)(key >> key32_shift(g.J));
        keys[i] = key;
        keys32[i] = k32;
    }
    uint32_t b = 0;
    const int64_t i0 = (int64_t)blockIdx.x * SORT_TB + (threadIdx.x & ~63u);
    const uint32_t t = __builtin_amdgcn_readfirstlane(min((uint32_t)(i0 / SORT_B), nb - 1));
    const uint64_t lo_s = t == 0 ? 0ull : spl[t];
    const uint64_t hi_s = t + 1 < nb ? spl[t + 1] : ~0ull;
    if (valid) {
        const uint64_t v = ((uint64_t)k32 << 32) | (uint64_t)i;
        if (lo_s <= v && (v < hi_s || t + 1 == nb)) b = t;
        else b = find_bucket(spl, nb, v, (uint32_t)(i / SORT_B));
    }
    if (!valid) return;
    const uint32_t myoff = bucket_offset(b, counts);
    bkt[i] = b;
    off[i] = myoff;
}

__global__ __launch_bounds__(SORT_TB) void k_bucket_scatter(int64_t n,
                                                            const uint32_t *__restrict__ keys32,
                                                            const uint32_t *__restrict__ bkt,
                                                            const uint32_t *__restrict__ off,
                                                            const uint32_t *__restrict__ starts,
                                                            uint64_t *__restrict__ comp) {
    chain_prio();
    const int64_t i = (int64_t)blockIdx.x * SORT_TB + threadIdx.x;
    if (i >= n) return;
    comp[starts[bkt[i]] + off[i]] = ((uint64_t)keys32[i] << 32) | (uint64_t)i;
}

// Bitonic network in its all-ascending form (the first step of every merge compares mirrored
// pairs): a comparator never moves the larger value down, so the elements past `s` can stay
// virtual +infinity -- sizes need no padding.  `A` is LDS or global memory of this workgroup.
// (Measured at C4: batching a stage's loads, and skipping the barrier between stages whose
// pairs stay inside one wave's 128-element block, were both slower than this plain form.)
template <bool LDS>
__device__ __forceinline__ void bitonic_sort(uint64_t *A, uint32_t s) {
    int lP = 0;
    while ((1u << lP) < s) ++lP;
    const uint32_t half = (1u << lP) >> 1;
    for (int lk = 1; lk <= lP; ++lk) {
        for (int lj = lk - 1; lj >= 0; --lj) {
            const uint32_t j = 1u << lj;
            const uint32_t flip = lj == lk - 1 ? (1u << lk) - 1 : 0u;  // mirrored partner
            for (uint32_t q = threadIdx.x; q < half; q += SORT_TB) {
                const uint32_t lo = ((q >> lj) << (lj + 1)) | (q & (j - 1));  // bit lj clear
                const uint32_t hi = flip ? (lo ^ flip) : (lo | j);
                if (hi < s) {
                    const uint64_t a = A[lo], c = A[hi];
                    if (c < a) {
                        A[lo] = c;
                        A[hi] = a;
                    }
                }
            }
            if (!LDS) __threadfence_block();
            __syncthreads();
        }
    }
}

// Buckets of up to RADIX_CAP elements: one counting pass on the top 8 bits of the key
// prefix's span inside the bucket (bins are key ranges, so bins in order are sorted relative
// to each other), then every element's rank inside its bin -- bins hold a few elements, ties
// of equal prefixes included, ordered by the whole composite.  A bin above RADIX_MAXBIN
// (clustered keys) sends the bucket to the bitonic network instead.
constexpr int RADIX_CAP = SORT_CAP / 2;  // the bin-grouped copy lives in the upper half of L
constexpr int RADIX_BINS = 256;
constexpr uint32_t RADIX_MAXBIN = 48;
// A bucket whose key prefixes are all equal (the dead bodies' sentinel run -- the LET subset's
// padding --, or a dense depth-16 cell) is binned by its slots instead: the composites' order is
// then the slot order, and the bins are slot ranges.
#ifndef BH_SORT_SLOT_RADIX
#define BH_SORT_SLOT_RADIX 1
#endif
// Any other bucket of up to SORT_CAP elements (keys clustered in a few bins -- a bucket that
// spans a gap of the subset's key ranges --, or above RADIX_CAP -- the bucket that new halo
// cells fall into after a drift): an LDS radix sort of its composites compressed to the bits
// they span, (key32 - min) : (slot - min); else the bitonic network.
#ifndef BH_SORT_BLOCK_RADIX
#define BH_SORT_BLOCK_RADIX 1
#endif
using BucketRadix = rocprim::block_radix_sort<unsigned long long, SORT_TB, SORT_CAP / SORT_TB>;
// Buckets of up to BH_SORT_BITONIC_MAX elements that the bin radix cannot take go to the bitonic
// network instead of the block radix sort.
#ifndef BH_SORT_BITONIC_MAX
#define BH_SORT_BITONIC_MAX 0
#endif
// Buckets of up to BH_SORT_RANK_MAX elements (a multiple of SORT_TB) that the bin radix cannot
// take -- a few per build, whose key span holds an outlier: all but one element in one bin -- are
// sorted by counting each element's rank in LDS instead of the block radix sort (0: off).
#ifndef BH_SORT_RANK_MAX
#define BH_SORT_RANK_MAX 1024
#endif
static_assert(BH_SORT_RANK_MAX % SORT_TB == 0 && BH_SORT_RANK_MAX <= SORT_CAP, "rank sort size");

#ifdef BH_SORT_STATS  // diagnostic build: which path each bucket took (radix / bitonic / global)
__device__ unsigned long long g_sort_stats[8];
// per launch (ring of SORT_LOG): largest bucket, buckets through the LDS bitonic network, through
// the global one, elements of the latter
constexpr int SORT_LOG = 256;
__device__ unsigned long long g_sort_log[SORT_LOG][4];
#define SORT_STAT(q, v) (threadIdx.x == 0 ? (void)atomicAdd(&g_sort_stats[(q)], (unsigned long long)(v)) : (void)0)
#define SORT_LOGV(q, v) (threadIdx.x == 0 ? (void)atomicAdd(&g_sort_log[seq % SORT_LOG][(q)], (unsigned long long)(v)) : (void)0)
#else
#define SORT_STAT(q, v) (void)0
#define SORT_LOGV(q, v) (void)0
#endif
__global__ __launch_bounds__(SORT_TB) void k_bucket_sort(const uint32_t *__restrict__ starts,
                                                         uint32_t *__restrict__ counts,
                                                         uint64_t *comp,
                                                         const uint64_t *__restrict__ keys,
                                                         uint32_t *__restrict__ keys32_s,
                                                         uint32_t *__restrict__ perm,
                                                         uint64_t *keys_s, uint32_t seq) {
    chain_prio();
    (void)seq;
    __shared__ union {
        uint64_t L[SORT_CAP];
        BucketRadix::storage_type brs;  // (after L is read into registers)
    } shm;
    uint64_t *L = shm.L;
    __shared__ uint32_t s_cnt[RADIX_BINS], s_start[RADIX_BINS];
    __shared__ uint32_t s_min, s_max, s_maxbin, s_smin, s_smax;
    const uint32_t t = blockIdx.x;
    const uint32_t b0 = starts[t], s = starts[t + 1] - b0;
    if (threadIdx.x == 0) counts[t] = 0;  // ready for the next build (counts were scanned)
#ifdef BH_SORT_STATS
    if (threadIdx.x == 0) atomicMax(&g_sort_log[seq % SORT_LOG][0], (unsigned long long)s);
#endif
    auto emit = [&](uint32_t j, uint64_t v) __attribute__((always_inline)) {
        const uint32_t src = (uint32_t)v;
        keys32_s[b0 + j] = (uint32_t)(v >> 32);
        perm[b0 + j] = src;
        keys_s[b0 + j] = keys[src];  // comp and keys_s share storage: L holds the bucket
    };
    if (s <= (uint32_t)SORT_CAP) {
        if (threadIdx.x == 0) {
            s_min = s_smin = 0xFFFFFFFFu;
            s_max = s_smax = 0;
            s_maxbin = 0;
        }
        if (threadIdx.x < RADIX_BINS) s_cnt[threadIdx.x] = 0;
        __syncthreads();
        uint32_t kmin = 0xFFFFFFFFu, kmax = 0, smin = 0xFFFFFFFFu, smax = 0;
        for (uint32_t j = threadIdx.x; j < s; j += SORT_TB) {
            const uint64_t v = comp[b0 + j];
            L[j] = v;
            kmin = min(kmin, (uint32_t)(v >> 32));
            kmax = max(kmax, (uint32_t)(v >> 32));
            smin = min(smin, (uint32_t)v);
            smax = max(smax, (uint32_t)v);
        }
        bool radix = s <= (uint32_t)RADIX_CAP;
        const bool need_minmax = radix || BH_SORT_BLOCK_RADIX;
        const bool need_slots = BH_SORT_SLOT_RADIX || BH_SORT_BLOCK_RADIX;
        if (need_minmax) {  // wave minima / maxima first: one LDS atomic per wave
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o, 64));
                kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
                if (need_slots) {
                    smin = min(smin, (uint32_t)__shfl_xor((int)smin, o, 64));
                    smax = max(smax, (uint32_t)__shfl_xor((int)smax, o, 64));
                }
            }
            if ((threadIdx.x & 63) == 0) {
                atomicMin(&s_min, kmin);
                atomicMax(&s_max, kmax);
                if (need_slots) {
                    atomicMin(&s_smin, smin);
                    atomicMax(&s_smax, smax);
                }
            }
        }
        __syncthreads();
        if (radix) {
            // (uniform) equal prefixes: bin by slot (the low half of the composite)
            const bool by_slot = BH_SORT_SLOT_RADIX && s_min == s_max;
            const int hs = by_slot ? 0 : 32;
            const uint32_t lo = by_slot ? s_smin : s_min;
            const uint32_t span = by_slot ? s_smax - s_smin : s_max - s_min;
            const int shift = span >= RADIX_BINS ? (32 - __clz(span)) - 8 : 0;  // span >> shift < 256
            uint32_t bin[RADIX_CAP / SORT_TB], off[RADIX_CAP / SORT_TB];
#pragma unroll
            for (int r = 0; r < RADIX_CAP / SORT_TB; ++r) {
                const uint32_t j = threadIdx.x + r * SORT_TB;
                if (j < s) {
                    bin[r] = ((uint32_t)(L[j] >> hs) - lo) >> shift;
                    off[r] = atomicAdd(&s_cnt[bin[r]], 1u);
                }
            }
            __syncthreads();
            static_assert(RADIX_BINS == SORT_TB, "one bin per thread");
            {  // inclusive scan of the bin counts: within each wave by shuffles, then wave sums
                const uint32_t c = s_cnt[threadIdx.x];
                atomicMax(&s_maxbin, c);
                const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
                uint32_t v = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t u = __shfl_up(v, d, 64);
                    if (lane >= d) v += u;
                }
                if (lane == 63) s_start[w] = v;  // wave totals (slots 0..3, rewritten below)
                __syncthreads();
                uint32_t add = 0;
                for (int q = 0; q < w; ++q) add += s_start[q];
                __syncthreads();
                s_start[threadIdx.x] = v + add;
            }
            __syncthreads();
            radix = s_maxbin <= RADIX_MAXBIN;  // uniform
            if (radix) {
                uint64_t *G = L + RADIX_CAP;  // bin-grouped copy
#pragma unroll
                for (int r = 0; r < RADIX_CAP / SORT_TB; ++r) {
                    const uint32_t j = threadIdx.x + r * SORT_TB;
                    if (j < s) G[s_start[bin[r]] - s_cnt[bin[r]] + off[r]] = L[j];
                }
                __syncthreads();
#pragma unroll
                for (int r = 0; r < RADIX_CAP / SORT_TB; ++r) {
                    const uint32_t j = threadIdx.x + r * SORT_TB;
                    if (j < s) {
                        const uint32_t be = s_start[bin[r]], bs = be - s_cnt[bin[r]];
                        const uint64_t v = L[j];
                        uint32_t rank = 0;
                        for (uint32_t q = bs; q < be; ++q) rank += G[q] < v ? 1u : 0u;
                        emit(bs + rank, v);
                    }
                }
                SORT_STAT(0, 1);
                SORT_STAT(1, s);
                return;
            }
        }
        SORT_STAT(2, 1);
        SORT_STAT(3, s);
        SORT_LOGV(1, 1);
        if (s <= (uint32_t)BH_SORT_RANK_MAX) {
            // every element's rank = the number of smaller composites (distinct: the slot is in
            // them), counted against the whole bucket in LDS -- broadcast reads, no barriers
            constexpr int RPT = BH_SORT_RANK_MAX > 0 ? BH_SORT_RANK_MAX / SORT_TB : 1;
            uint64_t v[RPT];
            uint32_t r[RPT];
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const uint32_t j = threadIdx.x + q * SORT_TB;
                v[q] = j < s ? L[j] : 0ull;
                r[q] = 0;
            }
#pragma unroll 4
            for (uint32_t j = 0; j < s; ++j) {
                const uint64_t u = L[j];
#pragma unroll
                for (int q = 0; q < RPT; ++q) r[q] += u < v[q] ? 1u : 0u;
            }
#pragma unroll
            for (int q = 0; q < RPT; ++q)
                if (threadIdx.x + q * SORT_TB < s) emit(r[q], v[q]);
            return;
        }
        if (BH_SORT_BLOCK_RADIX && s > (uint32_t)BH_SORT_BITONIC_MAX) {
            constexpr int IPT = SORT_CAP / SORT_TB;
            const uint32_t kmn = s_min, smn = s_smin;
            const uint32_t kspan = s_max - kmn, sspan = s_smax - smn;
            const int sb = sspan ? 32 - __clz(sspan) : 0;  // bits of the slot offset
            const int kb = kspan ? 32 - __clz(kspan) : 0;
            uint64_t v[IPT];  // blocked: thread t holds elements t * IPT + q
#pragma unroll
            for (int q = 0; q < IPT; ++q) {
                const uint32_t j = threadIdx.x * IPT + q;
                const uint64_t c = L[min(j, s - 1)];
                v[q] = j < s ? ((uint64_t)((uint32_t)(c >> 32) - kmn) << sb) |
                                   (uint64_t)((uint32_t)c - smn)
                             : ~0ull;  // past the bucket: last (stable: after every element)
            }
            __syncthreads();  // L is read: its storage becomes the sort's
            BucketRadix().sort(reinterpret_cast<unsigned long long(&)[IPT]>(v), shm.brs, 0u,
                               (unsigned)max(kb + sb, 1));
            const uint64_t smask = sb ? (~0ull >> (64 - sb)) : 0ull;
#pragma unroll
            for (int q = 0; q < IPT; ++q) {
                const uint32_t j = threadIdx.x * IPT + q;
                if (j < s)
                    emit(j, ((uint64_t)((uint32_t)(v[q] >> sb) + kmn) << 32) |
                                (uint64_t)((uint32_t)(v[q] & smask) + smn));
            }
            return;
        }
        bitonic_sort<true>(L, s);
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < s; j += SORT_TB) emit(j, L[j]);
    } else {  // oversized bucket: the same network on global memory, in place
        SORT_STAT(4, 1);
        SORT_STAT(5, s);
        SORT_LOGV(2, 1);
        SORT_LOGV(3, s);
        uint64_t *A = comp + b0;
        bitonic_sort<false>(A, s);
        for (uint32_t j = threadIdx.x; j < s; j += SORT_TB) emit(j, A[j]);  // own j: in place
    }
}

// After the 32-bit-prefix sort: keys_s = keys[perm] (k_key_gather), then every run of equal
// prefixes (bodies sharing a depth-16 cell — short: at most 5 in C3) re-sorted by (full key,
// original index) by the thread of its first element (k_key_fixup), so the result equals a
// stable sort of the full keys.  The run of out-of-root / merged-away bodies (one shared
// sentinel key) is already in index order and is left alone.
__global__ __launch_bounds__(TB) void k_key_gather(int64_t n, const uint64_t *__restrict__ keys,
                                                   const uint32_t *__restrict__ perm,
                                                   uint64_t *__restrict__ keys_s) {
    chain_prio();
    const int64_t a = (int64_t)xcd_block() * TB + threadIdx.x;
    if (a < n) keys_s[a] = keys[perm[a]];
}

__device__ __forceinline__ void key_fixup(int64_t a, int64_t n, int J,
                                          const uint32_t *__restrict__ keys32_s,
                                          uint64_t *__restrict__ keys_s,
                                          uint32_t *__restrict__ perm) {
    if (a + 1 >= n) return;
    const uint32_t k = keys32_s[a];
    if (keys32_s[a + 1] != k || (a > 0 && keys32_s[a - 1] == k)) return;  // not a run start
    if (k == (uint32_t)(sentinel_key(J) >> key32_shift(J))) return;        // sentinel run
    int64_t e = a + 2;
    while (e < n && keys32_s[e] == k) ++e;
    for (int64_t i = a + 1; i < e; ++i) {  // insertion sort by (full key, original index)
        const uint64_t ki = keys_s[i];
        const uint32_t pi = perm[i];
        int64_t j = i;
        while (j > a && (keys_s[j - 1] > ki || (keys_s[j - 1] == ki && perm[j - 1] > pi))) {
            keys_s[j] = keys_s[j - 1];
            perm[j] = perm[j - 1];
            --j;
        }
        keys_s[j] = ki;
        perm[j] = pi;
    }
}

__global__ __launch_bounds__(TB) void k_key_fixup(int64_t n, int J,
                                                  const uint32_t *__restrict__ keys32_s,
                                                  uint64_t *__restrict__ keys_s,
                                                  uint32_t *__restrict__ perm) {
    chain_prio();
    key_fixup((int64_t)blockIdx.x * TB + threadIdx.x, n, J, keys32_s, keys_s, perm);
}

struct HeavyList {  // TreeBuffers::heavy (null list: not wanted)
    uint32_t *list, *count;
    double thr;
};

// k_prep's body for one sorted body a < n: the state gathered into the new order, the splitters,
// the old -> new slot map, c(a) and the node count (returned); the heavy list
__device__ __forceinline__ uint32_t prep_one(int64_t a, int64_t n, int J,
                                             const uint64_t *__restrict__ keys_s,
                                             const uint32_t *__restrict__ perm, BodyState src,
                                             BodyState dst, int8_t *__restrict__ cpl,
                                             uint32_t *__restrict__ cnt,
                                             uint64_t *__restrict__ spl,
                                             uint32_t *__restrict__ inv, const HeavyList &hl) {
    const uint64_t SENT = sentinel_key(J);
    uint64_t k = keys_s[a];
    uint32_t i = perm[a];  // nearly the identity: the state is kept in the last Morton order
    inv[i] = (uint32_t)a;  // old slot -> new slot (carries the traversal's lane map, lane_order)
    if (a % SORT_B == 0)  // splitters of the next build's bucket sort
        spl[a / SORT_B] = ((k >> key32_shift(J)) << 32) | (uint64_t)a;
    dst.x[a] = src.x[i];
    dst.y[a] = src.y[i];
    // null: the velocities are still being written (the pipelined step) / a subset build carries
    // only the replicated slot in vx (LET)
    if (src.vx) dst.vx[a] = src.vx[i];
    if (src.vy) dst.vy[a] = src.vy[i];
    const double mi = src.m[i];
    const uint32_t ci = src.cidx[i];
    dst.m[a] = mi;
    dst.cidx[a] = ci;
    // the merge rule's heavy bodies in this order (k_heavy's test, BHA:474): masses change only in
    // the merge rule, so the list stays right until the rule that follows this build has run
    if (hl.list && mi > hl.thr && !(ci & CIDX_DEAD)) hl.list[atomicAdd(hl.count, 1u)] = (uint32_t)a;
    int c_cur = -1, c_prev = -1;
    if (k != SENT) {
        if (a + 1 < n) {
            uint64_t k2 = keys_s[a + 1];
            if (k2 != SENT) c_cur = common_digits(k, k2, J);
        }
        if (a > 0) c_prev = common_digits(keys_s[a - 1], k, J);
    }
    cpl[a] = (int8_t)c_cur;
    // internal nodes starting at a: depths c_prev+1 .. c_cur; plus a's leaf.
    const uint32_t c = (k == SENT) ? 0u : 1u + (uint32_t)max(0, c_cur - c_prev);
    cnt[a] = c;
    return c;
}

// The base scan (BH_BASE_SCAN): k_prep also sums its tile's counts into tsum[tile], and
// k_base_scan turns counts and tile sums into base -- two launches without inter-block waits in
// place of rocprim's lookback state initialisation and scan.
#ifndef BH_BASE_SCAN
#define BH_BASE_SCAN 1
#endif
constexpr int BS_TB = 1024;  // k_base_scan: BS_TB * PER counts per block

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__global__ __launch_bounds__(TB) void k_prep(int64_t n, int J, const uint64_t *__restrict__ keys_s,
                                             const uint32_t *__restrict__ perm, BodyState src,
                                             BodyState dst, int8_t *__restrict__ cpl,
                                             uint32_t *__restrict__ cnt,
                                             uint64_t *__restrict__ spl,
                                             uint32_t *__restrict__ inv,
                                             uint32_t *__restrict__ tsum, HeavyList hl) {
    chain_prio();
    const uint32_t tile = xcd_block();
    const int64_t a = (int64_t)tile * TB + threadIdx.x;
    uint32_t c = 0;
    if (a < n) c = prep_one(a, n, J, keys_s, perm, src, dst, cpl, cnt, spl, inv, hl);
    else if (a == n) cnt[n] = 0;
    if (tsum) {  // the tile's count sum for k_base_scan
        __shared__ uint32_t s_w[TB / 64];
        c = wave_sum_u32(c);
        if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
#pragma unroll
            for (int w = 0; w < TB / 64; ++w) t += s_w[w];
            tsum[tile] = t;
        }
    }
}

// base[i] = sum cnt[0..i) for i < n1: block b takes BS_TB * PER consecutive counts, its
// prefix the sum of the tile sums before them
template <int PER>
__global__ __launch_bounds__(BS_TB) void k_base_scan(int64_t n1, const uint32_t *__restrict__ cnt,
                                                     const uint32_t *__restrict__ tsum,
                                                     uint32_t *__restrict__ base) {
    chain_prio();
    __shared__ uint32_t s_w[BS_TB / 64];
    __shared__ uint32_t s_pre;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the prefix: tile sums [0, TILES * blockIdx.x)
    constexpr uint32_t TILES = BS_TB * PER / TB;
    uint32_t p = 0;
    for (uint32_t t = threadIdx.x; t < TILES * blockIdx.x; t += BS_TB) p += tsum[t];
    p = wave_sum_u32(p);
    if (lane == 0) s_w[w] = p;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < BS_TB / 64; ++k) t += s_w[k];
        s_pre = t;
    }
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * (BS_TB * PER) + (int64_t)threadIdx.x * PER;
    uint32_t v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) v[j] = i0 + j < n1 ? cnt[i0 + j] : 0u;
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) sum += v[j];
    uint32_t inc = sum;  // the wave's inclusive scan of the threads' sums
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += u;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t wpre = s_pre;
    for (uint32_t k = 0; k < w; ++k) wpre += s_w[k];
    uint32_t run = wpre + inc - sum;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (i0 + j < n1) base[i0 + j] = run;
        run += v[j];
    }
}


// First sorted body of every depth-D0 cell (bins 0 .. 4^D0; the sentinel's prefix is 4^D0,
// so bin 4^D0 starts at the first out-of-root body, i.e. at the in-root count).
// Also fills the span super list [0, n_super) with 0xFF bytes for k_span_find (in place of a
// memset launch; nothing reads it before k_span_find).
__device__ __forceinline__ void cells(int64_t bin, int64_t stride, int64_t n, int J, int D0,
                                      const uint64_t *__restrict__ keys_s,
                                      uint32_t *__restrict__ cell_start,
                                      uint32_t *__restrict__ super_list, int64_t n_super) {
    for (int64_t k = bin; k < n_super; k += stride) super_list[k] = 0xFFFFFFFFu;
    const int64_t nbins = (int64_t)1 << (2 * D0);
    if (bin > nbins) return;
    const int shift = 2 * (J - D0);
    int64_t lo = 0, hi = n;  // first index with (key >> shift) >= bin
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((int64_t)(keys_s[mid] >> shift) < bin) lo = mid + 1; else hi = mid;
    }
    cell_start[bin] = (uint32_t)lo;
}

__global__ __launch_bounds__(TB) void k_cells(int64_t n, int J, int D0,
                                              const uint64_t *__restrict__ keys_s,
                                              uint32_t *__restrict__ cell_start,
                                              uint32_t *__restrict__ super_list, int64_t n_super) {
    chain_prio();
    cells((int64_t)blockIdx.x * TB + threadIdx.x, (int64_t)gridDim.x * TB, n, J, D0, keys_s,
          cell_start, super_list, n_super);
}

// k_key_fixup and k_cells in one launch (BH_FIXUP_CELLS): the depth-D0 cell starts depend on the
// 32-bit prefixes only, final before the fixup -- which reorders bodies inside runs of one
// prefix, so a search probing a run mid-reorder compares the same prefix whichever it reads
#ifndef BH_FIXUP_CELLS
#define BH_FIXUP_CELLS 1
#endif
__global__ __launch_bounds__(TB) void k_fixup_cells(int64_t n, int J, int D0,
                                                    const uint32_t *__restrict__ keys32_s,
                                                    uint64_t *__restrict__ keys_s,
                                                    uint32_t *__restrict__ perm,
                                                    uint32_t *__restrict__ cell_start,
                                                    uint32_t *__restrict__ super_list,
                                                    int64_t n_super) {
    chain_prio();
    const int64_t t = (int64_t)blockIdx.x * TB + threadIdx.x;
    cells(t, (int64_t)gridDim.x * TB, n, J, D0, keys_s, cell_start, super_list, n_super);
    key_fixup(t, n, J, keys32_s, keys_s, perm);
}

// ---- the front of a small list's build in one workgroup ----------------------------------
// Up to BH_SMALL_FRONT_MAX (4 096) bodies, the build's first five launches -- the Morton keys,
// the bucket sort's three (bucket starts, scatter, the buckets' sorts), k_fixup_cells, k_prep and
// k_base_scan: ~45 us at C1 'R', each a latency chain after a launch boundary -- run as the phases
// of one 1 024-thread workgroup: the keys; a bitonic network over all composites
// (key32 << 32 | slot) in LDS, the same total order as the bucket sort's (the composites are
// distinct), so the same permutation; then key_fixup, cells and prep_one -- the very functions the
// separate kernels run -- per body, and the exclusive scan of the node counts into base.  It also
// clears the bucket counts the drifting traversal may have made, as k_bucket_sort does for the
// next build.  (The network alone over 16 384 composites -- C1 code -- is bound by one CU's LDS
// bandwidth: ~110 us, C1 code 0.339 -> 0.572 ms per step, profiles/r06s_small_sort_ab.txt.)
constexpr int SF_TB = 1024;
constexpr int64_t SMALL_FRONT_CAP = 4096;  // (P * 8 bytes of LDS: 32 KB)
#ifdef BH_SF_TIMING  // diagnostic build: phase stamps of the last k_small_front launches (ring)
constexpr int SF_T_REC = 64, SF_T_W = 8;
__device__ uint64_t g_sf_times[SF_T_REC * SF_T_W];
__device__ uint32_t g_sf_launch;
#define SF_STAMP(q)                                                                      \
    do {                                                                                 \
        if (threadIdx.x == 0) sf_t[(q)] = wall_clock64();                                 \
    } while (0)
#else
#define SF_STAMP(q) (void)0
#endif
#ifndef BH_SMALL_FRONT_MAX
#define BH_SMALL_FRONT_MAX SMALL_FRONT_CAP
#endif
__global__ __launch_bounds__(SF_TB) void k_small_front(
    int64_t n, uint32_t P, bool need_keys, Geometry g, int D0, BodyState src, BodyState dst,
    uint64_t *__restrict__ keys, uint32_t *__restrict__ keys32, uint32_t *__restrict__ keys32_s,
    uint32_t *__restrict__ perm, uint64_t *__restrict__ keys_s, uint32_t *__restrict__ counts,
    uint32_t nb, uint32_t *__restrict__ cell_start, uint32_t *__restrict__ super_list,
    int64_t n_super, int8_t *__restrict__ cpl, uint32_t *__restrict__ cnt,
    uint64_t *__restrict__ spl, HeavyList hl, uint32_t *__restrict__ base) {
    chain_prio();
    extern __shared__ uint64_t sf_L[];  // P = the power of two >= n, padded with ~0
    __shared__ uint32_t s_w[SF_TB / 64];
#ifdef BH_SF_TIMING
    __shared__ uint64_t sf_t[SF_T_W];
#endif
    const int J = g.J;
    const uint32_t t = threadIdx.x;
    SF_STAMP(0);
    // (k_morton) the keys, or the drifting traversal's
    for (uint32_t i = t; i < P; i += SF_TB) {
        uint64_t v = ~0ull;
        if ((int64_t)i < n) {
            uint32_t k32;
            if (need_keys) {
                const uint64_t key = morton_key(g, src.x[i], src.y[i], (src.cidx[i] & CIDX_DEAD) != 0u);
                k32 = (uint32_t)(key >> key32_shift(J));
                keys[i] = key;
            } else {
                k32 = keys32[i];
            }
            v = ((uint64_t)k32 << 32) | (uint64_t)i;
        }
        sf_L[i] = v;
    }
    for (uint32_t i = t; i <= nb; i += SF_TB) counts[i] = 0u;
    __syncthreads();
    SF_STAMP(1);
    // (the bucket sort) all composites, ascending.  A stage is bound by the LDS (~0.27 us for
    // 2 048 elements with 16 waves; 17.8 us of the front's ~33 at C1 'R', tools/sf_timing.py):
    // skipping the barrier of stages whose pairs stay inside a wave, and keeping the closest
    // stages in registers (fewer threads on the LDS stages), both measured no faster
    // (profiles/r06sk_small_front_sort_variants.txt).
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t q = t; q < P / 2; q += SF_TB) {  // pair (lo, lo + j), bit j of lo clear
                const uint32_t lo = ((q & ~(j - 1)) << 1) | (q & (j - 1));
                const uint32_t hi = lo | j;
                const uint64_t a = sf_L[lo], c = sf_L[hi];
                if ((a > c) == ((lo & k) == 0)) {
                    sf_L[lo] = c;
                    sf_L[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    SF_STAMP(2);
    for (uint32_t a = t; (int64_t)a < n; a += SF_TB) {
        const uint64_t v = sf_L[a];
        const uint32_t i = (uint32_t)v;
        keys32_s[a] = (uint32_t)(v >> 32);
        perm[a] = i;
        keys_s[a] = keys[i];
    }
    __syncthreads();
    SF_STAMP(3);
    // (k_fixup_cells) runs of equal prefixes by (full key, index) -- a run start is found in LDS,
    // only the (rare) starts read the global arrays --; the depth-D0 cell starts, searched in LDS:
    // the depth-D0 prefix is in the 32-bit one (2 (J - D0) >= key32_shift(J)) and the fixup
    // reorders inside runs of one 32-bit prefix only
    for (uint32_t a = t; (int64_t)a + 1 < n; a += SF_TB) {
        const uint32_t k = (uint32_t)(sf_L[a] >> 32);
        if ((uint32_t)(sf_L[a + 1] >> 32) == k && (a == 0 || (uint32_t)(sf_L[a - 1] >> 32) != k))
            key_fixup(a, n, J, keys32_s, keys_s, perm);
    }
    const int sh32 = 2 * (J - D0) - key32_shift(J);
    const int64_t nbins = (int64_t)1 << (2 * D0);
    const int64_t cells_hi = nbins + 1 > n_super ? nbins + 1 : n_super;
    if (sh32 >= 0) {
        for (int64_t k = t; k < n_super; k += SF_TB) super_list[k] = 0xFFFFFFFFu;
        for (int64_t bin = t; bin <= nbins; bin += SF_TB) {
            int64_t lo = 0, hi = n;  // first index with its depth-D0 prefix >= bin (cells())
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if ((int64_t)((uint32_t)(sf_L[mid] >> 32) >> sh32) < bin) lo = mid + 1;
                else hi = mid;
            }
            cell_start[bin] = (uint32_t)lo;
        }
        __syncthreads();
    } else {
        __syncthreads();
        for (int64_t bin = t; bin < cells_hi; bin += SF_TB)
            cells(bin, SF_TB, n, J, D0, keys_s, cell_start, super_list, n_super);
        __syncthreads();
    }
    SF_STAMP(4);
    // (k_prep) the state in the new order, c(a), node counts -- kept in LDS for the scan
    uint32_t *c_l = reinterpret_cast<uint32_t *>(sf_L);  // (n + 1 <= 2 P counts)
    for (uint32_t a = t; (int64_t)a <= n; a += SF_TB) {
        uint32_t c = 0;
        if ((int64_t)a < n) c = prep_one(a, n, J, keys_s, perm, src, dst, cpl, cnt, spl, keys32, hl);
        else cnt[n] = 0;
        c_l[a] = c;
    }
    __syncthreads();
    SF_STAMP(5);
    // (k_base_scan) base[i] = sum cnt[0..i), i <= n: each thread a run of E counts
    const uint32_t n1 = (uint32_t)n + 1u, E = (n1 + SF_TB - 1) / SF_TB;
    const uint32_t i0 = t * E;
    uint32_t sum = 0;
    for (uint32_t e = 0; e < E; ++e)
        if (i0 + e < n1) sum += c_l[i0 + e];
    const uint32_t lane = t & 63u, w = t >> 6;
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += u;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (uint32_t k = 0; k < w; ++k) run += s_w[k];
    for (uint32_t e = 0; e < E; ++e) {
        if (i0 + e < n1) {
            base[i0 + e] = run;
            run += c_l[i0 + e];
        }
    }
#ifdef BH_SF_TIMING
    __syncthreads();
    SF_STAMP(6);
    if (t == 0) {
        const uint32_t r = atomicAdd(&g_sf_launch, 1u) % SF_T_REC;
        for (int q = 0; q < 7; ++q) g_sf_times[r * SF_T_W + q] = sf_t[q];
    }
#endif
}

#ifdef BH_SF_TIMING
extern "C" int bh_debug_sf_times(uint64_t *out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sf_times), sizeof(uint64_t) * SF_T_REC * SF_T_W);
}
#endif

static bool small_front(int64_t n, uint32_t &P) {
    static const int64_t lim = [] {
        const char *v = std::getenv("BH_SMALL_FRONT_MAX");
        const int64_t x = v ? (int64_t)std::atoll(v) : (int64_t)BH_SMALL_FRONT_MAX;
        return x < SMALL_FRONT_CAP ? x : SMALL_FRONT_CAP;
    }();
    if (n <= 0 || n > lim) return false;
    P = 1;
    while ((int64_t)P < n) P <<= 1;
    return true;
}

// Largest e in [from, limit] with (keys_s[e] >> shift) == pref (keys_s[from] matches).
__device__ __forceinline__ int64_t run_end(const uint64_t *__restrict__ keys_s, int64_t limit,
                                           int64_t from, int shift, uint64_t pref) {
    int64_t lo = from, step = 1;
    while (lo + step <= limit && (keys_s[lo + step] >> shift) == pref) {
        lo += step;
        step <<= 1;
    }
    int64_t hi = min(lo + step, limit + 1);  // keys_s[hi] does not match (or hi > limit)
    while (hi - lo > 1) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if ((keys_s[mid] >> shift) == pref) lo = mid; else hi = mid;
    }
    return lo;
}

// c(j) + 1 of a window of WIN sorted positions starting at the chunk's first body, in LDS:
// a node's end is found by a word-wise SWAR scan of the window (most nodes end inside it);
// only nodes that outrun the window gallop over the keys in global memory.
// first j in [from, c0 + WIN) with c(j) < L, or -1; w[i] = c(c0 + i) + 1 in [0, 42];
// wm[k] = min of w over the 8-byte word k, bm[b] = min over the 64-byte block b.  SWAR tests
// on from's word, then on the word minima of the rest of its block, then on the block minima
// locate the first word holding a match: 3 LDS reads per search, at most 5 + WIN / 512 (a node
// near the top of a dense region ends thousands of bodies later; one such lane used to hold
// its wave and, at the phase barrier, its workgroup).
template <int WIN>
__device__ __forceinline__ int64_t lds_scan(const uint64_t *w, const uint64_t *wm,
                                            const uint64_t *bm, int64_t c0, int64_t from, int L) {
    static_assert(WIN % 512 == 0, "whole words of block minima");
    const uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
    const uint64_t sub = ones * (uint64_t)(L + 1);
    auto first = [&](uint64_t x) { return (x - sub) & ~x & highs; };  // bytes with c + 1 < L + 1
    const int64_t o = from - c0;
    if (o >= WIN) return -1;
    // from's word, bytes before `from` raised to 0x7F (>= L + 1): they neither match nor borrow
    const int wi = (int)(o >> 3);
    const uint64_t t0 = first(w[wi] | (~(~0ull << (8 * (o & 7))) & 0x7F7F7F7F7F7F7F7Full));
    if (t0) return c0 + 8 * (int64_t)wi + (__builtin_ctzll(t0) >> 3);
    // the later words of from's block, by their minima; then the matching word itself
    const int blk = wi >> 3;
    const uint64_t lo1 = (wi & 7) == 7 ? ~0ull : ~(~0ull << (8 * ((wi & 7) + 1)));
    const uint64_t t1 = first(wm[blk] | (lo1 & 0x7F7F7F7F7F7F7F7Full));
    int q = -1;
    if (t1) {
        q = 8 * blk + (__builtin_ctzll(t1) >> 3);
    } else {  // later blocks, by their minima
        const int b = blk + 1;
        if (b >= WIN / 64) return -1;
        uint64_t bpad = ~(~0ull << (8 * (b & 7))) & 0x7F7F7F7F7F7F7F7Full;
        for (int bw = b >> 3; bw < WIN / 512; ++bw) {
            const uint64_t t = first(bm[bw] | bpad);
            if (t) {
                const int b2 = 8 * bw + (__builtin_ctzll(t) >> 3);  // the block holds a match
                q = 8 * b2 + (__builtin_ctzll(first(wm[b2])) >> 3);
                break;
            }
            bpad = 0;
        }
        if (q < 0) return -1;
    }
    return c0 + 8 * (int64_t)q + (__builtin_ctzll(first(w[q])) >> 3);
}

// ---- exact replay of BHA:125-156 inside one jitter cell (depth J, h_J < 1e-3) ---------
struct JitterCtx {
    double *x, *y;
    uint32_t *err;
};

// BHA:146-151: x += (lsb(x)==0 ? +eps : -eps); y += (lsb(y)==0 ? -eps : +eps).  The
// mutation is permanent in the reference (the Body object is shared): it is applied to the
// body state itself.
__device__ __forceinline__ void jitter(const JitterCtx &c, int64_t j) {
    const double eps = 1e-3;
    double px = c.x[j], py = c.y[j];
    px += ((__double_as_longlong(px) & 1ll) == 0) ? +eps : -eps;
    py += ((__double_as_longlong(py) & 1ll) == 0) ? -eps : +eps;
    c.x[j] = px;
    c.y[j] = py;
}

// insertIntoChild on a depth-(J+1) cell: the body is jittered and must then land in a
// grandchild of width h_J < 1e-3 — impossible after a 1e-3 move, so it is dropped
// (BHA:126).  If geometry ever allowed it we flag instead of guessing.
__device__ void into_child_deep(const JitterCtx &c, int64_t j, double qcx, double qcy, double qh) {
    jitter(c, j);
    double px = c.x[j], py = c.y[j];
    double hh = qh / 2.0;
    double gcx = (px < qcx) ? qcx - hh : qcx + hh;
    double gcy = (py < qcy) ? qcy - hh : qcy + hh;
    if (quad_contains(gcx, gcy, hh, px, py)) atomicOr(c.err, 1u);
}

// in-place heapsort of ord[0..k) by key cidx[ord[i]] (caller-list order of a jitter run)
__device__ void sort_by_cidx(uint32_t *ord, int64_t k, const uint32_t *__restrict__ cidx) {
    auto sift = [&](int64_t root, int64_t end) {
        while (2 * root + 1 < end) {
            int64_t child = 2 * root + 1;
            if (child + 1 < end && cidx[ord[child]] < cidx[ord[child + 1]]) ++child;
            if (cidx[ord[root]] < cidx[ord[child]]) {
                uint32_t t = ord[root];
                ord[root] = ord[child];
                ord[child] = t;
                root = child;
            } else {
                return;
            }
        }
    };
    for (int64_t st = k / 2 - 1; st >= 0; --st) sift(st, k);
    for (int64_t end = k - 1; end > 0; --end) {
        uint32_t t = ord[0];
        ord[0] = ord[end];
        ord[end] = t;
        sift(0, end);
    }
}

// Replay of BHA:125-156 inside the jitter cell whose run of sorted bodies starts at `a`
// (c(a) == J, c(a-1) != J): the run's positions are mutated in place and the cell's k child
// slots s0.. are produced through put(slot, record) -- leaves in child order 0..3, then
// massless dead slots.  Returns the mask of subdivided children (for visitQuads).
template <typename Put>
__device__ uint32_t jitter_run(int64_t n, const Geometry &g, int64_t a, int cp,
                               const uint64_t *__restrict__ keys_s, const int8_t *__restrict__ cpl,
                               const uint32_t *__restrict__ base, double *x, double *y,
                               const double *__restrict__ m, const uint32_t *__restrict__ cidx,
                               uint32_t *scratch, uint32_t *err, Put put) {
    const int J = g.J;
    int64_t b = a;
    while (b < n && (int)cpl[b] == J) ++b;  // run = sorted bodies a..b
    const int64_t k = b - a + 1;

    // BHA:363 inserts in list order: order the run by caller index
    uint32_t *ord = scratch + a;
    for (int64_t i = 0; i < k; ++i) ord[i] = (uint32_t)(a + i);
    sort_by_cidx(ord, k, cidx);

    JitterCtx c{x, y, err};
    double ccx, ccy;
    cell_centre(g, keys_s[a], J, ccx, ccy);
    const double hc = g.h[J + 1];

    // state of the 4 children: -1 empty, >= 0 leaf body (slot), -2 subdivided
    int64_t ch[4] = {-1, -1, -1, -1};
    int64_t occ = -1;
    bool sub = false;

    auto into_child = [&](int64_t j) {  // BHA:145-156 on the jitter cell
        jitter(c, j);
        double px = c.x[j], py = c.y[j];
        int ix = (px < ccx) ? 0 : 1;
        int iy = (py < ccy) ? 0 : 2;
        int q = ix + iy;
        double qcx = (q & 1) ? ccx + hc : ccx - hc;
        double qcy = (q & 2) ? ccy + hc : ccy - hc;
        if (!quad_contains(qcx, qcy, hc, px, py)) return;  // BHA:126 dropped
        if (ch[q] == -1) {                                // BHA:127-129
            ch[q] = j;
            return;
        }
        if (ch[q] >= 0) {  // BHA:131-135 subdivide, push existing down
            int64_t e = ch[q];
            ch[q] = -2;
            into_child_deep(c, e, qcx, qcy, hc);
        }
        into_child_deep(c, j, qcx, qcy, hc);  // BHA:136
    };

    for (int64_t i = 0; i < k; ++i) {
        const int64_t j = ord[i];
        if (!sub && occ < 0) {
            occ = j;
            continue;
        }
        if (!sub) {
            sub = true;
            int64_t e = occ;
            occ = -1;
            into_child(e);
        }
        into_child(j);
    }

    // The cell's children into its k contiguous slots, child order 0..3.
    const uint32_t s0 = base[a] + (uint32_t)(J - cp);
    uint32_t w = 0;
    uint32_t jmask = 0;
    for (int q = 0; q < 4; ++q) {
        if (ch[q] == -2) jmask |= 1u << q;
        if (ch[q] < 0) continue;
        int64_t j = ch[q];
        double mm = m[j];
        Node leaf;
        leaf.comX = x[j];
        leaf.comY = y[j];
        leaf.mass = mm;
        leaf.next = s0 + w + 1;
        leaf.meta = NODE_LEAF | (uint32_t)j | (mm == 0.0 ? NODE_SKIP : 0u);
        put(s0 + w, leaf);
        ++w;
    }
    for (; w < (uint32_t)k; ++w) {
        Node dead;
        dead.comX = 0.0;
        dead.comY = 0.0;
        dead.mass = 0.0;
        dead.next = s0 + w + 1;
        dead.meta = NODE_SKIP;
        put(s0 + w, dead);
    }
    return jmask;
}

// BHA:173-202 for one internal node: children 0..3 in pre-order, skipping mass <= 0.
__device__ __forceinline__ void node_com(Node *nodes, uint32_t ni, const Geometry &g,
                                         uint64_t key, int L) {
    Node nd = nodes[ni];
    double mSum = 0.0, cx = 0.0, cy = 0.0;
    uint32_t c = ni + 1;
    while (c < nd.next) {  // children in pre-order == child order 0..3
        Node ch = nodes[c];
        if (ch.mass > 0.0) {
            mSum += ch.mass;
            cx += ch.comX * ch.mass;
            cy += ch.comY * ch.mass;
        }
        c = max(ch.next, c + 1);
    }
    nd.mass = mSum;
    if (mSum > 0.0) {
        nd.comX = cx / mSum;
        nd.comY = cy / mSum;
    } else {  // BHA:197-199 (never visited: mass == 0; a skip-leaf, see NODE_SKIP)
        cell_centre(g, key, L, nd.comX, nd.comY);
        nd.meta |= NODE_SKIP | NODE_LEAF;
    }
    nodes[ni] = nd;
}

constexpr uint32_t NO_SPAN = 0xFFFFFFFFu;
constexpr uint32_t SPAN_REF = 1u << 31;  // child list entry: owner slot of a span child
// span_list entry flag: the node also crosses a GROUP boundary (groups of SPAN_GROUP chunk
// boundaries, finished by one workgroup each); such nodes are finished by k_com_span_top
constexpr uint32_t SPAN_SUPER = 1u << 31;
constexpr int SPAN_GROUP = 1024;
#ifndef BH_EMIT_SPANS
#define BH_EMIT_SPANS 1
#endif
struct SpanOut {  // k_emit_com's span-list outputs (BH_EMIT_SPANS)
    uint32_t *list;
    uint32_t stride;
    uint32_t *super_list;
    uint32_t n_groups;
};

// Chunk-local centre of mass (k_emit_com below): LDS capacity per chunk and its encoding.
#ifndef BH_COM_CAP
#define BH_COM_CAP 2048
#endif
constexpr int COM_CAP = BH_COM_CAP;  // nodes staged per chunk (C3 at 1e6, 1024-body chunks: max 1814)
constexpr uint16_t NO_CHILD = (uint16_t)COM_CAP;  // the massless pad entry
constexpr uint16_t SPAN_CHILD = 0xFFFFu;         // s_ch.x of a chunk-spanning node

// ---- node emission, jitter replay and chunk-local centre of mass in one pass -----------
// One workgroup per 2^COM_CHUNK_SHIFT-body chunk of the Morton order.  Its bodies' node
// skeletons and leaves are produced straight into LDS (the chunk's pre-order slot range
// [base[c0], base[c1])), the jitter cells whose run starts in the chunk are replayed by one
// thread each (BHA:125-156, jitter_run), and the chunk-local internal nodes get their centre
// of mass level by level; every record is written to HBM once: leaves and
// jitter slots when produced, local internal nodes complete at the end, chunk-spanning nodes
// as skeletons for the span passes.  A chunk whose slot range exceeds the LDS capacity runs
// the same steps on global memory.  Jitter slots of a run that started in an earlier chunk are
// written by that chunk's workgroup; here they are inert leaves (no local node owns them).
#ifdef BH_EC_TIMING  // diagnostic build only: per-workgroup phase stamps (wall clock), slots, levels
constexpr int EC_TIMING_MAX = 1 << 16, EC_TIMING_W = 8;  // 7 stamps, slots | levels | CU
__device__ uint64_t g_ec_times[EC_TIMING_W * EC_TIMING_MAX];
#endif
constexpr int EC_WIN = (1 << COM_CHUNK_SHIFT) + 2048;  // c(j) + 1 of the chunk + look-ahead
#ifndef BH_EC_TB
#define BH_EC_TB 512
#endif
constexpr int EC_TB = BH_EC_TB;  // 2 bodies per thread (measured: 256 and 1024 threads slower)
constexpr int EC_PER = (1 << COM_CHUNK_SHIFT) / EC_TB;
#ifndef BH_EC_LVL
#define BH_EC_LVL 4
#endif
constexpr int EC_LVL = BH_EC_LVL;  // skeleton levels whose loads are batched
constexpr uint32_t EC_SPAN = 1u << 31;
constexpr uint32_t EC_LEAF = 1u << 30;
constexpr uint32_t EC_NEXT_MASK = 0xFFFFu;  // next - S0 (<= COM_CAP)
constexpr int EC_JMASK_SHIFT = 16;          // jitter cell: subdivided children
constexpr int EC_D2_SHIFT = 20;             // 2 x depth
constexpr uint16_t EC_OWN_DONE = 0xFFFFu;   // s_own: a leaf, or a node finished body-wise
constexpr uint32_t EC_OWN_BODY_MASK = (1u << COM_CHUNK_SHIFT) - 1;  // s_own: body - c0
constexpr int EC_OWN_L_SHIFT = COM_CHUNK_SHIFT;                      // s_own: depth
static_assert(COM_CHUNK_SHIFT + 5 <= 16, "s_own packs body and depth (depth <= J <= 30)");
static_assert(COM_CAP <= (int)EC_NEXT_MASK, "LDS next offsets must fit 16 bits");

__global__ __launch_bounds__(EC_TB) void k_emit_com(int64_t n, Geometry g, int D0,
                                                     const uint64_t *__restrict__ keys_s,
                                                     const int8_t *__restrict__ cpl,
                                                     const uint32_t *__restrict__ base,
                                                     const uint32_t *__restrict__ cell_start,
                                                     double *x, double *y,
                                                     const double *__restrict__ m,
                                                     const uint32_t *__restrict__ cidx,
                                                     uint32_t *scratch, Node *nodes,
                                                     uint32_t *err,
                                                     const uint32_t *__restrict__ inv,
                                                     uint32_t *__restrict__ lanes, SpanOut so,
                                                     TravCopy tc) {
    chain_prio();
    __shared__ double s_m[COM_CAP + 1], s_x[COM_CAP + 1], s_y[COM_CAP + 1];  // [COM_CAP]: pad
    __shared__ uint32_t s_next[COM_CAP];
    __shared__ ushort4 s_ch[COM_CAP];
    __shared__ uint64_t win[EC_WIN / 8];
    __shared__ uint64_t win_min[EC_WIN / 512];  // per 64-byte block of win: its minimum byte
    __shared__ uint64_t win_wmin[EC_WIN / 64];  // per 8-byte word of win: its minimum byte
    __shared__ int s_lmax;
#ifdef BH_EC_TIMING
    uint64_t t_ph[7];
    t_ph[0] = wall_clock64();
#define EC_STAMP(q) t_ph[q] = wall_clock64()
#else
#define EC_STAMP(q) (void)0
#endif
    const int J = g.J;
    const int64_t c0 = (int64_t)blockIdx.x << COM_CHUNK_SHIFT;
    const int64_t c1 = min(c0 + (1 << COM_CHUNK_SHIFT), n);
    const int64_t a0 = c0 + (int64_t)threadIdx.x * EC_PER;
    uint32_t lv[EC_PER];  // lane map entries, loaded first: the remap's second load waits on them
    if (lanes) {
#pragma unroll
        for (int i = 0; i < EC_PER; ++i) lv[i] = lanes[min(a0 + i, n - 1)];
    }
    int cps[EC_PER], ccs[EC_PER];
    uint32_t bases[EC_PER];
    // the bodies' keys and leaf data too: every independent load of the thread is in flight
    // before the first barrier (unconditional, clamped: a branch per load serialises them),
    // none waits behind the window or the skeleton's dependent chains
    uint64_t ks[EC_PER];
    double xs[EC_PER], ys[EC_PER], ms[EC_PER];
    int lmax = -1;
#pragma unroll
    for (int i = 0; i < EC_PER; ++i) {
        const int64_t a = a0 + i;
        const int64_t ac = min(a, n - 1);
        const int cp = (int)cpl[max(ac - 1, (int64_t)0)], cc = (int)cpl[ac];
        const uint32_t ba = base[ac];
        ks[i] = keys_s[ac];
        xs[i] = x[ac];
        ys[i] = y[ac];
        ms[i] = m[ac];
        cps[i] = a < n ? (a > 0 ? cp : -1) : -1;
        ccs[i] = a < n ? cc : -1;
        bases[i] = a < n ? ba : 0u;
        lmax = max(lmax, ccs[i]);
    }
    if (tc.m) {  // the second traversal's copies (k_trav_inputs): masses, flags, node count
        uint32_t cs[EC_PER];
#pragma unroll
        for (int i = 0; i < EC_PER; ++i) cs[i] = cidx[min(a0 + i, n - 1)];
#pragma unroll
        for (int i = 0; i < EC_PER; ++i) {
            if (a0 + i < n) {
                tc.m[a0 + i] = ms[i];
                tc.cidx[a0 + i] = cs[i];
            }
        }
        if (blockIdx.x == 0) {
            if (threadIdx.x == 0) *tc.T = base[n];
            if (tc.box_header && threadIdx.x < sizeof(MergeHeader) / sizeof(uint32_t))
                tc.box_header[threadIdx.x] = 0u;
        }
    }
    {
        // one 8-byte word of c(j) + 1 per thread (EC_WIN / 8 threads): the word minimum in
        // registers, the 64-byte block minimum over 8 neighbouring lanes
        uint8_t *mb = reinterpret_cast<uint8_t *>(win_min);
        uint8_t *wm = reinterpret_cast<uint8_t *>(win_wmin);
        constexpr int NW = EC_WIN / 8;
        static_assert(NW <= EC_TB && NW % 64 == 0, "one word per thread, whole waves");
        const int t = (int)threadIdx.x;
        if (t < NW) {
            const int64_t j = c0 + 8 * (int64_t)t;
            const int64_t valid = n - j;  // bytes past the last body: c = -1
            // a word that starts below n ends within cpl's 32 bytes of slack past cap
            uint64_t wv = *reinterpret_cast<const uint64_t *>(cpl + (valid > 0 ? j : 0));
            // c + 1 per byte without carries (c in [-1, 41]): -1 -> 0
            wv = ((wv & 0x7F7F7F7F7F7F7F7Full) + 0x0101010101010101ull) ^ (wv & 0x8080808080808080ull);
            if (valid < 8) wv = valid <= 0 ? 0ull : (wv & ~(~0ull << (8 * valid)));
            int mv = 0xFF;
#pragma unroll
            for (int q = 0; q < 8; ++q) mv = min(mv, (int)((wv >> (8 * q)) & 0xFFu));
            win[t] = wv;
            wm[t] = (uint8_t)mv;
#pragma unroll
            for (int off = 1; off < 8; off <<= 1) mv = min(mv, __shfl_xor(mv, off));
            if ((t & 7) == 0) mb[t >> 3] = (uint8_t)mv;
        }
    }
    if (threadIdx.x == 0) s_lmax = -1;
    const uint32_t chunk = blockIdx.x;
    if (BH_EMIT_SPANS) {  // this boundary's span list column: none until a skeleton says so
        if ((int)threadIdx.x <= J) so.list[(size_t)threadIdx.x * so.stride + chunk] = NO_SPAN;
        if (chunk + 1 == gridDim.x)  // (and every column past the last chunk)
            for (uint32_t q = threadIdx.x; q < (uint32_t)(J + 1) * so.stride; q += EC_TB)
                if (q % so.stride > chunk) so.list[q] = NO_SPAN;
    }
    // a chunk-spanning node at depth L, slot ni, ending at body e: listed by this boundary; the
    // owner (this chunk) rides in its comX for k_span_children; SUPER when it also contains the
    // first body past this chunk's group (k_com_span_top finishes it)
    auto span_node = [&](uint32_t ni, int L, int64_t e, uint32_t nx) __attribute__((always_inline)) {
        Node nd;
        nd.comX = BH_EMIT_SPANS ? __longlong_as_double((long long)chunk) : 0.0;
        nd.comY = 0.0;
        nd.mass = 0.0;
        nd.next = nx;
        nd.meta = (uint32_t)(2 * L) | NODE_SPAN;  // 2 x depth
        nodes[ni] = nd;
        if (BH_EMIT_SPANS) {
            const int64_t kG = (int64_t)(chunk / SPAN_GROUP) * SPAN_GROUP + SPAN_GROUP - 1;
            const int64_t bG = (kG << COM_CHUNK_SHIFT) + (1 << COM_CHUNK_SHIFT) - 1;
            const bool super = e > bG;
            so.list[(size_t)L * so.stride + chunk] = ni | (super ? SPAN_SUPER : 0u);
            if (super) so.super_list[(size_t)L * so.n_groups + (uint32_t)(kG / SPAN_GROUP)] = chunk;
        }
    };
    if (lanes) {  // the traversal's lane map through this build's permutation (lane_order)
        uint32_t nl[EC_PER];
#pragma unroll
        for (int i = 0; i < EC_PER; ++i) nl[i] = inv[lv[i]];
#pragma unroll
        for (int i = 0; i < EC_PER; ++i)
            if (a0 + i < n) lanes[a0 + i] = nl[i];
        if (tc.lanes) {
#pragma unroll
            for (int i = 0; i < EC_PER; ++i)
                if (a0 + i < n) tc.lanes[a0 + i] = nl[i];
        }
    }
    const uint32_t S0 = base[c0], S1 = base[c1];
    const uint32_t cnt = S1 - S0;
    const bool lds = cnt <= (uint32_t)COM_CAP;
    __syncthreads();
    EC_STAMP(1);
    atomicMax(&s_lmax, lmax);
    // Phases exchange data through LDS only (in the LDS mode): the barriers wait for LDS, not
    // for the global stores of leaves and skeletons, which nothing in this kernel reads back.
    auto phase_barrier = [&]() __attribute__((always_inline)) {
        if (lds) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
            __builtin_amdgcn_s_barrier();
        } else {
            __threadfence_block();
            __syncthreads();
        }
    };

    // ---- skeletons and leaves (BHA:125-137, 159-166, 176-178) ----
    const uint64_t SENT = sentinel_key(J);
    const int shift0 = 2 * (J - D0);
    // LDS mode: the slots' owners (body, depth) until the child lists reuse the space; the
    // nodes deeper than D0 are then finished slot by slot (below), 4 slots per thread, instead
    // of body by body (a body that starts 7 nested cells held its whole wave)
    uint16_t *s_own = reinterpret_cast<uint16_t *>(s_ch);
#pragma unroll
    for (int i = 0; i < EC_PER; ++i) {  // leaves first: their data is already loaded
        const int64_t a = a0 + i;
        if (a >= n || ks[i] == SENT) continue;  // not in the tree: no slots
        const int cp = cps[i], cc = ccs[i];
        const uint32_t li = bases[i] + (uint32_t)max(0, cc - cp);
        if (lds) s_own[li - S0] = EC_OWN_DONE;
        if (cc == J || cp == J) {  // a jitter run's slot: written by the run's replay below
            if (lds) {
                s_m[li - S0] = 0.0;
                s_x[li - S0] = 0.0;
                s_y[li - S0] = 0.0;
                s_next[li - S0] = (li + 1 - S0) | EC_LEAF;
            }
            continue;
        }
        const double mm = ms[i];
        Node leaf;
        leaf.comX = xs[i];  // BHA:176-178
        leaf.comY = ys[i];
        leaf.mass = mm;
        leaf.next = li + 1;
        leaf.meta = NODE_LEAF | (uint32_t)a | (mm == 0.0 ? NODE_SKIP : 0u);
        nodes[li] = leaf;
        if (lds) {
            s_m[li - S0] = mm;
            s_x[li - S0] = leaf.comX;
            s_y[li - S0] = leaf.comY;
            s_next[li - S0] = (li + 1 - S0) | EC_LEAF;
        }
    }
#pragma unroll
    for (int i = 0; i < EC_PER; ++i) {
        const int64_t a = a0 + i;
        const uint64_t k = ks[i];
        if (a >= n || k == SENT) continue;
        const int cp = cps[i], cc = ccs[i];
        const uint32_t b0 = bases[i];
        int64_t end = a;
        int top = cc;
        if (lds) {  // depths D0 < L <= cc: recorded for the slot pass; the rest are done here
            for (int L = cc; L > max(cp, D0); --L) {
                const uint32_t ni = b0 + (uint32_t)(L - cp - 1) - S0;
                s_own[ni] = (uint16_t)((uint32_t)(a - c0) | ((uint32_t)L << EC_OWN_L_SHIFT));
            }
            for (int L = min(cc, D0); L > cp; --L) s_own[b0 + (uint32_t)(L - cp - 1) - S0] = EC_OWN_DONE;
            top = min(cc, D0);
        }
        // deepest first (the LDS scans start at the deeper level's end: ends are nested), in
        // groups of EC_LVL levels whose end and slot loads are all in flight together: the
        // depth-<= D0 ends and the successors' slots do not depend on each other within a group
        for (int Lh = top; Lh > cp; Lh -= EC_LVL) {
            int64_t e[EC_LVL];
#pragma unroll
            for (int q = 0; q < EC_LVL; ++q) {  // below depth D0: LDS scans, nested
                const int L = Lh - q;
                int64_t b = end;
                if (L > cp && L > D0) {  // inside a's depth-D0 cell: LDS window, then galloping
                    b = lds_scan<EC_WIN>(win, win_wmin, win_min, c0, end, L);
                    if (b < 0) {
                        const int64_t limit = (int64_t)cell_start[(k >> shift0) + 1] - 1;
                        const int shift = 2 * (J - L);
                        b = run_end(keys_s, limit, c0 + EC_WIN - 1, shift, k >> shift);
                    }
                    end = b;
                }
                e[q] = b;
            }
            uint32_t cs[EC_LVL];
#pragma unroll
            for (int q = 0; q < EC_LVL; ++q) {  // depth <= D0: the next depth-L cell's start,
                const int L = Lh - q;           // every load issued unconditionally
                const bool sh = L > cp && L <= D0;
                cs[q] = cell_start[sh ? ((k >> (2 * (J - L))) + 1) << (2 * (D0 - L)) : 0];
            }
#pragma unroll
            for (int q = 0; q < EC_LVL; ++q) {
                const int L = Lh - q;
                if (L > cp && L <= D0) e[q] = (int64_t)cs[q] - 1;
            }
            uint32_t nxs[EC_LVL];
#pragma unroll
            for (int q = 0; q < EC_LVL; ++q) nxs[q] = base[Lh - q > cp ? e[q] + 1 : 0];
#pragma unroll
            for (int q = 0; q < EC_LVL; ++q) {
                const int L = Lh - q;
                if (L <= cp) break;
                const bool span = (a >> COM_CHUNK_SHIFT) != (e[q] >> COM_CHUNK_SHIFT);
                const uint32_t ni = b0 + (uint32_t)(L - cp - 1);
                const uint32_t nx = nxs[q];
                if (span) {
                    span_node(ni, L, e[q], nx);
                } else if (!lds) {
                    Node nd;
                    nd.comX = 0.0;
                    nd.comY = 0.0;
                    nd.mass = 0.0;
                    nd.next = nx;
                    nd.meta = (uint32_t)(2 * L);  // 2 x depth
                    nodes[ni] = nd;
                }
                if (lds)
                    s_next[ni - S0] =
                        span ? EC_SPAN : ((nx - S0) | ((uint32_t)(2 * L) << EC_D2_SHIFT));
            }
        }
    }
    if (lds) {  // the nodes below depth D0, by slot (s_own)
        phase_barrier();
        constexpr int SL = COM_CAP / EC_TB;
        static_assert(COM_CAP % EC_TB == 0, "whole slots per thread");
        int64_t as[SL], e[SL];
        int Ls[SL];
#pragma unroll
        for (int r = 0; r < SL; ++r) {
            const uint32_t i = threadIdx.x + (uint32_t)r * EC_TB;
            const uint32_t ow = i < cnt ? s_own[i] : EC_OWN_DONE;
            const bool live = ow != EC_OWN_DONE;
            as[r] = c0 + (ow & EC_OWN_BODY_MASK);
            Ls[r] = live ? (int)(ow >> EC_OWN_L_SHIFT) : -1;
            int64_t b = as[r];
            if (live) {  // the LDS window, then bounded galloping over the keys
                b = lds_scan<EC_WIN>(win, win_wmin, win_min, c0, as[r], Ls[r]);
                if (b < 0) {
                    const uint64_t k = keys_s[as[r]];
                    const int64_t limit = (int64_t)cell_start[(k >> shift0) + 1] - 1;
                    const int shift = 2 * (J - Ls[r]);
                    b = run_end(keys_s, limit, c0 + EC_WIN - 1, shift, k >> shift);
                }
            }
            e[r] = b;
        }
        uint32_t nxs[SL];
#pragma unroll
        for (int r = 0; r < SL; ++r) nxs[r] = base[Ls[r] >= 0 ? e[r] + 1 : 0];
#pragma unroll
        for (int r = 0; r < SL; ++r) {
            if (Ls[r] < 0) continue;
            const uint32_t i = threadIdx.x + (uint32_t)r * EC_TB;
            const int L = Ls[r];
            const bool span = (as[r] >> COM_CHUNK_SHIFT) != (e[r] >> COM_CHUNK_SHIFT);
            if (span) span_node(S0 + i, L, e[r], nxs[r]);
            s_next[i] = span ? EC_SPAN : ((nxs[r] - S0) | ((uint32_t)(2 * L) << EC_D2_SHIFT));
        }
    }
    phase_barrier();
    EC_STAMP(2);

    // ---- jitter cells whose run starts in this chunk (BHA:145-156) ----
#pragma unroll
    for (int i = 0; i < EC_PER; ++i) {
        const int64_t a = a0 + i;
        if (a >= n || ccs[i] != J || cps[i] == J) continue;
        const uint32_t jm = jitter_run(
            n, g, a, cps[i], keys_s, cpl, base, x, y, m, cidx, scratch, err,
            [&](uint32_t slot, const Node &nd) {
                nodes[slot] = nd;
                if (lds && slot >= S0 && slot < S1) {
                    s_m[slot - S0] = nd.mass;
                    s_x[slot - S0] = nd.comX;
                    s_y[slot - S0] = nd.comY;
                    s_next[slot - S0] = (slot + 1 - S0) | EC_LEAF;
                }
            });
        const uint32_t ni = bases[i] + (uint32_t)(J - cps[i] - 1);  // the jitter cell
        if (lds && !(s_next[ni - S0] & EC_SPAN))
            s_next[ni - S0] |= jm << EC_JMASK_SHIFT;
        else
            nodes[ni].meta |= jm << NODE_JMASK_SHIFT;  // skeleton written above by this thread
    }
    phase_barrier();
    EC_STAMP(3);

    // ---- centre of mass of the chunk-local internal nodes (BHA:173-202) ----
    if (lds) {
        if (threadIdx.x == 0) {
            s_m[COM_CAP] = 0.0;
            s_x[COM_CAP] = 0.0;
            s_y[COM_CAP] = 0.0;
        }
        for (uint32_t i = threadIdx.x; i < cnt; i += EC_TB) {
            const uint32_t nx = s_next[i];
            if (nx & EC_LEAF) continue;
            if (nx & EC_SPAN) {
                s_ch[i] = make_ushort4(SPAN_CHILD, SPAN_CHILD, SPAN_CHILD, SPAN_CHILD);
                continue;
            }
            const uint32_t e2 = nx & EC_NEXT_MASK;
            uint16_t ch[4] = {NO_CHILD, NO_CHILD, NO_CHILD, NO_CHILD};
            uint32_t c = i + 1;
            for (int q = 0; q < 4 && c < e2; ++q) {
                ch[q] = (uint16_t)c;
                c = max(s_next[c] & EC_NEXT_MASK, c + 1);
            }
            s_ch[i] = make_ushort4(ch[0], ch[1], ch[2], ch[3]);
        }
    }
    phase_barrier();
    EC_STAMP(4);
    const int top = s_lmax;
    for (int L = top; L >= 0; --L) {
        uint32_t mask = 0;
#pragma unroll
        for (int i = 0; i < EC_PER; ++i)
            if (ccs[i] >= L && cps[i] < L) mask |= 1u << i;
        if (lds) {
            while (mask) {
                const int i = __builtin_ctz(mask);
                mask &= mask - 1;
                int cpi = cps[0];
                uint32_t bi = bases[0];
#pragma unroll
                for (int q = 1; q < EC_PER; ++q)
                    if (i == q) {
                        cpi = cps[q];
                        bi = bases[q];
                    }
                const uint32_t li = bi + (uint32_t)(L - cpi - 1) - S0;
                const ushort4 chv = s_ch[li];
                if (chv.x == SPAN_CHILD) continue;  // finished by the span passes
                const uint16_t cs[4] = {chv.x, chv.y, chv.z, chv.w};
                double cm[4], ccx[4], ccy[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    cm[q] = s_m[cs[q]];
                    ccx[q] = s_x[cs[q]];
                    ccy[q] = s_y[cs[q]];
                }
                double mSum = 0.0, cx = 0.0, cy = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {  // children 0..3 in pre-order (BHA:189-192)
                    if (cm[q] > 0.0) {
                        mSum += cm[q];
                        cx += ccx[q] * cm[q];
                        cy += ccy[q] * cm[q];
                    }
                }
                double ox, oy;
                if (mSum > 0.0) {
                    ox = cx / mSum;
                    oy = cy / mSum;
                } else {
                    cell_centre(g, keys_s[a0 + i], L, ox, oy);
                }
                s_m[li] = mSum;
                s_x[li] = ox;
                s_y[li] = oy;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): LDS only inside the level loop
            __builtin_amdgcn_s_barrier();
        } else {
            while (mask) {
                const int i = __builtin_ctz(mask);
                mask &= mask - 1;
                const uint32_t ni = bases[i] + (uint32_t)(L - cps[i] - 1);
                if (!(nodes[ni].meta & NODE_SPAN)) node_com(nodes, ni, g, keys_s[a0 + i], L);
            }
            __threadfence_block();
            __syncthreads();
        }
    }
    EC_STAMP(5);
    if (lds) {  // the chunk's local internal nodes, complete, once
        phase_barrier();
        for (uint32_t i = threadIdx.x; i < cnt; i += EC_TB) {
            const uint32_t nx = s_next[i];
            if (nx & (EC_LEAF | EC_SPAN)) continue;
            const double mSum = s_m[i];
            Node nd;
            nd.comX = s_x[i];
            nd.comY = s_y[i];
            nd.mass = mSum;
            nd.next = (nx & EC_NEXT_MASK) + S0;
            nd.meta = ((nx >> EC_D2_SHIFT) & 0xFFu) |
                      (((nx >> EC_JMASK_SHIFT) & 0xFu) << NODE_JMASK_SHIFT) |
                      (mSum > 0.0 ? 0u : NODE_SKIP | NODE_LEAF);
            nodes[S0 + i] = nd;
        }
    }
#ifdef BH_EC_TIMING
    EC_STAMP(6);
    if (threadIdx.x == 0 && blockIdx.x < EC_TIMING_MAX) {
        uint64_t *o = g_ec_times + EC_TIMING_W * blockIdx.x;
        for (int q = 0; q < 7; ++q) o[q] = t_ph[q];
        o[7] = (uint64_t)(cnt & 0xFFFFu) | ((uint64_t)(s_lmax + 1) << 16) | ((uint64_t)__smid() << 32);
    }
#endif
#undef EC_STAMP
}

// The nodes crossing the boundary between chunk k and k+1 (bodies b = end of chunk k and
// b+1) are exactly b's ancestors at depths 0..c(b); each chunk-spanning node is listed once,
// by the boundary of the chunk it starts in: span_list[L * stride + k] (or NO_SPAN).  k_emit_com
// lists them as it writes their skeletons (BH_EMIT_SPANS); k_span_find is the separate pass.

__global__ __launch_bounds__(TB) void k_span_find(int64_t n, int J, int D0,
                                                  const uint64_t *__restrict__ keys_s,
                                                  const int8_t *__restrict__ cpl,
                                                  const uint32_t *__restrict__ base,
                                                  const uint32_t *__restrict__ cell_start,
                                                  uint32_t *__restrict__ span_list,
                                                  uint32_t span_stride,
                                                  uint32_t *__restrict__ super_list,
                                                  uint32_t n_groups, Node *nodes) {
    chain_prio();
    const int64_t k = (int64_t)blockIdx.x * TB + threadIdx.x;
    const int L = blockIdx.y;
    if (k >= (int64_t)span_stride) return;
    const int64_t chunk0 = k << COM_CHUNK_SHIFT;
    const int64_t b = chunk0 + (1 << COM_CHUNK_SHIFT) - 1;
    const int cb = (b + 1 < n) ? (int)cpl[b] : -1;
    uint32_t out = NO_SPAN;
    if (L <= cb) {
        const uint64_t key = keys_s[b];
        int64_t aL;  // first body of b's depth-L cell
        if (L <= D0) {
            aL = cell_start[(key >> (2 * (J - L))) << (2 * (D0 - L))];
        } else {
            const int shift = 2 * (J - L);
            const uint64_t pref = key >> shift;
            int64_t lo = cell_start[key >> (2 * (J - D0))], hi = b;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if ((keys_s[mid] >> shift) < pref) lo = mid + 1; else hi = mid;
            }
            aL = lo;
        }
        if (aL >= chunk0) {  // starts in chunk k: this boundary owns it
            const int cp = aL > 0 ? (int)cpl[aL - 1] : -1;
            const uint32_t ni = base[aL] + (uint32_t)(L - cp - 1);
            // the owner slot rides in the (not yet computed) comX of the span node, so its
            // parent's child list can refer to the slot (k_span_children)
            nodes[ni].comX = __longlong_as_double((long long)k);
            // does the node also contain the first group boundary at or after chunk k?
            const int64_t kG = (k / SPAN_GROUP) * SPAN_GROUP + SPAN_GROUP - 1;
            const int64_t bG = (kG << COM_CHUNK_SHIFT) + (1 << COM_CHUNK_SHIFT) - 1;
            const int shift = 2 * (J - L);
            const bool super = bG + 1 < n && (keys_s[bG + 1] >> shift) == (key >> shift);
            out = ni | (super ? SPAN_SUPER : 0u);
            if (super) super_list[(size_t)L * n_groups + (uint32_t)(kG / SPAN_GROUP)] = (uint32_t)k;
        }
    }
    span_list[(size_t)L * span_stride + k] = out;
}

// Children of every chunk-spanning node with the values of the local ones (final after
// k_emit_com), gathered in parallel so the level-by-level pass below reads one
// independent record per level.
__global__ __launch_bounds__(TB) void k_span_children(int J, const uint32_t *__restrict__ span_list,
                                                      uint32_t span_stride,
                                                      const Node *__restrict__ nodes,
                                                      SpanSlot *__restrict__ span_children) {
    chain_prio();
    const uint32_t L = blockIdx.y;
    for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < span_stride; i += gridDim.x * TB) {
        const size_t slot = (size_t)L * span_stride + i;
        const uint32_t e = span_list[slot];
        if (e == NO_SPAN) continue;  // empty slot: never read
        const uint32_t ni = e & ~SPAN_SUPER;
        SpanSlot out;
        const uint32_t end = nodes[ni].next;
        uint32_t c = ni + 1;
        for (int k = 0; k < 4; ++k) {
            out.ch[k] = 0xFFFFFFFFu;
            out.v[k][0] = 0.0;
            out.v[k][1] = 0.0;
            out.v[k][2] = 0.0;
            if (c >= end) continue;
            const Node cn = nodes[c];
            if (!(cn.meta & NODE_LEAF) && (cn.meta & NODE_SPAN)) {
                out.ch[k] = SPAN_REF | (uint32_t)__double_as_longlong(cn.comX);
            } else {
                out.ch[k] = c;
                if (cn.mass > 0.0) {
                    out.v[k][0] = cn.mass;
                    out.v[k][1] = cn.comX * cn.mass;
                    out.v[k][2] = cn.comY * cn.mass;
                }
            }
            c = max(cn.next, c + 1);
        }
        span_put(span_children, (size_t)(J + 1) * span_stride, slot, out);
    }
}

// Chunk-spanning nodes, levels J..0: workgroup g owns the chunk boundaries
// [g*SPAN_GROUP, (g+1)*SPAN_GROUP), thread = boundary, and finishes the span nodes that do
// not cross a group boundary (their span children are then in the same group).  The previous
// level's results live in LDS (a span child is referenced by its owner slot).  A thread first
// reads its whole span_list column (one latency) into a bit mask of the levels it owns a node
// at -- deep levels are mostly empty -- and then loads only those records, two levels ahead;
// stores to global stay in flight across the LDS-only barriers.
constexpr int SPAN_TB = SPAN_GROUP;

#ifdef BH_SPAN_TIMING  // diagnostic build: per-level wall-clock stamps of k_com_span's group 0
constexpr int SPAN_T_REC = 64, SPAN_T_W = 32;  // launches kept (ring), stamps per launch
__device__ uint64_t g_span_times[SPAN_T_REC * SPAN_T_W];
__device__ uint32_t g_span_launch;
#endif

struct SpanRegs {
    uint32_t ni;
    uint32_t ch[4];
    double v[4][3];
};

__device__ __forceinline__ void load_span(SpanRegs &r, const uint32_t *span_list,
                                          const SpanSlot *span_children, size_t P, size_t slot) {
    r.ni = span_list[slot];
    const SpanSlot q = span_get(span_children, P, slot);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        r.ch[k] = q.ch[k];
        r.v[k][0] = q.v[k][0];
        r.v[k][1] = q.v[k][1];
        r.v[k][2] = q.v[k][2];
    }
}

__global__ __launch_bounds__(SPAN_TB) void k_com_span(int J, const uint32_t *__restrict__ span_list,
                                                      uint32_t span_stride,
                                                      const SpanSlot *__restrict__ span_children,
                                                      Node *nodes) {
    chain_prio();
    __shared__ double r_m[2][SPAN_GROUP], r_x[2][SPAN_GROUP], r_y[2][SPAN_GROUP];
    const uint32_t g0 = blockIdx.x * SPAN_GROUP;
    const uint32_t kl = threadIdx.x, k = g0 + kl;
    const bool valid = k < span_stride;
#ifdef BH_SPAN_TIMING
    __shared__ uint64_t t_st[SPAN_T_W];
    int t_n = 0;  // (uniform)
    if (threadIdx.x == 0) t_st[0] = wall_clock64();
    t_n = 1;
#define SPAN_STAMP()                                                          \
    do {                                                                      \
        if (t_n < SPAN_T_W && threadIdx.x == 0) t_st[t_n] = wall_clock64();   \
        ++t_n;                                                                \
    } while (0)
#else
#define SPAN_STAMP() (void)0
#endif
    // levels (bit L) at which this boundary owns a node finished here (not group-crossing)
    uint64_t own = 0;
    if (valid) {
#pragma unroll 8
        for (int L = 0; L <= J; ++L) {
            const uint32_t e = span_list[(size_t)L * span_stride + k];
            if (e != NO_SPAN && !(e & SPAN_SUPER)) own |= 1ull << L;
        }
    }
#ifdef BH_SPAN_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    SPAN_STAMP();
#endif
    auto fetch = [&](SpanRegs &r, int L) __attribute__((always_inline)) {
        r.ni = NO_SPAN;
#ifdef BH_SPAN_NOLOAD  // (timing experiment only: results wrong)
        if (L >= 0 && ((own >> L) & 1ull)) {
            r.ni = 0u;
            for (int c = 0; c < 4; ++c) {
                r.ch[c] = 0xFFFFFFFFu;
                r.v[c][0] = r.v[c][1] = r.v[c][2] = 1.0;
            }
        }
#else
        if (L >= 0 && ((own >> L) & 1ull))
            load_span(r, span_list, span_children, (size_t)(J + 1) * span_stride,
                      (size_t)L * span_stride + k);
#endif
    };
    auto level = [&](const SpanRegs &C, int L) __attribute__((always_inline)) {
        const int cur = L & 1, prev = cur ^ 1;
        if (C.ni != NO_SPAN) {
            double mSum = 0.0, cx = 0.0, cy = 0.0;  // children 0..3 in order (BHA:189-192)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (C.ch[c] != 0xFFFFFFFFu && (C.ch[c] & SPAN_REF)) {
                    const uint32_t s2 = (C.ch[c] & ~SPAN_REF) - g0;
                    const double cm = r_m[prev][s2];
                    if (cm > 0.0) {
                        mSum += cm;
                        cx += r_x[prev][s2] * cm;
                        cy += r_y[prev][s2] * cm;
                    }
                } else {  // local child (or none): precomputed, zeros when skipped
                    mSum += C.v[c][0];
                    cx += C.v[c][1];
                    cy += C.v[c][2];
                }
            }
            double ox = 0.0, oy = 0.0;
            if (mSum > 0.0) {
                ox = cx / mSum;
                oy = cy / mSum;
            }
            r_m[cur][kl] = mSum;
            r_x[cur][kl] = ox;
            r_y[cur][kl] = oy;
            Node *dst = nodes + C.ni;
            dst->mass = mSum;
            dst->comX = ox;  // massless: never visited (the cell centre is not recorded)
            dst->comY = oy;
            if (!(mSum > 0.0)) dst->meta |= NODE_SKIP | NODE_LEAF;  // a skip-leaf
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): LDS results visible; stores fly on
        __builtin_amdgcn_s_barrier();
        SPAN_STAMP();
    };
    // a span child always sits one level below its parent and is owned by a boundary of the
    // same group, so the level pass needs no other synchronisation
#ifndef BH_SPAN_AHEAD
#define BH_SPAN_AHEAD 2  // levels whose records are in flight
#endif
    SpanRegs R[BH_SPAN_AHEAD];
#pragma unroll
    for (int j = 0; j < BH_SPAN_AHEAD; ++j) fetch(R[j], J - j);
    for (int L = J; L >= 0; L -= BH_SPAN_AHEAD) {
#pragma unroll
        for (int j = 0; j < BH_SPAN_AHEAD; ++j) {
            if (L - j >= 0) {
                level(R[j], L - j);
                fetch(R[j], L - j - BH_SPAN_AHEAD);
            }
        }
    }
#ifdef BH_SPAN_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    SPAN_STAMP();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint32_t rec = atomicAdd(&g_span_launch, 1u) % SPAN_T_REC;
        uint64_t *o = g_span_times + (size_t)rec * SPAN_T_W;
        for (int q = 0; q < SPAN_T_W; ++q) o[q] = q < t_n ? t_st[q] : 0ull;
        o[SPAN_T_W - 1] = (uint64_t)t_n;
    }
#endif
#undef SPAN_STAMP
}

// The nodes that cross a group boundary (few: at most one per group boundary and level),
// levels J..0, one workgroup, thread = group boundary.  Children come from the records
// (local ones) or from the node array (span children: finished by k_com_span, or by this
// kernel one level below).
__global__ __launch_bounds__(SPAN_TB) void k_com_span_top(int J,
                                                          const uint32_t *__restrict__ span_list,
                                                          uint32_t span_stride,
                                                          const SpanSlot *__restrict__ span_children,
                                                          const uint32_t *__restrict__ super_list,
                                                          uint32_t n_groups, Node *nodes) {
    chain_prio();
    for (int L = J; L >= 0; --L) {
        for (uint32_t gi = threadIdx.x; gi < n_groups; gi += SPAN_TB) {
            const uint32_t ko = super_list[(size_t)L * n_groups + gi];
            if (ko == NO_SPAN) continue;
            const size_t slot = (size_t)L * span_stride + ko;
            const uint32_t ni = span_list[slot] & ~SPAN_SUPER;
            const SpanSlot q = span_get(span_children, (size_t)(J + 1) * span_stride, slot);
            double mSum = 0.0, cx = 0.0, cy = 0.0;
            for (int c = 0; c < 4; ++c) {
                if (q.ch[c] != 0xFFFFFFFFu && (q.ch[c] & SPAN_REF)) {
                    const uint32_t ci =
                        span_list[(size_t)(L + 1) * span_stride + (q.ch[c] & ~SPAN_REF)] & ~SPAN_SUPER;
                    const Node cn = nodes[ci];
                    if (cn.mass > 0.0) {
                        mSum += cn.mass;
                        cx += cn.comX * cn.mass;
                        cy += cn.comY * cn.mass;
                    }
                } else {
                    mSum += q.v[c][0];
                    cx += q.v[c][1];
                    cy += q.v[c][2];
                }
            }
            Node *dst = nodes + ni;
            dst->mass = mSum;
            dst->comX = mSum > 0.0 ? cx / mSum : 0.0;
            dst->comY = mSum > 0.0 ? cy / mSum : 0.0;
            if (!(mSum > 0.0)) dst->meta |= NODE_SKIP | NODE_LEAF;  // a skip-leaf
        }
        __syncthreads();
    }
}

// The same pass with everything but the chain itself loaded up front (BH_SPAN_TOP_LDS, up to
// SPAN_TOP_PAIRS (level, group boundary) pairs): every pair's record, and the values of its
// children that are not group-crossing (local ones from the record, span ones from the node
// array: k_com_span finished them), are staged in LDS by all threads at once; the levels then
// run on LDS only -- a group-crossing child of (L, g) is the pair (L + 1, its owner's group).
// The old pass made ~5 dependent global loads per level, a 22-level chain of ~1 us steps.
#ifndef BH_SPAN_TOP_LDS
#define BH_SPAN_TOP_LDS 1
#endif
constexpr int SPAN_TOP_PAIRS = 256;
constexpr uint32_t TOP_CONST = 0xFFFFFFFFu;  // child value staged (no pair reference)
__global__ __launch_bounds__(SPAN_TB) void k_com_span_top_lds(
    int J, const uint32_t *__restrict__ span_list, uint32_t span_stride,
    const SpanSlot *__restrict__ span_children, const uint32_t *__restrict__ super_list,
    uint32_t n_groups, Node *nodes) {
    chain_prio();
    __shared__ uint32_t s_ni[SPAN_TOP_PAIRS];
    __shared__ uint32_t s_ref[SPAN_TOP_PAIRS][4];
    __shared__ double s_v[SPAN_TOP_PAIRS][4][3];
    __shared__ double s_res[SPAN_TOP_PAIRS][3];
    const uint32_t P = (uint32_t)(J + 1) * n_groups;
    for (uint32_t p = threadIdx.x; p < P; p += SPAN_TB) {
        const uint32_t L = p / n_groups, gi = p % n_groups;
        const uint32_t ko = super_list[(size_t)L * n_groups + gi];
        s_ni[p] = NO_SPAN;
        if (ko == NO_SPAN) continue;
        const size_t slot = (size_t)L * span_stride + ko;
        const uint32_t ni = span_list[slot] & ~SPAN_SUPER;
        const SpanSlot q = span_get(span_children, (size_t)(J + 1) * span_stride, slot);
        for (int c = 0; c < 4; ++c) {
            uint32_t ref = TOP_CONST;
            double v0 = q.v[c][0], v1 = q.v[c][1], v2 = q.v[c][2];
            if (q.ch[c] != 0xFFFFFFFFu && (q.ch[c] & SPAN_REF)) {
                const uint32_t kc = q.ch[c] & ~SPAN_REF;
                const uint32_t ec = span_list[(size_t)(L + 1) * span_stride + kc];
                if (ec & SPAN_SUPER) {  // finished below in this pass: pair (L + 1, kc's group)
                    ref = (L + 1) * n_groups + kc / SPAN_GROUP;
                } else {  // finished by k_com_span (BHA:189-192: mass > 0 only; zeros add nothing)
                    const Node cn = nodes[ec];
                    v0 = v1 = v2 = 0.0;
                    if (cn.mass > 0.0) {
                        v0 = cn.mass;
                        v1 = cn.comX * cn.mass;
                        v2 = cn.comY * cn.mass;
                    }
                }
            }
            s_ref[p][c] = ref;
            s_v[p][c][0] = v0;
            s_v[p][c][1] = v1;
            s_v[p][c][2] = v2;
        }
        s_ni[p] = ni;
    }
    __syncthreads();
    for (int L = J; L >= 0; --L) {
        for (uint32_t gi = threadIdx.x; gi < n_groups; gi += SPAN_TB) {
            const uint32_t p = (uint32_t)L * n_groups + gi;
            const uint32_t ni = s_ni[p];
            if (ni == NO_SPAN) continue;
            double mSum = 0.0, cx = 0.0, cy = 0.0;
            for (int c = 0; c < 4; ++c) {  // children 0..3 in order (BHA:189-192)
                const uint32_t ref = s_ref[p][c];
                if (ref != TOP_CONST) {
                    const double cm = s_res[ref][0];
                    if (cm > 0.0) {
                        mSum += cm;
                        cx += s_res[ref][1] * cm;
                        cy += s_res[ref][2] * cm;
                    }
                } else {
                    mSum += s_v[p][c][0];
                    cx += s_v[p][c][1];
                    cy += s_v[p][c][2];
                }
            }
            const double ox = mSum > 0.0 ? cx / mSum : 0.0;
            const double oy = mSum > 0.0 ? cy / mSum : 0.0;
            Node *dst = nodes + ni;
            dst->mass = mSum;
            dst->comX = ox;
            dst->comY = oy;
            if (!(mSum > 0.0)) dst->meta |= NODE_SKIP | NODE_LEAF;  // a skip-leaf
            s_res[p][0] = mSum;
            s_res[p][1] = ox;
            s_res[p][2] = oy;
        }
        __syncthreads();
    }
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + TB - 1) / TB); }

}  // namespace

// Stable LSD radix sort of the 32-bit key prefixes.  rocprim's default picks a merge sort for
// n <= BH_SORT_MERGE_LIMIT (2^20) and onesweep above.
#ifndef BH_SORT_MERGE_LIMIT
#define BH_SORT_MERGE_LIMIT (1024 * 1024)
#endif
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, BH_SORT_MERGE_LIMIT>;

int cell_table_depth(int J, int64_t n) {
    int d = 1;  // smallest depth with 4^d >= n, capped
    while (d < CELL_TABLE_MAX_DEPTH && ((int64_t)1 << (2 * d)) < n) ++d;
    return d < J ? d : J;
}

// ---- Hilbert lane order for the traversal (traverse.hip) ---------------------------------
// The traversal's wave walks the union of its 64 lanes' interaction lists, so how bodies are
// grouped into waves sets its work.  64 Hilbert-consecutive bodies form more compact groups than
// 64 Morton-consecutive ones (no Z jumps): 6.5 % fewer cursor stops and 7.7 % fewer point-force
// blocks at C3 and C4 (oracle union-walk model).  The lane map lane -> slot is made by sorting
// the bodies by the Hilbert index of their depth-16 cell (from the Morton key of the build) and
// carried through later builds by the builds' permutations, re-sorted every LANE_REFRESH builds.
// It only groups bodies into waves: every body's sum is unchanged.
__device__ __forceinline__ uint32_t hilbert16(uint64_t key, int J) {
    // de-interleave the top 16 Morton digits (digit = ix | iy << 1, root first)
    uint32_t ix = 0, iy = 0;
    const int lv = J < 16 ? J : 16;
    for (int d = 0; d < lv; ++d) {
        const uint32_t dig = (uint32_t)(key >> (2 * (J - 1 - d))) & 3u;
        ix = (ix << 1) | (dig & 1u);
        iy = (iy << 1) | (dig >> 1);
    }
    uint32_t h = 0;  // classic xy -> d over lv levels
    for (uint32_t sbit = 1u << (lv - 1); sbit > 0; sbit >>= 1) {
        const uint32_t rx = (ix & sbit) ? 1u : 0u, ry = (iy & sbit) ? 1u : 0u;
        h += sbit * sbit * ((3u * rx) ^ ry);
        if (ry == 0) {
            if (rx == 1) {
                ix = sbit - 1 - (ix & (sbit - 1)) + (ix & ~(sbit - 1));
                iy = sbit - 1 - (iy & (sbit - 1)) + (iy & ~(sbit - 1));
            }
            const uint32_t t = ix;
            ix = iy;
            iy = t;
        }
    }
    return h;
}

__global__ __launch_bounds__(TB) void k_hilbert_keys(int64_t n, int J, const uint64_t *__restrict__ keys_s,
                                                     uint32_t *__restrict__ hkey,
                                                     uint32_t *__restrict__ slot) {
    chain_prio();
    const int64_t a = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (a >= n) return;
    const uint64_t k = keys_s[a];
    hkey[a] = k == sentinel_key(J) ? 0xFFFFFFFFu : hilbert16(k, J);  // not in the tree: last
    slot[a] = (uint32_t)a;
}

__global__ __launch_bounds__(TB) void k_lane_remap(int64_t n, const uint32_t *__restrict__ inv,
                                                   uint32_t *__restrict__ lanes) {
    chain_prio();
    const int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (q < n) lanes[q] = inv[lanes[q]];
}

// The refresh sorts 24 bits (the depth-12 Hilbert cell: ~0.6 px at the 2400x800 root) with
// rocprim's onesweep radix sort (3 passes) -- its merge sort, the default below 2^20 keys, took
// ~150 us at C3.
using LaneSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                  rocprim::default_config, 1024>;
#ifndef BH_LANE_LO_BIT
#define BH_LANE_LO_BIT 8
#endif
constexpr unsigned LANE_SORT_LO_BIT = BH_LANE_LO_BIT;

// The pipelined step (engine.cpp): a build made while the previous evaluation still kicks the
// velocities leaves them out (src.vx = null); they follow with the build's permutation.
__global__ __launch_bounds__(TB) void k_permute_vel(int64_t n, const uint32_t *__restrict__ perm,
                                                    const double *__restrict__ svx,
                                                    const double *__restrict__ svy,
                                                    double *__restrict__ dvx,
                                                    double *__restrict__ dvy) {
    const int64_t a = (int64_t)xcd_block() * TB + threadIdx.x;
    if (a >= n) return;
    const uint32_t i = perm[a];
    dvx[a] = svx[i];
    dvy[a] = svy[i];
}

__global__ __launch_bounds__(TB) void k_spl_extend(uint64_t *__restrict__ spl, uint32_t from,
                                                   uint32_t to, uint64_t sent32) {
    const uint32_t t = from + blockIdx.x * TB + threadIdx.x;
    if (t < to) spl[t] = (sent32 << 32) | ((uint64_t)t * SORT_B);
}

void extend_splitters(uint64_t *spl, uint32_t from, uint32_t to, int J, hipStream_t s) {
    if (to <= from) return;
    k_spl_extend<<<(to - from + TB - 1) / TB, TB, 0, s>>>(spl, from, to,
                                                        sentinel_key(J) >> key32_shift(J));
}

void permute_velocities(int64_t n, const uint32_t *perm, const double *svx, const double *svy,
                        double *dvx, double *dvy, hipStream_t s) {
    if (n > 0) k_permute_vel<<<grid_for(n), TB, 0, s>>>(n, perm, svx, svy, dvx, dvy);
}

__global__ __launch_bounds__(TB) void k_unpermute_pos(int64_t n, const uint32_t *__restrict__ perm,
                                                      const double *__restrict__ sx,
                                                      const double *__restrict__ sy,
                                                      double *__restrict__ dx,
                                                      double *__restrict__ dy) {
    const int64_t a = (int64_t)xcd_block() * TB + threadIdx.x;
    if (a >= n) return;
    const uint32_t i = perm[a];
    dx[i] = sx[a];
    dy[i] = sy[a];
}

void unpermute_positions(int64_t n, const uint32_t *perm, const double *sx, const double *sy,
                         double *dx, double *dy, hipStream_t s) {
    if (n > 0) k_unpermute_pos<<<grid_for(n), TB, 0, s>>>(n, perm, sx, sy, dx, dy);
}

hipError_t lane_order(const TreeBuffers &b, int64_t n, int J, bool refresh, uint32_t *lanes,
                      hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (!refresh) {  // carry the grouping through this build's permutation (k_prep: keys32 =
                     // old slot -> new slot); tree_build does it inside k_emit_com when
                     // b.lanes_remap is set
        if (b.lanes_remap != lanes) k_lane_remap<<<grid_for(n), TB, 0, s>>>(n, b.keys32, lanes);
        return hipGetLastError();
    }
    // keys32 / keys32_s / idx are free once the build has run
    return lane_order_into(b.keys_s, n, J, b.keys32, b.keys32_s, b.idx, b.scratch, b.scratch_bytes,
                           lanes, s);
}

hipError_t lane_order_into(const uint64_t *keys_s, int64_t n, int J, uint32_t *hkey,
                           uint32_t *hkey_s, uint32_t *slot, void *scratch, size_t scratch_bytes,
                           uint32_t *lanes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_hilbert_keys<<<grid_for(n), TB, 0, s>>>(n, J, keys_s, hkey, slot);
    size_t bytes = scratch_bytes;
    return rocprim::radix_sort_pairs<LaneSortConfig>(scratch, bytes, hkey, hkey_s, slot, lanes,
                                                     (size_t)n, LANE_SORT_LO_BIT, 32u, s);
}

size_t lane_sort_bytes(int64_t n) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs<LaneSortConfig>(nullptr, bytes, (uint32_t *)nullptr,
                                                    (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                    (uint32_t *)nullptr, (size_t)n,
                                                    LANE_SORT_LO_BIT, 32u);
    return bytes;
}

size_t tree_scratch_bytes(int64_t n, int J) {
    size_t sort_bytes = 0, scan_bytes = 0;
    (void)J;
    (void)rocprim::radix_sort_pairs<SortConfig>(nullptr, sort_bytes, (uint32_t *)nullptr,
                                                (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                (uint32_t *)nullptr, (size_t)n, 0u, 32u);
    size_t lane_bytes = 0;
    (void)rocprim::radix_sort_pairs<LaneSortConfig>(nullptr, lane_bytes, (uint32_t *)nullptr,
                                                    (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                    (uint32_t *)nullptr, (size_t)n,
                                                    LANE_SORT_LO_BIT, 32u);
    sort_bytes = sort_bytes > lane_bytes ? sort_bytes : lane_bytes;
    (void)rocprim::exclusive_scan(nullptr, scan_bytes, (const uint32_t *)nullptr,
                                  (uint32_t *)nullptr, 0u, (size_t)(n + 1),
                                  rocprim::plus<uint32_t>());
    const size_t tsum_bytes = sizeof(uint32_t) * (size_t)((n + 1 + TB - 1) / TB + 1);  // k_prep
    scan_bytes = scan_bytes > tsum_bytes ? scan_bytes : tsum_bytes;
    return sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
}

hipError_t tree_build(const TreeBuffers &b, int64_t n, const Geometry &g, hipStream_t s) {
    if (n <= 0) return hipMemsetAsync(b.base, 0, sizeof(uint32_t), s);
    hipError_t st;
    const int D0 = cell_table_depth(g.J, n);
    const bool bucket = b.spl_nb > 0;
    const bool ready = bucket && b.keys_ready;  // the drifting traversal did both passes
    static_assert(TB == SORT_TB, "k_morton_count: one index space");
    uint32_t P = 0;
    const bool small = bucket && small_front(n, P);
    const uint32_t n_groups = span_groups(b.span_stride);
    const int64_t n_super = n_groups > 1 ? (int64_t)(g.J + 1) * n_groups : 0;
    const int64_t nbins1 = ((int64_t)1 << (2 * D0)) + 1;
    if (!ready && !bucket)
        k_morton<<<grid_for(n), TB, 0, s>>>(n, b.src.x, b.src.y, b.src.cidx, g, b.keys, b.keys32,
                                            b.idx);
    size_t bytes = b.scratch_bytes;
    if (small) {
        k_small_front<<<1, SF_TB, sizeof(uint64_t) * P, s>>>(
            n, P, !ready, g, D0, b.src, b.dst, b.keys, b.keys32, b.keys32_s, b.perm, b.keys_s,
            b.bcount, b.spl_nb, b.cell_start, b.super_list, n_super, b.cpl, b.cnt, b.spl,
            HeavyList{b.heavy, b.heavy_count, b.heavy_thr}, b.base);
    } else if (bucket) {  // bucket ids / offsets live in cnt / base until k_prep needs them
        const unsigned sg = (unsigned)((n + SORT_TB - 1) / SORT_TB);
        if (!ready)
            k_morton_count<<<sg, SORT_TB, 0, s>>>(n, b.src.x, b.src.y, b.src.cidx, g, b.keys,
                                                  b.keys32, b.spl, b.spl_nb, b.cnt, b.base,
                                                  b.bcount);
        st = rocprim::exclusive_scan(b.scratch, bytes, b.bcount, b.bstart, 0u,
                                     (size_t)b.spl_nb + 1, rocprim::plus<uint32_t>(), s);
        if (st != hipSuccess) return st;
        k_bucket_scatter<<<sg, SORT_TB, 0, s>>>(n, b.keys32, b.cnt, b.base, b.bstart, b.keys_s);
        uint32_t seq = 0;
#ifdef BH_SORT_STATS
        static uint32_t sort_seq = 0;  // (diagnostic build: one engine, one thread)
        seq = sort_seq++;
#endif
        k_bucket_sort<<<b.spl_nb, SORT_TB, 0, s>>>(b.bstart, b.bcount, b.keys_s, b.keys,
                                                   b.keys32_s, b.perm, b.keys_s, seq);
    } else {
        st = rocprim::radix_sort_pairs<SortConfig>(b.scratch, bytes, b.keys32, b.keys32_s, b.idx,
                                                   b.perm, (size_t)n, 0u, 32u, s);
        if (st != hipSuccess) return st;
        k_key_gather<<<grid_for(n), TB, 0, s>>>(n, b.keys, b.perm, b.keys_s);
    }
    if (small) {
    } else if (BH_FIXUP_CELLS)
        k_fixup_cells<<<grid_for(std::max<int64_t>(n, nbins1)), TB, 0, s>>>(
            n, g.J, D0, b.keys32_s, b.keys_s, b.perm, b.cell_start, b.super_list, n_super);
    else
        k_key_fixup<<<grid_for(n), TB, 0, s>>>(n, g.J, b.keys32_s, b.keys_s, b.perm);
    const int64_t prep_blocks = (n + 1 + TB - 1) / TB;
    // (above 4 M counts rocprim's single pass is faster: the blocks' prefix reads grow with n^2 /
    // block size -- C4 16.52-16.54 against 16.57-16.58 ms per step, profiles/r05y4_ab_c4.txt)
    const bool own_scan = BH_BASE_SCAN && n + 1 <= ((int64_t)1 << 22) &&
                          b.scratch_bytes >= sizeof(uint32_t) * (size_t)prep_blocks;
    uint32_t *tsum = own_scan ? static_cast<uint32_t *>(b.scratch) : nullptr;
    if (!small)
        k_prep<<<(unsigned)prep_blocks, TB, 0, s>>>(n, g.J, b.keys_s, b.perm, b.src, b.dst, b.cpl,
                                                    b.cnt, b.spl, b.keys32, tsum,
                                                    HeavyList{b.heavy, b.heavy_count, b.heavy_thr});
    if (small) {
    } else if (own_scan) {
        const int64_t per = (int64_t)BS_TB * 4;
        k_base_scan<4><<<(unsigned)((n + 1 + per - 1) / per), BS_TB, 0, s>>>(n + 1, b.cnt, tsum,
                                                                        b.base);
    } else {
        bytes = b.scratch_bytes;
        st = rocprim::exclusive_scan(b.scratch, bytes, b.cnt, b.base, 0u, (size_t)(n + 1),
                                     rocprim::plus<uint32_t>(), s);
        if (st != hipSuccess) return st;
    }
    if (!BH_FIXUP_CELLS && !small)
        k_cells<<<grid_for(nbins1), TB, 0, s>>>(n, g.J, D0, b.keys_s, b.cell_start, b.super_list,
                                                n_super);
    k_emit_com<<<(unsigned)((n + (1 << COM_CHUNK_SHIFT) - 1) >> COM_CHUNK_SHIFT), EC_TB, 0, s>>>(
        n, g, D0, b.keys_s, b.cpl, b.base, b.cell_start, b.dst.x, b.dst.y, b.dst.m, b.dst.cidx,
        b.idx, b.nodes, b.scalars + 1, b.keys32, b.lanes_remap,
        SpanOut{b.span_list, b.span_stride, b.super_list, n_groups}, b.tc);
    const dim3 span_grid((b.span_stride + TB - 1) / TB, g.J + 1);
    if (!BH_EMIT_SPANS)
        k_span_find<<<span_grid, TB, 0, s>>>(n, g.J, D0, b.keys_s, b.cpl, b.base, b.cell_start,
                                             b.span_list, b.span_stride, b.super_list, n_groups,
                                             b.nodes);
    k_span_children<<<span_grid, TB, 0, s>>>(g.J, b.span_list, b.span_stride, b.nodes,
                                             b.span_children);
    k_com_span<<<n_groups, SPAN_TB, 0, s>>>(g.J, b.span_list, b.span_stride, b.span_children,
                                            b.nodes);
    if (n_groups > 1 && BH_SPAN_TOP_LDS && (int64_t)(g.J + 1) * n_groups <= SPAN_TOP_PAIRS)
        k_com_span_top_lds<<<1, SPAN_TB, 0, s>>>(g.J, b.span_list, b.span_stride,
                                                 b.span_children, b.super_list, n_groups,
                                                 b.nodes);
    else if (n_groups > 1)
        k_com_span_top<<<1, SPAN_TB, 0, s>>>(g.J, b.span_list, b.span_stride, b.span_children,
                                             b.super_list, n_groups, b.nodes);
    return hipGetLastError();
}

#ifdef BH_SORT_STATS
extern "C" int bh_debug_sort_stats(unsigned long long *out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_stats), sizeof(unsigned long long) * 8);
}
extern "C" int bh_debug_sort_log(unsigned long long *out) {  // SORT_LOG x 4, by launch % SORT_LOG
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_log),
                                    sizeof(unsigned long long) * 4 * SORT_LOG);
}
#endif

#ifdef BH_SPAN_TIMING
extern "C" int bh_debug_span_times(uint64_t *out, uint32_t *launches) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_span_times),
                                       sizeof(uint64_t) * SPAN_T_REC * SPAN_T_W);
    if (e == hipSuccess) e = hipMemcpyFromSymbol(launches, HIP_SYMBOL(g_span_launch), 4);
    return (int)e;
}
#endif

#ifdef BH_EC_TIMING
extern "C" int bh_debug_ec_times(uint64_t *out, int n) {
    if (n > EC_TIMING_MAX) n = EC_TIMING_MAX;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ec_times),
                                    sizeof(uint64_t) * EC_TIMING_W * (size_t)n);
}
#endif

}  // namespace bh
