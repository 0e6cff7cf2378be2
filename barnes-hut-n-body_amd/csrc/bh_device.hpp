// Device-side data layout shared by the engine's HIP translation units.
//
// Bodies live in HBM as SoA fp64 arrays in MORTON ("slot") order — the order of the last
// tree build — plus `cidx`, each body's index in the caller's list (the reference's
// List<Body> order, which the jitter replay and the merge rule depend on).  Every build
// sorts, then permutes the state into the new order (nearly sequential: bodies move little
// between builds), so the traversal reads and writes coalesced and consecutive lanes hold
// spatial neighbours.
//
// The quadtree of the reference (BHA:95-202, a pointer tree of BHTree objects) is ONE flat
// array of 32-byte node records in depth-first PRE-ORDER with the reference's child order
// 0..3 (BHA:73-81 NW,NE,SW,SE == ascending Morton digit).  Only non-empty cells are stored:
// accumulateForce returns on mass == 0 (BHA:216), so an empty cell contributes nothing and is
// never descended.  Each record carries `next`, the pre-order index just past its subtree, so
// the traversal is stackless:
//     open    -> cur + 1      (first child)
//     skip    -> next         (accepted, leaf, or nobody in the wave opened it)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "bh_engine.h"  // BH_SHARD_ROUNDS

namespace bh {

struct __attribute__((aligned(32))) Node {
    double comX;    // BHTree.comX (BHA:106)
    double comY;    // BHTree.comY (BHA:109)
    double mass;    // BHTree.mass (BHA:103)
    uint32_t next;  // pre-order index after this subtree
    uint32_t meta;  // see NODE_* below
};
static_assert(sizeof(Node) == 32, "node record must be 32 bytes");

// meta bits
constexpr uint32_t NODE_LEAF = 1u << 31;             // leaf holding one body (BHA:97)
constexpr uint32_t NODE_SKIP = 1u << 30;             // mass == 0.0: never visited (BHA:216)
// An internal node of mass 0 (every child of mass <= 0, filtered out by computeMass, BHA:189-192)
// carries NODE_SKIP | NODE_LEAF: the reference returns there (BHA:216) and never reaches its
// children -- which may hold negative-mass bodies -- so the exact walk skips it, and the fast
// walk (which tests no flag) takes it as a leaf: an exact +-0 term, and the cursor moves past the
// subtree.  Such a node is told from a real leaf by next > index + 1.
constexpr uint32_t NODE_BODY_MASK = (1u << 30) - 1;  // leaf: body slot (Morton position)
constexpr uint32_t NODE_DEPTH2_MASK = 0xFFu;         // internal: 2 x depth (root = 0)
constexpr int NODE_JMASK_SHIFT = 8;                  // jitter cell: children that got subdivided
constexpr uint32_t NODE_SPAN = 1u << 12;             // internal: body range crosses a COM chunk

// Centre-of-mass chunking (tree_build.hip): nodes inside a 2^COM_CHUNK_SHIFT-body chunk of
// the Morton order are finished by one workgroup; the rest are listed per level.
#ifndef BH_COM_CHUNK_SHIFT
#define BH_COM_CHUNK_SHIFT 10
#endif
constexpr int COM_CHUNK_SHIFT = BH_COM_CHUNK_SHIFT;
__host__ __device__ inline uint32_t span_stride_for(int64_t n) {
    return (uint32_t)((n >> COM_CHUNK_SHIFT) + 2);
}
// chunk boundaries are grouped by 1024 (one span workgroup each, tree_build.hip)
__host__ __device__ inline uint32_t span_groups(uint32_t span_stride) {
    return (span_stride + 1023) / 1024;
}

// Adaptive bucket sort (tree_build.hip): splitter spacing of the previous build's sorted
// order = the expected bucket size.  512 (LDS capacity 2 048 per bucket, 17 KB per workgroup:
// up to 9 buckets in flight per CU) against 1 024 (4 096, 34 KB): build 5.8 -> 5.35 ms per 20 C3
// steps, C4 10.5 -> 9.8 ms per 5 steps; 384 within noise of 512, 256 and 2 048 slower (round 4,
// profiles/r04t_sort_bucket_ab.txt).  98-99 % of the buckets take the LDS bin radix path
// (tools/sort_stats.py).
#ifndef BH_SORT_B
#define BH_SORT_B 512
#endif
constexpr int SORT_B = BH_SORT_B;
__host__ __device__ inline uint32_t sort_buckets(int64_t n) {
    return (uint32_t)((n + SORT_B - 1) / SORT_B);
}

// Cell-start table: first sorted body of every depth-D0 cell, so the end of any node at
// depth <= D0 is one load, and deeper searches stay inside one depth-D0 cell.
constexpr int CELL_TABLE_MAX_DEPTH = 8;

constexpr int MAX_DEPTH_TAB = 40;

// Root cell and per-depth geometry, computed on the host exactly as the reference does:
// root Quad(W/2, H/2, max(W,H)/2 + 2) (BHA:360-361); child h = h / 2.0 (BHA:74).
struct Geometry {
    double root_cx, root_cy, root_h;
    int J;                     // first depth whose h < 1e-3: the jitter depth (BHA:146)
    double h[MAX_DEPTH_TAB];   // h at depth d
    double s2[MAX_DEPTH_TAB];  // (h*2.0)^2 at depth d (BHA:226)
};

// Key of a body outside the root cell (never inserted, BHA:126): sorts after every
// in-root key and differs from all of them at every prefix length.
__host__ __device__ inline uint64_t sentinel_key(int J) { return 1ull << (2 * J); }
// The build sorts the top 32 bits of the (2J+1)-bit keys and fixes the rare equal-prefix runs.
__host__ __device__ inline int key32_shift(int J) { return 2 * J + 1 > 32 ? 2 * J + 1 - 32 : 0; }

// Force-evaluation constants (BHA:225,253,256,378).
struct ForceParams {
    double G, soft2, theta2;
};

// Body state in slot order.
struct BodyState {
    double *x, *y, *vx, *vy, *m;
    uint32_t *cidx;  // caller (list) index; CIDX_DEAD marks a merged-away body until compaction
};
constexpr uint32_t CIDX_DEAD = 1u << 31;

// A chunk-spanning node's children, gathered once its local children are final: per child
// either a reference to another span node (SPAN_REF | owner boundary) with zero values, or
// the child's (mass, comX*mass, comY*mass) — zeros for mass <= 0 (BHA:189-192 skip those;
// adding +0.0 leaves the running sums bit-identical).
struct __attribute__((aligned(16))) SpanSlot {
    uint32_t ch[4];
    double v[4][3];
};
// (accessors: the records were also tried as field planes -- coalesced per field -- with no
// gain: the level pass is bound by the line requests one CU can keep in flight, round 4)
__device__ __forceinline__ void span_put(SpanSlot *base, size_t, size_t slot, const SpanSlot &s) {
    base[slot] = s;
}
__device__ __forceinline__ SpanSlot span_get(const SpanSlot *base, size_t, size_t slot) {
    return base[slot];
}

// Wave priority of the kernels that the pipelined one-GPU step runs next to the second traversal
// (merge rule, next tree build; engine.cpp evaluate_pipelined): they are latency-bound chains on
// the critical path once the traversal's last workgroups are placed, and at the default priority
// a traversal wave sharing their SIMD wins half the issue slots (k_merge_replay, one workgroup:
// 8-24 us alone, 170 us in the traversal's tail).  s_setprio only orders issue between the waves
// of one SIMD; alone on the GPU it changes nothing.
#ifndef BH_CHAIN_PRIO
#define BH_CHAIN_PRIO 1
#endif
__device__ __forceinline__ void chain_prio() {
    if (BH_CHAIN_PRIO) asm volatile("s_setprio 3");
}

// Workgroup i of a launch runs on XCD i % 8 (8 XCDs, each with its own 4 MB L2).  For gathers
// whose neighbouring blocks read overlapping lines, xcd_block() remaps the hardware block index
// so that every XCD takes runs of BH_XCD_RUN consecutive logical blocks (0: identity; 16 is
// ~1% faster for k_prep/k_key_gather and the old per-body emit kernel at C3 and C4 than the identity, A/B on one box).
#ifndef BH_XCD_RUN
#define BH_XCD_RUN 16
#endif
#ifdef __HIP__  // HIP translation units only (engine.cpp is host C++)
// Max over the wave of max(|vx|, |vy|) (every lane of the wave must call it; lanes without a body
// pass 0) into *vmax as the bits of a non-negative double -- ordered like the values -- with one
// atomic per wave; a non-finite speed counts as +inf.
__device__ __forceinline__ void wave_vmax(unsigned long long *vmax, double vx, double vy) {
    const double ax = __builtin_fabs(vx), ay = __builtin_fabs(vy);
    double v = ax > ay ? ax : ay;
    if (!(ax <= 1.7976931348623157e308 && ay <= 1.7976931348623157e308)) v = __builtin_inf();
    unsigned long long b = (unsigned long long)__double_as_longlong(v);
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long c = __shfl_xor(b, o, 64);
        b = c > b ? c : b;
    }
    if ((threadIdx.x & 63) == 0 && b) atomicMax(vmax, b);
}

template <uint32_t RUN = BH_XCD_RUN>
__device__ __forceinline__ uint32_t xcd_block() {
    uint32_t b = blockIdx.x;
    if (RUN > 0) {
        constexpr uint32_t C = RUN, G = 8 * C;
        const uint32_t full = gridDim.x / G;
        if (b < full * G) b = (b / 8 / C) * G + (b % 8) * C + (b / 8) % C;
    }
    return b;
}

// Morton key of one body (BHA:126,153-154): the depth-J cell by exact grid-line compares, the
// sentinel for a body outside the root or merged away (k_morton, the fused traversal epilogue).
__device__ __forceinline__ uint64_t morton_key(const Geometry &g, double px, double py, bool dead) {
    const double cx = g.root_cx, cy = g.root_cy, h = g.root_h;
    if (!(px >= cx - h && px < cx + h && py >= cy - h && py < cy + h) || dead)
        return sentinel_key(g.J);  // BHA:126 -- not inserted (or merged away this call)
    // The descent (BHA:153-154 at every depth: digit = p >= cell centre) ends in the depth-J
    // cell [x0 + i w, x0 + (i + 1) w) that holds p: every centre it compares against is a grid
    // line x0 + k w, exact in binary64 (dyadic, < 40 significant bits), and p stays in the
    // current cell, so i = floor((p - x0) / w) in exact arithmetic.  It is taken from the
    // rounded quotient (off by at most one near a line) and settled by two exact compares
    // against the grid lines, the same compares the descent makes.
    const double w = 2.0 * g.h[g.J];
    const double x0 = cx - h, y0 = cy - h;
    const int64_t top = ((int64_t)1 << g.J) - 1;
    auto cell = [&](double p, double o) __attribute__((always_inline)) {
        int64_t c = (int64_t)((p - o) * (1.0 / w));
        c = c < 0 ? 0 : (c > top ? top : c);
        if (p < o + (double)c * w) --c;
        else if (c < top && p >= o + (double)(c + 1) * w) ++c;
        return (uint64_t)c;
    };
    auto spread = [](uint64_t v) __attribute__((always_inline)) {  // bit k -> bit 2k
        v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
        v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
        v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
        v = (v | (v << 2)) & 0x3333333333333333ull;
        return (v | (v << 1)) & 0x5555555555555555ull;
    };
    return spread(cell(px, x0)) | (spread(cell(py, y0)) << 1);  // digit = ix | iy << 1
}

__device__ __forceinline__ bool spl_le(const uint64_t *__restrict__ spl, uint32_t t, uint64_t v) {
    return t == 0 || spl[t] <= v;  // spl[0] acts as -infinity: bucket 0 takes everything below
}

// largest t in [0, nb) with spl[t] <= v, galloping from `guess`
__device__ inline uint32_t find_bucket(const uint64_t *__restrict__ spl, uint32_t nb, uint64_t v,
                                       uint32_t guess) {
    uint32_t t = min(guess, nb - 1);
    uint32_t lo, hi;  // spl_le(lo) holds; hi == nb or !spl_le(hi)
    if (spl_le(spl, t, v)) {
        lo = t;
        uint32_t step = 1;
        for (;;) {
            const uint32_t j = lo + step;
            if (j >= nb) {
                hi = nb;
                break;
            }
            if (!spl_le(spl, j, v)) {
                hi = j;
                break;
            }
            lo = j;
            step <<= 1;
        }
    } else {  // t > 0
        hi = t;
        uint32_t step = 1;
        for (;;) {
            if (step >= hi) {
                lo = 0;
                break;
            }
            const uint32_t j = hi - step;
            if (spl_le(spl, j, v)) {
                lo = j;
                break;
            }
            hi = j;
            step <<= 1;
        }
    }
    while (hi - lo > 1) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (spl_le(spl, mid, v)) lo = mid; else hi = mid;
    }
    return lo;
}

// One atomic per distinct bucket among the wave's active lanes: the lane's offset inside bucket b
// (any order inside a bucket: each bucket is sorted whole by (key32, slot) afterwards).
__device__ __forceinline__ uint32_t bucket_offset(uint32_t b, uint32_t *__restrict__ counts) {
    uint64_t todo = __ballot(1);
    uint32_t myoff = 0;
    while (todo) {
        const int leader = __builtin_ctzll(todo);
        const uint32_t bl = __builtin_amdgcn_readlane(b, leader);
        const uint64_t same = __ballot(b == bl);
        uint32_t o = 0;
        if ((int)__lane_id() == leader) o = atomicAdd(&counts[bl], (uint32_t)__popcll(same));
        o = __builtin_amdgcn_readlane(o, leader);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(same >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)same, 0u));
        if (b == bl) myoff = o + below;
        todo &= ~same;
    }
    return myoff;
}
#endif

// ---- launchers (tree_build.hip) --------------------------------------------------
// The pipelined step's traversal copies of what the overlapped merge rule and build overwrite
// while the second traversal reads it (k_trav_inputs' job, integrate.hip), written by k_emit_com
// when m is set: masses and flags in the new order, the carried lane map, the node count; the
// merge rule's mailbox header cleared.
struct TravCopy {
    double *m = nullptr;
    uint32_t *cidx = nullptr;
    uint32_t *lanes = nullptr;  // (with lanes_remap only)
    uint32_t *T = nullptr;
    uint32_t *box_header = nullptr;
};

struct TreeBuffers {
    BodyState src;  // state before the build (previous slot order)
    BodyState dst;  // receives the state in the new Morton order (positions may be jittered)
    uint64_t *keys, *keys_s;
    uint32_t *keys32, *keys32_s;  // sort keys (32-bit prefixes) before / after the sort
    uint32_t *idx, *perm;
    int8_t *cpl;           // c(a): common digit count between sorted keys a, a+1; -1 at ends
    uint32_t *cnt, *base;  // node slots per sorted body; exclusive scan (n + 1 entries)
    uint32_t *cell_start;  // [4^D0 + 1] first sorted body of each depth-D0 cell
    uint32_t *lanes_remap = nullptr;  // traversal lane map to carry through this build (or null)
    Node *nodes;
    uint32_t *scalars;     // [1] = error flags
    uint32_t *span_list;   // [(J + 1) * span_stride]: chunk-spanning node per (level, boundary)
    uint32_t span_stride;
    struct SpanSlot *span_children;  // [(J + 1) * span_stride]
    uint32_t *super_list;  // [(J + 1) * span_groups]: group-crossing span node per (level, group)
    void *scratch;
    size_t scratch_bytes;
    // adaptive bucket sort: splitters of the previous build (spl_nb of them, 0 = none: rocprim
    // sort), bucket counts (kept zeroed between builds) and starts, sort_buckets(cap) + 2 each
    uint64_t *spl;
    uint32_t spl_nb;
    uint32_t *bcount, *bstart;
    bool keys_ready = false;  // keys, keys32 and the bucket counts were written by the traversal
    // the merge rule's heavy bodies (live, m > heavy_thr, BHA:474) listed by k_prep in this
    // build's slot order, any order: heavy[atomicAdd(heavy_count, 1)] = slot (null: not wanted;
    // *heavy_count is zero before the build -- k_merge_replay clears it after its use)
    uint32_t *heavy = nullptr, *heavy_count = nullptr;
    double heavy_thr = 0.0;
    TravCopy tc{};  // (m null: none)
};

int cell_table_depth(int J, int64_t n);
size_t tree_scratch_bytes(int64_t n, int J);
hipError_t tree_build(const TreeBuffers &b, int64_t n, const Geometry &g, hipStream_t s);
// Splitters spl[from, to) for a bucket sort over more slots than the build that wrote spl[0,
// from): (sentinel prefix, t * SORT_B) -- the tail of a grown subset capacity is dead padding
// (sentinel keys in slot order), which would otherwise fall into one oversized last bucket.
void extend_splitters(uint64_t *spl, uint32_t from, uint32_t to, int J, hipStream_t s);
// dst.v[a] = src.v[perm[a]]: the velocities of a build made with src.vx = null (k_prep skips them)
void permute_velocities(int64_t n, const uint32_t *perm, const double *svx, const double *svy,
                        double *dvx, double *dvy, hipStream_t s);
// After a tree_build: lanes = the bodies in Hilbert order of their cells (refresh), or the
// previous lane map carried through this build's permutation (k_prep leaves old slot -> new
// slot in keys32).  Uses keys32 / keys32_s / idx.
hipError_t lane_order(const TreeBuffers &b, int64_t n, int J, bool refresh, uint32_t *lanes,
                      hipStream_t s);
// The refresh half of lane_order on its own buffers (the pipelined step runs it beside the next
// first traversal, engine.cpp): Hilbert keys of the sorted Morton keys, radix-sorted with slots.
hipError_t lane_order_into(const uint64_t *keys_s, int64_t n, int J, uint32_t *hkey,
                           uint32_t *hkey_s, uint32_t *slot, void *scratch, size_t scratch_bytes,
                           uint32_t *lanes, hipStream_t s);
size_t lane_sort_bytes(int64_t n);

// ---- launchers (traverse.hip) ----------------------------------------------------
// Accelerations F/m of slots [lo, hi), written interleaved to a2[2p], a2[2p+1].
// node_cap: allocated node records (reads may run up to one record past the tree's last one).
// kick (optional, one GPU, no visit counting): the KDK update of the evaluated slots is applied
// in the kernel's epilogue instead of writing a2 -- KICK_DRIFT = k_kick_drift (BHA:414-422),
// KICK_ONLY = k_kick (BHA:429-432), same operations in the same order.
// KICK_OWN_DRIFT / KICK_OWN_ONLY (multi-rank LET, owner integration): the lane applies
// k_kick_drift / k_kick to its own body in the replicated state (velocities at slot rep[q]) and
// writes the body's new position (x + v dt, or x as the build left it) to a2[2q..2q+1] -- the
// peers take positions from the exchange, velocities once per call (engine.cpp).
enum KickMode {
    KICK_NONE = 0, KICK_DRIFT = 1, KICK_ONLY = 2, KICK_OWN_DRIFT = 3, KICK_OWN_ONLY = 4
};
// The next build's first two passes done by the drifting traversal (KICK_DRIFT of the pipelined
// one-GPU step): every lane writes its body's Morton key (k_morton) and bucket / in-bucket offset
// of the adaptive sort (k_bucket_count) right after the drift; the build then starts at the scan.
struct MortonFuse {
    uint64_t *keys = nullptr;  // null: off
    uint32_t *keys32 = nullptr;
    const uint64_t *spl = nullptr;  // the previous build's splitters (spl_nb > 0)
    uint32_t spl_nb = 0;
    uint32_t *bkt = nullptr, *off = nullptr, *counts = nullptr;
};
struct KickArgs {
    KickMode mode;
    double *vx, *vy;  // x, y are the traversal's own position arrays (KICK_OWN_*: replicated v)
    double dtHalf, dt;
    const uint32_t *rep = nullptr;  // KICK_OWN_*: lane -> replicated slot (null: the lane)
    MortonFuse mf{};
    // KICK_ONLY / KICK_DRIFT after a build that left the velocities in the previous slot order:
    // v[p] = sv[perm[p]] + a dt/2 (the build's permutation of v, fused; null: in place)
    const double *svx = nullptr, *svy = nullptr;
    const uint32_t *perm = nullptr;
    // KICK_OWN_DRIFT: max over the launch's bodies of max(|vx|, |vy|) after the kick, as the bits
    // of a non-negative double (atomicMax; non-finite -> +inf): the drift's displacement bound
    unsigned long long *vmax = nullptr;
};
// Diagnostic counters of the counting walk (all per evaluation): per body, the non-empty
// nodes visited (BHA:216 passed) and the point-force contributions (accepted internal nodes
// + other bodies' leaves, BHA:219-221,228-230); per wavefront, the nodes the shared cursor
// stopped at and the point-force blocks it executed.
struct TraverseCounters {
    uint32_t *visits, *contrib;
    uint32_t *wave_iters, *wave_blocks;
};
// A lane mapped to LANE_IDLE neither walks nor writes (the LET evaluation after a subset
// overflow, whose call is replayed).
constexpr uint32_t LANE_IDLE = 0xFFFFFFFFu;
// lanes (nullable): lane -> body slot map (the Hilbert grouping made by lane_order in
// tree_build.hip); [lo, hi) is then a range of lanes and a2 is written by lane; null = lane q
// walks slot q and a2 is written by slot.
// Longest-first dispatch of the traversal's waves (traverse.hip wave_order): `cost` receives
// every wave's duration (wall-clock ticks) and `order` the dispatch order of the XCD runs of
// waves, costliest first, made from the previous evaluation's costs.  Only the order in which
// waves start changes -- every body's sum is the same.
struct WaveOrder {
    const uint32_t *order = nullptr;
    uint32_t *cost = nullptr;
};
size_t wave_order_runs(int64_t n);  // runs of a launch over n lanes (0: too many to order)
// Whether traverse() walks [lo, hi) breadth first, one body per wave (traverse.hip bfs_walk)
bool traverse_is_bfs(size_t node_cap, int64_t lo, int64_t hi, int kick_mode, bool counting);
hipError_t wave_order(const uint32_t *cost, int64_t n, uint32_t *order, hipStream_t s);
void traverse(const Node *nodes, size_t node_cap, const uint32_t *d_T, double *x, double *y,
              const double *m, const uint32_t *cidx, int64_t lo, int64_t hi, const Geometry &g,
              const ForceParams &fp, double *a2, const TraverseCounters *cnt,
              hipStream_t s, const KickArgs *kick = nullptr, const uint32_t *lanes = nullptr,
              const WaveOrder *wo = nullptr);
// multi-GPU shard pieces (bh_shard_range): `rounds` x `world` pieces of whole wavefronts
__host__ __device__ inline int64_t shard_sub(int64_t n, int world, int rounds) {
    const int64_t parts = (int64_t)world * rounds;
    const int64_t c = (n + parts - 1) / parts;
    return (c + 63) / 64 * 64;
}
// Rank r owns lanes [r * span, (r + 1) * span), span = rounds * sub; its round k is the lanes
// [r * span + off[k], r * span + off[k + 1]) (whole wavefronts; rounds of unequal size: the
// first ones fill the GPU, the last ones are small so that little of the exchange is exposed).
// Lane q = r * span + off[k] + i sits in the exchange buffer at world * off[k] + r * size_k + i,
// so that the pieces of a round are adjacent (in-place all-gather).  span == 0: the identity.
struct GatherLayout {
    int64_t span;
    int64_t off[BH_SHARD_ROUNDS + 1];
    int world;
};
GatherLayout shard_layout(int64_t n, int world);  // engine.cpp (bh_shard_range's layout)
__host__ __device__ inline int64_t gather_slot(const GatherLayout &L, int64_t q) {
    if (L.span == 0) return q;
    const int64_t r = q / L.span, t = q - r * L.span;
    int k = 0;
#pragma unroll
    for (int j = 1; j < BH_SHARD_ROUNDS; ++j) k += t >= L.off[j] ? 1 : 0;
    return L.world * L.off[k] + r * (L.off[k + 1] - L.off[k]) + (t - L.off[k]);
}

// Exactness check of the traversal's in-range sqrt/reciprocal sequences against the IEEE
// operations on n generated operands; adds the mismatch count to *d_bad.
hipError_t selftest_fast_math(int64_t n, uint64_t seed, unsigned long long *d_bad, hipStream_t s);

// ---- launchers (let.hip): the multi-rank build as a locally essential tree -------------
// Every rank keeps the full replicated state but builds only the bodies of the depth-LET_P
// cells within reach of the bodies it evaluates (its pieces); the rest of the tree is the top
// (depth < LET_P) assembled from every rank's depth-LET_P cell values, with remote cells as
// childless records every local body provably accepts.  See let.hip.
constexpr int LET_P = 8;
constexpr int64_t LET_CELLS = (int64_t)1 << (2 * LET_P);
// an exchange table: LET_CELLS cell records + one status record (cnt = subset overflow)
constexpr int64_t LET_TSTRIDE = LET_CELLS + 1;
struct __attribute__((aligned(32))) LetCell {
    double comX, comY, mass;
    uint32_t cnt;  // in-tree bodies of the cell, saturated at 2 (0 empty, 1 leaf, 2 internal)
    uint32_t tag;  // exchange table: 1 = provided; levels: depth-LET_P cell of a 1-body node
};
static_assert(sizeof(LetCell) == 32, "LET cell record must be 32 bytes");
struct LetPieces {  // rank `rank` owns lanes [(k*world + rank)*sub, +sub) for k < rounds
    int64_t n, sub;
    int world, rank, rounds;
    const uint32_t *lanes;  // lane -> replicated slot (the Hilbert wave map), or null: identity
};
struct LetBufs {
    uint8_t *ecell, *hcell;   // [LET_CELLS] cells of own bodies / cells built locally
    uint8_t *own;             // [n] replicated slot evaluated by this rank
    uint32_t *subpos;         // [n] replicated slot -> subset slot (subset bodies)
    uint32_t *flag_all;       // [1] a non-finite own body: every cell is built
    uint8_t *flag8;           // [n] subset flag per replicated slot
    uint32_t *sel, *selpos;   // [n / 256 + 2] subset count per 256-slot block, its scan
    uint32_t *cstart;         // [LET_CELLS + 1] first sorted subset body of each cell
    LetCell *table, *tables;  // own exchange table, all ranks' tables [world][LET_CELLS]
    LetCell *levels;          // depths 0..LET_P, level d at ((4^d - 1) / 3)
    uint32_t *w, *posc, *bsz; // [LET_CELLS + 1] nodes per cell, their scan, block sizes
    uint32_t *csrc, *ccnt, *cpos;  // [LET_CELLS + 1] local block: first subset node, nodes, scan
    Node *nodes;              // the assembled tree, pre-order
    uint32_t node_cap;        // records allocated for it (every write is bounded by it)
    uint32_t *lanes;          // [n] lane -> subset slot (own pieces)
    void *scratch;
    size_t scratch_bytes;
    // the selection's restriction to candidate slot blocks (let_select, LetSweep)
    uint8_t *own_blk;         // [n / 256 + 2] the block holds an own body
    uint32_t *rowmask;        // [256 * 8] built cells as one 256-bit mask per grid row
    unsigned long long *vmax; // [nvmax] drift speed bounds: own, then every rank's (cleared
    int nvmax;                //   by the selection, after every reader of the last ones)
};
// Which 256-slot blocks of the replicated state the selection scans.  The state keeps the slot
// order of the last full build between full builds, so each block's bodies then occupied a small
// box of depth-LET_P cells (box: col_lo | col_hi << 8 | row_lo << 16 | row_hi << 24; lo > hi: no
// body in the root).  Since then no body moved farther than disp[0] (the drifts' bound: max
// speed x dt per drift, every rank's maximum exchanged) + allow (jitter, 2 x 2e-3 per build), so a
// body that lies in a built cell now lies in its block's box widened by floor(D / w) + 1 cells.
// Blocks whose widened box holds no built cell and no own body are skipped: the subset is the
// same, bit for bit (valid = false, or a bound beyond 64 cells: every block is scanned).
struct LetSweep {
    const uint32_t *box;
    const double *disp;
    double allow;
    bool valid;
};
// the boxes of the state's 256-slot blocks (after a full build, every rank alike)
void let_boxes(int64_t n, const BodyState &st, const Geometry &g, uint32_t *box, hipStream_t s);
// disp[0] += max(bits of vmax[0 .. k)) x dt (non-finite: +inf)
void let_disp_add(double *disp, const unsigned long long *vmax, int k, double dt, hipStream_t s);
// Largest gap^2 (in cells) at which a depth-LET_P cell may still be opened by a body of a cell
// at that gap; cells beyond it are accepted by every such body.  < 0: the LET does not apply.
double let_include_gap2(const Geometry &g, double theta2, double soft2);
size_t let_scratch_bytes(int64_t n);
inline int64_t let_sel_blocks(int64_t n) { return (n + 255) / 256; }
// own cells, halo, subset flags + scan + gather into `sub` (vx carries the replicated slot);
// the subset has selpos[let_sel_blocks(n)] bodies.  The build runs over a host-chosen capacity S without a host
// round trip: `sub` is padded with dead bodies (sentinel keys: not in the tree) up to S, and
// selpos[n] > S is an overflow (the status record of the table; scal[5] = max subset size)
// Where the selection reads body positions: the replica (a2 == null), or -- between LET
// evaluations, whose new positions are not copied into the replica -- the exchange buffer: lane
// q's position at a2[2 gather_slot(gl, q)], and slot i's at a2[2 gslot[i]] (gslot: the gather
// slot of the lane that holds slot i, made once per lane map by let_gather_slots).
struct PosSrc {
    const double *a2;
    GatherLayout gl;
    const uint32_t *gslot;
};
// mf.keys non-null: the gather also writes the subset build's Morton keys and bucket
// assignment (k_morton + k_bucket_count of tree_build, which then sets keys_ready)
hipError_t let_select(const BodyState &st, const PosSrc &ps, const Geometry &g,
                      const LetPieces &pc, double gap2, const LetBufs &L, const BodyState &sub,
                      int64_t S, uint32_t *scal, hipStream_t s, const MortonFuse &mf = {},
                      const LetSweep &sw = {}, bool clean = false);
// gslot[lanes[q]] = gather_slot(gl, q) (lanes null: the identity map)
void let_gather_slots(int64_t n, const uint32_t *lanes, GatherLayout gl, uint32_t *gslot,
                      hipStream_t s);
// after tree_build over the subset: the own cells' exchange table
hipError_t let_table(int64_t n_sub, const Geometry &g, const LetBufs &L, const TreeBuffers &tb,
                     hipStream_t s);
// after the exchange (L.tables, LET_TSTRIDE per rank): any rank's overflow -> scal[4]; top
// levels, layout, node array, lane map; tree size posc[LET_CELLS].  *cleaned: the lane-map kernel
// also cleared the selection's marks for the next selection (which may then skip k_let_clear)
hipError_t let_assemble(int64_t n_sub, const Geometry &g, const LetPieces &pc, const LetBufs &L,
                        const TreeBuffers &tb, uint32_t *scal, hipStream_t s,
                        bool *cleaned = nullptr);
// owner integration: a2 (gather slots) holds every lane's (x, y) -> the replicated state; the
// solo fill writes the current positions of all lanes first
void let_set_pos(int64_t n, const uint32_t *lanes, const double *a2, GatherLayout gl, double *x,
                 double *y, const uint32_t *skip, hipStream_t s);
void let_fill_pos(int64_t n, const uint32_t *lanes, const double *x, const double *y, double *a2,
                  GatherLayout gl, hipStream_t s);
// velocity exchange of the owner integration: own lanes' (vx, vy) into a2, all lanes' back out
void let_pack_vel(const LetPieces &pc, const double *vx, const double *vy, double *a2,
                  GatherLayout gl, hipStream_t s);
void let_unpack_vel(int64_t n, const uint32_t *lanes, const double *a2, GatherLayout gl,
                    double *vx, double *vy, hipStream_t s);

// ---- launchers (direct.hip): theta = 0 all-pairs ---------------------------------
// Non-empty leaves of the last tree in pre-order (the reference's theta = 0 summation order).
struct LeafList {
    double *rec;  // 32 B per leaf: x, y, m, body slot (low 32 bits; self-skip), in pre-order
};
size_t leaf_select_bytes(int64_t node_cap);
// cover: 2 (node_cap + 1) int32 of scratch (leaves under a mass-0 node are never visited)
hipError_t leaf_list_build(const Node *nodes, const uint32_t *d_T, int64_t node_cap,
                           uint8_t *flags, uint32_t *sel, uint32_t *d_count, const LeafList &L,
                           int64_t n, int32_t *cover, void *tmp, size_t tmp_bytes, hipStream_t s);
void direct_forces(const LeafList &L, const uint32_t *d_count, const double *x, const double *y,
                   const double *m, int64_t lo, int64_t hi, double G, double soft2, double *a2,
                   hipStream_t s);

// ---- launchers (integrate.hip) ---------------------------------------------------
// a2 indexed by traversal lane when lanes != null (lane i holds body slot lanes[i])
// lane q's acceleration at a2[2 * gather_slot(gl, q)]
void kick_drift(int64_t n, const double *a2, double *x, double *y, double *vx, double *vy,
                double dtHalf, double dt, hipStream_t s, const uint32_t *lanes = nullptr,
                GatherLayout gl = GatherLayout{}, unsigned long long *vmax = nullptr);
struct MergePair;
// (box: the merge mailbox, whose header it clears for the overlapped merge rule, or null)
void copy_trav_inputs(int64_t n, const double *m, double *m_t, const uint32_t *cidx,
                      uint32_t *cidx_t, const uint32_t *lanes, uint32_t *lanes_t,
                      const uint32_t *T, uint32_t *T_t, hipStream_t s, MergePair *box = nullptr);
// k_kick_drift of a2 written by lane (lanes: lane -> slot, or null) plus, when mf.keys is set, the
// next build's keys and bucket assignment -- the drifting traversal's epilogue as its own pass
void kick_drift_keys(int64_t n, const double *a2, double *x, double *y, double *vx, double *vy,
                     const uint32_t *cidx, double dtHalf, double dt, const uint32_t *lanes,
                     const Geometry &g, const MortonFuse &mf, hipStream_t s);
void kick(int64_t n, const double *a2, double *vx, double *vy, double dtHalf, hipStream_t s,
          const uint32_t *lanes = nullptr, GatherLayout gl = GatherLayout{});
void iota_u32(uint32_t *p, int64_t n, hipStream_t s);
// caller-order copies: dst_k[cidx[s]] = src_k[s]
void scatter_to_caller(int64_t n, const uint32_t *cidx, int k, const double *const *src,
                       double *const *dst, hipStream_t s);
void scatter_acc_to_caller(int64_t n, const uint32_t *cidx, const double *a2, double *ax,
                           double *ay, hipStream_t s, const uint32_t *lanes = nullptr,
                           GatherLayout gl = GatherLayout{});
// The pinned caller-order mirror: keep[c] / pos[c] over the caller indices of a state whose
// tombstones still hold theirs (keep, pos: n entries; tmp: compact_scratch_bytes(n)), then
// dst_j[pos[c]] = src_j[slot] for the live bodies -- the list after the call's removals.
hipError_t mirror_index(int64_t n, const uint32_t *cidx, uint32_t *keep, uint32_t *pos, void *tmp,
                        size_t tmp_bytes, hipStream_t s);
// For bh_step_positions, one array for one copy: out[0..4) = scalars[0..4) (tree flags, removals,
// mailbox overflow) and zeros up to MIRROR_HDR, then out[MIRROR_HDR + pos[c]] = c for every caller
// index c < n with keep[c] -- survivor j's index in the list before the call (ascending in j).
constexpr int MIRROR_HDR = 16;
void mirror_survivors(int64_t n, const uint32_t *keep, const uint32_t *pos, const uint32_t *scalars,
                      uint32_t *out, hipStream_t s);
void mirror_scatter(int64_t n, const uint32_t *cidx, const uint32_t *pos, int k,
                    const double *const *src, double *const *dst, hipStream_t s);
// *dst = *src by one thread at the chain's wave priority (a 4-byte hipMemcpyAsync beside the
// traversal is a blit kernel that waits ~0.5 ms for a wave slot, with the merge rule behind it)
void copy_u32(uint32_t *dst, const uint32_t *src, hipStream_t s);
// *dst |= *src | set; *src = 0 (one thread): hands a flag word over to another
void take_u32(uint32_t *dst, uint32_t *src, hipStream_t s, uint32_t set = 0u);
// The end-of-call read-back of the merge bookkeeping in one copy: out[0..3] = scal[0..3],
// out[4..11] = the mailbox header, out[12] = scal[8], out[16 + i] = dlog[i] for i < ahead
void pack_readback(const uint32_t *scal, const MergePair *box, const uint32_t *dlog, uint32_t ahead,
                   uint32_t *out, hipStream_t s);
// dst[perm[a]] = src[a] for x and y: positions of a sorted build (jitter included) back into the
// state's own slot order (multi-rank getTreeForDebug, engine.cpp bh_get_quads)
void unpermute_positions(int64_t n, const uint32_t *perm, const double *sx, const double *sy,
                         double *dx, double *dy, hipStream_t s);

struct MergePair {
    uint32_t h_cidx, v_cidx;  // heavy body and candidate victim, caller indices
    uint32_t h_slot, v_slot;
    double h_mass, v_mass;
};
// mailbox header (pairs[0] reinterpreted): pair count, heavy count
struct MergeHeader {
    uint32_t pairs, heavies, pad0, pad1;
    double pad2, pad3;
};
static_assert(sizeof(MergeHeader) == sizeof(MergePair), "mailbox header size");
// heavy = live m > thr (BHA:474) -> slot list (any order); then the distance test (BHA:493-501)
// heavy_count: the list was made by the last build (TreeBuffers::heavy): no k_heavy pass
void merge_candidates(int64_t n, const double *x, const double *y, const double *m,
                      const uint32_t *cidx, double thr, double minD2, uint32_t *heavy,
                      MergePair *box, uint32_t cap, hipStream_t s, bool header_zeroed = false,
                      const uint32_t *heavy_count = nullptr);
// Sequential merge rule on the device (one workgroup): removals become tombstones
// (cidx |= CIDX_DEAD) logged in dlog[scal[2]++]; scal[3] = pair count if the mailbox overflowed.
// skeys/sidx: scratch of 2 x cap entries (long lists); bits: (n_cap >> 5) + 1 words and
// slot_of: n_cap entries, n_cap > every caller index (the bitmap replay of long lists); n bounds
// the caller indices (radix sort width).
// heavy_count (nullable): the build's heavy-list counter, cleared for the next build
void merge_replay(const MergePair *box, uint32_t cap, double *m, uint32_t *cidx, uint32_t *scal,
                  uint32_t *dlog, uint64_t *skeys, uint32_t *sidx, uint32_t *bits,
                  uint32_t *slot_of, int64_t n, hipStream_t s, uint32_t *heavy_count = nullptr);
size_t compact_scratch_bytes(int64_t n);
// Remove tombstoned slots preserving order; caller indices are renumbered past the removed
// ones (dead_cidx sorted ascending, n_dead entries).  keep, pos: n-entry scratch.
// The traversal's lane map through compact_state (keep / pos of that call): surviving lanes in
// order, renumbered to the new slots, into out.  flag, qpos: n-entry scratch.
hipError_t compact_lanes(int64_t n, const uint32_t *lanes, const uint32_t *keep,
                         const uint32_t *pos, uint32_t *flag, uint32_t *qpos, uint32_t *out,
                         void *tmp, size_t tmp_bytes, hipStream_t s);
// (flag, qpos of that compact_lanes call) interleaved pairs by lane: out[2 qpos[q]..] = a2[2 q..]
void compact_lane_pairs(int64_t n, const uint32_t *flag, const uint32_t *qpos, const double *a2,
                        double *out, hipStream_t s);
void compact_pair(int64_t n, const uint32_t *keep, const uint32_t *pos, const double *sx,
                  const double *sy, double *dx, double *dy, hipStream_t s);
hipError_t compact_state(int64_t n, uint32_t *keep, const BodyState &src, const BodyState &dst,
                         const uint32_t *dead_cidx, uint32_t n_dead, uint32_t *pos, void *tmp,
                         size_t tmp_bytes, hipStream_t s);

}  // namespace bh
