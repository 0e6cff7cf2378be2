// Force evaluation — replaces BHTree.accumulateForce/pointForceAcc and the coroutine driver
// PhysicsEngine.computeAccelerations (BHA:215-259, BHA:374-395).
//
// One lane = one body, bodies in Morton order so a wavefront's 64 bodies are spatial
// neighbours.  The wave walks ONE shared pre-order cursor over the flattened tree:
//   * the node record is wave-uniform (one 32-byte scalar load serves 64 bodies);
//   * every lane evaluates the reference's own criterion s2 < theta2*dist2 (BHA:228) for
//     itself; a lane that accepts a node adds its point force and ignores that node's
//     subtree (resume = node.next); the cursor descends (cur + 1) iff at least one lane
//     opened the node (__ballot), otherwise it skips the subtree (cur = next).
// Because the cursor order is the reference's DFS order and each lane only sums the nodes
// its own recursive DFS would have summed, every body's force is the reference's sum in the
// reference's order: bit-identical, not merely close (no Burtscher "open for all").
//
// The kernel is bound by fp64 VALU issue (the IEEE sqrt and two IEEE divisions per
// interaction), not by HBM: the node stream is shared by 64 lanes and served from the
// scalar cache / L2.  See DESIGN.md for the roofline accounting.
// Small lists (bfs_walk below): the first walk of a step over <= 4 096 bodies serves one body
// per wave and examines the tree level by level, the terms added in pre-order -- the same sum.
#include <cstdlib>

#include "bh_device.hpp"
#include "fastmath.hpp"

namespace bh {
namespace {

// Workgroups in runs of BH_TRAV_XCD_RUN consecutive waves per XCD (bh_device.hpp): neighbouring
// waves walk nearly the same nodes, so a run shares its XCD's L2 (C3 -1.5 % at runs of 32..512
// against the round-robin default).
#ifndef BH_TRAV_XCD_RUN
#define BH_TRAV_XCD_RUN 64
#endif
constexpr int TB = 64;  // one wave per workgroup: finest dispatch granularity (C4 -1.5 %, C3 -0.5 %)
// Waves per workgroup of k_traverse: up to MAX_WPB, chosen per launch (waves_per_group below).
// A workgroup's waves share one CU and its scalar data cache, and neighbouring waves walk nearly
// the same node records.
constexpr int MAX_WPB = 8;
static_assert(BH_TRAV_XCD_RUN % MAX_WPB == 0, "an XCD run holds whole workgroups");

typedef double double4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// Node record through an explicit scalar load whose wait is placed by hand (nwait): the next
// record is requested as soon as the cursor decision is made and waited for only after the
// point-force block, so its latency hides behind that block's fp64 work.  (The compiler would
// sink a plain load below the block, to its first use.)
__device__ __forceinline__ u32x8 nload(const Node *p) {
    u32x8 v;
    asm volatile("s_load_dwordx8 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
    return v;
}
// Same, addressed as base + 32-bit byte offset (s_load's SGPR offset): one shift per
// iteration instead of a 64-bit address computation.  Only for node arrays below 4 GiB.
__device__ __forceinline__ u32x8 nload_off(const Node *base, uint32_t idx) {
    u32x8 v;
    asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(v) : "s"(base), "s"(idx << 5) : "memory");
    return v;
}
__device__ __forceinline__ void nwait(u32x8 &v) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(v)); }
__device__ __forceinline__ double as_f64(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Which lanes are active at a stop (cur >= the lane's resume point).  BH_TRAV_STACK 0: a per-lane
// compare at every stop and a per-lane `resume = next` in every point-force block.  1 (round 6):
// the active set is a wave-uniform mask that changes only at "mixed" internal nodes -- some
// active lanes accept the node, others open it: the accepting lanes park until the cursor reaches
// the node's `next`.  Parked subtrees nest (a node pushed later lies inside the earlier ones), so
// their `next` values form a stack: its top in an SGPR, the entries below in one VGPR, entry i in
// lane i (v_writelane / v_readlane), the parked lanes' `next` in a per-lane VGPR written only at
// mixed nodes.  When the cursor reaches the top, every lane whose `next` equals it is active
// again (one compare per pop).  The mask is the per-lane compare's at every stop, exactly: a lane
// active again keeps a stale `next` below every entry pushed after it.  At C3: ~645 stops and
// ~548 blocks per wave against ~106 mixed nodes.  Measured (profiles/r06p_*):
// bit-exact, VALU per wave 21572 -> 20758 (-3.8 %), but SALU 10416 -> 15537 (the pop test at
// every stop, the park test at every internal node) and k_traverse 0.768 -> 0.797 ms (+3.7 %):
// the wave is issue-bound over both units, so the trade loses.  Off by default.
#ifndef BH_TRAV_STACK
#define BH_TRAV_STACK 0
#endif
// (the stack holds one entry per tree level above the cursor: depth < MAX_DEPTH_TAB <= 64 lanes)
static_assert(MAX_DEPTH_TAB <= 64, "the parked-subtree stack holds one level per lane");
// v_writelane_b32 (the lane select goes through M0; no clang builtin on this toolchain)
extern "C" __device__ int bh_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
template <bool FAST, bool COUNT, bool OFF32>
__device__ __forceinline__ void walk(const Node *__restrict__ nodes, uint32_t T, double bx,
                                     double by, double Gm, double soft2, double theta2,
                                     double s2root, uint32_t self, uint32_t resume, double &fx,
                                     double &fy, uint32_t &nvis, uint32_t &niters,
                                     uint32_t &ncontrib, uint32_t &nblocks) {
    uint32_t cur = 0;
#if BH_TRAV_STACK
    uint64_t active = __builtin_amdgcn_ballot_w64(resume == 0u);  // (idle lanes never are)
    uint32_t top = 0xFFFFFFFFu, sp = 0u;  // the stack's top and its entries below, wave-uniform
    uint32_t below = 0u;                  // entry i of those in lane i
#endif
    // one iteration on record `rec`; the next record is requested into `nrec`.  The loop body
    // is unrolled twice with the two records swapping roles (no SGPR copies per iteration).
    // Loading node T (past the last one) is harmless: the node array has slack beyond T.
    auto iter = [&](const u32x8 &rec, u32x8 &nrec) __attribute__((always_inline)) {
        const double comX = as_f64(rec[0], rec[1]), comY = as_f64(rec[2], rec[3]);
        const double mass = as_f64(rec[4], rec[5]);
        uint32_t meta = rec[7];
        asm volatile("" : "+s"(meta));  // keep the flag tests scalar (s_bitcmp)
        uint32_t next = rec[6];
        next = next > cur ? next : cur + 1;  // structural guard: the cursor always advances
        // mass == 0.0 (BHA:216): not visited.  The fast path needs no test: a massless leaf's
        // term is an exact +-0 (mass 0, finite f), and a massless internal node carries the leaf
        // flag too (bh_device.hpp NODE_SKIP), so the wave never descends below it -- only the
        // visit-counting variant must skip it.
        if ((!FAST || COUNT) && (meta & NODE_SKIP)) {
            cur = next;
            nrec = OFF32 ? nload_off(nodes, cur) : nload(nodes + cur);
            nwait(nrec);
            return;
        }
        // lane masks in SGPRs straight from the compares; per-lane booleans via inverse ballot
#if BH_TRAV_STACK
        while (cur >= top) {  // the cursor left a parked subtree: its lanes walk again
            active |= __builtin_amdgcn_ballot_w64(resume == top);
            if (sp == 0u) {
                top = 0xFFFFFFFFu;
            } else {
                --sp;
                top = (uint32_t)__builtin_amdgcn_readlane((int)below, (int)sp);
            }
        }
        const uint64_t act_m = active;
#else
        const uint64_t act_m = __builtin_amdgcn_ballot_w64(cur >= resume);
#endif
        if (COUNT) {
            nvis += __builtin_amdgcn_inverse_ballot_w64(act_m) ? 1u : 0u;
            niters += 1;
        }
        const double dx = comX - bx;  // BHA:223-225 == BHA:251-253
        const double dy = comY - by;
        const double d2 = dx * dx + dy * dy + soft2;
        uint64_t contrib_m, open_m;  // lanes that take / open this node
        if (meta & NODE_LEAF) {  // BHA:217-221: skip self by identity
            // fast path: the own leaf's term is an exact +-0 (fastmath.hpp, lane_self_ok)
            contrib_m = FAST ? act_m
                             : act_m & __builtin_amdgcn_ballot_w64((meta & NODE_BODY_MASK) != self);
            open_m = 0;
        } else {
            // s2 = (h_d * 2.0)^2 with h_d = h_0 / 2^d exactly, so s2 = s2_0 * 4^-d exactly
            // (a power-of-two scaling commutes with rounding), and s2 < t2 <=> s2_0 < t2 * 4^d:
            // the scaling of t2 is exact too (up from a subnormal included) or overflows to
            // +inf where s2 < t2 holds anyway.  The record carries 2d: one scalar mask.
            // Fast path: s2 itself, the reference's own comparison, built on the scalar unit by
            // subtracting 2d from s2_0's exponent field (exact: s2_0 >= 2^-760 keeps it normal
            // for every 2d <= 255, fast_s2_ok) -- one v_ldexp_f64 less per internal node.
            uint64_t acc_m;
            if (FAST) {
                const uint64_t s2b = (uint64_t)__double_as_longlong(s2root) -
                                     ((uint64_t)(meta & NODE_DEPTH2_MASK) << 52);
                acc_m = __builtin_amdgcn_ballot_w64(__longlong_as_double((long long)s2b) <
                                                    theta2 * d2);  // BHA:226-228
            } else {
                const double t2 = __builtin_ldexp(theta2 * d2, (int)(meta & NODE_DEPTH2_MASK));
                acc_m = __builtin_amdgcn_ballot_w64(s2root < t2);  // BHA:226-228
            }
            contrib_m = act_m & acc_m;
            open_m = act_m & ~acc_m;
#if BH_TRAV_STACK
            if (open_m != 0ull && contrib_m != 0ull) {  // mixed: the accepting lanes park
                if (top != 0xFFFFFFFFu) {
                    below = (uint32_t)bh_writelane((int)top, (int)sp, (int)below);
                    ++sp;
                }
                top = next;  // (<= the entry below: this node lies inside that subtree)
                active &= ~contrib_m;
                if (__builtin_amdgcn_inverse_ballot_w64(contrib_m)) resume = next;
            }
#endif
        }
        const uint32_t ncur = open_m != 0ull ? cur + 1 : next;  // descend iff some lane opened
        nrec = OFF32 ? nload_off(nodes, ncur) : nload(nodes + ncur);
        if (COUNT) {  // contributions in the reference's sense: the own leaf is not one
            const bool own = (meta & NODE_LEAF) && (meta & NODE_BODY_MASK) == self;
            ncontrib += (__builtin_amdgcn_inverse_ballot_w64(contrib_m) && !own) ? 1u : 0u;
            nblocks += contrib_m != 0ull ? 1u : 0u;
        }
        if (__builtin_amdgcn_inverse_ballot_w64(contrib_m)) {  // BHA:250-259, order as written
            double invR, invR2;
            if (FAST) {
                double h;
                const double r = sqrt_rn_inrange_h(d2, h);
                invR = rcp_rn_seeded(r, h + h);
                invR2 = rcp_rn_seeded(d2, invR * invR);
            } else {
                invR = 1.0 / sqrt(d2);
                invR2 = 1.0 / d2;
            }
            const double f = Gm * mass * invR2;
            fx += f * dx * invR;
            fy += f * dy * invR;
#if !BH_TRAV_STACK
            resume = next;
#endif
        }
        nwait(nrec);
        cur = ncur;
    };
    if (T == 0) return;  // no body inside the root cell: an empty tree
    u32x8 r0 = nload(nodes), r1;
    nwait(r0);
    // (a `while (cur < T)` head with one exit test in the middle made the compiler keep a dead
    // v_readfirstlane per two stops)
    while (true) {
        iter(r0, r1);
        if (cur >= T) break;
        iter(r1, r0);
        if (cur >= T) break;
    }
}


// ---- one body per wave, breadth first (small launches) -----------------------------------
// A walk is a chain of dependent stops -- the next node is known only after the criterion at
// this one -- so a launch of a few thousand waves (C1's 2 000 or 12 500 bodies) lasts as long as
// one wave's ~250-350 stops of ~0.3 us, however wide the GPU.  Here the whole wave serves ONE
// body and examines the tree level by level: every lane takes one child of an opened node of the
// current level, so the chain is the tree's depth (~15 levels), not the body's visit count.
// The lane that takes an opened node examines its children, from node + 1 along `next` (each
// sibling's record requested before the criterion at the previous one).  Accepted nodes are marked in an LDS bitmap over node indices;
// the flattened tree is in pre-order, so the reference's DFS order of the terms (BHA:215-239)
// IS ascending node index and the set bits, read in ascending order, give the terms in the order
// walk() adds them.  The terms are evaluated 64 at a time, one per lane, and added into the sums
// in that order by one lane each (fx: lane 0, fy: lane 1).  Each term is the expression of
// walk<true>, and each sum the same additions from +0.0: bit-identical.  A body whose levels or
// accepted set overflow the LDS buffers, or whose tree exceeds the bitmap, is walked by walk()
// instead (the caller), so every body gets its exact sum.
// LDS of one wave (~5 KB at C1's 12 500 bodies: 31 waves per CU): the bitmap -- after the scan,
// the terms of one round of 64 --, the level buffers or the accepted list, two counters.
constexpr uint32_t BFS_E_CAP = 128;  // opened nodes per level (two buffers of (node, next))
constexpr uint32_t BFS_A_CAP = 384;  // accepted nodes per body (in the level buffers' space)
// (children blocks -- each internal node's child records side by side, built by a kernel before
// the walk, one gather per child -- measured the same as the chase: C1 'R' 40.5 against 40.0 us
// per evaluation, profiles/r06z5_bfs_child_blocks_ab.txt)
constexpr uint32_t BFS_E_WORDS = 2u;  // words per level entry
constexpr uint32_t BFS_R_WORDS = BFS_A_CAP > 2 * BFS_E_CAP * BFS_E_WORDS
                                     ? BFS_A_CAP : 2 * BFS_E_CAP * BFS_E_WORDS;
constexpr uint32_t BFS_TERM_WORDS = 2 * 64 * 2;  // 64 x (tx, ty) doubles
__host__ __device__ constexpr uint32_t bfs_bm_space(uint32_t bm_words) {
    return bm_words > BFS_TERM_WORDS ? bm_words : BFS_TERM_WORDS;
}
__host__ __device__ constexpr size_t bfs_lds_bytes(uint32_t bm_words) {
    return sizeof(uint32_t) * ((size_t)bfs_bm_space(bm_words) + BFS_R_WORDS + 4);
}

__device__ __forceinline__ double rfl_f64(double v) {  // lane 0's value in every lane
    const long long b = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t &total) {
    uint32_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    total = (uint32_t)__shfl((int)x, 63, 64);
    return x - v;
}

#ifdef BH_BFS_TIMING  // diagnostic build only: per-wave phase stamps of bfs_walk
constexpr int BFS_T_W = 16384, BFS_T_REC = 24;
__device__ uint64_t g_bfs_times[BFS_T_W * BFS_T_REC];
#define BFS_STAMP(slot)                                                                     \
    do {                                                                                    \
        const uint32_t wv_ = blockIdx.x;                                                    \
        if (lane == 0 && wv_ < (uint32_t)BFS_T_W) g_bfs_times[wv_ * BFS_T_REC + (slot)] = wall_clock64(); \
    } while (0)
#define BFS_NOTE(slot, v)                                                                    \
    do {                                                                                     \
        const uint32_t wv_ = blockIdx.x;                                                     \
        if (lane == 0 && wv_ < (uint32_t)BFS_T_W) g_bfs_times[wv_ * BFS_T_REC + (slot)] = (v); \
    } while (0)
#else
#define BFS_STAMP(slot) (void)0
#define BFS_NOTE(slot, v) (void)0
#endif

// false: a buffer overflowed (the caller walks the body with walk()).  fx, fy: wave-uniform.
__device__ bool bfs_walk(const Node *__restrict__ nodes, uint32_t T,
                         double bx, double by, double Gm, double soft2, double theta2,
                         double s2root, uint32_t *lds, uint32_t bm_words, double &fx, double &fy) {
    const uint32_t lane = threadIdx.x & 63u;
    fx = 0.0;
    fy = 0.0;
    if (T == 0) return true;  // an empty tree
    const uint32_t nbw = (T + 31u) / 32u;
    if (nbw > bm_words) return false;
    uint32_t *bits = lds;
    uint32_t *E0 = lds + bfs_bm_space(bm_words);
    uint32_t *E1 = E0 + BFS_E_CAP * BFS_E_WORDS;
    uint32_t *ctr = E0 + BFS_R_WORDS;  // [0]: next level's count, [1]: overflow
    double *terms = reinterpret_cast<double *>(lds);  // (the bitmap's space, after the scan)
    BFS_STAMP(0);
    for (uint32_t w = lane; w < nbw; w += 64) bits[w] = 0u;
    // the criterion (BHA:216-228 in walk<true>'s fast form): does the body open this node?
    auto opens = [&](const Node &r) __attribute__((always_inline)) -> bool {
        if (r.meta & NODE_LEAF) return false;  // (massless cells carry the leaf flag too)
        const double dx = r.comX - bx, dy = r.comY - by;
        const double d2 = dx * dx + dy * dy + soft2;
        const uint64_t s2b = (uint64_t)__double_as_longlong(s2root) -
                             ((uint64_t)(r.meta & NODE_DEPTH2_MASK) << 52);
        return !(__longlong_as_double((long long)s2b) < theta2 * d2);
    };
    uint32_t nE = 0;
    {
        const Node r = nodes[0];  // (every lane: the same address)
        if (opens(r)) {
            if (lane == 0) {
                E0[0] = 0u;
                E0[1] = r.next > 0u ? r.next : 1u;
            }
            nE = 1;
        } else if (lane == 0) {
            bits[0] = 1u;
        }
    }
    if (lane == 0) {
        ctr[0] = 0u;
        ctr[1] = 0u;
    }
    __syncthreads();
    BFS_STAMP(1);
    uint32_t level = 0;
    while (nE > 0) {
        for (uint32_t j = lane; j < nE; j += 64) {  // lane: every child of opened node j
            const uint32_t k = E0[2 * j], end = E0[2 * j + 1];
            uint32_t c = k + 1u;  // first child (pre-order)
            if (c >= end) continue;
            Node r = nodes[c];
            while (true) {
                const uint32_t nx = r.next > c ? r.next : c + 1u;
                const bool more = nx < end;
                Node rn;
                if (more) rn = nodes[nx];  // the next sibling's record, before this criterion
                if (opens(r)) {
                    const uint32_t at = atomicAdd(&ctr[0], 1u);
                    if (at < BFS_E_CAP) {
                        E1[2 * at] = c;
                        E1[2 * at + 1] = nx;
                    } else {
                        ctr[1] = 1u;
                    }
                } else {
                    atomicOr(&bits[c >> 5], 1u << (c & 31u));
                }
                if (!more) break;
                r = rn;
                c = nx;
            }
        }
        __syncthreads();
        nE = __builtin_amdgcn_readfirstlane(ctr[0]);
        const uint32_t over = __builtin_amdgcn_readfirstlane(ctr[1]);
        __syncthreads();
        if (over) return false;
        if (lane == 0) ctr[0] = 0u;
        uint32_t *t = E0;
        E0 = E1;
        E1 = t;
        __syncthreads();
        ++level;
        BFS_STAMP(2 + min(level, 15u));
    }
    BFS_NOTE(20, level);
    (void)level;
    // the accepted nodes in ascending order: each lane a contiguous run of bitmap words, read
    // 16 at a time (at most 32 per lane: BFS_MAX_BM_WORDS)
    uint32_t *A = lds + bfs_bm_space(bm_words);  // (the level buffers' space)
    const uint32_t per = (nbw + 63u) / 64u, w0 = min(lane * per, nbw), w1 = min(w0 + per, nbw);
    uint32_t cnt = 0;
    for (uint32_t b0 = w0; b0 < w1; b0 += 16) {
        uint32_t wv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) wv[u] = b0 + u < w1 ? bits[b0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < 16; ++u) cnt += (uint32_t)__popc(wv[u]);
    }
    uint32_t nA = 0;
    uint32_t at = wave_excl_scan(cnt, lane, nA);
    if (nA > BFS_A_CAP) return false;
    for (uint32_t b0 = w0; b0 < w1; b0 += 16) {
        uint32_t wv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) wv[u] = b0 + u < w1 ? bits[b0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            uint32_t b = wv[u];
            while (b) {
                A[at++] = (b0 + u) * 32u + (uint32_t)__ffs((int)b) - 1u;
                b &= b - 1u;
            }
        }
    }
    __syncthreads();
    BFS_STAMP(18);
    BFS_NOTE(21, nA);
    // the terms, 64 at a time (the next round's records requested before this round's terms);
    // lane 0 adds the x terms and lane 1 the y terms, in order
    double acc = 0.0;
    Node rn;
    if (lane < nA) rn = nodes[A[lane]];
    for (uint32_t base = 0; base < nA; base += 64) {
        const uint32_t i = base + lane;
        const Node r = rn;
        if (i + 64 < nA) rn = nodes[A[i + 64]];
        if (i < nA) {
            const double dx = r.comX - bx;  // BHA:251-253
            const double dy = r.comY - by;
            const double d2 = dx * dx + dy * dy + soft2;
            double h;
            const double sr = sqrt_rn_inrange_h(d2, h);
            const double invR = rcp_rn_seeded(sr, h + h);
            const double invR2 = rcp_rn_seeded(d2, invR * invR);
            const double f = Gm * r.mass * invR2;  // BHA:256
            terms[lane] = f * dx * invR;           // BHA:257-258
            terms[64 + lane] = f * dy * invR;
        }
        __syncthreads();
        if (lane < 2) {  // (reads issued 16 ahead of the dependent additions)
            const uint32_t m = min(64u, nA - base);
            const double *tl = terms + 64 * lane;
            uint32_t j = 0;
            for (; j + 16 <= m; j += 16) {
                double t[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) t[u] = tl[j + u];
#pragma unroll
                for (int u = 0; u < 16; ++u) acc += t[u];
            }
            for (; j < m; ++j) acc += tl[j];
        }
        __syncthreads();
    }
    fx = __shfl(acc, 0, 64);
    fy = __shfl(acc, 1, 64);
    BFS_STAMP(19);
    return true;
}

#ifdef BH_TRAV_TIMING  // diagnostic build only: per-wave wall-clock start / end, hardware ids
constexpr int TRAV_TIMING_MAX = 1 << 18;
__device__ uint64_t g_trav_times[4 * TRAV_TIMING_MAX];
#endif

// k_kick_drift / k_kick of lane q's own body, operation for operation (BHA:412-432): the new
// position -- drifted, or as the build left it -- goes to the exchange, the velocity stays with
// the owner.  (ax, ay) = F / m (BHA:390-391).
template <int KICK>
__device__ __forceinline__ void own_kick(int64_t q, double bx, double by, double ax, double ay,
                                         const KickArgs &kick, double *__restrict__ a2,
                                         double &vxi, double &vyi) {
    typedef double double2_t __attribute__((ext_vector_type(2)));
    const int64_t r = kick.rep ? (int64_t)kick.rep[q] : q;
    vxi = kick.vx[r] + ax * kick.dtHalf;
    vyi = kick.vy[r] + ay * kick.dtHalf;
    kick.vx[r] = vxi;
    kick.vy[r] = vyi;
    double2_t o;
    if (KICK == KICK_OWN_DRIFT) {
        o.x = bx + vxi * kick.dt;
        o.y = by + vyi * kick.dt;
    } else {
        o.x = bx;
        o.y = by;
    }
    *reinterpret_cast<double2_t *>(a2 + 2 * q) = o;
}

// KICK (KickMode): the integration step that follows the evaluation is applied by the lane
// itself after its walk -- the body's x, y are only ever read by its own lane (other lanes see
// it through the leaf records), so the update in place is race-free and a2 is not written.
// Wave v evaluates the bpw lanes [lo + bpw v, lo + bpw v + bpw) (64 = one body per lane; fewer
// for small launches, the wave's other lanes idle -- see traverse()): walk, then the epilogue.
template <bool COUNT, bool OFF32, int KICK, bool BFS>
__device__ __forceinline__ void trav_wave(uint32_t v, uint32_t bpw, uint64_t t_start,
                                          const Node *__restrict__ nodes,
                                          const uint32_t *__restrict__ d_T, double *x, double *y,
                                          const double *__restrict__ m,
                                          const uint32_t *__restrict__ cidx, int64_t lo,
                                          int64_t hi, const ForceParams &fp, const Geometry &g,
                                          double *__restrict__ a2, const TraverseCounters &cnt,
                                          const KickArgs &kick,
                                          const uint32_t *__restrict__ lanes,
                                          const WaveOrder &wo, uint32_t *lds,
                                          uint32_t bm_words) {
    const uint32_t lane = threadIdx.x & 63u;
    const bool in_wave = lane < bpw;
    const int64_t q = lo + (int64_t)v * bpw + lane;  // lane
    const uint32_t lp = lanes && in_wave && q < hi ? lanes[q] : (uint32_t)q;
    const bool valid = in_wave && q < hi && (!lanes || lp != LANE_IDLE);
    const int64_t p = lanes ? (int64_t)lp : q;  // its body's slot
    // A body merged away earlier in this bh_step call (a tombstone until the call's compaction)
    // needs no force: it does not walk.  Tombstones sort to the tail with the out-of-root
    // bodies and are flung across the domain by the heavy body that absorbed them, so a tail
    // wave of walking tombstones visits the union of 64 unrelated interaction lists -- it set
    // the kernel's duration (0.8 -> 2 ms over 20 steps at C3) before this test.
    const bool walks = valid && !(cidx[p] & CIDX_DEAD);
    const double bx = valid ? x[p] : 0.0;
    const double by = valid ? y[p] : 0.0;
    const double bm = valid ? m[p] : 1.0;
    const double Gm = fp.G * bm;  // (Config.G * b.m) is evaluated first (BHA:256)
    const double soft2 = fp.soft2, theta2 = fp.theta2;
    const double s2root = g.s2[0];
    const uint32_t self = (uint32_t)p;
    double fx = 0.0, fy = 0.0;
    uint32_t nvis = 0, niters = 0, ncontrib = 0, nblocks = 0;
    // lane is active for node `cur` iff cur >= resume; invalid lanes and tombstones never are.
    const uint32_t resume = walks ? 0u : 0xFFFFFFFFu;
    const uint32_t T = __builtin_amdgcn_readfirstlane(*d_T);
    const bool fast = fast_s2_ok(s2root) &&
        __ballot(walks && !(lane_fast_ok(bx, by, soft2) && lane_self_ok(Gm, bm))) == 0ull;
    bool walked = false;
    if (BFS && fast && (__ballot(walks) & 1ull)) {  // one body per wave: lane 0's (bpw == 1)
        double ux, uy;
        walked = bfs_walk(nodes, T, rfl_f64(bx), rfl_f64(by), rfl_f64(Gm), soft2, theta2, s2root,
                          lds, bm_words, ux, uy);
        if (walked) {
            fx = ux;
            fy = uy;
        }
    }
    if (walked) {
    } else if (fast)
        walk<true, COUNT, OFF32>(nodes, T, bx, by, Gm, soft2, theta2, s2root, self, resume, fx,
                                 fy, nvis, niters, ncontrib, nblocks);
    else
        walk<false, COUNT, OFF32>(nodes, T, bx, by, Gm, soft2, theta2, s2root, self, resume, fx,
                                  fy, nvis, niters, ncontrib, nblocks);
    if (wo.cost && lane == 0 && q < hi)
        wo.cost[v] = (uint32_t)(wall_clock64() - t_start < 0xFFFFFFull
                                    ? wall_clock64() - t_start : 0xFFFFFFull);
    if (COUNT && lane == 0 && lo + (int64_t)v * bpw < hi) {  // (a workgroup's last waves may be empty)
        cnt.wave_iters[v] = niters;
        cnt.wave_blocks[v] = nblocks;
    }
#ifdef BH_TRAV_TIMING
    if (lane == 0 && v < TRAV_TIMING_MAX) {
        uint64_t *t = g_trav_times + 4 * v;
        t[0] = t_start;
        t[1] = wall_clock64();
        t[2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID: wave, SIMD, CU, SE
        t[3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
    }
#endif
    if (KICK == KICK_OWN_DRIFT && kick.vmax) {  // the drift's speed bound: every lane takes part
        double vxi = 0.0, vyi = 0.0;
        if (valid) own_kick<KICK>(q, bx, by, fx / bm, fy / bm, kick, a2, vxi, vyi);
        wave_vmax(kick.vmax, vxi, vyi);
        if (COUNT && valid) {
            cnt.visits[p] = nvis;
            cnt.contrib[p] = ncontrib;
        }
        return;
    }
    if (!valid) return;
    // BHA:390-391, interleaved (ax, ay): coalesced 16-byte stores in Morton order
    typedef double double2_t __attribute__((ext_vector_type(2)));
    double2_t acc;
    acc.x = fx / bm;
    acc.y = fy / bm;
    if (KICK == KICK_NONE) {  // by lane with a lane map (the multi-GPU pieces stay contiguous)
        *reinterpret_cast<double2_t *>(a2 + 2 * q) = acc;
    } else if (KICK == KICK_OWN_DRIFT || KICK == KICK_OWN_ONLY) {
        double vxi, vyi;
        own_kick<KICK>(q, bx, by, acc.x, acc.y, kick, a2, vxi, vyi);
    } else {  // k_kick_drift / k_kick (integrate.hip), operation for operation
        double v0x, v0y;
        if ((KICK == KICK_ONLY || KICK == KICK_DRIFT) && kick.perm) {
            const uint32_t sp = kick.perm[p];
            v0x = kick.svx[sp];
            v0y = kick.svy[sp];
        } else {
            v0x = kick.vx[p];
            v0y = kick.vy[p];
        }
        const double vxi = v0x + acc.x * kick.dtHalf;
        const double vyi = v0y + acc.y * kick.dtHalf;
        kick.vx[p] = vxi;
        kick.vy[p] = vyi;
        if (KICK == KICK_DRIFT) {
            const double nx = bx + vxi * kick.dt, ny = by + vyi * kick.dt;
            x[p] = nx;
            y[p] = ny;
            if (kick.mf.keys) {  // the next build's k_morton and k_bucket_count for this body
                const uint64_t key = morton_key(g, nx, ny, (cidx[p] & CIDX_DEAD) != 0u);
                const uint32_t k32 = (uint32_t)(key >> key32_shift(g.J));
                kick.mf.keys[p] = key;
                kick.mf.keys32[p] = k32;
                const uint32_t b = find_bucket(kick.mf.spl, kick.mf.spl_nb,
                                               ((uint64_t)k32 << 32) | (uint64_t)p,
                                               (uint32_t)(p / SORT_B));
                kick.mf.bkt[p] = b;
                kick.mf.off[p] = bucket_offset(b, kick.mf.counts);
            }
        }
    }
    if (COUNT) {
        cnt.visits[p] = nvis;
        cnt.contrib[p] = ncontrib;
    }
}

template <bool COUNT, bool OFF32, int KICK, bool BFS>
__global__ __launch_bounds__(TB * MAX_WPB) void k_traverse(const Node *__restrict__ nodes,
                                                 const uint32_t *__restrict__ d_T, double *x,
                                                 double *y, const double *__restrict__ m,
                                                 const uint32_t *__restrict__ cidx,
                                                 int64_t lo, int64_t hi, ForceParams fp,
                                                 Geometry g, double *__restrict__ a2,
                                                 TraverseCounters cnt, KickArgs kick,
                                                 const uint32_t *__restrict__ lanes,
                                                 WaveOrder wo, uint32_t bpw, uint32_t wpb,
                                                 uint32_t bm_words) {
    extern __shared__ uint32_t trav_lds[];  // (bfs_walk only: bfs_lds_bytes(bm_words))
#if defined(BH_TRAV_TIMING)
    const uint64_t t_start = wall_clock64();
#else
    const uint64_t t_start = wo.cost ? wall_clock64() : 0;
#endif
    // xcd_block() with runs of BH_TRAV_XCD_RUN / wpb workgroups (= BH_TRAV_XCD_RUN waves)
    uint32_t b = blockIdx.x;
    {
        const uint32_t C = BH_TRAV_XCD_RUN / wpb, G = 8 * C, full = gridDim.x / G;
        if (b < full * G) b = (b / 8 / C) * G + (b % 8) * C + (b / 8) % C;
    }
    uint32_t v = b * wpb + (threadIdx.x >> 6);
    if (wo.order)  // the v-th run to start is the order[v]-th run of waves (wave_order)
        v = wo.order[v / BH_TRAV_XCD_RUN] * BH_TRAV_XCD_RUN + v % BH_TRAV_XCD_RUN;
    trav_wave<COUNT, OFF32, KICK, BFS>(v, bpw, t_start, nodes, d_T, x, y, m, cidx, lo, hi, fp, g,
                                       a2, cnt, kick, lanes, wo, trav_lds, bm_words);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Operands d2 in the fast-path range [2^-600, 2^503]: random; mantissas near 1.0 / near 2.0;
// squares of random doubles +- a few ulp (sqrt ties region); the physical range [1, 2^24).
constexpr int STB = 256;  // self-test block

__global__ __launch_bounds__(STB) void k_selftest_math(int64_t n, uint64_t seed,
                                                      unsigned long long *bad) {
    uint32_t local = 0;
    for (int64_t i = (int64_t)blockIdx.x * STB + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * STB) {
        const uint64_t r0 = mix64(seed ^ (uint64_t)i), r1 = mix64(r0);
        const int kind = (int)(r1 >> 62);
        uint64_t mant = r0 & ((1ull << 52) - 1);
        int ex = (int)(r1 % 1104) - 600;  // [-600, 503]
        if (kind == 1) mant = (r1 & 1) ? (mant & 0xFFF) : (((1ull << 52) - 1) ^ (mant & 0xFFF));
        double d2;
        if (kind == 2) {
            const double s0 = __builtin_ldexp(__longlong_as_double((long long)((1023ull << 52) | mant)),
                                              ex / 2);
            d2 = __longlong_as_double(__double_as_longlong(s0 * s0) + (long long)((r1 >> 8) % 5) - 2);
        } else {
            if (kind == 3) ex = (int)(r1 % 24);
            d2 = __builtin_ldexp(__longlong_as_double((long long)((1023ull << 52) | mant)), ex);
        }
        if (!(d2 >= 0x1p-600 && d2 <= 0x1p503)) continue;
        double h;
        const double sr = sqrt_rn_inrange_h(d2, h);
        const double invR = rcp_rn_seeded(sr, h + h);
        const double invR2 = rcp_rn_seeded(d2, invR * invR);
        const double wantR = 1.0 / sqrt(d2), wantR2 = 1.0 / d2;
        if (__double_as_longlong(sr) != __double_as_longlong(sqrt(d2))) ++local;
        if (__double_as_longlong(invR) != __double_as_longlong(wantR)) ++local;
        if (__double_as_longlong(invR2) != __double_as_longlong(wantR2)) ++local;
        if (__double_as_longlong(rcp_rn_inrange(d2)) != __double_as_longlong(wantR2)) ++local;
    }
    if (local) atomicAdd(bad, (unsigned long long)local);
}

// Dispatch order of the XCD runs (BH_TRAV_XCD_RUN consecutive waves, one XCD's L2): costliest
// first by the previous evaluation's wave durations, ties (no costs yet: all zero) in run order.
// The waves of a launch come in two to three dispatch generations at C3 whose durations span
// 170-540 us: in run order the dense disk centres start late and end the kernel alone.
constexpr int WO_TB = 1024;
constexpr int WO_MAX_RUNS = 4096;

__global__ __launch_bounds__(WO_TB) void k_wave_order(const uint32_t *__restrict__ cost,
                                                      uint32_t waves, uint32_t runs,
                                                      uint32_t *__restrict__ order) {
    __shared__ uint64_t key[WO_MAX_RUNS];
    uint32_t P = 1;
    while (P < runs) P <<= 1;
    for (uint32_t r = threadIdx.x; r < P; r += WO_TB) {
        uint64_t k = ~0ull;
        if (r < runs) {
            uint32_t sum = 0;
            const uint32_t w0 = r * BH_TRAV_XCD_RUN;
            const uint32_t w1 = min(w0 + (uint32_t)BH_TRAV_XCD_RUN, waves);
            for (uint32_t w = w0; w < w1; ++w) sum += cost[w];  // <= 64 x 2^24
            k = ((uint64_t)(~sum) << 32) | r;
        }
        key[r] = k;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += WO_TB) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = key[i], b = key[l];
                    if (((i & k) == 0) == (a > b)) {
                        key[i] = b;
                        key[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t r = threadIdx.x; r < runs; r += WO_TB) order[r] = (uint32_t)key[r];
}

}  // namespace

size_t wave_order_runs(int64_t n) {
    const int64_t waves = (n + TB - 1) / TB;
    const int64_t G = 8 * (int64_t)BH_TRAV_XCD_RUN;  // xcd_block remaps whole groups only
    const int64_t runs = (waves + G - 1) / G * 8;
    return runs <= WO_MAX_RUNS ? (size_t)runs : 0;
}

hipError_t wave_order(const uint32_t *cost, int64_t n, uint32_t *order, hipStream_t s) {
    const size_t runs = wave_order_runs(n);
    if (runs == 0) return hipErrorInvalidValue;
    k_wave_order<<<1, WO_TB, 0, s>>>(cost, (uint32_t)((n + TB - 1) / TB), (uint32_t)runs, order);
    return hipGetLastError();
}

hipError_t selftest_fast_math(int64_t n, uint64_t seed, unsigned long long *d_bad, hipStream_t s) {
    k_selftest_math<<<4096, STB, 0, s>>>(n, seed, d_bad);
    return hipGetLastError();
}

// Bodies per wave of a small launch.  A wave walks the union of its bodies' interaction lists,
// one dependent fp64 chain per stop, and a launch of a few thousand waves leaves most of the 1 024
// SIMDs with one wave or none: the kernel then lasts as long as its slowest wave's walk (C1's
// 12 500 bodies = 196 waves, C2's 1e5 = 1 563).  Fewer bodies per wave -- the wave's other lanes
// idle -- make more, shorter walks (the union of fewer lists) that fill the SIMDs: halved until
// the launch has BH_TRAV_MIN_WAVES waves or BH_TRAV_MIN_BPW bodies per wave.  Each body's sum is
// untouched (its own criterion and order), so the results are bit-identical for any grouping.
#ifndef BH_TRAV_MIN_WAVES
#define BH_TRAV_MIN_WAVES 1024
#endif
#ifndef BH_TRAV_MIN_BPW
#define BH_TRAV_MIN_BPW 1
#endif
uint32_t bodies_per_wave(int64_t lanes) {
    // (environment overrides for A/B sweeps; BH_TRAV_MIN_WAVES=0: always 64)
    static const int64_t min_waves = [] {
        const char *v = std::getenv("BH_TRAV_MIN_WAVES");
        return v ? (int64_t)std::atoll(v) : (int64_t)BH_TRAV_MIN_WAVES;
    }();
    static const uint32_t min_bpw = [] {
        const char *v = std::getenv("BH_TRAV_MIN_BPW");
        const long b = v ? std::atol(v) : (long)BH_TRAV_MIN_BPW;
        return (uint32_t)(b < 1 ? 1 : b > TB ? TB : b);
    }();
    uint32_t bpw = TB;
    while (bpw > min_bpw && (lanes + bpw - 1) / bpw < min_waves) bpw >>= 1;
    return bpw;
}

// Waves per workgroup for a launch of `waves` waves (profiles/r06s_*, r06t_wpb_sweep.jsonl, two
// interleaved rounds; ms per step for 1 / 2 / 4 / 8 waves per group):
//   C2 (1 563 waves)   0.507 / 0.489 / 0.500 / 0.478  -- 8 neighbouring waves on one CU share its
//                      scalar cache (196 groups: a quarter of the CUs idle, still the fastest)
//   C3 (15.6 K waves)  1.770 / 1.782 / 1.757 / 1.801
//   C4 (156 K waves)   16.45 / 16.51 / 16.38 / 16.40;  the solo C4 / 8 rank step within noise
//   C1 (1 563 waves of 8 bodies)  +1.5 % with 2: short walks keep one wave per group.
// BH_TRAV_WPB (1, 2, 4, 8) overrides.
#ifndef BH_TRAV_WPB_FULL_WAVES
#define BH_TRAV_WPB_FULL_WAVES 8192
#endif
static uint32_t waves_per_group(uint32_t waves, uint32_t bpw) {
    static const long over = [] {
        const char *v = std::getenv("BH_TRAV_WPB");
        return v ? std::atol(v) : 0L;
    }();
    if (over == 1 || over == 2 || over == 4 || over == 8) return (uint32_t)over;
    if (bpw < TB) return 1u;  // (short walks of a few bodies: C1 +1.5 % with 2)
    return waves >= BH_TRAV_WPB_FULL_WAVES ? 4u : waves >= 1024 ? 8u : 1u;
}

// Breadth-first walks (bfs_walk, one body per wave) for launches of up to BH_TRAV_BFS_MAX bodies
// (environment override; 0: never).  Measured (profiles/r06z2_*): C1 'R' (2 000 bodies) traversal
// 67.5 -> 39.8 us; C1 code default (12 500) 102 -> 135 us -- 12 500 one-body waves are ~3
// generations of ~40 us walks, against 1 563 eight-body union walks of ~100 us.  The bitmap covers min(node capacity, 2.25 x bodies + 256, 64 K)
// node indices -- a tree beyond it is walked by walk() body by body.
#ifndef BH_TRAV_BFS_MAX
#define BH_TRAV_BFS_MAX 4096
#endif
// The kick-only walk -- the pipelined step's second, which shares the GPU with the overlapped merge
// rule and next build -- keeps the cursor walk up to BH_TRAV_BFS_MAX_KICK bodies (0: always): the
// breadth-first walk's LDS would keep those kernels off the CUs until it ends.  C1 'R', 3
// interleaved rounds (profiles/r06e_bfs_first_walk_only_ab.txt): breadth first for both walks
// 0.277 ms per step, for the first only 0.272 (0.295 with neither).
#ifndef BH_TRAV_BFS_MAX_KICK
#define BH_TRAV_BFS_MAX_KICK 0
#endif
constexpr uint32_t BFS_MAX_BM_WORDS = 2048;
static int64_t env_or(const char *name, int64_t dflt) {
    const char *e = std::getenv(name);
    return e ? (int64_t)std::atoll(e) : dflt;
}
static int64_t bfs_max_bodies(int kick_mode) {
    static const int64_t v = env_or("BH_TRAV_BFS_MAX", BH_TRAV_BFS_MAX);
    static const int64_t vk = env_or("BH_TRAV_BFS_MAX_KICK", BH_TRAV_BFS_MAX_KICK);
    return kick_mode == KICK_ONLY ? vk : v;
}

// (one-GPU evaluations of the whole list only: a rank's lane range walks a tree of every rank's
// bodies, which the bitmap's size estimate does not cover)
bool traverse_is_bfs(size_t node_cap, int64_t lo, int64_t hi, int kick_mode, bool counting) {
    const bool off32 = node_cap * sizeof(Node) < (size_t(1) << 32);
    return !counting && off32 && lo == 0 && hi > 0 && hi <= bfs_max_bodies(kick_mode) &&
           kick_mode != KICK_OWN_DRIFT && kick_mode != KICK_OWN_ONLY;
}

void traverse(const Node *nodes, size_t node_cap, const uint32_t *d_T, double *x, double *y,
              const double *m, const uint32_t *cidx, int64_t lo, int64_t hi, const Geometry &g,
              const ForceParams &fp, double *a2, const TraverseCounters *cnt,
              hipStream_t s, const KickArgs *kick, const uint32_t *lanes, const WaveOrder *wo) {
    if (hi <= lo) return;
    // node records addressed by a 32-bit byte offset while the array stays below 4 GiB
    const bool off32 = node_cap * sizeof(Node) < (size_t(1) << 32);
    const bool bfs = traverse_is_bfs(node_cap, lo, hi, kick ? kick->mode : KICK_NONE, cnt);
    uint32_t bm_words = 0;
    if (bfs) {
        // (a one-GPU tree has ~1.7 nodes per body: C1 21 565 for 12 500, 3 511 for 2 000)
        const size_t bits = std::min<size_t>(node_cap, (size_t)(9 * (hi - lo) / 4 + 256));
        bm_words = (uint32_t)std::min<size_t>((bits + 31) / 32, BFS_MAX_BM_WORDS);
    }
    // (the counting walk keeps 64 bodies per wave: its per-wave counters define lane efficiency)
    const uint32_t bpw = cnt ? (uint32_t)TB : bfs ? 1u : bodies_per_wave(hi - lo);
    unsigned grid = (unsigned)((hi - lo + bpw - 1) / bpw);  // waves
    const WaveOrder w = wo && bpw == TB && wave_order_runs(hi - lo) ? *wo : WaveOrder{};
    if (w.order)  // whole runs: every run index the order maps to exists in the grid
        grid = (unsigned)(wave_order_runs(hi - lo) * BH_TRAV_XCD_RUN);
    const uint32_t wpb = waves_per_group(grid, bpw);
    grid = (grid + wpb - 1) / wpb;  // workgroups
    const size_t lds = bfs ? bfs_lds_bytes(bm_words) : 0;
    const KickArgs ka = kick ? *kick : KickArgs{KICK_NONE, nullptr, nullptr, 0.0, 0.0, nullptr};
    const TraverseCounters tc = cnt ? *cnt : TraverseCounters{nullptr, nullptr, nullptr, nullptr};
#define BH_TRAV(C, O, K, B)                                                                  \
    k_traverse<C, O, K, B><<<grid, TB * wpb, lds, s>>>(nodes, d_T, x, y, m, cidx, lo, hi, fp, g, \
                                                       a2, tc, ka, lanes, w, bpw, wpb, bm_words)
    if (cnt) {  // diagnostic counting walk: accelerations out, never fused
        if (off32) BH_TRAV(true, true, KICK_NONE, false);
        else BH_TRAV(true, false, KICK_NONE, false);
    } else if (bfs) {
        if (ka.mode == KICK_DRIFT) BH_TRAV(false, true, KICK_DRIFT, true);
        else if (ka.mode == KICK_ONLY) BH_TRAV(false, true, KICK_ONLY, true);
        else if (ka.mode == KICK_OWN_DRIFT) BH_TRAV(false, true, KICK_OWN_DRIFT, true);
        else if (ka.mode == KICK_OWN_ONLY) BH_TRAV(false, true, KICK_OWN_ONLY, true);
        else BH_TRAV(false, true, KICK_NONE, true);
    } else if (off32) {
        if (ka.mode == KICK_DRIFT) BH_TRAV(false, true, KICK_DRIFT, false);
        else if (ka.mode == KICK_ONLY) BH_TRAV(false, true, KICK_ONLY, false);
        else if (ka.mode == KICK_OWN_DRIFT) BH_TRAV(false, true, KICK_OWN_DRIFT, false);
        else if (ka.mode == KICK_OWN_ONLY) BH_TRAV(false, true, KICK_OWN_ONLY, false);
        else BH_TRAV(false, true, KICK_NONE, false);
    } else {
        if (ka.mode == KICK_DRIFT) BH_TRAV(false, false, KICK_DRIFT, false);
        else if (ka.mode == KICK_ONLY) BH_TRAV(false, false, KICK_ONLY, false);
        else if (ka.mode == KICK_OWN_DRIFT) BH_TRAV(false, false, KICK_OWN_DRIFT, false);
        else if (ka.mode == KICK_OWN_ONLY) BH_TRAV(false, false, KICK_OWN_ONLY, false);
        else BH_TRAV(false, false, KICK_NONE, false);
    }
#undef BH_TRAV
}

#ifdef BH_BFS_TIMING
extern "C" int bh_debug_bfs_times(uint64_t *out, int waves) {
    if (waves > BFS_T_W) waves = BFS_T_W;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bfs_times),
                                    sizeof(uint64_t) * BFS_T_REC * (size_t)waves);
}
#endif

#ifdef BH_TRAV_TIMING
extern "C" int bh_debug_trav_times(uint64_t *out, int waves) {
    if (waves > TRAV_TIMING_MAX) waves = TRAV_TIMING_MAX;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trav_times), sizeof(uint64_t) * 4 * (size_t)waves);
}
#endif

}  // namespace bh
