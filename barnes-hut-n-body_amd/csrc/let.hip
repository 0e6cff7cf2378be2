// Multi-rank tree build as a locally essential tree (LET): the build is sharded instead of
// replicated.  Replaces, per rank, PhysicsEngine.buildTree (BHA:359-366) for the bodies the rank
// evaluates in computeAccelerations (BHA:374-395), with forces bit-identical to the full tree.
//
// Every rank holds the full replicated state (engine.cpp) and evaluates its pieces of the slot
// order.  A traversal from body b visits a node iff b opened its parent (BHA:226-236), so a rank
// needs the full subtree only where its bodies may open nodes:
//   * own cells: the depth-P cells (P = LET_P) holding a body the rank evaluates;
//   * the halo: every depth-P cell that some own cell's body might open -- cells farther away
//     are accepted as a whole (BHA:228 holds for every body of every own cell, with a margin for
//     jitter and rounding), so their children are never visited;
//   * the subset = all bodies of own + halo cells (+ own bodies outside the tree): built with the
//     ordinary pipeline (tree_build.hip); a depth-P cell's subtree depends only on its bodies
//     (jitter replays stay inside depth-J cells), so those nodes are the full tree's, bit for bit;
//   * the top (depth < P): a node's centre of mass is a function of its children's values
//     (BHA:184-200), so every rank computes it from the depth-P cell values all ranks exchange
//     (32 B per cell, one all-gather), and lays the tree out in pre-order: top nodes, local
//     subtrees copied with shifted `next`, remote cells as childless records.
// The traversal kernel then walks this array unchanged (traverse.hip), one lane per own body.
// Jitter (BHA:146-151) mutates positions during the build: each lane kicks its own body in the
// traversal's epilogue and sends the body's new position (x + v dt, or x as the build left it),
// and every replica takes all positions from the exchange (let_set_pos); velocities stay with
// the owners until the next full build (engine.cpp sync_velocities).
#include <algorithm>
#include <cmath>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/zip_iterator.hpp>

#include "bh_device.hpp"

namespace bh {
namespace {

constexpr int TB = 256;
inline unsigned grid_for(int64_t n) { return (unsigned)((n + TB - 1) / TB); }

__device__ __forceinline__ uint32_t spread16(uint32_t v) {  // bit k -> bit 2k
    v = (v | (v << 8)) & 0x00FF00FFu;
    v = (v | (v << 4)) & 0x0F0F0F0Fu;
    v = (v | (v << 2)) & 0x33333333u;
    return (v | (v << 1)) & 0x55555555u;
}
__device__ __forceinline__ uint32_t compact16(uint32_t v) {  // bit 2k -> bit k
    v &= 0x55555555u;
    v = (v | (v >> 1)) & 0x33333333u;
    v = (v | (v >> 2)) & 0x0F0F0F0Fu;
    v = (v | (v >> 4)) & 0x00FF00FFu;
    return (v | (v >> 8)) & 0x0000FFFFu;
}

// Column of p on the grid o + k w, clamped to [0, top]: exact for p inside (settled by the same
// exact grid-line compares as k_morton); outside, the column of p's projection onto the root.
__device__ __forceinline__ uint32_t grid_col(double p, double o, double w, int top) {
    double q = (p - o) * (1.0 / w);  // off by at most one: settled below
    if (!(q >= 0.0)) q = 0.0;
    if (q > (double)top) q = (double)top;
    int c = (int)q;
    if (c > 0 && p < o + (double)c * w) --c;
    else if (c < top && p >= o + (double)(c + 1) * w) ++c;
    return (uint32_t)c;
}

__device__ __forceinline__ bool in_root(const Geometry &g, double x, double y) {  // BHA:61-62
    return x >= g.root_cx - g.root_h && x < g.root_cx + g.root_h && y >= g.root_cy - g.root_h &&
           y < g.root_cy + g.root_h;
}

__device__ __forceinline__ uint32_t cell_of(const Geometry &g, double x, double y) {
    const double w = 2.0 * g.h[LET_P];
    const int top = (1 << LET_P) - 1;
    return spread16(grid_col(x, g.root_cx - g.root_h, w, top)) |
           (spread16(grid_col(y, g.root_cy - g.root_h, w, top)) << 1);
}


// Cell centre at depth d of cell index i (BHA:73-81 applied d times, as tree_build's cell_centre).
__device__ void cell_centre_at(const Geometry &g, uint32_t i, int d, double &cx, double &cy) {
    cx = g.root_cx;
    cy = g.root_cy;
    for (int l = 0; l < d; ++l) {
        const uint32_t digit = (i >> (2 * (d - 1 - l))) & 3u;
        const double hh = g.h[l + 1];
        cx = (digit & 1u) ? cx + hh : cx - hh;
        cy = (digit & 2u) ? cy + hh : cy - hh;
    }
}

__host__ __device__ constexpr int64_t level_off(int d) { return (((int64_t)1 << (2 * d)) - 1) / 3; }

// ---- selection ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t own_lane(const LetPieces &pc, int64_t t) {  // t-th own lane
    return (int64_t)pc.rank * pc.rounds * pc.sub + t;  // one contiguous range per rank
}

__device__ __forceinline__ void slot_pos(const PosSrc &ps, const double *__restrict__ x,
                                         const double *__restrict__ y, int64_t i, double &px,
                                         double &py) {
    if (ps.a2) {
        const int64_t g = ps.gslot[i];
        px = ps.a2[2 * g];
        py = ps.a2[2 * g + 1];
    } else {
        px = x[i];
        py = y[i];
    }
}

__global__ __launch_bounds__(TB) void k_let_mark(LetPieces pc, PosSrc ps,
                                                 const double *__restrict__ x,
                                                 const double *__restrict__ y,
                                                 const uint32_t *__restrict__ cidx, Geometry g,
                                                 uint8_t *__restrict__ own,
                                                 uint8_t *__restrict__ own_blk,
                                                 uint8_t *__restrict__ ecell,
                                                 uint32_t *__restrict__ flag_all) {
    const int64_t t = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (t >= (int64_t)pc.rounds * pc.sub) return;
    const int64_t q = own_lane(pc, t);
    if (q >= pc.n) return;
    const int64_t i = pc.lanes ? (int64_t)pc.lanes[q] : q;
    own[i] = 1;
    own_blk[i >> 8] = 1;  // the selection scans this slot's block whatever its box
    if (cidx[i] & CIDX_DEAD) return;  // tombstones do not walk
    double px, py;
    if (ps.a2) {  // lane q's position in the exchange buffer
        const int64_t gs = gather_slot(ps.gl, q);
        px = ps.a2[2 * gs];
        py = ps.a2[2 * gs + 1];
    } else {
        px = x[i];
        py = y[i];
    }
    if (!__builtin_isfinite(px) || !__builtin_isfinite(py)) {
        *flag_all = 1u;
        return;
    }
    ecell[cell_of(g, px, py)] = 1;  // outside the root: the cell of the projection
}

// A cell is built locally iff some own cell lies within gap^2 <= gap2 cells of it (gap =
// whole cells between the two squares per axis).
__global__ __launch_bounds__(TB) void k_let_halo(const uint8_t *__restrict__ ecell,
                                                 const uint32_t *__restrict__ flag_all,
                                                 double gap2, int K,
                                                 uint8_t *__restrict__ hcell,
                                                 uint32_t *__restrict__ rowmask) {
    const int64_t c = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (c >= LET_CELLS) return;
    uint8_t h = (*flag_all != 0u) ? 1 : ecell[c];
    const int ix = (int)compact16((uint32_t)c), iy = (int)compact16((uint32_t)c >> 1);
    const int top = (1 << LET_P) - 1;
    for (int dy = -K; dy <= K && !h; ++dy) {
        const int ny = iy + dy;
        if (ny < 0 || ny > top) continue;
        const int gy = abs(dy) > 0 ? abs(dy) - 1 : 0;
        for (int dx = -K; dx <= K; ++dx) {
            const int nx = ix + dx;
            if (nx < 0 || nx > top) continue;
            const int gx = abs(dx) > 0 ? abs(dx) - 1 : 0;
            if ((double)(gx * gx + gy * gy) > gap2) continue;
            if (ecell[spread16((uint32_t)nx) | (spread16((uint32_t)ny) << 1)]) {
                h = 1;
                break;
            }
        }
    }
    hcell[c] = h;
    if (h) atomicOr(rowmask + iy * 8 + (ix >> 5), 1u << (ix & 31));
}

// Whether the rectangle [c0, c1] x [r0, r1] of grid cells holds a built cell (rowmask): the
// wave's lanes take a row each.
__device__ __forceinline__ bool rect_any(const uint32_t *__restrict__ rowmask, int c0, int c1,
                                         int r0, int r1) {
    bool any = false;
    const int w0 = c0 >> 5, w1 = c1 >> 5;
    for (int r = r0 + (int)(threadIdx.x & 63); r <= r1 && !any; r += 64)
        for (int w = w0; w <= w1; ++w) {
            uint32_t m = rowmask[r * 8 + w];
            if (w == w0) m &= ~0u << (c0 & 31);
            if (w == w1 && (c1 & 31) != 31) m &= (2u << (c1 & 31)) - 1u;
            if (m) {
                any = true;
                break;
            }
        }
    return __ballot(any) != 0ull;
}

// The box of depth-LET_P cells of each 256-slot block's bodies (one wave per block, four slots
// per lane): live bodies with a finite position, those outside the root by the cell of their
// projection (grid_col clamps; a clamped column moves no more than the body does).
__global__ __launch_bounds__(64) void k_let_boxes(int64_t n, const double *__restrict__ x,
                                                  const double *__restrict__ y,
                                                  const uint32_t *__restrict__ cidx, Geometry g,
                                                  uint32_t *__restrict__ box) {
    const int64_t b0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const double w = 2.0 * g.h[LET_P];
    const int top = (1 << LET_P) - 1;
    uint32_t clo = 255, chi = 0, rlo = 255, rhi = 0;
    bool any = false;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t i = b0 + 64 * u;
        if (i >= n || (cidx[i] & CIDX_DEAD)) continue;
        const double px = x[i], py = y[i];
        if (!__builtin_isfinite(px) || !__builtin_isfinite(py)) continue;
        const uint32_t c = grid_col(px, g.root_cx - g.root_h, w, top);
        const uint32_t r = grid_col(py, g.root_cy - g.root_h, w, top);
        clo = min(clo, c);
        chi = max(chi, c);
        rlo = min(rlo, r);
        rhi = max(rhi, r);
        any = true;
    }
    for (int o = 32; o > 0; o >>= 1) {
        clo = min(clo, (uint32_t)__shfl_xor((int)clo, o, 64));
        chi = max(chi, (uint32_t)__shfl_xor((int)chi, o, 64));
        rlo = min(rlo, (uint32_t)__shfl_xor((int)rlo, o, 64));
        rhi = max(rhi, (uint32_t)__shfl_xor((int)rhi, o, 64));
    }
    const bool some = __ballot(any) != 0ull;
    if (threadIdx.x == 0)
        box[blockIdx.x] = some ? (clo | chi << 8 | rlo << 16 | rhi << 24) : 0x00FF00FFu;
}

__global__ void k_let_disp_add(double *disp, const unsigned long long *vmax, int k, double dt) {
    unsigned long long b = 0;
    for (int q = 0; q < k; ++q) b = vmax[q] > b ? vmax[q] : b;
    const double v = __longlong_as_double((long long)b);
    const double d = disp[0] + v * dt;
    disp[0] = d >= 0.0 ? d : __builtin_inf();  // (NaN: no bound)
}

// the subset: bodies of built cells, and own bodies outside the tree (they still walk it, or
// idle); a flag byte per slot and the count of every 256-slot block (scanned: block offsets)
static_assert(TB == 256, "one 256-slot block per workgroup");
// One wave per 256-slot block, four slots per lane (slot base + lane + 64 u): four independent
// position loads and cell lookups in flight per lane, the block's count from four ballots.
__global__ __launch_bounds__(64) void k_let_flags(LetPieces pc, PosSrc ps,
                                                  const double *__restrict__ x,
                                                  const double *__restrict__ y,
                                                  const uint32_t *__restrict__ cidx, Geometry g,
                                                  const uint8_t *__restrict__ hcell,
                                                  const uint8_t *__restrict__ own,
                                                  uint8_t *__restrict__ flag8,
                                                  uint32_t *__restrict__ bcnt, LetBufs L,
                                                  LetSweep sw) {
    const int64_t b0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (sw.valid && *L.flag_all == 0u && !L.own_blk[blockIdx.x]) {
        // a candidate block: its box widened by the displacement bound holds a built cell
        const uint32_t bx = sw.box[blockIdx.x];
        const int clo = (int)(bx & 255u), chi = (int)((bx >> 8) & 255u);
        const int rlo = (int)((bx >> 16) & 255u), rhi = (int)(bx >> 24);
        const double D = (sw.disp[0] + sw.allow) * (1.0 + 1e-9);
        const double mw = D * (1.0 / (2.0 * g.h[LET_P]));
        bool cand = true;
        if (clo > chi) {
            cand = false;  // no live finite body in this block at the full build
        } else if (mw < 64.0) {
            const int m = (int)mw + 1;
            const int top = (1 << LET_P) - 1;
            cand = rect_any(L.rowmask, max(clo - m, 0), min(chi + m, top), max(rlo - m, 0),
                            min(rhi + m, top));
        }
        if (!cand) {  // (flag8 stays stale here: k_let_gather skips empty blocks)
            if (threadIdx.x == 0) {
                bcnt[blockIdx.x] = 0u;
                if (blockIdx.x + 1 == gridDim.x) bcnt[gridDim.x] = 0u;
            }
            return;
        }
    }
    uint32_t count = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t i = b0 + 64 * u;
        uint32_t f = 0;
        if (i < pc.n) {
            double px, py;
            slot_pos(ps, x, y, i, px, py);
            if (!(cidx[i] & CIDX_DEAD) && in_root(g, px, py)) f = hcell[cell_of(g, px, py)];
            else f = own[i];
            flag8[i] = (uint8_t)f;
        }
        count += (uint32_t)__popcll(__ballot(f != 0));
    }
    if (threadIdx.x == 0) {
        bcnt[blockIdx.x] = count;
        if (blockIdx.x + 1 == gridDim.x) bcnt[gridDim.x] = 0u;  // the scan's last entry
    }
}

// k_morton and k_bucket_count of the subset build for subset body j with Morton key `key`
__device__ __forceinline__ void let_fuse_key(const Geometry &g, const MortonFuse &mf, int64_t j,
                                             uint64_t key) {
    const uint32_t k32 = (uint32_t)(key >> key32_shift(g.J));
    mf.keys[j] = key;
    mf.keys32[j] = k32;
    const uint32_t b = find_bucket(mf.spl, mf.spl_nb, ((uint64_t)k32 << 32) | (uint64_t)j,
                                   (uint32_t)(j / SORT_B));
    mf.bkt[j] = b;
    mf.off[j] = bucket_offset(b, mf.counts);
}

// also pads subset slots [n_real, S) as dead bodies (sentinel keys: never in the tree, never
// evaluated) and writes the status: overflow when n_real > S (the build then misses bodies: the
// call is replayed); the grid covers n >= S threads
__global__ __launch_bounds__(TB) void k_let_gather(int64_t n, PosSrc ps,
                                                   const uint8_t *__restrict__ flag8,
                                                   const uint32_t *__restrict__ bpos,
                                                   BodyState st, BodyState sub, int64_t S,
                                                   const uint32_t *__restrict__ count,
                                                   LetCell *__restrict__ table,
                                                   uint32_t *__restrict__ scal, Geometry g,
                                                   MortonFuse mf) {
    __shared__ uint32_t s_w[TB / 64];
    const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
    {
        const int64_t n_real = *count;
        if (i == 0) {
            table[LET_CELLS] = LetCell{0.0, 0.0, 0.0, n_real > S ? 1u : 0u, 0u};
            atomicMax(scal + 5, (uint32_t)n_real);
        }
        if (i < S && i >= n_real) {
            sub.x[i] = 0.0;
            sub.y[i] = 0.0;
            sub.vx[i] = __longlong_as_double(-1ll);  // no replicated slot (vy: unused)
            sub.m[i] = 0.0;
            sub.cidx[i] = CIDX_DEAD;
            if (mf.keys) let_fuse_key(g, mf, i, sentinel_key(g.J));
        }
    }
    if (bpos[blockIdx.x + 1] == bpos[blockIdx.x]) return;  // nothing selected (or not scanned)
    const bool f = i < n && flag8[i];
    const uint64_t m = __ballot(f);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    if (!f) return;
    uint32_t j = bpos[blockIdx.x];
    for (uint32_t q = 0; q < w; ++q) j += s_w[q];
    j += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    double px, py;
    slot_pos(ps, st.x, st.y, i, px, py);
    sub.x[j] = px;
    sub.y[j] = py;
    sub.vx[j] = __longlong_as_double((long long)i);  // payload: the replicated slot (vy unused)
    sub.m[j] = st.m[i];
    const uint32_t ci = st.cidx[i];
    sub.cidx[j] = ci;
    if (mf.keys && (int64_t)j < S)  // (an overflowing subset is replayed: keys only below S)
        let_fuse_key(g, mf, j, morton_key(g, px, py, (ci & CIDX_DEAD) != 0u));
}

// a tree larger than its array can only come from a broken invariant: no walk (node count 0), and
// the call is replayed (bh_step) instead of reading past the array (the writers above check
// every position against node_cap)
__device__ __forceinline__ void let_guard(const LetBufs &L, uint32_t *__restrict__ scal) {
    if (L.posc[LET_CELLS] + 1u >= L.node_cap) {
        scal[4] = 1u;
        L.posc[LET_CELLS] = 0u;
    }
}
__global__ void k_let_guard(LetBufs L, uint32_t *__restrict__ scal) { let_guard(L, scal); }

// ---- after the subset build ----------------------------------------------------------------
// depth-P node of a cell with >= 2 subset bodies starting at sorted a: the internal nodes whose
// first body is a are depths c(a-1)+1 .. c(a) at base[a] + (depth - c(a-1) - 1) (k_prep)
__device__ __forceinline__ uint32_t cell_node(const TreeBuffers &tb, uint32_t a) {
    const int cp = a > 0 ? (int)tb.cpl[a - 1] : -1;
    return tb.base[a] + (uint32_t)(LET_P - cp - 1);
}

// first sorted subset index with (key >> shift) >= bin (sentinel: 4^P)
__device__ __forceinline__ uint32_t let_cell_start(int64_t n, int shift,
                                                   const uint64_t *__restrict__ keys_s,
                                                   int64_t bin) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)(keys_s[mid] >> shift) < bin) lo = mid + 1; else hi = mid;
    }
    return (uint32_t)lo;
}

// cstart (first subset body of every depth-P cell) and this rank's cell table in one launch:
// each cell's thread finds its own start and the next cell's
__global__ __launch_bounds__(TB) void k_let_table(int64_t n_sub, int J, LetBufs L, TreeBuffers tb) {
    const int64_t c = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (c > LET_CELLS) return;
    const int shift = 2 * (J - LET_P);
    const uint32_t a = let_cell_start(n_sub, shift, tb.keys_s, c);
    L.cstart[c] = a;
    if (c == LET_CELLS) return;
    LetCell r{0.0, 0.0, 0.0, 0u, 0u};
    if (L.ecell[c]) {
        const uint32_t cn = let_cell_start(n_sub, shift, tb.keys_s, c + 1) - a;
        r.tag = 1u;
        if (cn == 1) {
            r.comX = tb.dst.x[a];
            r.comY = tb.dst.y[a];
            r.mass = tb.dst.m[a];
            r.cnt = 1u;
        } else if (cn >= 2) {
            const Node nd = tb.nodes[cell_node(tb, a)];
            r.comX = nd.comX;
            r.comY = nd.comY;
            r.mass = nd.mass;
            r.cnt = 2u;
        }
    }
    L.table[c] = r;
}

// computeMass (BHA:184-200) of a top node from its 4 children in order 0..3 with the mass > 0
// filter; a one-body cell passes its body through (a leaf).
__device__ LetCell let_parent(const LetCell *c, int d, uint32_t i, const Geometry &g) {
    uint32_t total = 0;
    for (int q = 0; q < 4; ++q) total += c[q].cnt;
    LetCell r{0.0, 0.0, 0.0, 0u, 0u};
    if (total == 1u) {
        for (int q = 0; q < 4; ++q)
            if (c[q].cnt) r = c[q];
    } else if (total >= 2u) {
        double mSum = 0.0, cx = 0.0, cy = 0.0;
        for (int q = 0; q < 4; ++q) {
            if (c[q].mass > 0.0) {
                mSum += c[q].mass;
                cx += c[q].comX * c[q].mass;
                cy += c[q].comY * c[q].mass;
            }
        }
        r.mass = mSum;
        if (mSum > 0.0) {
            r.comX = cx / mSum;
            r.comY = cy / mSum;
        } else {
            cell_centre_at(g, i, d, r.comX, r.comY);
        }
        r.cnt = 2u;
    }
    return r;
}

// Depths LET_P .. 4 of one depth-4 cell per workgroup (256 depth-8 cells): the exchanged values
// (first rank that provided the cell), then the levels up, in LDS.
static_assert(LET_P == 8, "k_let_top_hi assumes 256 depth-LET_P cells per depth-4 cell");
#ifndef BH_LET_TOP_BATCH
#define BH_LET_TOP_BATCH 8  // one round of loads for up to 8 ranks
#endif
__global__ __launch_bounds__(256) void k_let_top_hi(int world, Geometry g,
                                                    const LetCell *__restrict__ tables,
                                                    LetCell *__restrict__ levels,
                                                    uint32_t *__restrict__ scal) {
    __shared__ LetCell sh[256];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    if (b == 0 && t == 0)  // some rank's subset overflowed: every rank replays the call
        for (int q = 0; q < world; ++q)
            if (tables[(int64_t)q * LET_TSTRIDE + LET_CELLS].cnt) scal[4] = 1u;
    {
        const uint32_t c = b * 256u + t;
        LetCell r{0.0, 0.0, 0.0, 0u, 0u};
        // the ranks' entries BH_LET_TOP_BATCH at a time: independent loads in flight, the first
        // tagged wins
        bool found = false;
        for (int q0 = 0; q0 < world && !found; q0 += BH_LET_TOP_BATCH) {
            LetCell v[BH_LET_TOP_BATCH];
#pragma unroll
            for (int j = 0; j < BH_LET_TOP_BATCH; ++j)
                if (q0 + j < world) v[j] = tables[(int64_t)(q0 + j) * LET_TSTRIDE + c];
#pragma unroll
            for (int j = 0; j < BH_LET_TOP_BATCH; ++j)
                if (!found && q0 + j < world && v[j].tag) {
                    r = v[j];
                    found = true;
                }
        }
        r.tag = r.cnt == 1u ? c : 0u;
        levels[level_off(LET_P) + c] = r;
        sh[t] = r;
    }
    __syncthreads();
    uint32_t width = 64;  // this workgroup's nodes at depth d
    for (int d = LET_P - 1; d >= 4; --d, width >>= 2) {
        LetCell r{};
        if (t < width) {
            r = let_parent(sh + 4 * t, d, b * width + t, g);
            levels[level_off(d) + b * width + t] = r;
        }
        __syncthreads();
        if (t < width) sh[t] = r;  // the level becomes the next level's children
        __syncthreads();
    }
}

// Depths 3 .. 0 (85 nodes) by one workgroup from depth 4.
__global__ __launch_bounds__(256) void k_let_top_lo(Geometry g, LetCell *__restrict__ levels) {
    __shared__ LetCell sh[256];
    const uint32_t t = threadIdx.x;
    sh[t] = levels[level_off(4) + t];
    __syncthreads();
    uint32_t width = 64;
    for (int d = 3; d >= 0; --d, width >>= 2) {
        LetCell r{};
        if (t < width) {
            r = let_parent(sh + 4 * t, d, t, g);
            levels[level_off(d) + t] = r;
        }
        __syncthreads();
        if (t < width) sh[t] = r;
        __syncthreads();
    }
}

__device__ __forceinline__ bool node_exists(const LetCell *__restrict__ levels, int d, uint32_t i) {
    if (levels[level_off(d) + i].cnt == 0u) return false;
    return d == 0 || levels[level_off(d - 1) + (i >> 2)].cnt >= 2u;
}

// nodes per depth-P cell: its own node(s) (a locally built subtree, or one record) plus the
// top nodes whose cell range starts at it; pre-order = order of (first cell, depth).
__global__ __launch_bounds__(TB) void k_let_w(LetBufs L, TreeBuffers tb,
                                              uint32_t *__restrict__ scal) {
    const int64_t c = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (c > LET_CELLS) return;
    if (c == LET_CELLS || scal[4]) {
        // after a subset overflow (some rank's subset missed bodies: the call is replayed) the
        // local cells need not hold what the exchanged counts say: an empty tree
        L.w[c] = 0u;
        L.ccnt[c] = 0u;
        L.bsz[c] = 0u;
        L.csrc[c] = 0u;
        return;
    }
    uint32_t bs = 0, copy = 0, ni = 0;
    if (node_exists(L.levels, LET_P, (uint32_t)c)) {
        if (L.levels[level_off(LET_P) + c].cnt >= 2u && L.hcell[c]) {
            if (L.cstart[c + 1] - L.cstart[c] < 2u) {  // cannot happen (replicated positions):
                scal[4] = 1u;                          // replay rather than read a wrong node
                bs = 1u;
            } else {
                ni = cell_node(tb, L.cstart[c]);
                bs = copy = tb.nodes[ni].next - ni;
            }
        } else {
            bs = 1u;
        }
    }
    L.csrc[c] = ni;
    L.ccnt[c] = copy;
    uint32_t anc = 0;
    for (int d = 0; d < LET_P; ++d) {
        const int sh = 2 * (LET_P - d);
        if (((uint64_t)c & ((1ull << sh) - 1)) == 0 && node_exists(L.levels, d, (uint32_t)(c >> sh)))
            ++anc;
    }
    L.bsz[c] = bs;
    L.w[c] = bs + anc;
}

__device__ __forceinline__ uint32_t leaf_slot(const LetBufs &L, uint32_t bc) {
    // the body of a one-body cell: its subset slot if the cell was built here (self-skip,
    // BHA:219), else a slot no local body has
    return L.hcell[bc] ? L.cstart[bc] : NODE_BODY_MASK;
}

__device__ __forceinline__ void let_write_top(const LetBufs &L, int64_t t) {
    int d = 0;
    while (t >= ((int64_t)1 << (2 * d))) {
        t -= (int64_t)1 << (2 * d);
        ++d;
    }
    const uint32_t i = (uint32_t)t;
    if (!node_exists(L.levels, d, i)) return;
    const int sh = 2 * (LET_P - d);
    uint32_t pos = L.posc[(uint64_t)i << sh];
    for (int d2 = 0; d2 < d; ++d2) {  // ancestors that start at the same cell come first
        const int s2 = 2 * (d - d2);
        if ((i & ((1u << s2) - 1u)) == 0u && node_exists(L.levels, d2, i >> s2)) ++pos;
    }
    const LetCell v = L.levels[level_off(d) + i];
    Node nd;
    nd.comX = v.comX;
    nd.comY = v.comY;
    nd.mass = v.mass;
    if (v.cnt >= 2u) {
        nd.next = L.posc[((uint64_t)i + 1) << sh];
        nd.meta = (uint32_t)(2 * d) | (v.mass > 0.0 ? 0u : NODE_SKIP | NODE_LEAF);
    } else {
        nd.next = pos + 1;
        nd.meta = NODE_LEAF | leaf_slot(L, v.tag) | (v.mass == 0.0 ? NODE_SKIP : 0u);
    }
    if (pos < L.node_cap) L.nodes[pos] = nd;
}

// one record per depth-P cell that is not copied: a remote internal cell (accepted by every local
// body: never opened) or a one-body leaf
__device__ __forceinline__ void let_write_cell(const LetBufs &L, int64_t c) {
    const uint32_t bs = L.bsz[c];
    if (bs != 1u || L.ccnt[c] != 0u) return;
    const uint32_t pos = L.posc[c + 1] - 1u;
    const LetCell v = L.levels[level_off(LET_P) + c];
    Node nd;
    nd.comX = v.comX;
    nd.comY = v.comY;
    nd.mass = v.mass;
    nd.next = pos + 1;
    if (v.cnt >= 2u)
        nd.meta = (uint32_t)(2 * LET_P) | (v.mass > 0.0 ? 0u : NODE_SKIP | NODE_LEAF);
    else
        nd.meta = NODE_LEAF | leaf_slot(L, (uint32_t)c) | (v.mass == 0.0 ? NODE_SKIP : 0u);
    if (pos < L.node_cap) L.nodes[pos] = nd;
}

// the top records (threads [0, level_off(P))) and the per-cell records (the next LET_CELLS
// threads) in one launch: disjoint node slots, the same inputs
__global__ __launch_bounds__(TB) void k_let_write_top_cells(LetBufs L) {
    const int64_t t = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (t < level_off(LET_P)) let_write_top(L, t);
    else if (t < level_off(LET_P) + LET_CELLS) let_write_cell(L, t - level_off(LET_P));
}

// the locally built subtrees, one thread per node (grid-stride over cpos[LET_CELLS] nodes): node t
// of the concatenated blocks belongs to the cell c with cpos[c] <= t < cpos[c + 1]; its `next`
// moves with the block.  The cell is found by the whole wave: a 64-ary search for the cell of
// the wave's first node (three rounds of 64 parallel loads instead of a 16-step chain of
// dependent loads by one lane), then each lane's own cell in the 64-cell window after it
// (one load, a binary search over the window by lane shuffles); a lane past the window (many
// empty cells between two pieces) gallops from the window's end.
#ifndef BH_LET_COPY_GRID
#define BH_LET_COPY_GRID 8192  // workgroups of the grid-stride copy (one search per 64 nodes)
#endif
__global__ __launch_bounds__(TB) void k_let_copy_blocks(LetBufs L, const Node *__restrict__ src) {
    const uint32_t total = L.cpos[LET_CELLS];
    const uint32_t lane = threadIdx.x & 63u, stride = gridDim.x * TB;
    constexpr uint32_t NC = (uint32_t)LET_CELLS;
    for (uint32_t base = blockIdx.x * TB + (threadIdx.x & ~63u); base < total; base += stride) {
        // largest c < NC with cpos[c] <= base (cpos is non-decreasing, cpos[0] = 0): the lanes
        // whose probe satisfies it form a prefix, its length picks the next range
        uint32_t c0 = 0, span = NC;
        while (span > 1u) {
            const uint32_t step = (span + 63u) >> 6;
            const bool in = lane * step < span;
            const bool le = in && L.cpos[c0 + lane * step] <= base;
            const uint32_t k = (uint32_t)__popcll(__ballot(le));  // >= 1
            c0 += (k - 1u) * step;
            const uint32_t rest = span - (k - 1u) * step;
            span = rest < step ? rest : step;
        }
        const uint32_t t = base + lane;
        // the window: cells c0 .. c0 + 63 (past the last cell: never <= t)
        const uint32_t w = c0 + lane < NC ? L.cpos[c0 + lane] : 0xFFFFFFFFu;
        uint32_t j = 0;  // largest j with w_j <= t (w_0 = cpos[c0] <= base <= t)
#pragma unroll
        for (uint32_t sft = 32; sft >= 1u; sft >>= 1) {
            const uint32_t wj = (uint32_t)__shfl((int)w, (int)(j + sft));
            if (wj <= t) j += sft;
        }
        if (t >= total) continue;
        uint32_t c = c0 + j;
        if (j == 63u && c + 1u < NC && L.cpos[c + 1] <= t) {  // past the window: gallop
            uint32_t lo = c + 1, step = 1, hi;
            for (;;) {  // cpos[lo] <= t holds
                hi = lo + step;
                if (hi >= NC || L.cpos[hi] > t) break;
                lo = hi;
                step <<= 1;
            }
            if (hi > NC) hi = NC;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (L.cpos[mid] <= t) lo = mid; else hi = mid;
            }
            c = lo;
        }
        const uint32_t k = t - L.cpos[c];
        const uint32_t ni = L.csrc[c], dst = L.posc[c + 1] - L.bsz[c];
        Node nd = src[ni + k];
        nd.next = nd.next - ni + dst;
        if (dst + k < L.node_cap) L.nodes[dst + k] = nd;
    }
}

__global__ __launch_bounds__(TB) void k_let_subpos(int64_t n_sub, int64_t n,
                                                   const double *__restrict__ rep,
                                                   uint32_t *__restrict__ subpos, LetBufs L,
                                                   uint32_t *__restrict__ scal) {
    const int64_t s = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (s == 0) let_guard(L, scal);  // before k_let_lanes reads scal[4]
    if (s >= n_sub) return;
    const int64_t i = (int64_t)__double_as_longlong(rep[s]);
    if (i >= 0 && i < n) subpos[i] = (uint32_t)s;
}

// own lane -> subset slot of its body
// The selection's marks cleared for the next selection (k_let_clear's stores, grid-strided):
// the build's last kernel does it, none of its inputs being read after the assembly
__device__ __forceinline__ void let_clear_marks(int64_t t, int64_t stride, int64_t n,
                                                const LetBufs &L, int64_t nb) {
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    const int64_t nv = n >> 4;
    for (int64_t i = t; i < nv; i += stride) reinterpret_cast<uint4 *>(L.own)[i] = z;
    if (t < (n & 15)) L.own[(nv << 4) + t] = 0;
    for (int64_t i = t; i < LET_CELLS / 16; i += stride) reinterpret_cast<uint4 *>(L.ecell)[i] = z;
    for (int64_t i = t; i < nb; i += stride) L.own_blk[i] = 0;
    for (int64_t i = t; i < 256 * 8; i += stride) L.rowmask[i] = 0u;
    if (t < L.nvmax) L.vmax[t] = 0ull;
    if (t == 0) *L.flag_all = 0u;
}

__global__ __launch_bounds__(TB) void k_let_lanes(LetPieces pc, uint32_t n_sub,
                                                  const uint32_t *__restrict__ subpos,
                                                  const uint32_t *__restrict__ scal,
                                                  uint32_t *__restrict__ lanes, LetBufs L,
                                                  int64_t nb_clear) {
    const int64_t t = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (nb_clear >= 0) let_clear_marks(t, (int64_t)gridDim.x * TB, pc.n, L, nb_clear);
    if (t >= (int64_t)pc.rounds * pc.sub) return;
    const int64_t q = own_lane(pc, t);
    if (q >= pc.n) return;
    // every own body is in the subset (its cell is an own cell, or it is listed as own); the
    // clamp only keeps a broken invariant inside the subset
    const uint32_t s = subpos[pc.lanes ? (int64_t)pc.lanes[q] : q];
    // after a subset overflow (the call is replayed) the lanes sit out: no walk, no kick
    lanes[q] = scal[4] ? LANE_IDLE : (s < n_sub ? s : 0u);
}

__global__ __launch_bounds__(TB) void k_let_set_pos(int64_t n, const uint32_t *__restrict__ lanes,
                                                    const double *__restrict__ a2, GatherLayout gl,
                                                    double *__restrict__ x, double *__restrict__ y,
                                                    const uint32_t *__restrict__ skip) {
    const int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (q >= n || (skip && *skip)) return;  // skip: a subset overflow left the state as it was
    const int64_t i = lanes ? (int64_t)lanes[q] : q, g = gather_slot(gl, q);
    x[i] = a2[2 * g];
    y[i] = a2[2 * g + 1];
}

__global__ __launch_bounds__(TB) void k_let_fill_pos(int64_t n, const uint32_t *__restrict__ lanes,
                                                     const double *__restrict__ x,
                                                     const double *__restrict__ y,
                                                     double *__restrict__ a2, GatherLayout gl) {
    const int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (q >= n) return;
    const int64_t i = lanes ? (int64_t)lanes[q] : q, g = gather_slot(gl, q);
    a2[2 * g] = x[i];
    a2[2 * g + 1] = y[i];
}

__global__ __launch_bounds__(TB) void k_let_pack_vel(LetPieces pc, const double *__restrict__ vx,
                                                     const double *__restrict__ vy,
                                                     double *__restrict__ a2, GatherLayout gl) {
    const int64_t t = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (t >= (int64_t)pc.rounds * pc.sub) return;
    const int64_t q = own_lane(pc, t);
    if (q >= pc.n) return;
    const int64_t i = pc.lanes ? (int64_t)pc.lanes[q] : q, g = gather_slot(gl, q);
    a2[2 * g] = vx[i];
    a2[2 * g + 1] = vy[i];
}

__global__ __launch_bounds__(TB) void k_let_gather_slots(int64_t n,
                                                         const uint32_t *__restrict__ lanes,
                                                         GatherLayout gl,
                                                         uint32_t *__restrict__ gslot) {
    const int64_t q = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (q < n) gslot[lanes ? (int64_t)lanes[q] : q] = (uint32_t)gather_slot(gl, q);
}

}  // namespace

void let_gather_slots(int64_t n, const uint32_t *lanes, GatherLayout gl, uint32_t *gslot,
                      hipStream_t s) {
    if (n > 0) k_let_gather_slots<<<grid_for(n), TB, 0, s>>>(n, lanes, gl, gslot);
}

void let_set_pos(int64_t n, const uint32_t *lanes, const double *a2, GatherLayout gl, double *x,
                 double *y, const uint32_t *skip, hipStream_t s) {
    if (n > 0) k_let_set_pos<<<grid_for(n), TB, 0, s>>>(n, lanes, a2, gl, x, y, skip);
}

void let_fill_pos(int64_t n, const uint32_t *lanes, const double *x, const double *y, double *a2,
                  GatherLayout gl, hipStream_t s) {
    if (n > 0) k_let_fill_pos<<<grid_for(n), TB, 0, s>>>(n, lanes, x, y, a2, gl);
}

void let_pack_vel(const LetPieces &pc, const double *vx, const double *vy, double *a2,
                  GatherLayout gl, hipStream_t s) {
    const int64_t m = (int64_t)pc.rounds * pc.sub;
    if (m > 0 && pc.n > 0) k_let_pack_vel<<<grid_for(m), TB, 0, s>>>(pc, vx, vy, a2, gl);
}

void let_unpack_vel(int64_t n, const uint32_t *lanes, const double *a2, GatherLayout gl,
                    double *vx, double *vy, hipStream_t s) {
    // the same copy as the positions' (lane's gather slot -> its body's slot)
    if (n > 0) k_let_set_pos<<<grid_for(n), TB, 0, s>>>(n, lanes, a2, gl, vx, vy, nullptr);
}

double let_include_gap2(const Geometry &g, double theta2, double soft2) {
    if (!(theta2 > 0.0) || g.J <= LET_P + 1) return -1.0;
    // a cell at distance D from the own bodies is accepted by all of them when
    // theta2 * ((D - m)^2 + soft2) >= s2_P (1 + 1e-6): m covers jitter (<= 2e-3 per axis) and the
    // rounding of centres of mass; the criterion's own rounding is far inside the 1e-6
    const double w = 2.0 * g.h[LET_P], m = 0.01;
    const double q = g.s2[LET_P] * (1.0 + 1e-6) / theta2 - soft2;
    const double r = (m + std::sqrt(q > 0.0 ? q : 0.0)) / w;
    const double gap2 = r * r;
    return gap2 > 16.0 * 16.0 ? -1.0 : gap2;  // a halo this wide: the replicated build
}

// The assembly's two per-cell scans (record counts -> posc, copied-cell counts -> cpos) as one
// scan of pairs (BH_LET_PAIR_SCAN): one lookback launch pair instead of two.
#ifndef BH_LET_PAIR_SCAN
#define BH_LET_PAIR_SCAN 1
#endif
using U32Pair = rocprim::tuple<uint32_t, uint32_t>;
struct PairPlus {
    __host__ __device__ U32Pair operator()(const U32Pair &a, const U32Pair &b) const {
        return U32Pair(rocprim::get<0>(a) + rocprim::get<0>(b),
                       rocprim::get<1>(a) + rocprim::get<1>(b));
    }
};
hipError_t pair_scan(void *scratch, size_t &bytes, const uint32_t *a, const uint32_t *b,
                     uint32_t *sa, uint32_t *sb, size_t count, hipStream_t s) {
    auto in = rocprim::make_zip_iterator(rocprim::make_tuple(a, b));
    auto out = rocprim::make_zip_iterator(rocprim::make_tuple(sa, sb));
    return rocprim::exclusive_scan(scratch, bytes, in, out, U32Pair(0u, 0u), count, PairPlus(), s);
}

size_t let_scratch_bytes(int64_t n) {
    size_t a = 0, b = 0, c = 0;
    (void)rocprim::exclusive_scan(nullptr, a, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u,
                                  (size_t)(n + 1), rocprim::plus<uint32_t>());
    (void)rocprim::exclusive_scan(nullptr, b, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u,
                                  (size_t)(LET_CELLS + 1), rocprim::plus<uint32_t>());
    (void)pair_scan(nullptr, c, nullptr, nullptr, nullptr, nullptr, (size_t)(LET_CELLS + 1),
                    nullptr);
    return std::max({a, b, c});
}

// The selection's three clears in one launch (16-byte stores; the buffers are hipMalloc'd):
// own[0, n), ecell[0, LET_CELLS), *flag_all.
static_assert(LET_CELLS % 16 == 0, "ecell is cleared in 16-byte stores");
__global__ __launch_bounds__(TB) void k_let_clear(int64_t n, uint8_t *__restrict__ own,
                                                  uint8_t *__restrict__ ecell,
                                                  uint32_t *__restrict__ flag_all,
                                                  uint8_t *__restrict__ own_blk, int64_t nb,
                                                  uint32_t *__restrict__ rowmask,
                                                  unsigned long long *__restrict__ vmax,
                                                  int nvmax) {
    const int64_t t = (int64_t)blockIdx.x * TB + threadIdx.x;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    const int64_t nv = n >> 4;
    if (t < nv) reinterpret_cast<uint4 *>(own)[t] = z;
    if (t < (n & 15)) own[(nv << 4) + t] = 0;
    if (t < LET_CELLS / 16) reinterpret_cast<uint4 *>(ecell)[t] = z;
    if (t < nb) own_blk[t] = 0;
    if (t < 256 * 8) rowmask[t] = 0u;
    if (t < nvmax) vmax[t] = 0ull;  // the drift bound's words (read at the last evaluation's end)
    if (t == 0) *flag_all = 0u;
}

hipError_t let_select(const BodyState &st, const PosSrc &ps, const Geometry &g,
                      const LetPieces &pc, double gap2, const LetBufs &L, const BodyState &sub,
                      int64_t S, uint32_t *scal, hipStream_t s, const MortonFuse &mf,
                      const LetSweep &sw, bool clean) {
    if (pc.n <= 0) {
        hipError_t e = hipMemsetAsync(L.ecell, 0, LET_CELLS, s);
        return e == hipSuccess ? hipMemsetAsync(L.flag_all, 0, sizeof(uint32_t), s) : e;
    }
    const int64_t nb = let_sel_blocks(pc.n);
    const int64_t clear = std::max<int64_t>({pc.n >> 4, LET_CELLS / 16, nb, 256 * 8});
    if (!clean)  // (else the previous LET build's lane map cleared them)
        k_let_clear<<<grid_for(clear), TB, 0, s>>>(pc.n, L.own, L.ecell, L.flag_all, L.own_blk,
                                                   nb, L.rowmask, L.vmax, L.nvmax);
    hipError_t e;
    const int64_t marks = (int64_t)pc.rounds * pc.sub;
    if (marks > 0)
        k_let_mark<<<grid_for(marks), TB, 0, s>>>(pc, ps, st.x, st.y, st.cidx, g, L.own,
                                                  L.own_blk, L.ecell, L.flag_all);
    const int K = (int)std::floor(std::sqrt(gap2 > 0.0 ? gap2 : 0.0)) + 1;
    k_let_halo<<<grid_for(LET_CELLS), TB, 0, s>>>(L.ecell, L.flag_all, gap2, K, L.hcell,
                                                  L.rowmask);
    k_let_flags<<<(unsigned)nb, 64, 0, s>>>(pc, ps, st.x, st.y, st.cidx, g, L.hcell, L.own,
                                            L.flag8, L.sel, L, sw);
    size_t bytes = L.scratch_bytes;
    e = rocprim::exclusive_scan(L.scratch, bytes, L.sel, L.selpos, 0u, (size_t)(nb + 1),
                                rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    k_let_gather<<<(unsigned)nb, TB, 0, s>>>(pc.n, ps, L.flag8, L.selpos, st, sub, S,
                                             L.selpos + nb, L.table, scal, g, mf);
    return hipGetLastError();
}

void let_boxes(int64_t n, const BodyState &st, const Geometry &g, uint32_t *box, hipStream_t s) {
    if (n > 0)
        k_let_boxes<<<(unsigned)let_sel_blocks(n), 64, 0, s>>>(n, st.x, st.y, st.cidx, g, box);
}

void let_disp_add(double *disp, const unsigned long long *vmax, int k, double dt, hipStream_t s) {
    k_let_disp_add<<<1, 1, 0, s>>>(disp, vmax, k, dt);
}

hipError_t let_table(int64_t n_sub, const Geometry &g, const LetBufs &L, const TreeBuffers &tb,
                     hipStream_t s) {
    k_let_table<<<grid_for(LET_CELLS + 1), TB, 0, s>>>(n_sub, g.J, L, tb);
    return hipGetLastError();
}

#ifndef BH_LET_CLEAR_AHEAD
#define BH_LET_CLEAR_AHEAD 1
#endif
hipError_t let_assemble(int64_t n_sub, const Geometry &g, const LetPieces &pc, const LetBufs &L,
                        const TreeBuffers &tb, uint32_t *scal, hipStream_t s, bool *cleaned) {
    if (cleaned) *cleaned = false;
    k_let_top_hi<<<256, 256, 0, s>>>(pc.world, g, L.tables, L.levels, scal);
    k_let_top_lo<<<1, 256, 0, s>>>(g, L.levels);
    k_let_w<<<grid_for(LET_CELLS + 1), TB, 0, s>>>(L, tb, scal);
    size_t bytes = L.scratch_bytes;
    hipError_t e;
    if (BH_LET_PAIR_SCAN) {
        e = pair_scan(L.scratch, bytes, L.w, L.ccnt, L.posc, L.cpos, (size_t)(LET_CELLS + 1), s);
        if (e != hipSuccess) return e;
    } else {
        e = rocprim::exclusive_scan(L.scratch, bytes, L.w, L.posc, 0u, (size_t)(LET_CELLS + 1),
                                    rocprim::plus<uint32_t>(), s);
        if (e != hipSuccess) return e;
        bytes = L.scratch_bytes;
        e = rocprim::exclusive_scan(L.scratch, bytes, L.ccnt, L.cpos, 0u, (size_t)(LET_CELLS + 1),
                                    rocprim::plus<uint32_t>(), s);
        if (e != hipSuccess) return e;
    }
    k_let_write_top_cells<<<grid_for(level_off(LET_P) + LET_CELLS), TB, 0, s>>>(L);
    k_let_copy_blocks<<<BH_LET_COPY_GRID, TB, 0, s>>>(L, tb.nodes);
    if (n_sub > 0)
        k_let_subpos<<<grid_for(n_sub), TB, 0, s>>>(n_sub, pc.n, tb.dst.vx, L.subpos, L, scal);
    else
        k_let_guard<<<1, 1, 0, s>>>(L, scal);
    const int64_t own_lanes = (int64_t)pc.rounds * pc.sub;
    if (own_lanes > 0 && pc.n > 0) {
        const bool clear = BH_LET_CLEAR_AHEAD && cleaned;
        k_let_lanes<<<grid_for(own_lanes), TB, 0, s>>>(pc, (uint32_t)n_sub, L.subpos, scal,
                                                        L.lanes, L,
                                                        clear ? let_sel_blocks(pc.n) : -1);
        if (clear) *cleaned = true;
    }
    return hipGetLastError();
}

}  // namespace bh
