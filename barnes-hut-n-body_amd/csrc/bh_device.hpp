// Device-side data layout shared by the engine's HIP translation units.
//
// The quadtree of the reference (BHA:95-202, a pointer tree of BHTree objects) is held in
// HBM as ONE flat array of 32-byte node records in depth-first PRE-ORDER with the
// reference's child order 0..3 (BHA:73-81 NW,NE,SW,SE == ascending Morton digit).
// Only non-empty cells are stored: accumulateForce returns on mass == 0 (BHA:216), so an
// empty cell contributes nothing and is never descended.  Each record carries `next`, the
// pre-order index just past its subtree, so the traversal is stackless:
//     open    -> cur + 1      (first child)
//     skip    -> next         (accepted, leaf, or nobody in the wave opened it)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

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
constexpr uint32_t NODE_LEAF = 1u << 31;        // leaf holding one body (BHA:97)
constexpr uint32_t NODE_SKIP = 1u << 30;        // mass == 0.0: never visited (BHA:216)
constexpr uint32_t NODE_BODY_MASK = (1u << 30) - 1;  // leaf: Morton-sorted body position
constexpr uint32_t NODE_DEPTH_MASK = 0xFFu;     // internal: depth (root = 0)
constexpr int NODE_JMASK_SHIFT = 8;             // jitter cell: which children got subdivided
constexpr uint32_t NODE_SPAN = 1u << 12;        // internal: body range crosses a COM chunk

// Centre-of-mass chunking (tree_build.hip): nodes inside a 2^COM_CHUNK_SHIFT-body chunk of
// the Morton order are finished by one workgroup; the rest are listed per level.
constexpr int COM_CHUNK_SHIFT = 10;
__host__ __device__ inline uint32_t span_stride_for(int64_t n) {
    return (uint32_t)((n >> COM_CHUNK_SHIFT) + 2);
}

constexpr int MAX_DEPTH_TAB = 40;

// Root cell and per-depth geometry, computed on the host exactly as the reference does:
// root Quad(W/2, H/2, max(W,H)/2 + 2) (BHA:360-361); child h = h / 2.0 (BHA:74).
struct Geometry {
    double root_cx, root_cy, root_h;
    int J;                        // first depth whose h < 1e-3: the jitter depth (BHA:146)
    double h[MAX_DEPTH_TAB];      // h at depth d
    double s2[MAX_DEPTH_TAB];     // (h*2.0)^2 at depth d (BHA:226)
};

// Key of a body outside the root cell (never inserted, BHA:126): sorts after every
// in-root key and differs from all of them at every prefix length.
__host__ __device__ inline uint64_t sentinel_key(int J) { return 1ull << (2 * J); }

// Force-evaluation constants (BHA:225,253,256,378).
struct ForceParams {
    double G, soft2, theta2;
};

// ---- launchers (tree_build.hip) --------------------------------------------------
struct TreeBuffers {
    // inputs: positions in caller order (mutated by the jitter), masses
    double *x, *y;
    const double *m;
    // workspace
    uint64_t *keys, *keys_s;
    uint32_t *idx, *perm;
    double *sx, *sy, *sm;  // Morton-sorted copies (sm: mass)
    int8_t *cpl;           // c(a): common digit count between sorted keys a, a+1; -1 at ends
    uint32_t *cnt, *base;  // node slots per sorted body; exclusive scan (n + 1 entries)
    Node *nodes;
    uint32_t *scalars;     // [0] = node count T, [1] = error flags
    uint32_t *span_cnt;    // [J + 1] chunk-spanning internal nodes per level
    uint32_t *span_list;   // [(J + 1) * span_stride]
    uint32_t span_stride;
    uint4 *span_children;  // [(J + 1) * span_stride]
    void *cub_tmp;
    size_t cub_bytes;
};

size_t tree_cub_bytes(int64_t n, int J);
hipError_t tree_build(const TreeBuffers &b, int64_t n, const Geometry &g, hipStream_t s);

// ---- launchers (traverse.hip) ----------------------------------------------------
// Accelerations for Morton-sorted positions [lo, hi).  If a_sorted == nullptr the result
// F/m is scattered to ax/ay in caller order through perm; otherwise it is written
// interleaved (ax, ay) to a_sorted[2p], a_sorted[2p+1] for the multi-GPU all-gather.
void traverse(const Node *nodes, const uint32_t *d_T, const double *sx, const double *sy,
              const double *sm, const uint32_t *perm, int64_t lo, int64_t hi, const Geometry &g,
              const ForceParams &fp, double *ax, double *ay, double *a_sorted, uint32_t *visits,
              uint32_t *wave_iters, hipStream_t s);
void scatter_sorted_acc(const double *a_sorted, const uint32_t *perm, int64_t n, double *ax,
                        double *ay, hipStream_t s);

// ---- launchers (integrate.hip) ---------------------------------------------------
void kick_drift(int64_t n, const double *ax, const double *ay, double *x, double *y, double *vx,
                double *vy, double dtHalf, double dt, hipStream_t s);
void kick(int64_t n, const double *ax, const double *ay, double *vx, double *vy, double dtHalf,
          hipStream_t s);

struct MergePair {
    uint32_t k;  // heavy list position
    uint32_t j;  // victim candidate body index
    double mj;   // candidate mass
};
size_t merge_cub_bytes(int64_t n);
// Ordered list of bodies with m > thr (BHA:474); returns via d_count.
hipError_t heavy_list(const double *m, int64_t n, double thr, uint32_t *heavy, uint32_t *d_count,
                void *tmp, size_t tmp_bytes, hipStream_t s);
void merge_candidates(int64_t n, const double *x, const double *y, const double *m,
                      const uint32_t *heavy, uint32_t H, double minD2, MergePair *pairs,
                      uint32_t cap, uint32_t *d_count, hipStream_t s);
// Remove flagged bodies (keep[i] == 0) preserving order; writes compacted arrays to dst.
hipError_t compact_bodies(int64_t n, const uint32_t *keep, const double *const src[5], double *const dst[5],
                    uint32_t *pos, uint32_t *d_count, void *tmp, size_t tmp_bytes, hipStream_t s);
// keep[dead[i]] = 0; m[upd_idx[i]] = upd_mass[i]
void apply_merge(uint32_t n_dead, const uint32_t *dead, uint32_t n_upd, const uint32_t *upd_idx,
                 const double *upd_mass, uint32_t *keep, double *m, hipStream_t s);
void gather_doubles(const uint32_t *idx, uint32_t cnt, const double *src, double *dst, hipStream_t s);

}  // namespace bh
