/*
 * bh_engine.h — C-ABI drop-in boundary of the MI355X Barnes–Hut engine.
 *
 * Replaces the reference's PhysicsEngine / Body / BHTree Kotlin surface
 * (/root/reference/src/main/kotlin/BarnesHutAlg.kt = BHA, Config.kt = CFG) as consumed by
 * NBodyPanel (NBodyPanel.kt = PNL).  Plain pointers and sizes only: a JNI / Panama / ctypes
 * shim binds these symbols directly (INTEGRATION.md shows the Kotlin-side binding).
 *
 * Semantics are the reference's, bit for bit in IEEE binary64:
 *   - bodies are SoA fp64 arrays (x, y, vx, vy, m) in the caller's list order (BHA:21-25);
 *   - one bh_step() == one PhysicsEngine.step() (BHA:405-439): build, a(t), kick, drift,
 *     build, a(t+dt), kick, merge (BHA:463-532), so N may shrink;
 *   - the quadtree jitter (BHA:146-151) mutates positions exactly as the reference does;
 *   - bodies outside the root cell are not inserted but still integrate (BHA:126).
 *
 * Errors: every int-returning call returns 0 on success and a negative BH_E* code on
 * failure; bh_last_error() returns a human-readable message.  Nothing aborts the process.
 * Threading: one host thread per engine handle; calls are synchronous (results are
 * visible to bh_get_bodies on return), like step() under runBlocking (BHA:408,426).
 */
#ifndef BH_ENGINE_H
#define BH_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BH_OK 0
#define BH_E_INVALID (-1)  /* bad argument */
#define BH_E_DEVICE (-2)   /* HIP runtime error */
#define BH_E_COMM (-3)     /* RCCL error */
#define BH_E_CAPACITY (-4) /* caller buffer too small; *n_out holds the required size */
#define BH_E_STATE (-5)    /* call not valid in this state */

/* The Config.kt fields the hot path reads live, plus the merge knobs.
 * Replaces: Config.G (CFG:11), Config.DT (CFG:14), Config.theta (CFG:23),
 * Config.SOFT2 (CFG:20), Config.WIDTH_PX/HEIGHT_PX (CFG:5,8; root cell BHA:360-361),
 * PhysicsEngine.mergeMaxMass (BHA:315), PhysicsEngine.mergeMinDist (BHA:321). */
typedef struct bh_params {
    double G;
    double dt;
    double theta;
    double soft2;
    int32_t width_px;
    int32_t height_px;
    double merge_max_mass;
    double merge_min_dist;
} bh_params;

/* Reference defaults (CFG:5-23, BHA:315,321). */
void bh_default_params(bh_params *p);

typedef struct bh_engine bh_engine;

/* new PhysicsEngine(...) (BHA:287) on HIP device `device`, single GPU. */
int bh_create(const bh_params *p, int device, bh_engine **out);

/* new PhysicsEngine(...) (BHA:287) over every GPU of `device_mask` (bit d = HIP device d; 0 = every
 * visible device) behind ONE handle: the reference's step() fans its force evaluation out over
 * worker threads and joins them (computeAccelerations, BHA:374-395, inside runBlocking, BHA:408,
 * 426); this handle fans every step out over the GPUs and returns when all are done, so the one
 * PhysicsEngine object of the front-end (NBodyPanel.kt:103, 290-293) drives all of them.
 * Inside: one member engine per GPU -- the ranks of bh_create_dist's decomposition (replicated
 * state, locally essential tree builds, every exchange an in-place RCCL all-gather over xGMI on
 * communicators made in this process by ncclCommInitAll) -- each driven by its own host thread
 * (member 0 by the caller's).  Every call of this header takes the handle: calls that change the
 * state run on every member, calls that read it read member 0's replica (complete at every API
 * boundary), bh_set_mirror / bh_map_bodies use member 0's mirror.  One set bit = bh_create (the
 * pipelined one-GPU engine).  Results are bit-identical to bh_create's on the paths tested: one
 * GPU, members that share a device (device-to-device copies) and a one-rank RCCL communicator;
 * the distinct-device RCCL path (more than one rank) has not run on hardware yet, so callers
 * should keep one GPU (mask 1, or bh_create) unless they opt in (the Kotlin drop-in's default).
 * A call that fails on one member -- or whose waits for the others exceed BH_COMM_TIMEOUT_S
 * seconds (default 300; 0 = forever) -- aborts the others' waits (RCCL: ncclCommAbort) and returns
 * an error from every member; the handle then returns BH_E_COMM for every call that uses the
 * bodies until bh_reset_bodies, which makes new communicators. */
int bh_create_multi(const bh_params *p, uint32_t device_mask, bh_engine **out);

/* The same over an explicit device list, repeats allowed: a device listed twice hosts two members
 * (RCCL refuses two ranks per device), so a list with repeats -- or BH_MULTI_EXCHANGE=copy in the
 * environment -- exchanges by device-to-device copies between the members (an in-process group,
 * bh_create_local) instead of RCCL; the pieces, rounds and layout are the same. */
int bh_create_multi_list(const bh_params *p, const int32_t *devices, int32_t count,
                         bh_engine **out);

/* Members of a multi-device handle (1 for any other engine) and member `rank`'s own handle, for
 * diagnostics (per-rank timings, LET statistics, collective logs, bh_debug_inject on one rank).
 * Owned by the handle: never bh_destroy a member, and never bh_step one on its own (its peers
 * would wait for it).  A plain engine is its own member 0. */
int bh_multi_world(const bh_engine *e);
bh_engine *bh_multi_member(bh_engine *e, int rank);

/* Multi-rank engines log every collective they issue, in host issue order: 4 int64 per entry --
 * the engine's state-changing API call count when it was issued, the site (1 a round of
 * accelerations, 2 a round of new positions, 3 a round of velocities, 4 the LET cell tables,
 * 5 the end-of-call LET status all-reduce, 6 the settings check at creation), the bytes every
 * rank receives, and the stream (0 the engine's, 1 the exchange stream).  Every rank of a
 * decomposition must log the same sequence: RCCL pairs the n-th call of every rank.  The
 * in-process exchange logs the same entries.  BH_E_CAPACITY + *n_out if cap is too small. */
int bh_collective_log(const bh_engine *e, int64_t *out4, int64_t cap, int64_t *n_out);
int bh_collective_log_clear(bh_engine *e);

/* Multi-GPU member: one process per GPU; `unique_id` is the 128-byte RCCL id produced by
 * bh_comm_unique_id() on rank 0 and broadcast by the caller (e.g. torch.distributed).
 * Replaces computeAccelerations' fan-out over worker threads (BHA:374-395) by a fan-out over
 * GPUs.  Every rank holds a replica of the state and owns one contiguous range of the Hilbert
 * wave order (bh_shard_range).  Per force evaluation a rank either
 *   - builds a locally essential tree (from 2 ranks up, or BH_LET=1): only the depth-8 cells its
 *     bodies can open, plus the top computed from every rank's cell values (one all-gather of
 *     2 MB cell tables); it evaluates its range, kicks (and drifts) its own bodies, and the new
 *     positions -- 16 B per body -- are all-gathered over RCCL in BH_SHARD_ROUNDS rounds into
 *     every replica; velocities stay with their owners and are all-gathered before the next
 *     full build; or
 *   - builds the full tree (the first build after a reset, every 32 builds): it evaluates its
 *     range and the accelerations are all-gathered, after which every rank integrates every body.
 * At the end of every bh_step call the positions and velocities are complete on every rank
 * (velocities all-gathered if the call ended with a LET build); bh_get_quads then builds the
 * last build's full tree on demand (lastTree) without changing the rank's state.
 * The merge rule is replicated (identical inputs).  world == 1 with a non-NULL id runs the same
 * RCCL path on one rank (used to test it on one GPU).  BH_LET and BH_ROUND_FRACS must be equal
 * on every rank (checked at creation: BH_E_INVALID on every rank otherwise). */
int bh_create_dist(const bh_params *p, int device, int rank, int world, const void *unique_id,
                   bh_engine **out);
int bh_comm_unique_id(void *out128);

/* RCCL's own view of the engine's communicator: *nranks = ncclCommCount, *rank =
 * ncclCommUserRank; *nranks = 0 (and *rank = the engine's rank) for an engine without one
 * (single GPU, in-process group, solo). */
int bh_comm_ranks(const bh_engine *e, int32_t *nranks, int32_t *rank);

/* Test hooks.  what == 1: the next locally essential tree build of this rank trips the node
 * array guard (let.hip k_let_guard), as a broken invariant on one rank would; the call must then
 * be replayed by every rank of the group alike.  what == 2 + k (k < 98): the k-th next full tree
 * build (k = 0: the next one) raises the jitter replay's error flag, as the unsupported-geometry
 * guard would; the bh_step call whose step uses that tree returns BH_E_STATE -- for a call's last
 * pipelined build (the next call's first tree) that is the next call; what == 99: that carried tree
 * (one GPU, after a call) raises its flag now (BH_E_STATE if there is none).  what == 100 + k: this rank
 * fails host-side (BH_E_COMM) right before its k-th next collective; what == 200 + k: before its
 * k-th next in-process group barrier -- a rank-local error between collectives: every rank of the
 * decomposition must then return an error within a bounded time, refuse further calls with
 * BH_E_COMM, and step bit-exactly again after bh_reset_bodies. */
int bh_debug_inject(bh_engine *e, int what);

/* Progress of an engine, safe to read from any thread while a call runs (a watchdog's
 * heartbeat): out4[0] state-changing API calls begun, [1] collectives issued, [2] the site of
 * the last one (as bh_collective_log), [3] bit 0 a call is running, bit 1 the last multi-rank
 * call failed (BH_E_COMM until bh_reset_bodies), bit 2 its RCCL communicator was aborted.  A
 * multi-device handle reports member 0's (bh_multi_member for the others). */
int bh_progress(const bh_engine *e, int64_t *out4);

/* In-process rank group (testing the multi-GPU decomposition on one device, where RCCL refuses
 * several ranks): `world` engines of one process, each driven by its own host thread with
 * identical calls, exchange the force pieces with device-to-device copies on the same pieces,
 * rounds and in-place layout as bh_create_dist's ncclAllGather. */
typedef struct bh_local_group bh_local_group;
int bh_local_group_create(int world, bh_local_group **out);
void bh_local_group_destroy(bh_local_group *g);  /* after its members' bh_destroy */
int bh_create_local(const bh_params *p, int device, int rank, bh_local_group *group,
                    bh_engine **out);

/* Measurement only: rank `rank` of a `world`-rank engine running alone on one device -- the
 * rank's own work of a multi-GPU step (its locally essential tree builds, the traversal of its
 * pieces, the integration of every body) without peers and without the exchange: the peers'
 * bodies get zero acceleration and the cell values of the peers' cells come from the last
 * full build.  Times one GPU's share of the north-star decomposition on a single GPU; the
 * results are NOT the reference's. */
int bh_create_solo(const bh_params *p, int device, int rank, int world, bh_engine **out);

void bh_destroy(bh_engine *e);
const char *bh_last_error(const bh_engine *e);

/* Live Config mutation (PNL:247-260 change theta/DT/G between steps). */
int bh_set_params(bh_engine *e, const bh_params *p);
int bh_get_params(const bh_engine *e, bh_params *p);

/* PhysicsEngine.resetBodies(newBodies) (BHA:342-349): copy-in of n bodies. */
int bh_reset_bodies(bh_engine *e, int64_t n, const double *x, const double *y, const double *vx,
                    const double *vy, const double *m);

/* On-disk state (checkpoint / resume): the Config fields and the body list in the caller's
 * order as one little-endian file: an 80-byte header -- the 8-byte magic "BHSTATE1", a uint32
 * holding the size of the block that follows the first 16 bytes (64: the bh_params fields and
 * the int64 N), a uint32 flags word (0), that block -- then x[N], y[N], vx[N], vy[N], m[N] fp64
 * from byte 16 + 64 = 80 (layout in csrc/state_io.cpp).  A file whose length is not
 * 80 + 40 N is rejected (BH_E_INVALID) before anything is allocated.  Loading = bh_set_params
 * + bh_reset_bodies (resetBodies, BHA:342-349) of the saved list, so a resumed run is
 * bit-identical to an uninterrupted one.  The file is written to path.tmp, then renamed. */
int bh_save_state(bh_engine *e, const char *path);
int bh_load_state(bh_engine *e, const char *path);

/* k x PhysicsEngine.step() (BHA:405-439). */
int bh_step(bh_engine *e, int32_t k);

/* bh_step(e, k) on a thread of the engine's own, for a caller that overlaps its own work with
 * the call (the drop-in shim: NBodyPanel's tick, PNL:290-306, around step(), BHA:405-439).
 * Needs the two-buffer mirror (bh_set_mirror(e, 2)), else BH_E_STATE.  Until bh_step_end the
 * caller may only read the mirror it mapped before (bh_map_bodies: the call writes the other
 * buffer) and call bh_step_positions (bh_step, bh_reset_bodies, bh_set_params, bh_get_bodies,
 * bh_map_bodies, bh_set_mirror, bh_get_quads and bh_compute_accelerations return BH_E_STATE); bh_step_end joins and returns bh_step's result (then
 * bh_last_removed, bh_map_bodies, ... as after bh_step).
 * bh_step_positions blocks until the call's positions and masses are final -- on one GPU that is
 * once its last merge rule is done, before its last traversal; else when the call ends -- and
 * returns the mirror planes x, y, m of the list after the call (n_out bodies; the other buffer
 * than the one mapped before) and survivors[j], ascending: survivor j's index in the list before
 * the call (n_before bodies) -- the removals are the indices missing from it (bh_last_removed
 * after bh_step_end).  vx and vy of the same buffer are final only after bh_step_end +
 * bh_map_bodies.  With x, y and m all NULL it returns as soon as the survivors are known (their
 * copy runs ahead of the planes').  If the call fails, bh_step_positions returns its error; if it
 * fails after the hand-off (an unsupported jitter geometry), bh_step_end does. */
int bh_step_begin(bh_engine *e, int32_t k);
int bh_step_positions(bh_engine *e, const double **x, const double **y, const double **m,
                      const uint32_t **survivors, int64_t *n_out, int64_t *n_before);
int bh_step_end(bh_engine *e);

/* getBodies().size */
int64_t bh_num_bodies(const bh_engine *e);

/* PhysicsEngine.getBodies() (BHA:335) copy-out; any pointer may be NULL to skip it.
 * Returns BH_E_CAPACITY with *n_out = N if cap < N. */
int bh_get_bodies(bh_engine *e, double *x, double *y, double *vx, double *vy, double *m,
                  int64_t cap, int64_t *n_out);

/* getBodies() without a copy (BHA:335; NBodyPanel reads every body after every step,
 * PNL:302-306): a pinned host mirror of the bodies in the caller's list order.
 * bh_set_mirror(e, 1) makes every bh_step call write it itself -- positions and masses while
 * its last traversal still runs, velocities right after -- so the device-to-host copy overlaps
 * the call's last tree build.  bh_map_bodies waits for that copy (or makes one if the state
 * changed since) and returns pointers to x[N], y[N], vx[N], vy[N], m[N] (any pointer may be
 * NULL).  They stay valid -- and the data unchanged -- until the next call on this engine that
 * changes or moves the bodies (bh_step, bh_reset_bodies, bh_get_quads, bh_compute_accelerations,
 * bh_load_state, bh_set_mirror, bh_destroy).
 * bh_set_mirror(e, 2): two pinned buffers -- the calls write the one bh_map_bodies did not hand
 * out last, so the mapped bodies stay valid and unchanged until the next bh_map_bodies (or
 * bh_set_mirror, bh_destroy), and a caller may read them on one thread while a bh_step runs
 * on another (the drop-in compares its list against them during the step).  enabled is 0, 1
 * or 2 (else BH_E_INVALID). */
int bh_set_mirror(bh_engine *e, int enabled);
int bh_map_bodies(bh_engine *e, const double **x, const double **y, const double **vx,
                  const double **vy, const double **m, int64_t *n_out);

/* buildTree() + computeAccelerations() (BHA:359-395) on the current state, exactly as
 * the first half of step() does it (including the jitter's position mutation).  ax/ay
 * (length N, caller order) receive F/m.  visits (nullable, length N) receives the number
 * of non-empty nodes each body's traversal visited (accumulateForce calls passing the
 * mass == 0 test, BHA:216) — the V of the roofline byte model. */
int bh_compute_accelerations(bh_engine *e, double *ax, double *ay, int64_t *visits);

/* Indices (into the list as it was before the last bh_step call, ascending) of the bodies the
 * merge rule removed during that call — what a shim needs to apply BHA:519's removeAt to the
 * caller's own list and keep Body identity.  BH_E_CAPACITY + *n_out if cap is too small. */
int bh_last_removed(const bh_engine *e, int64_t *idx, int64_t cap, int64_t *n_out);

/* getTreeForDebug().visitQuads{} (BHA:265-274,329-332): pre-order list of every cell
 * (cx, cy, h) of the last tree, or of a freshly built one if the cache was dropped
 * (after resetBodies or a merge, BHA:348,526).  BH_E_CAPACITY + *n_out if cap too small. */
int bh_get_quads(bh_engine *e, double *cx, double *cy, double *h, int64_t cap, int64_t *n_out);

/* Per-phase device timings (ms) of the last bh_step call, summed over its steps:
 * [0] tree build, [1] traversal, [2] integration, [3] merge, [4] all-gather. */
int bh_last_timings(const bh_engine *e, double *out5);

/* Number of tree nodes (non-empty + skip slots) of the last build; for byte models. */
int64_t bh_last_tree_nodes(const bh_engine *e);

/* Traversal kernel timing for roofline: average duration (ms) of the force-evaluation
 * kernel over the launches of the last bh_step, measured with HIP events on the
 * engine's own stream; *launches receives the count. */
int bh_traverse_kernel_ms(const bh_engine *e, double *avg_ms, int64_t *launches);

/* The same measurement per launch, in launch order (ms): min / median / max of the traversal
 * over a timed region.  BH_E_CAPACITY + *n_out if cap is too small. */
int bh_traverse_kernel_samples(const bh_engine *e, double *ms, int64_t cap, int64_t *n_out);

/* Lane efficiency of the last bh_compute_accelerations(..., visits != NULL): the sum over
 * bodies of visited nodes, the sum over wavefronts of nodes the wave's shared cursor stopped
 * at (union of its 64 bodies' traversals), and the number of wavefronts. */
int bh_traversal_stats(const bh_engine *e, int64_t *lane_visits, int64_t *wave_iters,
                       int64_t *waves);

/* All counters of the last bh_compute_accelerations(..., visits != NULL), summed over bodies /
 * wavefronts: [0] nodes visited, [1] point-force contributions (accepted internal nodes and
 * other bodies' leaves: the 20-flop work units of the FP64 roofline), [2] nodes the wavefronts'
 * shared cursors stopped at, [3] point-force blocks the wavefronts executed, [4] wavefronts.
 * Lane efficiency = [0] / (64 [2]); force-block lane use = ([1] + bodies) / (64 [3]). */
int bh_traversal_counters(const bh_engine *e, int64_t *out5);

/* Multi-rank build sharding (locally essential tree): out5[0] LET builds, out5[1] full-tree
 * builds since the engine was created, out5[2] bodies in the largest LET subset of the last
 * bh_step call (the cells this rank's bodies can open), out5[3] node records of the last LET
 * tree, out5[4] bh_step calls replayed because a subset outgrew its capacity (the capacity
 * follows the previous call's subsets, so the build needs no host round trip).  LET builds run
 * on every multi-rank engine (2 ranks up); BH_LET=1 in the environment before creating an engine
 * enables them also on one rank, BH_LET=0 keeps every build full. */
int bh_let_stats(const bh_engine *e, int64_t *out5);

/* Enable/disable per-phase event timing (default off: no events in the hot loop). */
int bh_set_profiling(bh_engine *e, int enabled);

/* Multi-GPU force evaluation runs in BH_SHARD_ROUNDS rounds.  Rank r owns the contiguous
 * lanes [r * rounds * sub, (r + 1) * rounds * sub) of the Hilbert wave order (one spatial
 * region: its locally essential tree has one halo), and round k evaluates its lanes
 * [lo, hi) = [(r * rounds + k) * sub, + sub) clipped to n, with sub = ceil(n / (world * rounds))
 * rounded up to whole wavefronts.  The accelerations of lane q are written to the exchange
 * buffer at bh_gather_slot(n, world, q) = (k * world + r) * sub + i (q = (r * rounds + k) * sub
 * + i): the pieces of round k are adjacent there and are all-gathered in place (one
 * ncclAllGather per round) on a second stream while round k + 1 is evaluated.  Host-only; used
 * by the engine itself. */
#ifndef BH_SHARD_ROUNDS
#define BH_SHARD_ROUNDS 4
#endif
int bh_shard_range(int64_t n, int rank, int world, int round, int64_t *lo, int64_t *hi);
int64_t bh_gather_slot(int64_t n, int world, int64_t lane);

/* Diagnostic: checks, on HIP device `device`, the traversal's reduced-range exact sequences
 * for sqrt(d2), 1/sqrt(d2) and 1/d2 (traverse.hip) bit-for-bit against the IEEE operations on
 * n generated operands (random, near powers of two, near perfect squares, physical range);
 * *mismatches receives the number of differing results (0 expected). */
int bh_selftest_fast_math(int device, int64_t n, uint64_t seed, int64_t *mismatches);

/* Block until all device work of this engine is complete. */
int bh_synchronize(bh_engine *e);

/* ---- scene generation (BodyFactory.kt = BF), host-side, deterministic -------------
 * Kotlin's kotlin.random.Random(seed) XorWow stream (kotlin-stdlib 2.2.20) restated so
 * that seeded scenes are reproducible; caller provides arrays of length n_total. */
int bh_scene_galaxy_disk(int32_t n_total, double eps_m2, double phi0, double bar_taper_r,
                         double radial_scale, double speed_jitter, double radial_jitter,
                         int32_t clockwise, int64_t seed, double vx, double vy, double x,
                         double y, double r, double min_r, double central_mass,
                         double total_satellite_mass, double G, double *ox, double *oy,
                         double *ovx, double *ovy, double *om);
int bh_scene_kepler_disk(int32_t n_total, int32_t clockwise, double radial_jitter,
                         double speed_jitter, int64_t seed, double vx, double vy, double x,
                         double y, double r, double G, double *ox, double *oy, double *ovx,
                         double *ovy, double *om);
int bh_scene_uniform(int32_t n, double m, int64_t seed, int32_t width_px, int32_t height_px,
                     double *ox, double *oy, double *ovx, double *ovy, double *om);

/* ---- fp32 3-D all-pairs engine: the physics of the reference's OpenGL compute shader
 * (gpu/GPU.kt:101-152 = "GPU").  a_i = sum_{j!=i} (G m_j) d / (d.d +
 * softening^2)^{3/2} with the hardware reciprocal square root (GLSL inversesqrt, GPU:140),
 * then v += a dt, x += v dt (GPU:145-146) — double-buffered instead of the reference's
 * in-place race.  fp32 throughout; parity is a tolerance, not bit-identity. */
typedef struct bh_nbody3d bh_nbody3d;
int bh_nbody3d_create(int device, bh_nbody3d **out);
void bh_nbody3d_destroy(bh_nbody3d *h);
const char *bh_nbody3d_last_error(const bh_nbody3d *h);
/* upload (replaces GpuNBody's SSBO upload of Body{x,y,z,vx,vy,vz,m}) */
int bh_nbody3d_set(bh_nbody3d *h, int64_t n, const float *x, const float *y, const float *z,
                   const float *vx, const float *vy, const float *vz, const float *m);
/* GpuNBody.simulate(dt, g, softening) x k (GPU:411-422) */
int bh_nbody3d_step(bh_nbody3d *h, int32_t k, float dt, float G, float softening);
/* one evaluation of the accelerations of the current state (no integration) */
int bh_nbody3d_accelerations(bh_nbody3d *h, float G, float softening, float *ax, float *ay,
                             float *az);
int bh_nbody3d_get(const bh_nbody3d *h, float *x, float *y, float *z, float *vx, float *vy,
                   float *vz, float *m, int64_t cap, int64_t *n_out);
/* device time (ms) of the last bh_nbody3d_step / bh_nbody3d_accelerations call */
double bh_nbody3d_last_ms(const bh_nbody3d *h);

#ifdef __cplusplus
}
#endif
#endif /* BH_ENGINE_H */
