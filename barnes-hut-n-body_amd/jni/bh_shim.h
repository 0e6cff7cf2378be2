/*
 * bh_shim.h -- the logic of the Kotlin drop-in's JNI natives, as plain C
 * over the C-ABI (include/bh_engine.h): no JNI types, so tests/c/abi_harness.c drives exactly
 * this code against the oracle, and bh_jni.c only moves Java arrays in and out.
 *
 * Array layouts are the Kotlin shim's (PhysicsEngine.soa() / pull() / QuadList (kotlin/PhysicsEngine.kt)):
 *   bodies  SoA, 5 n doubles: x[0..n) y[0..n) vx[0..n) vy[0..n) m[0..n)   (BHA:21-25)
 *   quads   interleaved triples cx, cy, h in visitQuads pre-order          (BHA:265-274)
 *   removed int32 list indices, ascending, relative to the list before the last step (BHA:519)
 * Every function returns BH_OK or a negative BH_E_* code (bh_last_error has the message).
 */
#ifndef BH_SHIM_H
#define BH_SHIM_H

#include <stdint.h>

#include "bh_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Native.create(deviceMask): PhysicsEngine's engine (BHA:287) over the HIP devices of
 * `device_mask` (bit d = device d, 0 = every visible device; bh_create_multi: one handle, the
 * step fanned out over the GPUs and joined), with the pinned body mirror on (every step writes
 * the caller-order bodies to host memory itself).  BH_DEVICES="0,1,..." in the environment
 * overrides the mask with an explicit device list (repeats allowed: bh_create_multi_list). */
int bh_shim_create(uint32_t device_mask, bh_engine **out);

/* Native.setParams: Config.G / DT / theta / SOFT2 / WIDTH_PX / HEIGHT_PX (CFG:5-23) and
 * mergeMaxMass / mergeMinDist (BHA:315,321), read live before every step. */
int bh_shim_set_params(bh_engine *e, double G, double dt, double theta, double soft2,
                       int32_t width_px, int32_t height_px, double merge_max_mass,
                       double merge_min_dist);

/* Native.reset(n, soa): resetBodies (BHA:342-349) from the 5 n SoA array. */
int bh_shim_reset(bh_engine *e, int64_t n, const double *soa);

/* Native.step(k): k x step() (BHA:405-439). */
int bh_shim_step(bh_engine *e, int32_t k);

/* Native.stepBegin / positions / stepEnd: step() with the shim's own work beside it
 * (bh_step_begin / bh_step_positions / bh_step_end).  positions: soa[0..5) point at the planes of
 * the mirror buffer the running call writes (x, y, m final; vx, vy after stepEnd + map), *n
 * bodies after the call, *n_before before it, survivors[j] = survivor j's list index before the
 * call (ascending) -- the merge rule's removals are the indices missing from it (BHA:519). */
int bh_shim_step_begin(bh_engine *e, int32_t k);
int bh_shim_positions(bh_engine *e, const double *soa[5], int64_t *n, int64_t *n_before,
                      const int32_t **survivors);
/* survivors alone: returns as soon as they are known, ahead of the planes' copy */
int bh_shim_survivors(bh_engine *e, const int32_t **survivors, int64_t *n, int64_t *n_before);
int bh_shim_step_end(bh_engine *e);

/* Native.get: getBodies() (BHA:335) into a 5 cap SoA array; *n = body count.  cap < n:
 * BH_E_CAPACITY with *n set (size query with soa = NULL, cap = 0). */
int bh_shim_get(bh_engine *e, double *soa, int64_t cap, int64_t *n);

/* Native.get's source: the engine's pinned caller-order mirror (bh_map_bodies) -- soa[0..5)
 * point at x, y, vx, vy, m of *n bodies, valid until the next call that changes the bodies. */
int bh_shim_map(bh_engine *e, const double *soa[5], int64_t *n);

/* Native.quads: getTreeForDebug().visitQuads{} (BHA:265-274, 329-332) as 3 cap interleaved
 * doubles; *nq = quad count.  cap < nq: BH_E_CAPACITY with *nq set (size query). */
int bh_shim_quads(bh_engine *e, double *q, int64_t cap, int64_t *nq);

/* Native.lastRemoved: the list indices the merge rule removed in the last step call (BHA:519),
 * as int32 (Kotlin IntArray).  cap < count: BH_E_CAPACITY with *count set (size query). */
int bh_shim_last_removed(const bh_engine *e, int32_t *idx, int64_t cap, int64_t *count);

#ifdef __cplusplus
}
#endif
#endif /* BH_SHIM_H */
