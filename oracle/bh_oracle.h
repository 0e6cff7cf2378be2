/* ORACLE — test infrastructure only (see bh_oracle.c header).  PARITY UNPINNED. */
#ifndef BH_ORACLE_H
#define BH_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Config.kt fields read by the hot path (CFG:5,8,11,14,20,23) + merge knobs (BHA:315,321). */
typedef struct {
    double G;              /* CFG:11 */
    double dt;             /* CFG:14 */
    double theta;          /* CFG:23 */
    double soft2;          /* CFG:20 */
    int32_t width_px;      /* CFG:5  */
    int32_t height_px;     /* CFG:8  */
    double merge_max_mass; /* BHA:315 */
    double merge_min_dist; /* BHA:321 */
    int32_t threads;       /* workers (0 = all host cores), BHA:292,377 */
    int32_t _pad;
} oracle_params;

typedef struct oracle_engine oracle_engine;

oracle_engine *oracle_create(const oracle_params *p, int64_t n, const double *x, const double *y,
                             const double *vx, const double *vy, const double *m);
void oracle_set_params(oracle_engine *e, const oracle_params *p);
void oracle_reset_bodies(oracle_engine *e, int64_t n, const double *x, const double *y,
                         const double *vx, const double *vy, const double *m);
int64_t oracle_num_bodies(const oracle_engine *e);
void oracle_get_bodies(const oracle_engine *e, double *x, double *y, double *vx, double *vy, double *m);
int oracle_step(oracle_engine *e, int k);
int oracle_accel(oracle_engine *e, int64_t count, const int64_t *subset, double *ax, double *ay,
                 int64_t *visits);
int64_t oracle_quads(oracle_engine *e, double *cx, double *cy, double *h, int64_t cap);
/* seconds spent by the last oracle_accel in the serial tree build and in the walk */
void oracle_last_timing(const oracle_engine *e, double *build_s, double *walk_s);
void oracle_tree_stats(oracle_engine *e, int64_t *n_nodes, int64_t *n_nonempty);
/* analysis: wave-union iterations of groups of `group` consecutive bodies of `order` */
int64_t oracle_group_union(oracle_engine *e, const int64_t *order, int64_t count, int group,
                           int64_t *lane_visits, int64_t *per_group);
/* of the last oracle_group_union: iterations with >= 1 contributing lane, contributions */
void oracle_union_force_stats(int64_t *force_iters, int64_t *contribs);
/* analysis: per-lane deferred-force queues of depth q, flushed when one is full or >= t lanes
 * have work (q = 0: off); flush count of the next oracle_group_union */
void oracle_deferred_model(int q, int t);
int64_t oracle_deferred_flushes(void);
void oracle_destroy(oracle_engine *e);

#ifdef __cplusplus
}
#endif
#endif
