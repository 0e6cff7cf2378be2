/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A CPU restatement, line by line, of the reference Barnes–Hut hot path
 * (/root/reference/src/main/kotlin/BarnesHutAlg.kt, "BHA" below; Config.kt "CFG").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker / the timed "reference-algorithm CPU path".  The product
 * (barnes-hut-n-body_amd/, libbh_engine.so) never links or calls anything here.
 *
 * PARITY UNPINNED: the reference is Kotlin/JVM with no tests, no fixtures and no
 * golden vectors, and no JVM exists in this image, so this
 * restatement cannot be checked against the reference's own outputs.  It is pinned
 * instead by (1) an independent pure-Python restatement (oracle/py_oracle.py) that
 * must agree bit for bit, (2) hand-computed known-answer tests, (3) physics
 * invariants (theta = 0 == direct sum), all under tests/.
 *
 * Numerics: JVM >= 17 floating point is strict IEEE-754 binary64 (JEP 306) with no
 * fused multiply-add, so this file is compiled with -ffp-contract=off and without
 * fast-math; every expression keeps the reference's left-to-right association.
 *
 * Structure mirrors the reference: a pointer quadtree (here: indices into a node
 * pool) with <= 1 body per leaf, built serially in body-index order; recursive
 * centre-of-mass; recursive per-body traversal; worker threads pulling body indices
 * from one atomic counter (BHA:374-395); kick-drift-kick (BHA:405-439); the merge
 * rule (BHA:463-532).
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "bh_oracle.h"

/* ---- Body (BHA:21-25) and Quad (BHA:53-82) ---------------------------------- */
typedef struct { double x, y, vx, vy, m; } Body;
typedef struct { double cx, cy, h; } Quad;

/* BHA:61-62 — half-open [cx-h, cx+h) x [cy-h, cy+h), bounds evaluated as written. */
static int quad_contains(const Quad *q, const Body *b) {
    return b->x >= q->cx - q->h && b->x < q->cx + q->h &&
           b->y >= q->cy - q->h && b->y < q->cy + q->h;
}

/* BHA:73-81 — child 0=(-,-), 1=(+,-), 2=(-,+), 3=(+,+); hh = h / 2.0. */
static Quad quad_child(const Quad *q, int which) {
    double hh = q->h / 2.0;
    Quad c;
    switch (which) {
    case 0: c.cx = q->cx - hh; c.cy = q->cy - hh; break;
    case 1: c.cx = q->cx + hh; c.cy = q->cy - hh; break;
    case 2: c.cx = q->cx - hh; c.cy = q->cy + hh; break;
    default: c.cx = q->cx + hh; c.cy = q->cy + hh; break;
    }
    c.h = hh;
    return c;
}

/* ---- BHTree (BHA:95-275) ------------------------------------------------------
 * Node pool: a node's 4 children are allocated consecutively by subdivide().
 * `body` is the body index (identity, BHA:219 `single === b`) or -1;
 * `child` is the index of child 0, or -1 for a leaf (BHA:100,112).               */
typedef struct {
    Quad q;
    int64_t body;
    int64_t child;
    double mass, comX, comY; /* BHA:103-109 */
} Node;

typedef struct {
    Node *nodes;
    int64_t n, cap;
    Body *bodies;
} Tree;

static int64_t tree_alloc4(Tree *t, const Quad *parent) {
    if (t->n + 4 > t->cap) {
        int64_t nc = t->cap ? t->cap * 2 : 1024;
        while (nc < t->n + 4) nc *= 2;
        t->nodes = (Node *)realloc(t->nodes, (size_t)nc * sizeof(Node));
        t->cap = nc;
    }
    int64_t first = t->n;
    for (int i = 0; i < 4; ++i) { /* BHA:160-165 */
        Node *c = &t->nodes[first + i];
        c->q = quad_child(parent, i);
        c->body = -1;
        c->child = -1;
        c->mass = 0.0; c->comX = 0.0; c->comY = 0.0;
    }
    t->n += 4;
    return first;
}

static void tree_insert(Tree *t, int64_t node, int64_t bi);

/* BHA:145-156 — deterministic jitter below h < 1e-3, then child by ix + iy. */
static void insert_into_child(Tree *t, int64_t node, int64_t bi) {
    Body *b = &t->bodies[bi];
    Quad q = t->nodes[node].q;
    if (q.h < 1e-3) {
        const double eps = 1e-3;
        uint64_t bx, by;
        memcpy(&bx, &b->x, 8);
        b->x += ((bx & 1ULL) == 0ULL) ? +eps : -eps;
        memcpy(&by, &b->y, 8);
        b->y += ((by & 1ULL) == 0ULL) ? -eps : +eps;
    }
    int ix = (b->x < q.cx) ? 0 : 1;
    int iy = (b->y < q.cy) ? 0 : 2;
    tree_insert(t, t->nodes[node].child + ix + iy, bi);
}

/* BHA:125-137 */
static void tree_insert(Tree *t, int64_t node, int64_t bi) {
    if (!quad_contains(&t->nodes[node].q, &t->bodies[bi])) return; /* BHA:126 dropped */
    if (t->nodes[node].body < 0 && t->nodes[node].child < 0) {      /* BHA:127-129 */
        t->nodes[node].body = bi;
        return;
    }
    if (t->nodes[node].child < 0) { /* BHA:131 subdivide (BHA:159-166) */
        Quad q = t->nodes[node].q;
        int64_t first = tree_alloc4(t, &q);
        t->nodes[node].child = first;
    }
    int64_t existing = t->nodes[node].body; /* BHA:132-135 */
    if (existing >= 0) {
        t->nodes[node].body = -1;
        insert_into_child(t, node, existing);
    }
    insert_into_child(t, node, bi); /* BHA:136 */
}

/* BHA:173-202 — post-order, children 0..3 in order, skipping mass <= 0. */
static void compute_mass(Tree *t, int64_t node) {
    Node *nd = &t->nodes[node];
    if (nd->child < 0) {
        if (nd->body >= 0) {
            const Body *b = &t->bodies[nd->body];
            nd->mass = b->m; nd->comX = b->x; nd->comY = b->y;
        } else {
            nd->mass = 0.0; nd->comX = nd->q.cx; nd->comY = nd->q.cy;
        }
        return;
    }
    double mSum = 0.0, cx = 0.0, cy = 0.0;
    int64_t ch = nd->child;
    for (int i = 0; i < 4; ++i) {
        compute_mass(t, ch + i);
        const Node *c = &t->nodes[ch + i];
        if (c->mass > 0.0) {
            mSum += c->mass;
            cx += c->comX * c->mass;
            cy += c->comY * c->mass;
        }
    }
    nd = &t->nodes[node];
    nd->mass = mSum;
    if (mSum > 0.0) {
        nd->comX = cx / mSum;
        nd->comY = cy / mSum;
    } else {
        nd->comX = nd->q.cx;
        nd->comY = nd->q.cy;
    }
}

typedef struct {
    double G, soft2, theta2;
} ForceCtx;

/* BHA:250-259 — ((G*b.m)*m)*invR2 ; fx += (f*dx)*invR. */
static inline void point_force_acc(const ForceCtx *c, const Body *b, double px, double py, double m,
                                   double *fx, double *fy) {
    double dx = px - b->x;
    double dy = py - b->y;
    double r2 = dx * dx + dy * dy + c->soft2;
    double invR = 1.0 / sqrt(r2);
    double invR2 = 1.0 / r2;
    double f = c->G * b->m * m * invR2;
    *fx += f * dx * invR;
    *fy += f * dy * invR;
}

/* BHA:215-239 — recursive DFS; `visits` counts calls that pass the mass == 0 test. */
static void accumulate_force(const Tree *t, const ForceCtx *c, int64_t node, int64_t bi,
                             double *fx, double *fy, int64_t *visits) {
    const Node *nd = &t->nodes[node];
    if (nd->mass == 0.0) return; /* BHA:216 */
    ++*visits;
    const Body *b = &t->bodies[bi];
    if (nd->child < 0) { /* BHA:217-222 */
        if (nd->body < 0 || nd->body == bi) return;
        point_force_acc(c, b, nd->comX, nd->comY, nd->mass, fx, fy);
        return;
    }
    double dx = nd->comX - b->x; /* BHA:223-226 */
    double dy = nd->comY - b->y;
    double dist2 = dx * dx + dy * dy + c->soft2;
    double hh = nd->q.h * 2.0;
    double s2 = hh * hh;
    if (s2 < c->theta2 * dist2) { /* BHA:228-230 */
        point_force_acc(c, b, nd->comX, nd->comY, nd->mass, fx, fy);
    } else { /* BHA:233-237 */
        int64_t ch = nd->child;
        accumulate_force(t, c, ch + 0, bi, fx, fy, visits);
        accumulate_force(t, c, ch + 1, bi, fx, fy, visits);
        accumulate_force(t, c, ch + 2, bi, fx, fy, visits);
        accumulate_force(t, c, ch + 3, bi, fx, fy, visits);
    }
}

/* ---- PhysicsEngine (BHA:287-532) ------------------------------------------- */
struct oracle_engine {
    oracle_params p;
    Body *bodies;
    int64_t n, cap;
    double *ax, *ay; /* BHA:298-301 */
    int64_t acc_cap;
    int64_t *visits; /* per-body visit counts of the last evaluation */
    Tree tree;       /* last built tree (BHA:304 lastTree) */
    int tree_valid;
    int threads;
    double t_build, t_walk; /* seconds of the last oracle_accel's build and walk (bench.py) */
};

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* BHA:359-366 — root Quad(W/2, H/2, max(W,H)/2 + 2); insert in list order. */
static void build_tree(oracle_engine *e) {
    Tree *t = &e->tree;
    t->n = 0;
    t->bodies = e->bodies;
    if (t->cap < 1) {
        t->cap = 1024;
        t->nodes = (Node *)realloc(t->nodes, (size_t)t->cap * sizeof(Node));
    }
    int W = e->p.width_px, H = e->p.height_px;
    double half = (double)(W > H ? W : H) / 2.0 + 2.0;
    Node *root = &t->nodes[0];
    root->q.cx = (double)W / 2.0;
    root->q.cy = (double)H / 2.0;
    root->q.h = half;
    root->body = -1; root->child = -1;
    root->mass = 0.0; root->comX = 0.0; root->comY = 0.0;
    t->n = 1;
    for (int64_t i = 0; i < e->n; ++i) tree_insert(t, 0, i);
    compute_mass(t, 0);
    e->tree_valid = 1;
}

typedef struct {
    oracle_engine *e;
    const int64_t *subset; /* NULL: all bodies */
    int64_t count;
    atomic_long next;
    ForceCtx ctx;
} AccJob;

static void *acc_worker(void *arg) {
    AccJob *j = (AccJob *)arg;
    oracle_engine *e = j->e;
    for (;;) { /* BHA:384-392 — one body per grab */
        long k = atomic_fetch_add(&j->next, 1);
        if (k >= j->count) break;
        int64_t i = j->subset ? j->subset[k] : k;
        double fx = 0.0, fy = 0.0;
        int64_t v = 0;
        accumulate_force(&e->tree, &j->ctx, 0, i, &fx, &fy, &v);
        const Body *b = &e->bodies[i];
        e->ax[i] = fx / b->m;
        e->ay[i] = fy / b->m;
        e->visits[i] = v;
    }
    return NULL;
}

/* BHA:374-395 — workers = min(cores, max(n,1)); theta2 from the live theta. */
static void compute_accelerations(oracle_engine *e, const int64_t *subset, int64_t count) {
    AccJob j;
    j.e = e;
    j.subset = subset;
    j.count = count;
    atomic_init(&j.next, 0);
    j.ctx.G = e->p.G;
    j.ctx.soft2 = e->p.soft2;
    j.ctx.theta2 = e->p.theta * e->p.theta;
    int64_t nw = e->threads;
    if (nw > (count > 1 ? count : 1)) nw = count > 1 ? count : 1;
    if (nw <= 1) {
        acc_worker(&j);
        return;
    }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nw);
    for (int64_t w = 0; w < nw; ++w) pthread_create(&th[w], NULL, acc_worker, &j);
    for (int64_t w = 0; w < nw; ++w) pthread_join(th[w], NULL);
    free(th);
}

static void ensure_acc(oracle_engine *e) {
    if (e->acc_cap < e->n) {
        e->acc_cap = e->n;
        e->ax = (double *)realloc(e->ax, sizeof(double) * (size_t)(e->n ? e->n : 1));
        e->ay = (double *)realloc(e->ay, sizeof(double) * (size_t)(e->n ? e->n : 1));
        e->visits = (int64_t *)realloc(e->visits, sizeof(int64_t) * (size_t)(e->n ? e->n : 1));
    }
}

/* BHA:463-532 — merge rule.  The reference scans [0,n) in parallel chunks and
 * concatenates victims in chunk order, then sorts them descending: the victim list is
 * therefore exactly {j != i : d2 < minD2} in descending order, which a serial scan
 * reproduces.  Mass is added in descending j, then i = indexOf(bi), then i++.        */
static void merge_close_bodies(oracle_engine *e) {
    double minDist = e->p.merge_min_dist;
    if (minDist <= 0.0 || e->n <= 1) return;
    double minD2 = minDist * minDist;
    int64_t *victims = NULL;
    int64_t vcap = 0;
    int64_t i = 0;
    while (i < e->n) {
        if (e->bodies[i].m > e->p.merge_max_mass) {
            int64_t n = e->n;
            if (n > 1) {
                int64_t nv = 0;
                double bix = e->bodies[i].x, biy = e->bodies[i].y;
                for (int64_t j = 0; j < n; ++j) {
                    if (j == i) continue;
                    double dx = e->bodies[j].x - bix;
                    double dy = e->bodies[j].y - biy;
                    if (dx * dx + dy * dy < minD2) {
                        if (nv == vcap) {
                            vcap = vcap ? vcap * 2 : 64;
                            victims = (int64_t *)realloc(victims, sizeof(int64_t) * (size_t)vcap);
                        }
                        victims[nv++] = j;
                    }
                }
                if (nv > 0) {
                    /* victims ascending by construction; remove in descending order */
                    int64_t bi_idx = i;
                    for (int64_t v = nv - 1; v >= 0; --v) {
                        int64_t j = victims[v];
                        /* BHA:518 bi.m += bj.m; BHA:519 removeAt(j) */
                        e->bodies[bi_idx].m += e->bodies[j].m;
                        memmove(&e->bodies[j], &e->bodies[j + 1], sizeof(Body) * (size_t)(e->n - j - 1));
                        e->n -= 1;
                        if (j < bi_idx) bi_idx -= 1; /* indexOf(bi) */
                    }
                    i = bi_idx; /* BHA:522-523 */
                    e->tree_valid = 0; /* BHA:526 lastTree = null */
                }
            }
        }
        ++i;
    }
    free(victims);
}

/* ---- exported API --------------------------------------------------------- */

oracle_engine *oracle_create(const oracle_params *p, int64_t n, const double *x, const double *y,
                             const double *vx, const double *vy, const double *m) {
    oracle_engine *e = (oracle_engine *)calloc(1, sizeof(oracle_engine));
    e->p = *p;
    e->threads = p->threads > 0 ? p->threads : (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (e->threads < 1) e->threads = 1;
    oracle_reset_bodies(e, n, x, y, vx, vy, m);
    return e;
}

void oracle_set_params(oracle_engine *e, const oracle_params *p) {
    e->p = *p;
    e->threads = p->threads > 0 ? p->threads : (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (e->threads < 1) e->threads = 1;
}

/* BHA:342-349 */
void oracle_reset_bodies(oracle_engine *e, int64_t n, const double *x, const double *y,
                         const double *vx, const double *vy, const double *m) {
    if (n > e->cap) {
        e->bodies = (Body *)realloc(e->bodies, sizeof(Body) * (size_t)n);
        e->cap = n;
    }
    for (int64_t i = 0; i < n; ++i) {
        e->bodies[i].x = x[i]; e->bodies[i].y = y[i];
        e->bodies[i].vx = vx[i]; e->bodies[i].vy = vy[i];
        e->bodies[i].m = m[i];
    }
    e->n = n;
    ensure_acc(e);
    e->tree_valid = 0;
}

int64_t oracle_num_bodies(const oracle_engine *e) { return e->n; }

void oracle_get_bodies(const oracle_engine *e, double *x, double *y, double *vx, double *vy, double *m) {
    for (int64_t i = 0; i < e->n; ++i) {
        x[i] = e->bodies[i].x; y[i] = e->bodies[i].y;
        vx[i] = e->bodies[i].vx; vy[i] = e->bodies[i].vy;
        m[i] = e->bodies[i].m;
    }
}

/* BHA:405-439 — one step = build, a(t), kick, drift, build, a(t+dt), kick, merge. */
int oracle_step(oracle_engine *e, int k) {
    for (int s = 0; s < k; ++s) {
        int64_t n = e->n;
        ensure_acc(e);
        build_tree(e);
        compute_accelerations(e, NULL, n);
        double dtHalf = e->p.dt * 0.5; /* BHA:412 */
        for (int64_t i = 0; i < n; ++i) {
            e->bodies[i].vx += e->ax[i] * dtHalf;
            e->bodies[i].vy += e->ay[i] * dtHalf;
        }
        for (int64_t i = 0; i < n; ++i) { /* BHA:419-422 */
            e->bodies[i].x += e->bodies[i].vx * e->p.dt;
            e->bodies[i].y += e->bodies[i].vy * e->p.dt;
        }
        build_tree(e);
        compute_accelerations(e, NULL, n);
        for (int64_t i = 0; i < n; ++i) {
            e->bodies[i].vx += e->ax[i] * dtHalf;
            e->bodies[i].vy += e->ay[i] * dtHalf;
        }
        merge_close_bodies(e); /* BHA:438 */
    }
    return 0;
}

/* buildTree + computeAccelerations on the current state (mutates positions through
 * the jitter exactly like the reference's build).  subset == NULL: every body.   */
int oracle_accel(oracle_engine *e, int64_t count, const int64_t *subset, double *ax, double *ay,
                 int64_t *visits) {
    ensure_acc(e);
    const double t0 = now_s();
    build_tree(e);
    const double t1 = now_s();
    if (!subset) count = e->n;
    compute_accelerations(e, subset, count);
    e->t_build = t1 - t0;
    e->t_walk = now_s() - t1;
    for (int64_t k = 0; k < count; ++k) {
        int64_t i = subset ? subset[k] : k;
        if (ax) ax[k] = e->ax[i];
        if (ay) ay[k] = e->ay[i];
        if (visits) visits[k] = e->visits[i];
    }
    return 0;
}

/* Timing of the last oracle_accel (the CPU baseline's bounded sample, bench.py). */
void oracle_last_timing(const oracle_engine *e, double *build_s, double *walk_s) {
    *build_s = e->t_build;
    *walk_s = e->t_walk;
}

/* BHA:265-274 visitQuads on getTreeForDebug() (BHA:329-332). */
static void visit_quads(const Tree *t, int64_t node, double *cx, double *cy, double *h, int64_t cap,
                        int64_t *k) {
    const Node *nd = &t->nodes[node];
    if (*k < cap) {
        cx[*k] = nd->q.cx; cy[*k] = nd->q.cy; h[*k] = nd->q.h;
    }
    ++*k;
    if (nd->child >= 0)
        for (int i = 0; i < 4; ++i) visit_quads(t, nd->child + i, cx, cy, h, cap, k);
}

int64_t oracle_quads(oracle_engine *e, double *cx, double *cy, double *h, int64_t cap) {
    if (!e->tree_valid) build_tree(e);
    int64_t k = 0;
    visit_quads(&e->tree, 0, cx, cy, h, cap, &k);
    return k;
}

/* Tree statistics for the roofline byte model. */
void oracle_tree_stats(oracle_engine *e, int64_t *n_nodes, int64_t *n_nonempty) {
    if (!e->tree_valid) build_tree(e);
    int64_t ne = 0;
    for (int64_t i = 0; i < e->tree.n; ++i) ne += e->tree.nodes[i].mass != 0.0;
    *n_nodes = e->tree.n;
    *n_nonempty = ne;
}

/* Analysis helper (not part of the reference): the GPU traversal walks one pre-order cursor per
 * wavefront over the UNION of its lanes' visit sets.  For groups of `group` consecutive bodies
 * of `order`, count that union (nodes reached by at least one lane: the GPU's wave iterations)
 * and the lanes' own visits; their ratio is the lane efficiency of that body ordering. */
static int64_t g_force_iters, g_contribs; /* analysis counters (single-threaded helper) */

/* Deferred-force model (analysis only): every lane queues its contributions (FIFO, depth
 * g_sim_q); a "flush" runs the force math once for every lane with a non-empty queue.  A flush
 * happens when some queue is full, or when at least g_sim_t lanes have work; the queues are
 * drained at the end of the walk.  g_sim_flushes counts flushes (force-block executions). */
static int g_sim_q, g_sim_t;
static int g_sim_cnt[64];
static int64_t g_sim_flushes;

/* Pair-merge model (analysis helper): a wave defers its point-force block by one iteration
 * and runs the next iteration's block together with it when the two lane sets are
 * disjoint (each lane still adds its terms in order).  Counts blocks under that rule. */
static uint64_t g_pm_pend;
static int64_t g_pm_blocks, g_pm_merges;

static void pm_push(uint64_t contrib) {
    if (g_pm_pend) {
        ++g_pm_blocks;
        if (contrib && !(contrib & g_pm_pend)) {
            ++g_pm_merges;
            g_pm_pend = 0;
            return;
        }
        g_pm_pend = 0;
    }
    g_pm_pend = contrib;
}

static void pm_drain(void) {
    if (g_pm_pend) ++g_pm_blocks;
    g_pm_pend = 0;
}

void oracle_pairmerge_stats(int64_t *blocks, int64_t *merges) {
    *blocks = g_pm_blocks;
    *merges = g_pm_merges;
}

static void sim_push(uint64_t contrib) {
    pm_push(contrib);
    if (!g_sim_q) return;
    int full = 0, nonempty = 0;
    for (int l = 0; l < 64; ++l) {
        if (contrib >> l & 1) ++g_sim_cnt[l];
        full |= g_sim_cnt[l] >= g_sim_q;
        nonempty += g_sim_cnt[l] > 0;
    }
    if (full || nonempty >= g_sim_t) {
        ++g_sim_flushes;
        for (int l = 0; l < 64; ++l)
            if (g_sim_cnt[l] > 0) --g_sim_cnt[l];
    }
}

static void sim_drain(void) {
    int mx = 0;
    for (int l = 0; l < 64; ++l) {
        if (g_sim_cnt[l] > mx) mx = g_sim_cnt[l];
        g_sim_cnt[l] = 0;
    }
    g_sim_flushes += mx;
}

/* Resume-stack model (analysis helper): a node some active lanes accept while others open it
 * ("mixed") parks the accepting lanes until the cursor leaves its subtree -- a stack entry of
 * (next, lane mask).  Counts the pushes and the largest stack depth per group (histogram). */
static int g_mix_sd, g_mix_max;
static int64_t g_mix_pushes, g_mix_hist[65];

void oracle_mixstack_stats(int64_t *pushes, int64_t *hist65) {
    *pushes = g_mix_pushes;
    for (int k = 0; k < 65; ++k) hist65[k] = g_mix_hist[k];
}

static int64_t union_walk(const Tree *t, const ForceCtx *c, int64_t node, const int64_t *bis,
                          uint64_t mask, int64_t *lane_visits) {
    const Node *nd = &t->nodes[node];
    if (nd->mass == 0.0 || !mask) return 0; /* BHA:216 */
    *lane_visits += __builtin_popcountll(mask);
    if (nd->child < 0) {
        uint64_t contrib = 0;
        for (uint64_t m = mask; m; m &= m - 1) {
            const int l = __builtin_ctzll(m);
            if (nd->body >= 0 && nd->body != bis[l]) contrib |= 1ull << l;
        }
        g_force_iters += contrib != 0;
        g_contribs += __builtin_popcountll(contrib);
        sim_push(contrib);
        return 1;
    }
    uint64_t open = 0;
    for (uint64_t m = mask; m; m &= m - 1) {
        const int l = __builtin_ctzll(m);
        const Body *b = &t->bodies[bis[l]];
        const double dx = nd->comX - b->x, dy = nd->comY - b->y;
        const double dist2 = dx * dx + dy * dy + c->soft2;
        const double hh = nd->q.h * 2.0, s2 = hh * hh;
        if (!(s2 < c->theta2 * dist2)) open |= 1ull << l;
    }
    const uint64_t acc = mask & ~open;
    g_force_iters += acc != 0;
    g_contribs += __builtin_popcountll(acc);
    sim_push(acc);
    int64_t it = 1;
    const int mixed = acc && open;
    if (mixed) {
        ++g_mix_pushes;
        if (++g_mix_sd > g_mix_max) g_mix_max = g_mix_sd;
    }
    if (open)
        for (int k = 0; k < 4; ++k) it += union_walk(t, c, nd->child + k, bis, open, lane_visits);
    g_mix_sd -= mixed;
    return it;
}

void oracle_union_force_stats(int64_t *force_iters, int64_t *contribs) {
    *force_iters = g_force_iters;
    *contribs = g_contribs;
}

/* Configure the deferred-force model for the next oracle_group_union (q = 0: off). */
void oracle_deferred_model(int q, int t) {
    g_sim_q = q;
    g_sim_t = t;
    for (int l = 0; l < 64; ++l) g_sim_cnt[l] = 0;
    g_sim_flushes = 0;
}

int64_t oracle_deferred_flushes(void) { return g_sim_flushes; }

int64_t oracle_group_union(oracle_engine *e, const int64_t *order, int64_t count, int group,
                           int64_t *lane_visits, int64_t *per_group) {
    if (group < 1 || group > 64) return -1;
    if (!e->tree_valid) {
        build_tree(e);
        e->tree_valid = 1;
    }
    ForceCtx c = {e->p.G, e->p.soft2, e->p.theta * e->p.theta};
    int64_t iters = 0, lv = 0;
    g_force_iters = g_contribs = 0;
    g_pm_blocks = g_pm_merges = 0;
    g_pm_pend = 0;
    g_mix_pushes = 0;
    for (int k = 0; k < 65; ++k) g_mix_hist[k] = 0;
    for (int64_t g0 = 0; g0 < count; g0 += group) {
        g_mix_sd = g_mix_max = 0;
        const int nb = (int)((count - g0) < group ? (count - g0) : group);
        const uint64_t mask = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        const int64_t it = union_walk(&e->tree, &c, 0, order + g0, mask, &lv);
        pm_drain();
        g_mix_hist[g_mix_max < 64 ? g_mix_max : 64]++;
        if (g_sim_q) sim_drain();
        if (per_group) per_group[g0 / group] = it;
        iters += it;
    }
    if (lane_visits) *lane_visits = lv;
    return iters;
}

void oracle_destroy(oracle_engine *e) {
    if (!e) return;
    free(e->bodies);
    free(e->ax); free(e->ay); free(e->visits);
    free(e->tree.nodes);
    free(e);
}
