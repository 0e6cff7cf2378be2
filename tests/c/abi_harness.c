/*
 * C-side replay of the Kotlin drop-in through its real JNI glue --
 * TEST INFRASTRUCTURE (links the oracle as the checker).
 *
 * The Kotlin shim cannot be compiled here (no JDK), so this harness performs exactly the calls
 * the Kotlin class makes, into the committed glue (barnes-hut-n-body_amd/jni/bh_jni.c + its
 * bh_shim.c helpers, compiled against tests/c/jni_stub/jni.h and run with the fake JVM of
 * fake_jvm.c): Native.create / setParams / reset / step / get / quads / lastRemoved, with the
 * shim's own logic (shadow copy, upload only when the caller's list changed, pull(afterStep)
 * applying lastRemoved once), driven by the frame sequence of NBodyPanel (PNL:103 ctor, :291 step,
 * :333-340 getTreeForDebug().visitQuads, :247-260 live Config edits, :262/:285 resetBodies,
 * :228-234 getBodies() + new disk).  After every frame the caller's list must equal the reference
 * restatement's list word for word, and every surviving light body must still be the same Body
 * object (its unique start mass).
 *
 * Exit status 0 = pass; the last line says what was checked.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "bh_engine.h"
#include "bh_oracle.h"
#include "fake_jvm.h"

/* ---- Config (CFG:5-23), read live ---------------------------------------------------- */
static double cfg_G = 80.0, cfg_DT = 0.005, cfg_theta = 0.5, cfg_SOFT2 = 1.0;
static int cfg_W = 2400, cfg_H = 800;

/* ---- the caller's MutableList<Body> (BHA:21-25): an ArrayList of references to Body
 * objects, as the JVM holds it (the objects allocated together, as a TLAB places them); `id`
 * names the object for the identity checks ------------------------------------------------- */
typedef struct {
    double x, y, vx, vy, m;
    long id;
} Body;
typedef struct {
    Body **b;
    long n, cap;
} List;

static double *start_mass; /* by id */
static long next_id;
static long jni_calls;

static void fail(const char *what, long frame) {
    fprintf(stderr, "abi_harness: FAIL at frame %ld: %s\n", frame, what);
    exit(1);
}

/* ---- the Kotlin shim, over the JNI natives -------------------------- */
typedef struct {
    jlong h; /* Native.create's handle */
    List *bodies;
    jdoubleArray shadow; /* the shim's reusable upload DoubleArray (grown only) */
    jlongArray info;     /* Native.map's [n, stride] */
    const double *mir;   /* the engine's pinned mirror, read in place (Native.map) */
    long mir_stride;
    long shadow_n;       /* bodies in the mapped mirror (-1: none) */
    const jint *rem;     /* lastRemoved, ascending, while a removal pass runs */
    long nrem;
    Body **spare;        /* the survivors' target list (grown only; swapped with bodies->b) */
    long spare_cap;
    double mergeMaxMass, mergeMinDist; /* BHA:315,321 */
    jlongArray info3;      /* Native.positions' [n, stride, n before] */
    const int32_t *surv;   /* Native.survivors: survivor j's list index before the step */
} Shim;

static JNIEnv *env;

static void jni_check(const char *call) { /* a RuntimeException thrown by the glue */
    ++jni_calls;
    const char *exc = fake_jvm_take_exception();
    if (exc) {
        fprintf(stderr, "abi_harness: Native.%s threw: %s\n", call, exc);
        exit(1);
    }
}

static long step_end_errors_replaced; /* stepEnd errors of speculative steps an upload replaced */
static void jni_clear(void) { /* a call whose exception the shim discards (PhysicsEngine.kt) */
    ++jni_calls;
    if (fake_jvm_take_exception()) ++step_end_errors_replaced;
}

static void shim_params(Shim *s) {
    Java_Native_setParams(env, NULL, s->h, cfg_G, cfg_DT, cfg_theta, cfg_SOFT2, cfg_W, cfg_H,
                          s->mergeMaxMass, s->mergeMinDist);
    jni_check("setParams");
}

static void soa_of(const List *l, double *a) {
    long n = l->n;
    for (long i = 0; i < n; ++i) {
        a[i] = l->b[i]->x;
        a[n + i] = l->b[i]->y;
        a[2 * n + i] = l->b[i]->vx;
        a[3 * n + i] = l->b[i]->vy;
        a[4 * n + i] = l->b[i]->m;
    }
}

static long shadow_allocs; /* DoubleArray allocations of the shim after its constructor */

static void shim_grow(Shim *s, long n) { /* `shadow = DoubleArray(5 n)` when too small */
    if (s->shadow && fake_jvm_length(s->shadow) >= 5 * n) return;
    if (s->shadow) fake_jvm_free(s->shadow);
    s->shadow = fake_jvm_double_array((jsize)(5 * n), NULL);
    ++shadow_allocs;
}

/* map(): the engine's pinned mirror as a direct buffer (Native.map), read in place; returns n */
static long shim_map(Shim *s) {
    jobject buf = Java_Native_map(env, NULL, s->h, s->info);
    jni_check("map");
    const jlong *in = fake_jvm_longs(s->info);
    jlong cap = 0;
    s->mir = (const double *)fake_jvm_direct_address(buf, &cap);
    s->mir_stride = (long)in[1];
    s->shadow_n = (long)in[0];
    if (cap != 5 * (jlong)sizeof(double) * in[1]) fail("map: buffer capacity is not 5 planes", -1);
    fake_jvm_free(buf); /* (the JVM's buffer object; the memory is the engine's) */
    return s->shadow_n;
}

static void shim_push(Shim *s) {
    long n = s->bodies->n;
    shim_grow(s, n);
    soa_of(s->bodies, fake_jvm_doubles(s->shadow));
    Java_Native_reset(env, NULL, s->h, (jint)n, s->shadow);
    jni_check("reset");
    shim_map(s); /* the engine's copy, as uploaded */
}

/* The shim's O(N) passes in chunks over worker threads, as PhysicsEngine.kt runs them on
 * Dispatchers.Default (the reference's own fan-out, BHA:374-395): a pool of persistent workers
 * (started once, as the JVM's shared pool is), 4 chunks per worker taken in turn (a worker that
 * shares its core with a spinning thread takes fewer); short lists stay serial. */
static int shim_threads = 8;
static long shim_par_min = 65536; /* BH_SHIM_PAR_MIN: shorter lists stay serial */
static struct {
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    long gen;
    int started, pending;
    Shim *s;
    long n, chunk;
    int (*fn)(Shim *, long, long);
    atomic_long next;
    atomic_int any;
} pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0, 0,
        NULL, 0, 0, NULL, 0, 0};
static void pool_chunks(void) {
    for (;;) {
        const long c = atomic_fetch_add(&pool.next, 1);
        const long lo = c * pool.chunk;
        if (lo >= pool.n) return;
        const long hi = lo + pool.chunk < pool.n ? lo + pool.chunk : pool.n;
        if (pool.fn(pool.s, lo, hi)) atomic_store(&pool.any, 1);
    }
}
static void *pool_worker(void *arg) {
    (void)arg;
    long seen = 0;
    for (;;) {
        pthread_mutex_lock(&pool.mu);
        while (pool.gen == seen) pthread_cond_wait(&pool.go, &pool.mu);
        seen = pool.gen;
        pthread_mutex_unlock(&pool.mu);
        pool_chunks();
        pthread_mutex_lock(&pool.mu);
        if (--pool.pending == 0) pthread_cond_signal(&pool.done);
        pthread_mutex_unlock(&pool.mu);
    }
    return NULL;
}
static int par_any(Shim *s, long n, int (*fn)(Shim *, long, long)) { /* OR of fn over chunks */
    const int w = n < shim_par_min ? 1 : shim_threads;
    if (w <= 1) return fn(s, 0, n);
    if (!pool.started) {
        for (int k = 1; k < w; ++k) {
            pthread_t t;
            if (pthread_create(&t, NULL, pool_worker, NULL)) fail("pthread_create", -1);
            pthread_detach(t);
        }
        pool.started = w;
    }
    pthread_mutex_lock(&pool.mu);
    pool.s = s;
    pool.n = n;
    pool.fn = fn;
    pool.chunk = (n + 4 * (long)w - 1) / (4 * (long)w);
    atomic_store(&pool.next, 0);
    atomic_store(&pool.any, 0);
    pool.pending = pool.started - 1;
    ++pool.gen;
    pthread_cond_broadcast(&pool.go);
    pthread_mutex_unlock(&pool.mu);
    pool_chunks(); /* the caller's thread takes chunks too */
    pthread_mutex_lock(&pool.mu);
    while (pool.pending > 0) pthread_cond_wait(&pool.done, &pool.mu);
    pthread_mutex_unlock(&pool.mu);
    return atomic_load(&pool.any);
}

/* changed(): field by field against the mapped mirror, in place (toRawBits compares) */
static int changed_part(Shim *s, long lo, long hi) {
    const long st = s->mir_stride;
    const double *a = s->mir;
    for (long i = lo; i < hi; ++i) {
        const Body *b = s->bodies->b[i];
        if (memcmp(&b->x, &a[i], 8) || memcmp(&b->y, &a[st + i], 8) ||
            memcmp(&b->vx, &a[2 * st + i], 8) || memcmp(&b->vy, &a[3 * st + i], 8) ||
            memcmp(&b->m, &a[4 * st + i], 8))
            return 1;
    }
    return 0;
}
static int shim_changed(Shim *s) {
    long n = s->bodies->n;
    if (n != s->shadow_n) return 1;
    return par_any(s, n, changed_part);
}

static void swap_spare(Shim *s) { /* the spare list becomes the list, and the list the spare */
    Body **b = s->bodies->b;
    const long cap = s->bodies->cap;
    s->bodies->b = s->spare;
    s->bodies->cap = s->spare_cap;
    s->spare = b;
    s->spare_cap = cap;
}
static long removed_below(const Shim *s, long i) { /* lower_bound over lastRemoved */
    long lo = 0, hi = s->nrem;
    while (lo < hi) {
        long mid = (lo + hi) / 2;
        if (s->rem[mid] < i) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
static int compact_part(Shim *s, long lo, long hi) {
    long q = removed_below(s, lo), w = lo - q;
    for (long i = lo; i < hi; ++i) {
        if (q < s->nrem && s->rem[q] == i) {
            ++q;
            continue;
        }
        s->spare[w++] = s->bodies->b[i];
    }
    return 0;
}

/* pull(afterStep): removals are applied once, right after the step that made them */
static void shim_apply_removed(Shim *s) {
    {
        jintArray rem = Java_Native_lastRemoved(env, NULL, s->h);
        jni_check("lastRemoved");
        const jint *r = fake_jvm_ints(rem);
        const jsize nr = fake_jvm_length(rem);
        for (jsize k = 1; k < nr; ++k)
            if (r[k - 1] >= r[k]) fail("lastRemoved is not ascending", -1);
        if (nr <= 2) {
            for (jsize k = nr; k-- > 0;) { /* removeAt, descending (BHA:519) */
                long j = (long)r[k];
                memmove(&s->bodies->b[j], &s->bodies->b[j + 1],
                        sizeof(Body *) * (s->bodies->n - j - 1));
                s->bodies->n -= 1;
            }
        } else if (s->bodies->n < shim_par_min || shim_threads <= 1) {
            /* PhysicsEngine.kt: the same survivors in one pass, then one range removal */
            long w = r[0], q = 0;
            for (long i = r[0]; i < s->bodies->n; ++i) {
                if (q < nr && r[q] == i) {
                    ++q;
                    continue;
                }
                s->bodies->b[w++] = s->bodies->b[i];
            }
            s->bodies->n = w;
        } else { /* in chunks: survivors into the spare list, which becomes the list (the Kotlin
                  * shim copies the references back instead, the caller's ArrayList stays) */
            const long n = s->bodies->n;
            if (s->spare_cap < n) {
                free(s->spare);
                s->spare = (Body **)malloc(sizeof(Body *) * n);
                s->spare_cap = n;
            }
            s->rem = r;
            s->nrem = nr;
            (void)par_any(s, n, compact_part);
            swap_spare(s);
            s->bodies->n = n - nr;
        }
        fake_jvm_free(rem);
    }
}

static int unpack_part(Shim *s, long lo, long hi) {
    const double *a = s->mir;
    const long st = s->mir_stride;
    for (long i = lo; i < hi; ++i) { /* into the SAME Body objects (BHA:414-432) */
        Body *b = s->bodies->b[i];
        b->x = a[i];
        b->y = a[st + i];
        b->vx = a[2 * st + i];
        b->vy = a[3 * st + i];
        b->m = a[4 * st + i];
    }
    return 0;
}
static int unpack_xym_part(Shim *s, long lo, long hi) { /* the hand-off: x, y, m final */
    const double *a = s->mir;
    const long st = s->mir_stride;
    for (long i = lo; i < hi; ++i) {
        Body *b = s->bodies->b[i];
        b->x = a[i];
        b->y = a[st + i];
        b->m = a[4 * st + i];
    }
    return 0;
}
static int unpack_v_part(Shim *s, long lo, long hi) { /* after the step: vx, vy */
    const double *a = s->mir;
    const long st = s->mir_stride;
    for (long i = lo; i < hi; ++i) {
        Body *b = s->bodies->b[i];
        b->vx = a[2 * st + i];
        b->vy = a[3 * st + i];
    }
    return 0;
}
/* the removals from the survivors' list: survivor j is the body at list index surv[j] */
static int gather_part(Shim *s, long lo, long hi) {
    for (long j = lo; j < hi; ++j) s->spare[j] = s->bodies->b[s->surv[j]];
    return 0;
}
static void shim_keep_survivors(Shim *s, long n) {
    if (s->spare_cap < s->bodies->n) {
        free(s->spare);
        s->spare = (Body **)malloc(sizeof(Body *) * s->bodies->n);
        s->spare_cap = s->bodies->n;
    }
    (void)par_any(s, n, gather_part);
    swap_spare(s);
    s->bodies->n = n;
}
static void shim_unpack(Shim *s, long n) {
    if (n != s->bodies->n) {
        fprintf(stderr, "abi_harness: engine N %ld vs caller list %ld\n", n, s->bodies->n);
        exit(1);
    }
    (void)par_any(s, n, unpack_part);
}

static void shim_pull(Shim *s, int after_step) {
    if (after_step) shim_apply_removed(s);
    shim_unpack(s, shim_map(s));
}

static void shim_create(Shim *s, List *initial, jint device_mask) {
    memset(s, 0, sizeof(*s));
    s->mergeMaxMass = 4000.0;
    s->mergeMinDist = 8.0;
    s->shadow_n = -1;
    s->info = fake_jvm_long_array(2);
    s->info3 = fake_jvm_long_array(3);
    s->h = Java_Native_createMask(env, NULL, device_mask); /* (-Dbh.deviceMask) */
    if (fake_jvm_take_exception() || !s->h) {
        fprintf(stderr, "abi_harness: Native.create failed (no GPU?)\n");
        exit(1);
    }
    s->bodies = initial;
    shim_params(s);
    shim_push(s);
}

static void shim_reset(Shim *s, List *l) {
    s->bodies = l;
    shim_push(s);
}

static long shim_steps_uploaded;
static double now_ms(void);
/* step(): Native.stepBegin (the step runs on the engine's thread), the list compared against the
 * mapped mirror meanwhile (the step writes the other buffer); an edited list is uploaded and
 * stepped again instead.  Else Native.positions waits for the step's hand-off -- positions and
 * masses final, its merge rule done -- and the removals (Native.survivors) and the x, y, m unpack
 * run while its last traversal still does; after Native.stepEnd only vx, vy are unpacked.
 * t (nullable): params, compare, wait for the survivors, removals, unpack x/y/m, wait for the
 * end, map + unpack vx/vy, wait for the planes -- ms, accumulated. */
static void shim_frame(Shim *s, double *t) {
    double a = now_ms(), b;
#define LAP(q) do { b = now_ms(); if (t) t[q] += b - a; a = b; } while (0)
    shim_params(s);
    LAP(0);
    if (s->bodies->n != s->shadow_n) { /* bodies added or removed: upload first */
        shim_push(s);
        ++shim_steps_uploaded;
        Java_Native_step(env, NULL, s->h, 1);
        jni_check("step");
        shim_pull(s, 1);
        return;
    }
    Java_Native_stepBegin(env, NULL, s->h, 1);
    jni_check("stepBegin");
    const int diff = shim_changed(s);
    LAP(1);
    if (diff) { /* the upload replaces that step's result -- and an error it met (PhysicsEngine.kt) */
        Java_Native_stepEnd(env, NULL, s->h);
        jni_clear();
        shim_push(s);
        ++shim_steps_uploaded;
        Java_Native_step(env, NULL, s->h, 1);
        jni_check("step");
        shim_pull(s, 1);
        return;
    }
    { /* the survivors first (ahead of the planes' copy): the removals run while it lasts */
        jobject sb = Java_Native_survivors(env, NULL, s->h);
        jni_check("survivors");
        jlong scap = 0;
        s->surv = (const int32_t *)fake_jvm_direct_address(sb, &scap);
        fake_jvm_free(sb);
        const long ns = (long)(scap / (jlong)sizeof(int32_t));
        LAP(2);
        if (ns != s->bodies->n) shim_keep_survivors(s, ns);
        LAP(3);
    }
    jobject buf = Java_Native_positions(env, NULL, s->h, s->info3);
    jni_check("positions");
    const jlong *in = fake_jvm_longs(s->info3);
    jlong cap = 0;
    s->mir = (const double *)fake_jvm_direct_address(buf, &cap);
    s->mir_stride = (long)in[1];
    const long n = (long)in[0];
    if (n != s->bodies->n) fail("positions: the list after the step", -1);
    fake_jvm_free(buf);
    LAP(7);
    (void)par_any(s, n, unpack_xym_part);
    LAP(4);
    Java_Native_stepEnd(env, NULL, s->h);
    jni_check("stepEnd");
    LAP(5);
    if (shim_map(s) != n) fail("map after the step: N", -1);
    (void)par_any(s, n, unpack_v_part);
    LAP(6);
#undef LAP
}
static void shim_step(Shim *s) { shim_frame(s, NULL); }

/* getTreeForDebug(): Native.quads (QuadList: interleaved triples), then pull(false);
 * returned de-interleaved (cx[], cy[], h[]) for the comparison with the oracle */
static double *shim_tree(Shim *s, int64_t *nq) {
    shim_params(s);
    jdoubleArray qa = Java_Native_quads(env, NULL, s->h);
    jni_check("quads");
    *nq = fake_jvm_length(qa) / 3;
    const double *t = fake_jvm_doubles(qa);
    double *q = malloc(sizeof(double) * (3 * *nq + 1));
    for (int64_t i = 0; i < *nq; ++i) {
        q[i] = t[3 * i];
        q[*nq + i] = t[3 * i + 1];
        q[2 * *nq + i] = t[3 * i + 2];
    }
    fake_jvm_free(qa);
    shim_pull(s, 0);
    return q;
}

/* ---- scenes --------------------------------------------------------------------------- */
static void list_append_soa(List *l, long n, const double *x, const double *y, const double *vx,
                            const double *vy, const double *m) {
    l->b = realloc(l->b, sizeof(Body *) * (l->n + n + 1));
    l->cap = l->n + n + 1;
    start_mass = realloc(start_mass, sizeof(double) * (next_id + n + 1));
    Body *objs = malloc(sizeof(Body) * (n + 1)); /* (owned by the scene for the whole run) */
    for (long i = 0; i < n; ++i) {
        /* a unique start mass per body (light bodies keep theirs: only heavies absorb) */
        double mi = m[i] <= 4000.0 ? m[i] * (1.0 + (double)(next_id + 1) * 0x1p-40) : m[i];
        Body b = {x[i], y[i], vx[i], vy[i], mi, next_id};
        start_mass[next_id++] = mi;
        objs[i] = b;
        l->b[l->n++] = &objs[i];
    }
}

static void add_galaxy(List *l, long n, double x, double y, double vx, double r, double mc,
                       double msat, long seed) {
    double *a = malloc(sizeof(double) * 5 * n);
    if (bh_scene_galaxy_disk((int32_t)n, 0.03, 0.0, -1.0, -1.0, 0.01, 0.0, 1, seed, vx, 0.0, x, y,
                             r, 8.0, mc, msat, 80.0, a, a + n, a + 2 * n, a + 3 * n, a + 4 * n) != 0)
        fail("bh_scene_galaxy_disk", -1);
    list_append_soa(l, n, a, a + n, a + 2 * n, a + 3 * n, a + 4 * n);
    free(a);
}

static void add_uniform(List *l, long n, double m, long seed) {
    double *a = malloc(sizeof(double) * 5 * n);
    if (bh_scene_uniform((int32_t)n, m, seed, cfg_W, cfg_H, a, a + n, a + 2 * n, a + 3 * n,
                         a + 4 * n) != 0)
        fail("bh_scene_uniform", -1);
    list_append_soa(l, n, a, a + n, a + 2 * n, a + 3 * n, a + 4 * n);
    free(a);
}

/* ---- the checker ---------------------------------------------------------------------- */
static oracle_params oparams(const Shim *s) {
    oracle_params p = {cfg_G, cfg_DT, cfg_theta, cfg_SOFT2, cfg_W, cfg_H, s->mergeMaxMass,
                       s->mergeMinDist, 0, 0};
    return p;
}

static oracle_engine *oracle_of(const List *l, const Shim *s) {
    long n = l->n;
    double *a = malloc(sizeof(double) * (5 * n + 1));
    soa_of(l, a);
    oracle_params p = oparams(s);
    oracle_engine *o = oracle_create(&p, n, a, a + n, a + 2 * n, a + 3 * n, a + 4 * n);
    free(a);
    return o;
}

static void compare(const List *l, oracle_engine *o, long frame) {
    long n = oracle_num_bodies(o);
    if (n != l->n) fail("N differs from the oracle", frame);
    double *a = malloc(sizeof(double) * (5 * n + 1)), *b = malloc(sizeof(double) * (5 * n + 1));
    oracle_get_bodies(o, a, a + n, a + 2 * n, a + 3 * n, a + 4 * n);
    soa_of(l, b);
    if (memcmp(a, b, sizeof(double) * 5 * n) != 0) fail("state differs from the oracle", frame);
    free(a);
    free(b);
    for (long i = 0; i < n; ++i) { /* identity: light bodies keep their unique start mass */
        const Body *bd = l->b[i];
        if (start_mass[bd->id] <= 4000.0 && bd->m != start_mass[bd->id])
            fail("a surviving Body is not the object the reference keeps", frame);
    }
}

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e3 + (double)t.tv_nsec * 1e-6;
}

/* --c3-frames K: the shim's per-frame host work at C3 (8e5 + 2e5 galaxy disks, NBodyPanel's
 * two disks scaled), timed beside the GPU step: NBodyPanel's tick() -> step() (PNL:290-293),
 * K frames after 5 warm-up frames.  Prints one JSON line.  (The list holds references to Body
 * objects, as an ArrayList does; C loops over them are a lower bound of the JVM's.) */
static int c3_frames(long frames, jint mask) {
    List list = {NULL, 0, 0};
    add_galaxy(&list, 800000, 1200.0, 400.0, 0.0, 300.0, 50000.0, 5000.0, 1);
    add_galaxy(&list, 200000, 1200.0, 160.0, -50.0, 100.0, 5000.0, 500.0, 2);
    Shim s;
    shim_create(&s, &list, mask);
    for (int w = 0; w < 5; ++w) shim_step(&s);
    const long allocs0 = shadow_allocs, uploads0 = shim_steps_uploaded;
    double t[8] = {0, 0, 0, 0, 0, 0, 0, 0}; /* shim_frame's phases */
    const long n0 = s.bodies->n;
    const double t0 = now_ms();
    for (long f = 0; f < frames; ++f) shim_frame(&s, t);
    const double total = now_ms() - t0;
    printf("{\"frames\": %ld, \"bodies\": %ld, \"devices\": %d, \"threads\": %d, \"ms_per_frame\": %.4f, "
           "\"params_ms\": %.4f, \"changed_ms\": %.4f, \"wait_survivors_ms\": %.4f, \"removals_ms\": %.4f, "
           "\"wait_planes_ms\": %.4f, \"unpack_xym_ms\": %.4f, \"wait_end_ms\": %.4f, \"unpack_v_ms\": %.4f, "
           "\"allocations_per_frame\": %.3f, \"uploads\": %ld}\n",
           frames, n0, bh_multi_world((bh_engine *)(intptr_t)s.h), shim_threads, total / frames,
           t[0] / frames, t[1] / frames, t[2] / frames, t[3] / frames, t[7] / frames, t[4] / frames,
           t[5] / frames, t[6] / frames, (double)(shadow_allocs - allocs0) / frames, shim_steps_uploaded - uploads0);
    bh_destroy((bh_engine *)(intptr_t)s.h);
    return 0;
}

int main(int argc, char **argv) {
    env = fake_jvm_env();
    const char *tv = getenv("BH_SHIM_THREADS");
    if (tv && atoi(tv) >= 1 && atoi(tv) <= 64) shim_threads = atoi(tv);
    const char *pm = getenv("BH_SHIM_PAR_MIN");
    if (pm && atol(pm) >= 1) shim_par_min = atol(pm);
    jint mask = 1; /* GPU 0; BH_DEVICES="0,0,0" in the environment: one handle over a list */
    long timing_frames = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--mask") && i + 1 < argc) mask = (jint)strtol(argv[++i], NULL, 0);
        else if (!strcmp(argv[i], "--c3-frames") && i + 1 < argc) timing_frames = atol(argv[++i]);
    }
    if (timing_frames > 0) return c3_frames(timing_frames, mask);
    List list = {NULL, 0, 0};
    /* defaultBodies() (PNL:83-100), scaled down */
    add_galaxy(&list, 3000, 1200.0, 400.0, 0.0, 300.0, 50000.0, 5000.0, 1);
    add_galaxy(&list, 800, 1200.0, 160.0, -50.0, 100.0, 5000.0, 500.0, 2);
    Shim s;
    shim_create(&s, &list, mask); /* PNL:103 */
    const long allocs0 = shadow_allocs;
    oracle_engine *o = oracle_of(&list, &s);
    List list2 = {NULL, 0, 0}, list3 = {NULL, 0, 0};
    long removed_total = 0, quads_checked = 0, removed_max = 0;
    for (long frame = 0; frame < 40; ++frame) {
        if (frame == 10) cfg_theta = 0.7; /* Z/X keys (PNL:247-248), read live */
        if (frame == 14) cfg_DT = 0.008;  /* O/P keys (PNL:255-257) */
        if (frame == 16) s.mergeMaxMass = 3000.0;
        if (frame == 20) { /* 'C' key: resetBodies(makeUniformRandom(...)) (PNL:282-286) */
            add_uniform(&list2, 2500, 0.5, 5);
            add_galaxy(&list2, 400, 600.0, 300.0, 20.0, 60.0, 8000.0, 400.0, 7);
            shim_reset(&s, &list2);
            oracle_destroy(o);
            o = oracle_of(&list2, &s);
        }
        if (frame == 30) { /* mouse release: getBodies() + new disk -> resetBodies (PNL:228-234) */
            for (long i = 0; i < s.bodies->n; ++i) {
                list3.b = realloc(list3.b, sizeof(Body *) * (list3.n + 1));
                list3.cap = list3.n + 1;
                list3.b[list3.n++] = s.bodies->b[i]; /* the same objects, re-listed */
            }
            add_galaxy(&list3, 500, 1700.0, 500.0, 0.0, 80.0, 6000.0, 300.0, 9);
            shim_reset(&s, &list3);
            oracle_destroy(o);
            o = oracle_of(&list3, &s);
        }
        if (frame == 25) { /* the caller edits a body in place (as a drag would): step() uploads */
            s.bodies->b[7]->vx += 1.0;
            s.bodies->b[s.bodies->n - 1]->y -= 3.0;
            oracle_destroy(o);
            o = oracle_of(s.bodies, &s); /* the reference steps the edited objects themselves */
        }
        if (frame == 25 && bh_multi_world((bh_engine *)(intptr_t)s.h) == 1)
            /* the tree the last frame left for this one -- which the edited frame's speculative
             * step takes over -- raises its error flag: the upload must replace that step's error
             * too (the edited list never uses that tree) */
            if (bh_debug_inject((bh_engine *)(intptr_t)s.h, 99) != 0) fail("bh_debug_inject", frame);
        oracle_params op = oparams(&s);
        oracle_set_params(o, &op);
        long before = s.bodies->n;
        shim_step(&s); /* PNL:291 */
        oracle_step(o, 1);
        removed_total += before - s.bodies->n;
        if (before - s.bodies->n > removed_max) removed_max = before - s.bodies->n;
        compare(s.bodies, o, frame);
        if (frame == 5) { /* Native.getInto (a copy into a Java array) agrees with the mapped mirror */
            jdoubleArray a = fake_jvm_double_array((jsize)(5 * s.bodies->n), NULL);
            const jint got = Java_Native_getInto(env, NULL, s.h, a);
            jni_check("getInto");
            const double *g = fake_jvm_doubles(a);
            const long n = s.bodies->n, st = s.mir_stride;
            if (got != (jint)n) fail("getInto's count", frame);
            for (int k = 0; k < 5; ++k)
                if (memcmp(g + k * n, s.mir + k * st, sizeof(double) * (size_t)n))
                    fail("getInto differs from the mapped mirror", frame);
            fake_jvm_free(a);
        }
        if (frame % 4 == 3) { /* showTree: getTreeForDebug().visitQuads (PNL:333-340) */
            int64_t nq = 0;
            double *q = shim_tree(&s, &nq);
            int64_t mq = oracle_quads(o, NULL, NULL, NULL, 0);
            double *w = malloc(sizeof(double) * (3 * mq + 1));
            oracle_quads(o, w, w + mq, w + 2 * mq, mq);
            if (mq != nq || memcmp(q, w, sizeof(double) * 3 * nq) != 0)
                fail("quads differ from the reference's visitQuads", frame);
            quads_checked += nq;
            free(q);
            free(w);
            compare(s.bodies, o, frame); /* a fresh debug build may jitter (BHA:146-151) */
        }
    }
    if (removed_total == 0) fail("the scene never merged: identity bookkeeping untested", 40);
    if (removed_max < 3) fail("no frame removed 3+ bodies: the one-pass removal is untested", 40);
    if (shim_steps_uploaded != 1) fail("the in-place edit of frame 25 was not uploaded exactly once", 40);
    if (bh_multi_world((bh_engine *)(intptr_t)s.h) == 1 && step_end_errors_replaced != 1)
        fail("the edited frame's speculative step did not meet the injected carried-tree error", 40);
    printf("abi_harness: 40 frames through the JNI glue on %d device(s) (%ld native calls) "
           "bit-identical to the oracle; %ld bodies merged away (at most %ld in one frame), %ld "
           "quads checked, %ld uploads after the constructor/resets, %ld shadow allocations after "
           "the constructor\n",
           bh_multi_world((bh_engine *)(intptr_t)s.h), jni_calls, removed_total, removed_max,
           quads_checked, shim_steps_uploaded, shadow_allocs - allocs0);
    oracle_destroy(o);
    bh_destroy((bh_engine *)(intptr_t)s.h); /* the Kotlin object lives as long as the app */
    return 0;
}
