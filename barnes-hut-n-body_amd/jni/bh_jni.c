/*
 * bh_jni.c -- JNI glue of the Kotlin drop-in PhysicsEngine: the
 * `external fun`s of `object Native` (class `Native`, default package).  Every native only moves
 * Java arrays in and out and calls the matching bh_shim_* helper (bh_shim.c), whose logic
 * tests/c/abi_harness.c runs against the oracle; errors become java.lang.RuntimeException with
 * bh_last_error's text.
 *
 * Build where a JDK exists (none in this image, so it is not part of __graft_entry__.build()):
 *   make -C barnes-hut-n-body_amd jni JAVA_HOME=/path/to/jdk     -> lib/libbh_jni.so
 * then run the Kotlin app with -Djava.library.path=barnes-hut-n-body_amd/lib.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "bh_shim.h"

static void throw_rt(JNIEnv *env, const bh_engine *e, const char *what) {
    jclass rt = (*env)->FindClass(env, "java/lang/RuntimeException");
    if (rt) (*env)->ThrowNew(env, rt, e ? bh_last_error(e) : what);
}

/* external fun createMask(deviceMask: Int): Long  (bit d = HIP device d; 0 = every visible GPU) */
JNIEXPORT jlong JNICALL Java_Native_createMask(JNIEnv *env, jobject self, jint deviceMask) {
    (void)self;
    bh_engine *e = NULL;
    if (bh_shim_create((uint32_t)deviceMask, &e) != BH_OK) {
        throw_rt(env, NULL, "bh_create failed (no HIP device?)");
        return 0;
    }
    return (jlong)(intptr_t)e;
}

/* external fun create(device: Int): Long  (one GPU: HIP device `device`) */
JNIEXPORT jlong JNICALL Java_Native_create(JNIEnv *env, jobject self, jint device) {
    if (device < 0 || device > 31) {
        throw_rt(env, NULL, "create: device index out of range (0..31)");
        return 0;
    }
    return Java_Native_createMask(env, self, (jint)(1u << device));
}

/* external fun setParams(h: Long, G: Double, dt: Double, theta: Double, soft2: Double,
 *                        w: Int, hgt: Int, mergeMaxMass: Double, mergeMinDist: Double) */
JNIEXPORT void JNICALL Java_Native_setParams(JNIEnv *env, jobject self, jlong h, jdouble G,
                                             jdouble dt, jdouble theta, jdouble soft2, jint w,
                                             jint hgt, jdouble mm, jdouble md) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    if (bh_shim_set_params(e, G, dt, theta, soft2, w, hgt, mm, md) != BH_OK)
        throw_rt(env, e, "setParams");
}

/* external fun reset(h: Long, n: Int, soa: DoubleArray)
 * The Java array is copied into a native buffer first (GetDoubleArrayRegion): no device work runs
 * while the JVM holds an array pinned, and the GC is never stalled by the upload. */
JNIEXPORT void JNICALL Java_Native_reset(JNIEnv *env, jobject self, jlong h, jint n,
                                         jdoubleArray soa) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    if (n < 0 || n > INT32_MAX / 5 || !soa || (*env)->GetArrayLength(env, soa) < 5 * (jsize)n) {
        throw_rt(env, NULL, "reset: the SoA array must hold 5 n doubles (n < 2^31 / 5)");
        return;
    }
    double *a = (double *)malloc(sizeof(double) * (5 * (size_t)n + 1));
    if (!a) {
        throw_rt(env, NULL, "reset: out of memory");
        return;
    }
    if (n > 0) (*env)->GetDoubleArrayRegion(env, soa, 0, 5 * (jsize)n, a);
    const int rc = bh_shim_reset(e, (int64_t)n, a);
    free(a);
    if (rc != BH_OK) throw_rt(env, e, "reset");
}

/* external fun step(h: Long, k: Int) */
JNIEXPORT void JNICALL Java_Native_step(JNIEnv *env, jobject self, jlong h, jint k) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    if (bh_shim_step(e, (int32_t)k) != BH_OK) throw_rt(env, e, "step");
}

/* external fun stepBegin(h: Long, k: Int)  (bh_step_begin: the step runs on the engine's thread) */
JNIEXPORT void JNICALL Java_Native_stepBegin(JNIEnv *env, jobject self, jlong h, jint k) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    if (bh_shim_step_begin(e, (int32_t)k) != BH_OK) throw_rt(env, e, "stepBegin");
}

/* external fun positions(h: Long, info: LongArray): ByteBuffer
 * The running call's hand-off (bh_step_positions): a direct buffer over the five planes of the
 * mirror buffer it writes -- x, y, m final, vx, vy only after stepEnd + map -- with info =
 * [n after the call, stride in doubles, n before it]. */
JNIEXPORT jobject JNICALL Java_Native_positions(JNIEnv *env, jobject self, jlong h,
                                                jlongArray info) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    const double *f[5] = {NULL, NULL, NULL, NULL, NULL};
    const int32_t *sv = NULL;
    int64_t n = 0, n0 = 0;
    static double empty[1];
    if (!info || (*env)->GetArrayLength(env, info) < 3) {
        throw_rt(env, NULL, "positions: info must hold 3 longs");
        return NULL;
    }
    if (bh_shim_positions(e, f, &n, &n0, &sv) != BH_OK) {
        throw_rt(env, e, "positions");
        return NULL;
    }
    const int64_t stride = (int64_t)(f[1] - f[0]);
    if (5 * stride * (int64_t)sizeof(double) > INT32_MAX) {
        throw_rt(env, NULL, "positions: more bodies than a direct buffer addresses");
        return NULL;
    }
    const jlong out[3] = {(jlong)n, (jlong)stride, (jlong)n0};
    (*env)->SetLongArrayRegion(env, info, 0, 3, out);
    return (*env)->NewDirectByteBuffer(env, n > 0 ? (void *)f[0] : (void *)empty,
                                       (jlong)(5 * stride * (int64_t)sizeof(double)));
}

/* external fun survivors(h: Long): ByteBuffer
 * The running call's survivors (bh_step_positions without the planes: as soon as they are
 * known): int32 list indices before the call, ascending, one per body after it -- the removals
 * are the indices missing (BHA:519); the buffer's capacity is 4 n. */
JNIEXPORT jobject JNICALL Java_Native_survivors(JNIEnv *env, jobject self, jlong h) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    const int32_t *sv = NULL;
    int64_t n = 0, n0 = 0;
    static int32_t empty[1];
    if (bh_shim_survivors(e, &sv, &n, &n0) != BH_OK) { /* (ahead of the planes' copy) */
        throw_rt(env, e, "survivors");
        return NULL;
    }
    return (*env)->NewDirectByteBuffer(env, n > 0 ? (void *)sv : (void *)empty,
                                       (jlong)(n * (int64_t)sizeof(int32_t)));
}

/* external fun stepEnd(h: Long)  (bh_step_end: joins; the step's error as an exception) */
JNIEXPORT void JNICALL Java_Native_stepEnd(JNIEnv *env, jobject self, jlong h) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    if (bh_shim_step_end(e) != BH_OK) throw_rt(env, e, "stepEnd");
}

/* external fun getInto(h: Long, soa: DoubleArray): Int  (n, or -n if soa is shorter than 5 n)
 * Fills the caller's reusable array from the engine's pinned caller-order mirror
 * (bh_map_bodies), which the step wrote itself: five SetDoubleArrayRegion copies, no allocation,
 * no device call while a Java array is held. */
JNIEXPORT jint JNICALL Java_Native_getInto(JNIEnv *env, jobject self, jlong h, jdoubleArray soa) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    const double *f[5] = {NULL, NULL, NULL, NULL, NULL};
    int64_t n = 0;
    if (!soa) {
        throw_rt(env, NULL, "getInto: null array");
        return 0;
    }
    if (bh_shim_map(e, f, &n) != BH_OK) {
        throw_rt(env, e, "getInto");
        return 0;
    }
    if (n > INT32_MAX / 5) {
        throw_rt(env, NULL, "getInto: more bodies than a Java array holds (5 n >= 2^31)");
        return 0;
    }
    if ((int64_t)(*env)->GetArrayLength(env, soa) < 5 * n) return (jint)(-n);
    for (int k = 0; k < 5 && n > 0; ++k)
        (*env)->SetDoubleArrayRegion(env, soa, (jsize)(k * n), (jsize)n, f[k]);
    return (jint)n;
}

/* external fun map(h: Long, info: LongArray): ByteBuffer
 * The engine's pinned caller-order mirror itself (bh_map_bodies), which the step filled: a direct
 * buffer over its five planes (x at 0, y at the stride, then vx, vy, m) and info = [n, stride in
 * doubles].  Nothing is copied -- the shim compares and unpacks straight from pinned host memory
 * -- and, with the shim's two mirror buffers (bh_set_mirror(e, 2)), the buffer stays valid and
 * unchanged until the next map: the shim compares its list against it while the next step runs
 * on another thread, then maps again. */
JNIEXPORT jobject JNICALL Java_Native_map(JNIEnv *env, jobject self, jlong h, jlongArray info) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    const double *f[5] = {NULL, NULL, NULL, NULL, NULL};
    int64_t n = 0;
    static double empty[1];
    if (!info || (*env)->GetArrayLength(env, info) < 2) {
        throw_rt(env, NULL, "map: info must hold 2 longs");
        return NULL;
    }
    if (bh_shim_map(e, f, &n) != BH_OK) {
        throw_rt(env, e, "map");
        return NULL;
    }
    const int64_t stride = n > 0 ? (int64_t)(f[1] - f[0]) : 0;
    if (n > 0 && 5 * stride * (int64_t)sizeof(double) > INT32_MAX) {
        throw_rt(env, NULL, "map: more bodies than a direct buffer addresses (40 stride >= 2^31)");
        return NULL;
    }
    const jlong out[2] = {(jlong)n, (jlong)stride};
    (*env)->SetLongArrayRegion(env, info, 0, 2, out);
    return (*env)->NewDirectByteBuffer(env, n > 0 ? (void *)f[0] : (void *)empty,
                                       (jlong)(5 * stride * (int64_t)sizeof(double)));
}

/* external fun quads(h: Long): DoubleArray  ([cx0, cy0, h0, cx1, ...], visitQuads order) */
JNIEXPORT jdoubleArray JNICALL Java_Native_quads(JNIEnv *env, jobject self, jlong h) {
    (void)self;
    bh_engine *e = (bh_engine *)(intptr_t)h;
    int64_t nq = 0;
    int rc = bh_shim_quads(e, NULL, 0, &nq); /* builds the tree if the cache was dropped */
    if (rc != BH_OK && rc != BH_E_CAPACITY) {
        throw_rt(env, e, "quads");
        return NULL;
    }
    if (nq > INT32_MAX / 3) {
        throw_rt(env, NULL, "quads: more cells than a Java array holds");
        return NULL;
    }
    double *q = (double *)malloc(sizeof(double) * (size_t)(3 * nq + 1));
    if (!q) {
        throw_rt(env, NULL, "quads: out of memory");
        return NULL;
    }
    rc = bh_shim_quads(e, q, nq, &nq);
    jdoubleArray out = NULL;
    if (rc == BH_OK) {
        out = (*env)->NewDoubleArray(env, (jsize)(3 * nq));
        if (out) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)(3 * nq), q);
    } else {
        throw_rt(env, e, "quads");
    }
    free(q);
    return out;
}

/* external fun lastRemoved(h: Long): IntArray */
JNIEXPORT jintArray JNICALL Java_Native_lastRemoved(JNIEnv *env, jobject self, jlong h) {
    (void)self;
    const bh_engine *e = (const bh_engine *)(intptr_t)h;
    int64_t cnt = 0;
    int rc = bh_shim_last_removed(e, NULL, 0, &cnt);
    if (rc != BH_OK && rc != BH_E_CAPACITY) {
        throw_rt(env, e, "lastRemoved");
        return NULL;
    }
    if (cnt > INT32_MAX) {
        throw_rt(env, NULL, "lastRemoved: more removals than a Java array holds");
        return NULL;
    }
    int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)(cnt + 1));
    if (!idx) {
        throw_rt(env, NULL, "lastRemoved: out of memory");
        return NULL;
    }
    rc = bh_shim_last_removed(e, idx, cnt, &cnt);
    jintArray out = NULL;
    if (rc == BH_OK) {
        out = (*env)->NewIntArray(env, (jsize)cnt);
        if (out) (*env)->SetIntArrayRegion(env, out, 0, (jsize)cnt, (const jint *)idx);
    } else {
        throw_rt(env, e, "lastRemoved");
    }
    free(idx);
    return out;
}
