/*
 * TEST INFRASTRUCTURE: an in-process stand-in for the JVM side of JNI, enough to call the real
 * glue (barnes-hut-n-body_amd/jni/bh_jni.c) from C: Java arrays are heap blocks, a thrown
 * exception is recorded and checked by the caller.
 */
#ifndef BH_FAKE_JVM_H
#define BH_FAKE_JVM_H

#include "jni.h"

JNIEnv *fake_jvm_env(void);
/* the message of a pending exception (NULL if none); clears it */
const char *fake_jvm_take_exception(void);

jdoubleArray fake_jvm_double_array(jsize len, const double *init); /* NULL init: zeros */
double *fake_jvm_doubles(jdoubleArray a);
jint *fake_jvm_ints(jintArray a);
jsize fake_jvm_length(jarray a);
jlongArray fake_jvm_long_array(jsize len);
jlong *fake_jvm_longs(jlongArray a);
/* a direct ByteBuffer's address and capacity (GetDirectBufferAddress / GetDirectBufferCapacity) */
void *fake_jvm_direct_address(jobject buf, jlong *capacity);
void fake_jvm_free(jarray a);

/* the glue's natives (bh_jni.c), declared for the harness */
jlong Java_Native_create(JNIEnv *env, jobject self, jint device);
jlong Java_Native_createMask(JNIEnv *env, jobject self, jint deviceMask);
void Java_Native_setParams(JNIEnv *env, jobject self, jlong h, jdouble G, jdouble dt,
                           jdouble theta, jdouble soft2, jint w, jint hgt, jdouble mm, jdouble md);
void Java_Native_reset(JNIEnv *env, jobject self, jlong h, jint n, jdoubleArray soa);
void Java_Native_step(JNIEnv *env, jobject self, jlong h, jint k);
jint Java_Native_getInto(JNIEnv *env, jobject self, jlong h, jdoubleArray soa);
jobject Java_Native_map(JNIEnv *env, jobject self, jlong h, jlongArray info);
void Java_Native_stepBegin(JNIEnv *env, jobject self, jlong h, jint k);
jobject Java_Native_positions(JNIEnv *env, jobject self, jlong h, jlongArray info);
jobject Java_Native_survivors(JNIEnv *env, jobject self, jlong h);
void Java_Native_stepEnd(JNIEnv *env, jobject self, jlong h);
jdoubleArray Java_Native_quads(JNIEnv *env, jobject self, jlong h);
jintArray Java_Native_lastRemoved(JNIEnv *env, jobject self, jlong h);

#endif
