/*
 * TEST INFRASTRUCTURE: the subset of the JNI interface (JDK <jni.h>) that
 * barnes-hut-n-body_amd/jni/bh_jni.c uses, so the glue compiles and runs in this image (no JDK)
 * against the in-process fake JVM of tests/c/fake_jvm.c.  Same type names, same call shape
 * ((*env)->Fn(env, ...)) as the real header; a real build uses the JDK's header instead.
 */
#ifndef BH_TEST_JNI_STUB_H
#define BH_TEST_JNI_STUB_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct fake_jobject *jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jdoubleArray;
typedef jarray jintArray;
typedef jarray jlongArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv *env, const char *name);
    jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);
    jdoubleArray (*NewDoubleArray)(JNIEnv *env, jsize len);
    void (*SetDoubleArrayRegion)(JNIEnv *env, jdoubleArray array, jsize start, jsize len,
                                 const jdouble *buf);
    void (*GetDoubleArrayRegion)(JNIEnv *env, jdoubleArray array, jsize start, jsize len,
                                 jdouble *buf);
    jintArray (*NewIntArray)(JNIEnv *env, jsize len);
    void (*SetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len,
                              const jint *buf);
    void (*SetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len,
                               const jlong *buf);
    jobject (*NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);
};

#endif
