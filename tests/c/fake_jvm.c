/* TEST INFRASTRUCTURE: the fake JVM of fake_jvm.h. */
#include "fake_jvm.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct fake_jobject {
    jsize len;
    size_t elem;
    unsigned char data[];
};

static char pending[512];
static int has_pending;
static struct fake_jobject runtime_exception_class;

static jclass find_class(JNIEnv *env, const char *name) {
    (void)env;
    return strcmp(name, "java/lang/RuntimeException") == 0 ? &runtime_exception_class : NULL;
}

static jint throw_new(JNIEnv *env, jclass clazz, const char *msg) {
    (void)env;
    (void)clazz;
    snprintf(pending, sizeof(pending), "%s", msg ? msg : "(null)");
    has_pending = 1;
    return 0;
}

static struct fake_jobject *new_array(jsize len, size_t elem) {
    struct fake_jobject *a = calloc(1, sizeof(*a) + elem * (size_t)(len > 0 ? len : 1));
    a->len = len;
    a->elem = elem;
    return a;
}

static jsize get_length(JNIEnv *env, jarray a) {
    (void)env;
    return a->len;
}
static jdoubleArray new_double_array(JNIEnv *env, jsize len) {
    (void)env;
    return new_array(len, sizeof(jdouble));
}
static void set_double_region(JNIEnv *env, jdoubleArray a, jsize start, jsize len,
                              const jdouble *buf) {
    (void)env;
    memcpy(a->data + sizeof(jdouble) * (size_t)start, buf, sizeof(jdouble) * (size_t)len);
}
static void get_double_region(JNIEnv *env, jdoubleArray a, jsize start, jsize len,
                              jdouble *buf) {
    (void)env;
    if (start < 0 || len < 0 || start + len > a->len) { /* ArrayIndexOutOfBoundsException */
        snprintf(pending, sizeof(pending), "GetDoubleArrayRegion out of bounds");
        has_pending = 1;
        return;
    }
    memcpy(buf, a->data + sizeof(jdouble) * (size_t)start, sizeof(jdouble) * (size_t)len);
}
static jintArray new_int_array(JNIEnv *env, jsize len) {
    (void)env;
    return new_array(len, sizeof(jint));
}
static void set_int_region(JNIEnv *env, jintArray a, jsize start, jsize len, const jint *buf) {
    (void)env;
    memcpy(a->data + sizeof(jint) * (size_t)start, buf, sizeof(jint) * (size_t)len);
}

static void set_long_region(JNIEnv *env, jlongArray a, jsize start, jsize len, const jlong *buf) {
    (void)env;
    if (start < 0 || len < 0 || start + len > a->len) {
        snprintf(pending, sizeof(pending), "SetLongArrayRegion out of bounds");
        has_pending = 1;
        return;
    }
    memcpy(a->data + sizeof(jlong) * (size_t)start, buf, sizeof(jlong) * (size_t)len);
}
/* a direct buffer: no elements of its own, the address and capacity in its data */
struct direct_buf {
    void *address;
    jlong capacity;
};
static jobject new_direct_buffer(JNIEnv *env, void *address, jlong capacity) {
    (void)env;
    struct fake_jobject *o = new_array((jsize)sizeof(struct direct_buf), 1);
    o->len = -1; /* not an array */
    struct direct_buf d = {address, capacity};
    memcpy(o->data, &d, sizeof(d));
    return o;
}

static const struct JNINativeInterface_ table = {
    .FindClass = find_class,
    .ThrowNew = throw_new,
    .GetArrayLength = get_length,
    .NewDoubleArray = new_double_array,
    .SetDoubleArrayRegion = set_double_region,
    .GetDoubleArrayRegion = get_double_region,
    .NewIntArray = new_int_array,
    .SetIntArrayRegion = set_int_region,
    .SetLongArrayRegion = set_long_region,
    .NewDirectByteBuffer = new_direct_buffer,
};
static JNIEnv env_ptr = &table;

JNIEnv *fake_jvm_env(void) { return &env_ptr; }

const char *fake_jvm_take_exception(void) {
    if (!has_pending) return NULL;
    has_pending = 0;
    return pending;
}

jdoubleArray fake_jvm_double_array(jsize len, const double *init) {
    struct fake_jobject *a = new_array(len, sizeof(double));
    if (init) memcpy(a->data, init, sizeof(double) * (size_t)len);
    return a;
}
double *fake_jvm_doubles(jdoubleArray a) { return (double *)a->data; }
jint *fake_jvm_ints(jintArray a) { return (jint *)a->data; }
jsize fake_jvm_length(jarray a) { return a->len; }
void fake_jvm_free(jarray a) { free(a); }

jlongArray fake_jvm_long_array(jsize len) { return new_array(len, sizeof(jlong)); }
jlong *fake_jvm_longs(jlongArray a) { return (jlong *)a->data; }
void *fake_jvm_direct_address(jobject buf, jlong *capacity) {
    struct direct_buf d;
    memcpy(&d, buf->data, sizeof(d));
    if (capacity) *capacity = d.capacity;
    return d.address;
}
