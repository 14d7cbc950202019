/* mock_vm.h — TEST-ONLY mock JNI VM shared by the shim drivers (jni_test.c: against the
 * scripted fake libpbx; jni_real.c: against the real lib/libpbx.so on the GPU): arrays,
 * strings, direct buffers and one pending exception, behind the minimal JNIEnv of jni.h. */
#ifndef PBX_MOCK_VM_H
#define PBX_MOCK_VM_H
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

#define J(name) Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_##name

/* ---- the mock VM: arrays, strings, direct buffers, one pending exception */
struct mock_obj {
    int kind;  /* 0 string, 1 byte[], 2 long[], 3 int[], 4 direct buffer, 5 class */
    size_t len;
    void* data;
    const char* name;
};
static char pending[256];
static int failures;

#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            failures++;                                                 \
        }                                                               \
    } while (0)

static jclass m_FindClass(JNIEnv* e, const char* n) {
    (void)e;
    static struct mock_obj c[8];
    static int k;
    struct mock_obj* o = &c[k++ % 8];
    o->kind = 5;
    o->name = n;
    return o;
}
static jint m_ThrowNew(JNIEnv* e, jclass c, const char* msg) {
    (void)e;
    snprintf(pending, sizeof pending, "%s: %s", c->name, msg);
    return 0;
}
static jboolean m_ExceptionCheck(JNIEnv* e) { (void)e; return pending[0] != 0; }
static const char* m_GetStringUTFChars(JNIEnv* e, jstring s, jboolean* c) { (void)e; (void)c; return (const char*)s->data; }
static void m_ReleaseStringUTFChars(JNIEnv* e, jstring s, const char* p) { (void)e; (void)s; (void)p; }
static jsize m_GetArrayLength(JNIEnv* e, jarray a) { (void)e; return (jsize)a->len; }
static int region_fail_after = -1;  /* > 0: that many GetByteArrayRegion calls succeed, the next throws */
static void m_GetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, jbyte* buf) {
    (void)e;
    if (region_fail_after == 0) {
        region_fail_after = -1;
        snprintf(pending, sizeof pending, "java/lang/InternalError");
        return;
    }
    if (region_fail_after > 0) region_fail_after--;
    if (s < 0 || n < 0 || (size_t)s + (size_t)n > a->len) {
        snprintf(pending, sizeof pending, "java/lang/ArrayIndexOutOfBoundsException");
        return;
    }
    memcpy(buf, (char*)a->data + s, (size_t)n);
}
static void m_SetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, const jbyte* buf) {
    (void)e;
    memcpy((char*)a->data + s, buf, (size_t)n);
}
static struct mock_obj made[64];
static int nmade;
static jbyteArray m_NewByteArray(JNIEnv* e, jsize n) {
    (void)e;
    struct mock_obj* o = &made[nmade++ % 64];
    o->kind = 1;
    o->len = (size_t)n;
    o->data = calloc((size_t)n + 1, 1);
    return o;
}
static jbyte* m_GetByteArrayElements(JNIEnv* e, jbyteArray a, jboolean* c) { (void)e; (void)c; return a->data; }
static void m_ReleaseByteArrayElements(JNIEnv* e, jbyteArray a, jbyte* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jlong* m_GetLongArrayElements(JNIEnv* e, jlongArray a, jboolean* c) { (void)e; (void)c; return a->data; }
static void m_ReleaseLongArrayElements(JNIEnv* e, jlongArray a, jlong* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jlongArray m_NewLongArray(JNIEnv* e, jsize n) {
    (void)e;
    struct mock_obj* o = &made[nmade++ % 64];
    o->kind = 2;
    o->len = (size_t)n;
    o->data = calloc((size_t)n + 1, 8);
    return o;
}
static void m_SetLongArrayRegion(JNIEnv* e, jlongArray a, jsize s, jsize n, const jlong* b) {
    (void)e;
    memcpy((jlong*)a->data + s, b, 8 * (size_t)n);
}
static void m_SetIntArrayRegion(JNIEnv* e, jintArray a, jsize s, jsize n, const jint* b) {
    (void)e;
    memcpy((jint*)a->data + s, b, 4 * (size_t)n);
}
static void m_GetIntArrayRegion(JNIEnv* e, jintArray a, jsize s, jsize n, jint* b) {
    (void)e;
    memcpy(b, (jint*)a->data + s, 4 * (size_t)n);
}
static void* m_GetDirectBufferAddress(JNIEnv* e, jobject b) { (void)e; return b && b->kind == 4 ? b->data : NULL; }
static jlong m_GetDirectBufferCapacity(JNIEnv* e, jobject b) { (void)e; return b && b->kind == 4 ? (jlong)b->len : -1; }

static const struct JNINativeInterface_ table = {
    m_FindClass, m_ThrowNew, m_ExceptionCheck, m_GetStringUTFChars, m_ReleaseStringUTFChars,
    m_GetArrayLength, m_GetByteArrayRegion, m_SetByteArrayRegion, m_NewByteArray,
    m_GetByteArrayElements, m_ReleaseByteArrayElements, m_GetLongArrayElements,
    m_ReleaseLongArrayElements, m_NewLongArray, m_SetLongArrayRegion, m_SetIntArrayRegion, m_GetIntArrayRegion,
    m_GetDirectBufferAddress, m_GetDirectBufferCapacity};
static JNIEnv envp = &table;
static JNIEnv* env = &envp;

static struct mock_obj str(const char* s) { struct mock_obj o = {0, strlen(s), (void*)s, NULL}; return o; }
static struct mock_obj arr(int kind, size_t len, size_t esz) {
    struct mock_obj o = {kind, len, calloc(len + 1, esz), NULL};
    return o;
}
static int threw(const char* cls) { return strncmp(pending, cls, strlen(cls)) == 0; }
#endif
