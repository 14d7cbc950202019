/* jni.h — TEST-ONLY minimal JNI environment for unit-testing jni/pbx_jni.c without a JDK
 * (this image has none).  Source-compatible with the calls the shim makes; the function
 * table is our own (not the JDK's binary layout): the shim is compiled against it and driven
 * by tests/jni_mock/jni_test.c with a fake libpbx (fake_pbx.c).  Never used for a real build:
 * `make -C jni` uses $JAVA_HOME/include/jni.h. */
#ifndef PBX_TEST_JNI_H
#define PBX_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT
#define JNICALL
#define JNI_ABORT 2
#define JNI_TRUE 1
#define JNI_FALSE 0

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef int32_t jsize;
typedef struct mock_obj* jobject;
typedef jobject jclass, jstring, jarray, jbyteArray, jlongArray, jintArray, jthrowable;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv*, const char*);
    jint (*ThrowNew)(JNIEnv*, jclass, const char*);
    jboolean (*ExceptionCheck)(JNIEnv*);
    const char* (*GetStringUTFChars)(JNIEnv*, jstring, jboolean*);
    void (*ReleaseStringUTFChars)(JNIEnv*, jstring, const char*);
    jsize (*GetArrayLength)(JNIEnv*, jarray);
    void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
    void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
    jbyteArray (*NewByteArray)(JNIEnv*, jsize);
    jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
    void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
    jlong* (*GetLongArrayElements)(JNIEnv*, jlongArray, jboolean*);
    void (*ReleaseLongArrayElements)(JNIEnv*, jlongArray, jlong*, jint);
    jlongArray (*NewLongArray)(JNIEnv*, jsize);
    void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
    void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
    void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
    jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
};
#endif
