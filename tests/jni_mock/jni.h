/*
 * jni.h — TEST-ONLY stand-in for the subset of the JNI interface that
 * raytracing-clj_amd/jni/rtclj_jni.c uses.  This image has no JDK; this file
 * lets the shim's own source compile unchanged against a function table that
 * tests/jni_mock/mock_env.c fills with recording fakes, so its argument
 * checks, array/string releases and error mapping can be exercised
 * (tests/test_jni_shim.py).  It is not a JVM and not a JDK header: only the
 * names, calling shape `(*env)->Fn(env, ...)` and the scalar type widths the
 * shim relies on are reproduced.  A JVM build uses the JDK's jni.h
 * (`make -C raytracing-clj_amd jni JAVA_HOME=...`).
 */
#ifndef RTCLJ_TEST_JNI_MOCK_H
#define RTCLJ_TEST_JNI_MOCK_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

typedef struct mock_obj* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jobject jthrowable;
typedef jarray jfloatArray;
typedef jarray jintArray;
typedef jarray jbyteArray;
typedef jarray jdoubleArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass cls, const char* msg);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  jsize (*GetArrayLength)(JNIEnv* env, jarray a);
  jfloat* (*GetFloatArrayElements)(JNIEnv* env, jfloatArray a, jboolean* is_copy);
  void (*ReleaseFloatArrayElements)(JNIEnv* env, jfloatArray a, jfloat* elems, jint mode);
  jint* (*GetIntArrayElements)(JNIEnv* env, jintArray a, jboolean* is_copy);
  void (*ReleaseIntArrayElements)(JNIEnv* env, jintArray a, jint* elems, jint mode);
  jbyte* (*GetByteArrayElements)(JNIEnv* env, jbyteArray a, jboolean* is_copy);
  void (*ReleaseByteArrayElements)(JNIEnv* env, jbyteArray a, jbyte* elems, jint mode);
  void (*GetFloatArrayRegion)(JNIEnv* env, jfloatArray a, jsize start, jsize len, jfloat* buf);
  void (*SetFloatArrayRegion)(JNIEnv* env, jfloatArray a, jsize start, jsize len, const jfloat* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray a, jsize start, jsize len, const jbyte* buf);
  void (*GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray a, jsize start, jsize len, jdouble* buf);
  const char* (*GetStringUTFChars)(JNIEnv* env, jstring s, jboolean* is_copy);
  void (*ReleaseStringUTFChars)(JNIEnv* env, jstring s, const char* chars);
};

#endif
