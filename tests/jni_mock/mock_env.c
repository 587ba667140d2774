/*
 * mock_env.c — TEST-ONLY recording JNI function table for
 * tests/test_jni_shim.py (see jni.h here).  Java arrays and strings are
 * heap objects with a pin count; every call is checked against the JNI rules
 * the shim must follow and violations are counted:
 *   - every Get<Type>ArrayElements / GetStringUTFChars is released once, with
 *     the pointer it returned (inputs: mode JNI_ABORT, nothing written back);
 *   - no JNI call other than ExceptionCheck and the releases while an
 *     exception is pending;
 *   - Get/Set<Type>ArrayRegion within the array's bounds.
 * mock_fail_get(k) makes the k-th following Get*Elements return NULL with a
 * pending OutOfMemoryError, as a JVM does when it cannot copy an array.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { T_FLOAT = 1, T_INT, T_BYTE, T_STRING, T_CLASS, T_DOUBLE };

struct mock_obj {
  int type;
  jsize len;
  void* data;   /* the array's contents (what Java sees) */
  void* pinned; /* the copy handed out by Get*Elements, or NULL */
  int gets, releases;
  char name[128];
};

#define MAX_OBJS 256
static struct mock_obj* objs[MAX_OBJS];
static int n_objs;

static struct {
  int pending;
  char cls[128], msg[512];
  int throws;
  int calls_while_pending;
  int bad_release;      /* wrong pointer, double release, mode != JNI_ABORT */
  int region_oob;
  int set_regions;
  int fail_get_in;      /* 0 = off; k = the k-th Get*Elements from now fails */
} st;

static void record_call(void) {
  if (st.pending) st.calls_while_pending++;
}

static struct mock_obj* new_obj(int type, jsize len, size_t esz, const void* src) {
  if (n_objs >= MAX_OBJS) return NULL;
  struct mock_obj* o = (struct mock_obj*)calloc(1, sizeof *o);
  o->type = type;
  o->len = len;
  o->data = calloc((size_t)len + 1, esz);
  if (src && len) memcpy(o->data, src, (size_t)len * esz);
  objs[n_objs++] = o;
  return o;
}

static size_t esize(int type) { return type == T_BYTE ? 1 : type == T_DOUBLE ? 8 : 4; }

static int fail_now(void) {
  if (st.fail_get_in <= 0) return 0;
  if (--st.fail_get_in == 0) {
    st.pending = 1;
    snprintf(st.cls, sizeof st.cls, "java/lang/OutOfMemoryError");
    snprintf(st.msg, sizeof st.msg, "mock: array copy failed");
    return 1;
  }
  return 0;
}

static void* get_elems(struct mock_obj* o, int type) {
  record_call();
  if (!o || o->type != type) return NULL;
  if (fail_now()) return NULL;
  if (o->pinned) { /* a second pin of the same array: allowed by JNI, but the shim never needs it */
    st.bad_release++;
    return NULL;
  }
  o->gets++;
  o->pinned = malloc((size_t)o->len * esize(type) + 1);
  memcpy(o->pinned, o->data, (size_t)o->len * esize(type));
  return o->pinned;
}

static void release_elems(struct mock_obj* o, int type, void* elems, jint mode) {
  if (!o || o->type != type || !o->pinned || elems != o->pinned || mode != JNI_ABORT) {
    st.bad_release++;
    return;
  }
  free(o->pinned);
  o->pinned = NULL;
  o->releases++;
}

static jclass m_FindClass(JNIEnv* env, const char* name) {
  (void)env;
  record_call();
  struct mock_obj* c = new_obj(T_CLASS, 0, 1, NULL);
  if (c) snprintf(c->name, sizeof c->name, "%s", name);
  return c;
}
static jint m_ThrowNew(JNIEnv* env, jclass cls, const char* msg) {
  (void)env;
  record_call();
  st.pending = 1;
  st.throws++;
  snprintf(st.cls, sizeof st.cls, "%s", cls ? cls->name : "?");
  snprintf(st.msg, sizeof st.msg, "%s", msg ? msg : "");
  return 0;
}
static jboolean m_ExceptionCheck(JNIEnv* env) {
  (void)env;
  return st.pending ? JNI_TRUE : JNI_FALSE;
}
static jsize m_GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  record_call();
  return a ? a->len : 0;
}
static jfloat* m_GetFloatArrayElements(JNIEnv* env, jfloatArray a, jboolean* c) {
  (void)env;
  if (c) *c = JNI_TRUE;
  return (jfloat*)get_elems(a, T_FLOAT);
}
static void m_ReleaseFloatArrayElements(JNIEnv* env, jfloatArray a, jfloat* e, jint mode) {
  (void)env;
  release_elems(a, T_FLOAT, e, mode);
}
static jint* m_GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* c) {
  (void)env;
  if (c) *c = JNI_TRUE;
  return (jint*)get_elems(a, T_INT);
}
static void m_ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* e, jint mode) {
  (void)env;
  release_elems(a, T_INT, e, mode);
}
static jbyte* m_GetByteArrayElements(JNIEnv* env, jbyteArray a, jboolean* c) {
  (void)env;
  if (c) *c = JNI_TRUE;
  return (jbyte*)get_elems(a, T_BYTE);
}
static void m_ReleaseByteArrayElements(JNIEnv* env, jbyteArray a, jbyte* e, jint mode) {
  (void)env;
  release_elems(a, T_BYTE, e, mode);
}
static void m_GetFloatArrayRegion(JNIEnv* env, jfloatArray a, jsize start, jsize len, jfloat* buf) {
  (void)env;
  record_call();
  if (!a || a->type != T_FLOAT || start < 0 || len < 0 || start + len > a->len) {
    st.region_oob++;
    st.pending = 1;
    snprintf(st.cls, sizeof st.cls, "java/lang/ArrayIndexOutOfBoundsException");
    return;
  }
  memcpy(buf, (float*)a->data + start, (size_t)len * 4);
}
static void m_SetFloatArrayRegion(JNIEnv* env, jfloatArray a, jsize start, jsize len, const jfloat* buf) {
  (void)env;
  record_call();
  st.set_regions++;
  if (!a || a->type != T_FLOAT || start < 0 || len < 0 || start + len > a->len) {
    st.region_oob++;
    st.pending = 1;
    snprintf(st.cls, sizeof st.cls, "java/lang/ArrayIndexOutOfBoundsException");
    return;
  }
  memcpy((float*)a->data + start, buf, (size_t)len * 4);
}
static void m_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize len, const jbyte* buf) {
  (void)env;
  record_call();
  st.set_regions++;
  if (!a || a->type != T_BYTE || start < 0 || len < 0 || start + len > a->len) {
    st.region_oob++;
    st.pending = 1;
    snprintf(st.cls, sizeof st.cls, "java/lang/ArrayIndexOutOfBoundsException");
    return;
  }
  memcpy((jbyte*)a->data + start, buf, (size_t)len);
}
static void m_GetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len, jdouble* buf) {
  (void)env;
  record_call();
  if (!a || a->type != T_DOUBLE || start < 0 || len < 0 || start + len > a->len) {
    st.region_oob++;
    st.pending = 1;
    snprintf(st.cls, sizeof st.cls, "java/lang/ArrayIndexOutOfBoundsException");
    return;
  }
  memcpy(buf, (double*)a->data + start, (size_t)len * 8);
}
static const char* m_GetStringUTFChars(JNIEnv* env, jstring s, jboolean* c) {
  (void)env;
  if (c) *c = JNI_TRUE;
  record_call();
  if (!s || s->type != T_STRING) return NULL;
  if (fail_now()) return NULL;
  if (s->pinned) {
    st.bad_release++;
    return NULL;
  }
  s->gets++;
  s->pinned = strdup((const char*)s->data);
  return (const char*)s->pinned;
}
static void m_ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* chars) {
  (void)env;
  if (!s || s->type != T_STRING || !s->pinned || chars != s->pinned) {
    st.bad_release++;
    return;
  }
  free(s->pinned);
  s->pinned = NULL;
  s->releases++;
}

static const struct JNINativeInterface_ table = {
    m_FindClass,           m_ThrowNew,
    m_ExceptionCheck,      m_GetArrayLength,
    m_GetFloatArrayElements, m_ReleaseFloatArrayElements,
    m_GetIntArrayElements, m_ReleaseIntArrayElements,
    m_GetByteArrayElements, m_ReleaseByteArrayElements,
    m_GetFloatArrayRegion, m_SetFloatArrayRegion,
    m_SetByteArrayRegion,  m_GetDoubleArrayRegion,
    m_GetStringUTFChars,   m_ReleaseStringUTFChars,
};
static JNIEnv the_env = &table;

/* ---- test API (ctypes) ---------------------------------------------------- */
JNIEXPORT JNIEnv* mock_env(void) { return &the_env; }

JNIEXPORT void mock_reset(void) {
  for (int i = 0; i < n_objs; ++i) {
    free(objs[i]->data);
    free(objs[i]->pinned);
    free(objs[i]);
  }
  n_objs = 0;
  memset(&st, 0, sizeof st);
}

JNIEXPORT jobject mock_float_array(const float* src, jsize len) { return new_obj(T_FLOAT, len, 4, src); }
JNIEXPORT jobject mock_int_array(const int32_t* src, jsize len) { return new_obj(T_INT, len, 4, src); }
JNIEXPORT jobject mock_byte_array(const int8_t* src, jsize len) { return new_obj(T_BYTE, len, 1, src); }
JNIEXPORT jobject mock_double_array(const double* src, jsize len) { return new_obj(T_DOUBLE, len, 8, src); }
JNIEXPORT jobject mock_string(const char* s) { return new_obj(T_STRING, (jsize)strlen(s), 1, s); }
JNIEXPORT void* mock_data(jobject o) { return o ? o->data : NULL; }
JNIEXPORT void mock_fail_get(int k) { st.fail_get_in = k; }

/* out[8]: pins outstanding (gets - releases over every object), bad releases,
 * calls while an exception was pending, throws, out-of-bounds regions,
 * Set<Float|Byte>ArrayRegion calls, exception pending, total gets. */
JNIEXPORT void mock_stats(int* out) {
  int outstanding = 0, gets = 0;
  for (int i = 0; i < n_objs; ++i) {
    outstanding += objs[i]->gets - objs[i]->releases;
    gets += objs[i]->gets;
  }
  out[0] = outstanding;
  out[1] = st.bad_release;
  out[2] = st.calls_while_pending;
  out[3] = st.throws;
  out[4] = st.region_oob;
  out[5] = st.set_regions;
  out[6] = st.pending;
  out[7] = gets;
}

/* The pending exception's class and message ("" when none). */
JNIEXPORT const char* mock_exception_class(void) { return st.pending ? st.cls : ""; }
JNIEXPORT const char* mock_exception_message(void) { return st.pending ? st.msg : ""; }
JNIEXPORT void mock_clear_exception(void) { st.pending = 0; }
