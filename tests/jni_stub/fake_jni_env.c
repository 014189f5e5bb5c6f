/* TEST-ONLY fake JNI environment that drives graph-embedding_amd/jni/
 * graphwalk_jni.c without a JVM (tests/test_jni_shim.py, through ctypes).
 *
 * Objects are heap records {kind, len, data}.  Get*ArrayElements and
 * GetStringUTFChars hand out COPIES (isCopy semantics), so the release mode
 * matters as in a JVM that copies: mode 0 copies back and frees, JNI_COMMIT
 * copies back, JNI_ABORT frees without copying.  The fake counts pins (every
 * Get must be Released), records the pending exception (class + message),
 * and can make the k-th pin fail with an OutOfMemoryError, as a JVM does
 * when it cannot pin or copy an array.                                     */
#define _POSIX_C_SOURCE 200809L /* strdup */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_STRING = 1, K_INT = 2, K_LONG = 3, K_DOUBLE = 4, K_OBJECT = 5, K_CLASS = 6 };

struct _jobject {
  int kind;
  jsize len;
  void* data;
};

static char g_exc_class[256];
static char g_exc_msg[1024];
static int g_pending = 0;
static int g_pins = 0;        /* outstanding Get* without a Release */
static int g_pin_calls = 0;   /* Get* calls so far */
static int g_fail_at = -1;    /* the Get* call (0-based) that fails, -1: none */
static int g_abort_copyback = 0;  /* JNI_ABORT releases whose copy differed from the array (input written) */

static jclass JNICALL f_FindClass(JNIEnv* env, const char* name) {
  (void)env;
  struct _jobject* c = (struct _jobject*)calloc(1, sizeof *c);
  c->kind = K_CLASS;
  c->data = strdup(name);
  return c;
}

static jint JNICALL f_ThrowNew(JNIEnv* env, jclass clazz, const char* msg) {
  (void)env;
  strncpy(g_exc_class, (const char*)clazz->data, sizeof g_exc_class - 1);
  strncpy(g_exc_msg, msg ? msg : "", sizeof g_exc_msg - 1);
  g_pending = 1;
  free(clazz->data);  /* the fake's class refs are single-use */
  free(clazz);
  return 0;
}

static void oom(void) {
  strcpy(g_exc_class, "java/lang/OutOfMemoryError");
  strcpy(g_exc_msg, "fake pin failure");
  g_pending = 1;
}

static int pin_fails(void) {
  if (g_pin_calls++ == g_fail_at) {
    oom();
    return 1;
  }
  return 0;
}

static jboolean JNICALL f_ExceptionCheck(JNIEnv* env) {
  (void)env;
  return (jboolean)(g_pending != 0);
}

static void JNICALL f_DeleteLocalRef(JNIEnv* env, jobject obj) {
  (void)env;
  (void)obj;  /* objects belong to the test */
}

static const char* JNICALL f_GetStringUTFChars(JNIEnv* env, jstring str, jboolean* isCopy) {
  (void)env;
  if (pin_fails()) return NULL;
  if (isCopy) *isCopy = JNI_TRUE;
  ++g_pins;
  return strdup((const char*)str->data);
}

static void JNICALL f_ReleaseStringUTFChars(JNIEnv* env, jstring str, const char* chars) {
  (void)env;
  (void)str;
  --g_pins;
  free((void*)chars);
}

static jsize JNICALL f_GetArrayLength(JNIEnv* env, jarray array) {
  (void)env;
  return array->len;
}

static jobject JNICALL f_GetObjectArrayElement(JNIEnv* env, jobjectArray array, jsize index) {
  (void)env;
  return ((jobject*)array->data)[index];
}

static size_t esize(int kind) { return kind == K_INT ? 4 : 8; }

static void* get_elems(jarray a, int kind, jboolean* isCopy) {
  if (a->kind != kind) abort();
  if (pin_fails()) return NULL;
  if (isCopy) *isCopy = JNI_TRUE;
  ++g_pins;
  void* p = malloc(esize(kind) * (size_t)(a->len > 0 ? a->len : 1));
  memcpy(p, a->data, esize(kind) * (size_t)a->len);
  return p;
}

static void release_elems(jarray a, void* elems, jint mode) {
  const size_t nb = esize(a->kind) * (size_t)a->len;
  if (mode == 0 || mode == JNI_COMMIT) memcpy(a->data, elems, nb);
  else if (mode == JNI_ABORT && memcmp(a->data, elems, nb) != 0) ++g_abort_copyback;
  if (mode != JNI_COMMIT) {
    --g_pins;
    free(elems);
  }
}

static jint* JNICALL f_GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* c) { (void)env; return (jint*)get_elems(a, K_INT, c); }
static jlong* JNICALL f_GetLongArrayElements(JNIEnv* env, jlongArray a, jboolean* c) { (void)env; return (jlong*)get_elems(a, K_LONG, c); }
static jdouble* JNICALL f_GetDoubleArrayElements(JNIEnv* env, jdoubleArray a, jboolean* c) { (void)env; return (jdouble*)get_elems(a, K_DOUBLE, c); }
static void JNICALL f_ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* e, jint m) { (void)env; release_elems(a, e, m); }
static void JNICALL f_ReleaseLongArrayElements(JNIEnv* env, jlongArray a, jlong* e, jint m) { (void)env; release_elems(a, e, m); }
static void JNICALL f_ReleaseDoubleArrayElements(JNIEnv* env, jdoubleArray a, jdouble* e, jint m) { (void)env; release_elems(a, e, m); }

static void JNICALL f_SetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len, const jdouble* buf) {
  (void)env;
  if (a->kind != K_DOUBLE || start < 0 || len < 0 || start + len > a->len) abort();
  memcpy((double*)a->data + start, buf, sizeof(double) * (size_t)len);
}

static const struct JNINativeInterface_ g_table = {
    f_FindClass, f_ThrowNew, f_ExceptionCheck, f_DeleteLocalRef, f_GetStringUTFChars, f_ReleaseStringUTFChars,
    f_GetArrayLength, f_GetObjectArrayElement, f_GetIntArrayElements, f_GetLongArrayElements,
    f_GetDoubleArrayElements, f_ReleaseIntArrayElements, f_ReleaseLongArrayElements, f_ReleaseDoubleArrayElements,
    f_SetDoubleArrayRegion};
static JNIEnv g_env = &g_table;

/* ---- the test's side (ctypes) -------------------------------------------- */
JNIEXPORT JNIEnv* fake_env(void) { return &g_env; }

JNIEXPORT jobject fake_string(const char* s) {
  struct _jobject* o = (struct _jobject*)calloc(1, sizeof *o);
  o->kind = K_STRING;
  o->data = strdup(s);
  return o;
}

/* kind: 2 int32, 3 int64, 4 float64; data copied in when non-NULL, else zeros */
JNIEXPORT jobject fake_array(int kind, jsize len, const void* data) {
  struct _jobject* o = (struct _jobject*)calloc(1, sizeof *o);
  o->kind = kind;
  o->len = len;
  o->data = calloc((size_t)(len > 0 ? len : 1), esize(kind));
  if (data) memcpy(o->data, data, esize(kind) * (size_t)len);
  return o;
}

JNIEXPORT jobject fake_object_array(jsize len, jobject* elems) {
  struct _jobject* o = (struct _jobject*)calloc(1, sizeof *o);
  o->kind = K_OBJECT;
  o->len = len;
  o->data = calloc((size_t)(len > 0 ? len : 1), sizeof(jobject));
  memcpy(o->data, elems, sizeof(jobject) * (size_t)len);
  return o;
}

JNIEXPORT void* fake_data(jobject o) { return o->data; }

JNIEXPORT void fake_free(jobject o) {
  if (!o) return;
  free(o->data);
  free(o);
}

/* pending exception class ("" if none) and message; fake_clear() resets it */
JNIEXPORT const char* fake_exception_class(void) { return g_pending ? g_exc_class : ""; }
JNIEXPORT const char* fake_exception_msg(void) { return g_pending ? g_exc_msg : ""; }
JNIEXPORT int fake_pins(void) { return g_pins; }
JNIEXPORT int fake_abort_copyback(void) { return g_abort_copyback; }

JNIEXPORT void fake_clear(int fail_at) {
  g_pending = 0;
  g_exc_class[0] = g_exc_msg[0] = 0;
  g_pin_calls = 0;
  g_fail_at = fail_at;
  g_abort_copyback = 0;
}
