/* TEST-ONLY stand-in for the JDK's <jni.h> (this image has no JDK).
 *
 * Declares exactly the JNIEnv members graph-embedding_amd/jni/graphwalk_jni.c
 * calls, with the JNI 1.x signatures and member names, so the shim compiles
 * unchanged against this header and against a real JDK's.  The function
 * table's member ORDER is not the JVM's (the real table has ~230 slots): a
 * shim built against this header is only ever driven by the fake environment
 * in tests/jni_stub/fake_jni_env.c, never loaded into a JVM.               */
#ifndef GW_TEST_JNI_STUB_H
#define GW_TEST_JNI_STUB_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef unsigned char jboolean;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass(JNICALL* FindClass)(JNIEnv* env, const char* name);
  jint(JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jboolean(JNICALL* ExceptionCheck)(JNIEnv* env);
  void(JNICALL* DeleteLocalRef)(JNIEnv* env, jobject obj);
  const char*(JNICALL* GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
  void(JNICALL* ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
  jsize(JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
  jobject(JNICALL* GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
  jint*(JNICALL* GetIntArrayElements)(JNIEnv* env, jintArray array, jboolean* isCopy);
  jlong*(JNICALL* GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
  jdouble*(JNICALL* GetDoubleArrayElements)(JNIEnv* env, jdoubleArray array, jboolean* isCopy);
  void(JNICALL* ReleaseIntArrayElements)(JNIEnv* env, jintArray array, jint* elems, jint mode);
  void(JNICALL* ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
  void(JNICALL* ReleaseDoubleArrayElements)(JNIEnv* env, jdoubleArray array, jdouble* elems, jint mode);
  void(JNICALL* SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
};

#endif
