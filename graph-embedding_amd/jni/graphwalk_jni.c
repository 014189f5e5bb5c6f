/* JNI shim: the Java host (DeepSim/TopSimAll's simrank.* / benchmark.*
 * drivers, e.g. Test_u_u_TopSim_singleSample.java:46-64) calling libgraphwalk's
 * C ABI (include/graphwalk.h).  Java class: simrank.GraphWalkNative.
 *
 * This image has no JDK (no jni.h, no javac): tests/test_jni_shim.py compiles
 * this file -Wall -Wextra -Werror against a test-only <jni.h> stand-in and
 * drives every entry point through a fake JNIEnv (no JVM).  build.py builds
 * the real shim only when $JAVA_HOME/include/jni.h exists:
 *   cc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      graph-embedding_amd/jni/graphwalk_jni.c -Lgraph-embedding_amd/gwamd -lgraphwalk \
 *      -o graph-embedding_amd/gwamd/libgraphwalk_jni.so
 *
 * Errors map to the exceptions the reference throws on the same inputs:
 * IOException (unreadable file, Graph.java:28-42), NumberFormatException
 * (a separator that does not split the line, Graph.java:38-39),
 * ArrayIndexOutOfBoundsException (ids >= V), RuntimeException otherwise. */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "graphwalk.h"

static void throw_gw(JNIEnv* env, int rc, const gw_graph* g) {
  const char* cls = rc == GW_ERR_IO      ? "java/io/IOException"
                    : rc == GW_ERR_PARSE ? "java/lang/NumberFormatException"
                    : rc == GW_ERR_RANGE ? "java/lang/ArrayIndexOutOfBoundsException"
                    : rc == GW_ERR_NOMEM ? "java/lang/OutOfMemoryError"
                                         : "java/lang/RuntimeException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, gw_last_error(g));
}

static gw_graph* G(jlong h) { return (gw_graph*)(intptr_t)h; }

static void throw_arg(JNIEnv* env, const char* msg) {
  jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (c) (*env)->ThrowNew(env, c, msg);
}

/* a Get*ArrayElements / GetStringUTFChars that returned NULL has already
 * thrown (OutOfMemoryError): the caller releases what it pinned and returns */

/* structures.Graph(path, V) with MyConfiguration.SEPARATOR (Graph.java:28-42), uploaded to `device` */
JNIEXPORT jlong JNICALL Java_simrank_GraphWalkNative_loadGraph(JNIEnv* env, jclass cls, jstring path, jstring sep,
                                                               jint V, jint device) {
  (void)cls;
  if (!path || !sep) {
    throw_arg(env, "path / separator is null");
    return 0;
  }
  const char* p = (*env)->GetStringUTFChars(env, path, 0);
  const char* s = p ? (*env)->GetStringUTFChars(env, sep, 0) : NULL;
  if (!p || !s) {
    if (p) (*env)->ReleaseStringUTFChars(env, path, p);
    return 0;
  }
  gw_graph* g = NULL;
  int rc = gw_graph_load_edgelist(p, s, GW_SEM_JAVA_MULTI, 0, 0, V, &g);
  if (rc == GW_OK) rc = gw_graph_to_device(g, device);
  (*env)->ReleaseStringUTFChars(env, path, p);
  (*env)->ReleaseStringUTFChars(env, sep, s);
  if (rc != GW_OK) {
    throw_gw(env, rc, g);
    if (g) gw_graph_free(g);
    return 0;
  }
  return (jlong)(intptr_t)g;
}

JNIEXPORT void JNICALL Java_simrank_GraphWalkNative_freeGraph(JNIEnv* env, jclass cls, jlong g) {
  (void)env;
  (void)cls;
  gw_graph_free(G(g));
}

JNIEXPORT jint JNICALL Java_simrank_GraphWalkNative_vertexCount(JNIEnv* env, jclass cls, jlong gh) {
  (void)cls;
  gw_graph_info_t inf;
  int rc = gw_graph_info(G(gh), &inf);
  if (rc != GW_OK) {
    throw_gw(env, rc, G(gh));
    return 0;
  }
  return (jint)inf.n;
}

/* TopSim (variant: GW_TOPSIM_*) for `sources`, top-k rows: ids [ns*k], scores [ns*k] */
JNIEXPORT void JNICALL Java_simrank_GraphWalkNative_topsimTopK(JNIEnv* env, jclass cls, jlong gh, jint variant,
                                                               jint sample, jint step, jdouble C, jlong seed,
                                                               jintArray sources, jint k, jintArray idsOut,
                                                               jdoubleArray scoresOut, jlongArray stats) {
  (void)cls;
  gw_graph* g = G(gh);
  if (!sources || !idsOut || !scoresOut || k < 0) {
    throw_arg(env, "null array or k < 0");
    return;
  }
  const jsize ns = (*env)->GetArrayLength(env, sources);
  const int64_t need = (int64_t)ns * (int64_t)k; /* 64-bit: ns * k can pass 2^31 */
  if ((int64_t)(*env)->GetArrayLength(env, idsOut) < need || (int64_t)(*env)->GetArrayLength(env, scoresOut) < need) {
    throw_arg(env, "idsOut / scoresOut shorter than sources.length * k");
    return;
  }
  if (stats && (*env)->GetArrayLength(env, stats) < 4) {
    throw_arg(env, "stats needs 4 entries");
    return;
  }
  jint* src = (*env)->GetIntArrayElements(env, sources, 0);
  jint* ids = src ? (*env)->GetIntArrayElements(env, idsOut, 0) : NULL;
  jdouble* sc = ids ? (*env)->GetDoubleArrayElements(env, scoresOut, 0) : NULL;
  jlong* st = (sc && stats) ? (*env)->GetLongArrayElements(env, stats, 0) : NULL;
  int rc = GW_ERR_NOMEM;
  if (src && ids && sc && (!stats || st))
    rc = gw_topsim_host(g, variant, sample, step, C, (uint64_t)seed, (const int32_t*)src, ns, k, (int32_t*)ids, sc,
                        NULL, (int64_t*)st);
  if (src) (*env)->ReleaseIntArrayElements(env, sources, src, JNI_ABORT);
  if (ids) (*env)->ReleaseIntArrayElements(env, idsOut, ids, 0);
  if (sc) (*env)->ReleaseDoubleArrayElements(env, scoresOut, sc, 0);
  if (st) (*env)->ReleaseLongArrayElements(env, stats, st, 0);
  if ((*env)->ExceptionCheck(env)) return; /* a pin failed: OutOfMemoryError pending */
  if (rc != GW_OK) throw_gw(env, rc, g);
}

/* TopSim compute() + utils.Print.printByOrder (TopSim_singleSample.java:47-54,
 * Print.java:25-53) for `sources`, Java-exact at any V (gw_topsim_write_text:
 * sparse rows, FixedMaxPQ replayed): path and path + ".sim.txt" */
JNIEXPORT void JNICALL Java_simrank_GraphWalkNative_topsimWriteText(JNIEnv* env, jclass cls, jlong gh, jint variant,
                                                                    jint sample, jint step, jdouble C, jlong seed,
                                                                    jintArray sources, jint topk, jstring path,
                                                                    jstring sep, jlongArray stats) {
  (void)cls;
  gw_graph* g = G(gh);
  if (!sources || !path || !sep || topk < 0) {
    throw_arg(env, "null argument or topk < 0");
    return;
  }
  if (stats && (*env)->GetArrayLength(env, stats) < 4) {
    throw_arg(env, "stats needs 4 entries");
    return;
  }
  const jsize ns = (*env)->GetArrayLength(env, sources);
  const char* p = (*env)->GetStringUTFChars(env, path, 0);
  const char* s = p ? (*env)->GetStringUTFChars(env, sep, 0) : NULL;
  jint* src = s ? (*env)->GetIntArrayElements(env, sources, 0) : NULL;
  jlong* st = (src && stats) ? (*env)->GetLongArrayElements(env, stats, 0) : NULL;
  int rc = GW_ERR_NOMEM;
  if (p && s && src && (!stats || st))
    rc = gw_topsim_write_text(g, variant, sample, step, C, (uint64_t)seed, (const int32_t*)src, ns, topk, p, s, 6,
                              (int64_t*)st);
  if (st) (*env)->ReleaseLongArrayElements(env, stats, st, 0);
  if (src) (*env)->ReleaseIntArrayElements(env, sources, src, JNI_ABORT);
  if (s) (*env)->ReleaseStringUTFChars(env, sep, s);
  if (p) (*env)->ReleaseStringUTFChars(env, path, p);
  if ((*env)->ExceptionCheck(env)) return;
  if (rc != GW_OK) throw_gw(env, rc, g);
}

/* dense rows (TopSim_singleSample.getResult(), TopSim_singleSample.java:56-58): simOut[r] = sim[sources[r]][*] */
JNIEXPORT void JNICALL Java_simrank_GraphWalkNative_topsimDense(JNIEnv* env, jclass cls, jlong gh, jint variant,
                                                                jint sample, jint step, jdouble C, jlong seed,
                                                                jintArray sources, jobjectArray simOut,
                                                                jlongArray stats) {
  (void)cls;
  gw_graph* g = G(gh);
  gw_graph_info_t inf;
  if (gw_graph_info(g, &inf) != GW_OK) {
    throw_gw(env, GW_ERR_INVALID, g);
    return;
  }
  if (!sources || !simOut) {
    throw_arg(env, "null array");
    return;
  }
  const jsize ns = (*env)->GetArrayLength(env, sources);
  if ((*env)->GetArrayLength(env, simOut) < ns || (stats && (*env)->GetArrayLength(env, stats) < 4)) {
    throw_arg(env, "simOut shorter than sources.length or stats shorter than 4");
    return;
  }
  double* rows = (double*)malloc(sizeof(double) * (size_t)ns * (size_t)(inf.n > 0 ? inf.n : 1));
  if (!rows) {
    throw_gw(env, GW_ERR_NOMEM, g);
    return;
  }
  jint* src = (*env)->GetIntArrayElements(env, sources, 0);
  jlong* st = (src && stats) ? (*env)->GetLongArrayElements(env, stats, 0) : NULL;
  int rc = GW_ERR_NOMEM;
  if (src && (!stats || st))
    rc = gw_topsim_host(g, variant, sample, step, C, (uint64_t)seed, (const int32_t*)src, ns, 0, NULL, NULL, rows,
                        (int64_t*)st);
  if (src) (*env)->ReleaseIntArrayElements(env, sources, src, JNI_ABORT);
  if (st) (*env)->ReleaseLongArrayElements(env, stats, st, 0);
  if (rc == GW_OK) {
    for (jsize r = 0; r < ns && !(*env)->ExceptionCheck(env); ++r) {
      jdoubleArray row = (jdoubleArray)(*env)->GetObjectArrayElement(env, simOut, r);
      if (!row || (*env)->GetArrayLength(env, row) < (jsize)inf.n) {
        if (row) (*env)->DeleteLocalRef(env, row);
        throw_arg(env, "simOut row null or shorter than V");
        break;
      }
      (*env)->SetDoubleArrayRegion(env, row, 0, (jsize)inf.n, rows + (size_t)r * (size_t)inf.n);
      (*env)->DeleteLocalRef(env, row);
    }
  }
  free(rows);
  if ((*env)->ExceptionCheck(env)) return;
  if (rc != GW_OK) throw_gw(env, rc, g);
}

/* simrank.SimRank(g).compute() + getResult() (SimRank.java:36-81): V*V row-major, diag 0 */
JNIEXPORT void JNICALL Java_simrank_GraphWalkNative_simrankNaive(JNIEnv* env, jclass cls, jlong gh, jdouble C,
                                                                 jint step, jdoubleArray out) {
  (void)cls;
  gw_graph* g = G(gh);
  gw_graph_info_t inf;
  if (gw_graph_info(g, &inf) != GW_OK) {
    throw_gw(env, GW_ERR_INVALID, g);
    return;
  }
  if (!out || (int64_t)(*env)->GetArrayLength(env, out) < (int64_t)inf.n * inf.n) {
    throw_arg(env, "out shorter than V * V");
    return;
  }
  jdouble* sim = (*env)->GetDoubleArrayElements(env, out, 0);
  if (!sim) return;
  int rc = gw_simrank_naive_host(g, C, step, sim);
  (*env)->ReleaseDoubleArrayElements(env, out, sim, 0);
  if (rc != GW_OK) throw_gw(env, rc, g);
}
