/* JNI shim: the Java host (DeepSim/TopSimAll's simrank.* / benchmark.*
 * drivers, e.g. Test_u_u_TopSim_singleSample.java:46-64) calling libgraphwalk's
 * C ABI (include/graphwalk.h).  Java class: simrank.GraphWalkNative.
 *
 * UNTESTED HERE: this image has no JDK (no jni.h, no javac), so build.py
 * compiles this file only when $JAVA_HOME/include/jni.h exists:
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

/* structures.Graph(path, V) with MyConfiguration.SEPARATOR (Graph.java:28-42), uploaded to `device` */
JNIEXPORT jlong JNICALL Java_simrank_GraphWalkNative_loadGraph(JNIEnv* env, jclass cls, jstring path, jstring sep,
                                                               jint V, jint device) {
  (void)cls;
  const char* p = (*env)->GetStringUTFChars(env, path, 0);
  const char* s = (*env)->GetStringUTFChars(env, sep, 0);
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
  jsize ns = (*env)->GetArrayLength(env, sources);
  if ((*env)->GetArrayLength(env, idsOut) < (jsize)ns * k || (*env)->GetArrayLength(env, scoresOut) < (jsize)ns * k) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (c) (*env)->ThrowNew(env, c, "idsOut / scoresOut shorter than sources.length * k");
    return;
  }
  jint* src = (*env)->GetIntArrayElements(env, sources, 0);
  jint* ids = (*env)->GetIntArrayElements(env, idsOut, 0);
  jdouble* sc = (*env)->GetDoubleArrayElements(env, scoresOut, 0);
  jlong* st = stats ? (*env)->GetLongArrayElements(env, stats, 0) : NULL;
  int rc = gw_topsim_host(g, variant, sample, step, C, (uint64_t)seed, (const int32_t*)src, ns, k, (int32_t*)ids, sc,
                          NULL, (int64_t*)st);
  (*env)->ReleaseIntArrayElements(env, sources, src, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, idsOut, ids, 0);
  (*env)->ReleaseDoubleArrayElements(env, scoresOut, sc, 0);
  if (st) (*env)->ReleaseLongArrayElements(env, stats, st, 0);
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
  jsize ns = (*env)->GetArrayLength(env, sources);
  double* rows = (double*)malloc(sizeof(double) * (size_t)ns * (size_t)(inf.n > 0 ? inf.n : 1));
  if (!rows) {
    throw_gw(env, GW_ERR_NOMEM, g);
    return;
  }
  jint* src = (*env)->GetIntArrayElements(env, sources, 0);
  jlong* st = stats ? (*env)->GetLongArrayElements(env, stats, 0) : NULL;
  int rc = gw_topsim_host(g, variant, sample, step, C, (uint64_t)seed, (const int32_t*)src, ns, 0, NULL, NULL, rows,
                          (int64_t*)st);
  (*env)->ReleaseIntArrayElements(env, sources, src, JNI_ABORT);
  if (st) (*env)->ReleaseLongArrayElements(env, stats, st, 0);
  if (rc == GW_OK) {
    for (jsize r = 0; r < ns; ++r) {
      jdoubleArray row = (jdoubleArray)(*env)->GetObjectArrayElement(env, simOut, r);
      (*env)->SetDoubleArrayRegion(env, row, 0, (jsize)inf.n, rows + (size_t)r * (size_t)inf.n);
      (*env)->DeleteLocalRef(env, row);
    }
  }
  free(rows);
  if (rc != GW_OK) throw_gw(env, rc, g);
}

/* simrank.SimRank(g).compute() + getResult() (SimRank.java:36-81): V*V row-major, diag 0 */
JNIEXPORT void JNICALL Java_simrank_GraphWalkNative_simrankNaive(JNIEnv* env, jclass cls, jlong gh, jdouble C,
                                                                 jint step, jdoubleArray out) {
  (void)cls;
  gw_graph* g = G(gh);
  jdouble* sim = (*env)->GetDoubleArrayElements(env, out, 0);
  int rc = gw_simrank_naive_host(g, C, step, sim);
  (*env)->ReleaseDoubleArrayElements(env, out, sim, 0);
  if (rc != GW_OK) throw_gw(env, rc, g);
}

/* utils.Print.printByOrder (Print.java:25-53) from top-k rows: path and path + ".sim.txt" */
JNIEXPORT void JNICALL Java_simrank_GraphWalkNative_writeTopK(JNIEnv* env, jclass cls, jstring path, jintArray ids,
                                                              jdoubleArray scores, jintArray rowIds, jint k,
                                                              jstring sep) {
  (void)cls;
  const char* p = (*env)->GetStringUTFChars(env, path, 0);
  const char* s = (*env)->GetStringUTFChars(env, sep, 0);
  jsize nr = (*env)->GetArrayLength(env, rowIds);
  jint* id = (*env)->GetIntArrayElements(env, ids, 0);
  jdouble* sc = (*env)->GetDoubleArrayElements(env, scores, 0);
  jint* rid = (*env)->GetIntArrayElements(env, rowIds, 0);
  int rc = gw_write_sim_text_topk(p, (const int32_t*)id, sc, (const int32_t*)rid, nr, k, s, 6);
  (*env)->ReleaseIntArrayElements(env, ids, id, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, scores, sc, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, rowIds, rid, JNI_ABORT);
  (*env)->ReleaseStringUTFChars(env, path, p);
  (*env)->ReleaseStringUTFChars(env, sep, s);
  if (rc != GW_OK) throw_gw(env, rc, NULL);
}
