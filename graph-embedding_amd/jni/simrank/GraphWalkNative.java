package simrank;

/**
 * Native bindings of libgraphwalk (include/graphwalk.h) through
 * graph-embedding_amd/jni/graphwalk_jni.c.
 *
 * No JVM in the build image: the C shim is compiled and driven through a fake
 * JNIEnv by tests/test_jni_shim.py; build.py compiles the real shim only
 * when $JAVA_HOME/include/jni.h exists.  Load order: libgraphwalk.so, then
 * libgraphwalk_jni.so (java.library.path = graph-embedding_amd/gwamd).
 */
public final class GraphWalkNative {
    static {
        System.loadLibrary("graphwalk");
        System.loadLibrary("graphwalk_jni");
    }

    /** include/graphwalk.h GW_TOPSIM_* variants. */
    public static final int TOPSIM_SINGLE_SAMPLE = 0, TOPSIM_ENUMERATE = 1, TOPSIM_SINGLE_RW = 2;

    private GraphWalkNative() {}

    /** structures.Graph(path, V) (Graph.java:28-42) with the given separator, on GPU `device`. */
    public static native long loadGraph(String path, String separator, int V, int device) throws java.io.IOException;

    public static native void freeGraph(long g);

    public static native int vertexCount(long g);

    /** TopSim rows for `sources` as dense V-length rows (getResult() of those sources). */
    public static native void topsimDense(long g, int variant, int sample, int step, double C, long seed,
                                          int[] sources, double[][] simOut, long[] stats);

    /** TopSim top-k rows for any V: ids / scores of length sources.length * k. */
    public static native void topsimTopK(long g, int variant, int sample, int step, double C, long seed,
                                         int[] sources, int k, int[] idsOut, double[] scoresOut, long[] stats);

    /** simrank.SimRank(g).compute() + getResult(): V*V row-major, diagonal 0 (SimRank.java:36-81). */
    public static native void simrankNaive(long g, double C, int step, double[] simOut);

    /**
     * TopSim compute() + utils.Print.printByOrder(sim, path, topk, ...) for `sources`
     * (TopSim_singleSample.java:47-54, Print.java:25-53): the reference's bytes at any V
     * (sparse rows, FixedMaxPQ replayed exactly); stats may be null or long[4].
     */
    public static native void topsimWriteText(long g, int variant, int sample, int step, double C, long seed,
                                              int[] sources, int topk, String path, String separator, long[] stats)
            throws java.io.IOException;
}
