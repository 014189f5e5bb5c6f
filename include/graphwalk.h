/*
 * graphwalk.h — C ABI of the MI355X-native node2vec walk generator (H1) and
 * TopSim random-walk SimRank (H2).
 *
 * Drop-in boundary.  The reference has no FFI on this path; its interfaces are
 * a Python class (H1) and Java classes (H2).  Every entry point below names
 * the reference symbol it replaces (file:line relative to the reference
 * checkout).  A maintainer binds these from Python with ctypes (see
 * graph-embedding_amd/gwamd/_lib.py) or from Java with the JNI stub shown in
 * INTEGRATION.md.
 *
 * Conventions
 *   - plain C types only; opaque handles; every call returns an int status
 *     (GW_OK == 0, negative = error); gw_last_error() gives the message.
 *   - no global mutable state: seeds, modes and device ordinals are explicit;
 *     one handle may be used from one thread at a time.
 *   - every call that touches a device runs on the graph's device (or the
 *     `device` argument) and restores the caller's current device on return.
 *   - "_dev" pointers are device (HBM) pointers on the graph's device,
 *     "stream" is a hipStream_t (NULL = the default stream).  gw_n2v_walks and
 *     gw_simrank_naive (after its first call sized the workspace) are
 *     asynchronous and launch-only (no allocation, no synchronisation), so they
 *     can be captured in a HIP graph.  The TopSim calls (gw_topsim,
 *     gw_topsim_dense, gw_topsim_m, gw_topsim_double, gw_topsim_dev,
 *     gw_double_random_walk) synchronise the stream before returning (they
 *     read the kernels' capacity flag to fail loudly) and size their
 *     workspace on first use (gw_topsim_prepare does it ahead of time).
 *   - all other pointers are host pointers, caller-allocated; size them with
 *     gw_graph_info() / the documented formulas.
 *   - vertex ids crossing the boundary are dense ids in [0, n) unless a
 *     function says "labels"; gw_graph_export_csr() gives the label map.
 */
#ifndef GRAPHWALK_H
#define GRAPHWALK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define GW_OK 0
#define GW_ERR_INVALID (-1)     /* bad argument (Python ValueError)            */
#define GW_ERR_IO (-2)          /* file open/read/write (Java IOException)     */
#define GW_ERR_PARSE (-3)       /* malformed edge line (NumberFormatException) */
#define GW_ERR_NOMEM (-4)       /* host or device allocation failed            */
#define GW_ERR_DEVICE (-5)      /* HIP runtime error / no GPU                  */
#define GW_ERR_STATE (-6)       /* call order (e.g. walks before prepare)      */
#define GW_ERR_UNSUPPORTED (-7) /* option not supported for this graph/mode    */
#define GW_ERR_RANGE (-8)       /* id out of [0,V) (ArrayIndexOutOfBounds)     */
#define GW_ERR_KEY (-9)         /* missing edge key (Python KeyError)          */
#define GW_ERR_ZERODIV (-10)    /* weights sum to 0 (ZeroDivisionError)        */
#define GW_ERR_CAPACITY (-11)   /* workspace too small for the frontier        */

/* ---- graph semantics ------------------------------ */
/* networkx simple graph as built by read_graph (node2vec/src/main.py:76-89):
 * duplicates merge (last weight wins, to_undirected resolves reciprocal pairs
 * by node order), node order = first appearance, neighbours sorted by label,
 * original integer labels kept.                                             */
#define GW_SEM_NX_SIMPLE 0
/* structures.Graph (DeepSim/TopSimAll/src/structures/Graph.java:28-57): each
 * line appends both directions, duplicates kept, insertion order, ids dense
 * in [0,V), V given by the caller.                                          */
#define GW_SEM_JAVA_MULTI 1

/* ---- node2vec modes ------------------------------------------------------ */
/* exact reference replay: per-node AND per-edge alias tables
 * (node2vec.py:83-113), uniforms supplied by the caller (MT19937 stream of
 * np.random, node2vec.py:156-157).  Needs sum(deg^2) table entries.        */
#define GW_N2V_REPLAY 0
/* scale mode: per-node alias only (or none when unweighted); second-order
 * bias by exact rejection sampling with the return edge as an outlier;
 * Philox4x32-10 keyed by (seed, walk, step, trial).  Unweighted undirected
 * NX_SIMPLE graphs: prepare builds 16 B slot entries {x, deg x, offsets x}
 * and per-row neighbour hash sets (16 B buckets); at q > 1 a step whose
 * deg(prev) < deg(cur) draws from the exact N(cur)/N(prev) mixture proposal,
 * otherwise from the uniform proposal with a lazy has_edge probe.  64 B
 * listed entries (common neighbours of each edge when they fit 40 B, which
 * answer most lazy probes) are built for q < 1 only, whatever
 * gw_options_t.listed says (at q >= 1 they would answer no probe), and are
 * skipped (same walks, 16 B entries) when they exceed half of the free HBM.
 * The walks never depend on which tables were built.                       */
#define GW_N2V_REJECTION 1
/* exact second-order sampling from per-edge common-neighbour bitsets (the
 * reference's per-edge alias tables compressed to 1 bit per entry, sum(deg^2)
 * bits; unweighted undirected NX_SIMPLE graphs): a step is a 3-way mixture
 * (return / common neighbour / other) with no has_edge probes.  Philox keyed
 * like GW_N2V_REJECTION.                                                   */
#define GW_N2V_BITSET 2
/* pick BITSET or REJECTION by modelled end-to-end time (prepare + the walk
 * steps announced in gw_options_t.expected_steps): the rejection sampler is
 * prepared (milliseconds) and a pilot of its walks counts its trials per
 * step (time = trials x a measured cost per trial); the bitset sampler's
 * time is its build model (sum over edges of min(deg u, deg v)) plus the
 * steps at its measured rate.  The choice is a function of the graph, p, q
 * and expected_steps (no timing), so runs repeat.  With expected_steps = 0
 * (unknown) the bitset sampler is taken whenever it applies and fits (the
 * throughput choice).  gw_graph_info().n2v_mode reports the choice.       */
#define GW_N2V_AUTO 3

/* ---- TopSim variants (DeepSim/TopSimAll/src/simrank/) --------------------- */
#define GW_TOPSIM_SINGLE_SAMPLE 0 /* TopSim_singleSample.java:62-203 (= _Basic) */
#define GW_TOPSIM_ENUMERATE 1     /* TopSim_Enumerate.java:61-136 (always enumerate) */
#define GW_TOPSIM_SINGLE_RW 2     /* SingleRandomWalk.java:53-92 (plain Monte-Carlo) */

typedef struct gw_graph gw_graph;

typedef struct gw_graph_info_t {
  int64_t n;          /* vertices (dense ids 0..n-1)                        */
  int64_t nnz;        /* adjacency entries (directed slots)                 */
  int64_t max_degree;
  int64_t edge_alias_entries; /* sum over slots of deg(dst); 0 until prepared */
  int32_t semantics;  /* GW_SEM_*                                           */
  int32_t directed;
  int32_t weighted;
  int32_t device;     /* -1 when not resident                               */
  int64_t sampler_bytes; /* HBM held by the prepared n2v sampler's per-slot tables
                            (bitset entries + regions, or rejection slot entries) */
  int32_t n2v_mode;   /* GW_N2V_* the last gw_n2v_prepare built (-1: none)    */
  int32_t listed;     /* 1: the rejection sampler has 64 B listed entries      */
} gw_graph_info_t;

/* Per-handle tuning (gw_graph_set_options).  Sizes and sampler choices
 * only: the walks and scores a call returns do not depend on any of them
 * (tested).  These replace what earlier versions read from environment
 * variables, so the library reads no process-global state.               */
typedef struct gw_options_t {
  /* cap on the node2vec sampler's per-slot tables (bitset entries + regions,
   * listed entries, 16 B slot entries); 0 = half of the free HBM at prepare */
  int64_t table_budget_bytes;
  /* walk steps the caller intends to run on one gw_n2v_prepare; with
   * listed = -1, GW_N2V_REJECTION builds its 64 B listed entries only when
   * their modelled build time is paid back over these steps; 0 = unknown   */
  int64_t expected_steps;
  /* GW_N2V_REJECTION listed entries, considered for q < 1 only (never built
   * at q >= 1): -1 = by expected_steps (unknown: build whenever they fit),
   * 0 = never, 1 = whenever they fit                                       */
  int32_t listed;
  /* gw_simrank_naive input row: 0 = in LDS when it fits, 1 = in HBM (same
   * result bits; exists for tests and very large m)                        */
  int32_t simrank_hbm_row;
  /* gw_n2v_walks_host staging chunk in bytes; 0 = 256 MB                   */
  int64_t host_chunk_bytes;
  /* TopSim (pipelined kernel, STEP >= 4): a heavy source's key-hash
   * partitions get 2^-k of their room (0..8; 0 = all).  A partition that
   * fills makes the call re-run without the append path (same scores);
   * exists to test that fallback                                          */
  int32_t topsim_part_shrink;
  int32_t reserved0;  /* 0 */
} gw_options_t;

typedef struct gw_topsim_stats_t {
  int64_t extensions;   /* path extensions (queue.add, TopSim_singleSample.java:115,147) */
  int64_t pair_updates; /* executions of TopSim_singleSample.java:189                     */
  int64_t max_frontier; /* largest per-source level size seen                             */
  int64_t walkers;      /* random children spawned (mass < degree branch)                 */
} gw_topsim_stats_t;

/* ---- library -------------------------------------------------------------- */
const char* gw_version(void);
/* message of the last failing call made with this handle (NULL: the last
 * failing handle-less call on this thread).                                 */
const char* gw_last_error(const gw_graph* g);
const char* gw_strerror(int code);
/* number of visible GPUs (0 and GW_ERR_DEVICE when none)                    */
int gw_device_count(int* count);
/* The counter-based generator behind every scale-mode draw (Philox4x32-10,
 * Salmon et al. SC'11; csrc/gw_philox.h), so a host can reproduce the walks'
 * and TopSim's draws: for i < n, in[6i..6i+5] = (c0, c1, c2, c3, k0, k1) ->
 * out[4i..4i+3] = (x, y, z, w).  device >= 0 evaluates the kernels' own
 * device build on that GPU; device = -1 evaluates the same source on the host
 * (no GPU needed).  Replaces no reference symbol (the reference draws from
 * np.random / java.util.Random streams, node2vec.py:156-157, Graph.java:17);
 * pinned to Random123's published known-answer vectors (tests).            */
int gw_philox4x32(int device, const uint32_t* in, int64_t n, uint32_t* out);

/* ---- graph construction (host) ------------------------------------------ */
/* Replaces read_graph (node2vec/src/main.py:76-89, sem NX_SIMPLE) and
 * new structures.Graph(path, V) (Graph.java:28-42, sem JAVA_MULTI).
 * delim: separator string (NULL or "" = any whitespace, as nx delimiter=None).
 * vcount: JAVA_MULTI only (ids must lie in [0,vcount)); pass -1 otherwise.  */
int gw_graph_load_edgelist(const char* path, const char* delim, int semantics,
                           int directed, int weighted, int64_t vcount,
                           gw_graph** out);
/* Same semantics from in-memory edge arrays (labels for NX_SIMPLE, dense ids
 * for JAVA_MULTI).  w may be NULL (unweighted, every weight 1).             */
int gw_graph_from_edges(int64_t m, const int64_t* src, const int64_t* dst,
                        const double* w, int semantics, int directed,
                        int64_t vcount, gw_graph** out);
/* A graph whose semantics are already resolved by the caller (e.g. a
 * networkx graph handed to node2vec.Graph, node2vec.py:7-11): CSR over dense
 * ids with rows in draw order (NX_SIMPLE: sorted by dense id, dense id order
 * == label order), weights[nnz] (NULL = unweighted), labels[n] (NULL =
 * identity), node_order[n] = dense ids in G.nodes() order (NULL = 0..n-1). */
int gw_graph_from_csr(int64_t n, const int64_t* offsets, const int32_t* nbrs,
                      const double* weights, const int64_t* labels,
                      const int32_t* node_order, int semantics, int directed,
                      gw_graph** out);
/* Graph500 R-MAT (a,b,c; d = 1-a-b-c), 2^scale vertices, edge_factor*2^scale
 * generated edges, symmetrised, deduplicated, self-loops dropped, isolated
 * vertices removed; NX_SIMPLE semantics, labels = generator ids.  Philox
 * keyed by seed: identical on every host.                                   */
int gw_graph_rmat(int scale, int edge_factor, double a, double b, double c,
                  uint64_t seed, gw_graph** out);
/* R-MAT over an arbitrary vertex count n with m generated lines, Java
 * multigraph semantics (the reference generator's quadrant recursion,
 * RMATGraphGenerator.java:119-145; each line added both ways, duplicates and
 * self loops kept), V = n.  TopSim synthetic input (P10M: n=1e7, m=1e8).  */
int gw_graph_rmat_java(int64_t n, int64_t m, double a, double b, double c,
                       uint64_t seed, gw_graph** out);
int gw_graph_info(const gw_graph* g, gw_graph_info_t* info);
/* offsets[n+1], nbrs[nnz] (dense ids, row order = draw order), weights[nnz]
 * (NULL ok), labels[n] (NULL ok), node_order[n] (dense ids in the
 * reference's G.nodes() order; NULL ok).                                    */
int gw_graph_export_csr(const gw_graph* g, int64_t* offsets, int32_t* nbrs,
                        double* weights, int64_t* labels, int32_t* node_order);
int gw_graph_free(gw_graph* g);

/* Options of this handle (defaults: all zero, listed = -1); opt NULL resets
 * the defaults.  Take effect at the next call that uses them.               */
int gw_graph_set_options(gw_graph* g, const gw_options_t* opt);
int gw_graph_get_options(const gw_graph* g, gw_options_t* opt);

/* Upload CSR (+degree, weight sums) to HBM of `device`.                     */
int gw_graph_to_device(gw_graph* g, int device);

/* ---- node2vec (H1) ------------------------------------------------------- */
/* Replaces Graph.preprocess_transition_probs (node2vec.py:83-113): builds the
 * alias tables on the GPU (alias_setup node2vec.py:116-147, get_alias_edge
 * :61-81).  mode GW_N2V_REPLAY builds per-edge tables (bit-exact with the
 * reference); GW_N2V_REJECTION builds only what rejection sampling needs.   */
int gw_n2v_prepare(gw_graph* g, double p, double q, int mode);
/* Copy the alias tables back (node2vec.py:112-113 alias_nodes/alias_edges):
 * node_J/node_q [nnz] in CSR slot order; edge_off [nnz+1], edge_J/edge_q
 * [edge_alias_entries] (REPLAY only; pass NULL to skip).                    */
int gw_n2v_export_alias(const gw_graph* g, int32_t* node_J, double* node_q,
                        int64_t* edge_off, int32_t* edge_J, double* edge_q);
/* Standalone alias_setup (node2vec.py:116-147) of one distribution on the
 * GPU: J[K], q[K] (J as int64 like np.int).                                 */
int gw_alias_setup(int device, const double* probs, int64_t K, int64_t* J,
                   double* q);

/* Exact reference replay of Graph.simulate_walks/node2vec_walk
 * (node2vec.py:13-59) for nwalks walks whose start vertices (dense ids, the
 * shuffled orders concatenated iteration-major) are given, consuming the
 * caller's uniform stream (np.random.rand() values in draw order, 2 per
 * step).  Host buffers: out_walks[nwalks*walk_len] (dense ids, -1 padded),
 * out_len[nwalks]; *uniforms_used = values consumed.  Requires
 * gw_n2v_prepare(..., GW_N2V_REPLAY).                                        */
int gw_n2v_walks_replay(gw_graph* g, int walk_len, int64_t nwalks,
                        const int32_t* starts, const double* uniforms,
                        int64_t n_uniforms, int32_t* out_walks, int32_t* out_len,
                        int64_t* uniforms_used);

/* Scale-mode walks (GW_N2V_REJECTION or REPLAY tables), device-resident.
 * Global walk index w in [walk_begin, walk_begin+walk_count): iteration
 * it = w / n, start = node_order[perm_it(w % n)] (shuffle != 0; perm is the
 * keyed Feistel bijection) or node_order[w % n] (shuffle == 0).  Output
 * row-major [walk_count][walk_len] dense ids (-1 padded), lens optional.
 * counters_dev (optional, 2 x uint64): += steps taken, += rejection trials. */
int gw_n2v_walks(gw_graph* g, int walk_len, uint64_t seed, int64_t walk_begin,
                 int64_t walk_count, int shuffle, int32_t* out_walks_dev,
                 int32_t* out_len_dev, uint64_t* counters_dev, void* stream);

/* Host-buffer form of gw_n2v_walks (stages through HBM in ~1 GB chunks and
 * synchronises): out_walks[walk_count*walk_len], out_len[walk_count] (NULL
 * ok), counters[2] (NULL ok).  For JNI / CLI callers.                       */
int gw_n2v_walks_host(gw_graph* g, int walk_len, uint64_t seed,
                      int64_t walk_begin, int64_t walk_count, int shuffle,
                      int32_t* out_walks, int32_t* out_len, uint64_t* counters);

/* ---- TopSim (H2) ------------------------------------------------------------ */
/* Allocate the per-workgroup workspace for up to `sample`/`step` (kept in the
 * handle; sizes the level arrays and the accumulator rows).                 */
int gw_topsim_prepare(gw_graph* g, int variant, int sample, int step, int topk);
/* Name of the kernel the handle's prepared TopSim workspace launches (e.g.
 * "k_topsim_pipe<5>", "k_topsim_2wg<5, 2>", "k_topsim_pipe_row<5>"; "" before
 * the first gw_topsim_prepare / gw_topsim* call).  Diagnostic: the choice
 * depends on V, SAMPLE and STEP (no reference counterpart).                 */
const char* gw_topsim_kernel(const gw_graph* g);
/* Registers per lane, private segment (scratch) bytes per lane and LDS bytes
 * per workgroup (static + dynamic) of that kernel (hipFuncGetAttributes).   */
int gw_topsim_kernel_attrs(gw_graph* g, int32_t* vgprs, int32_t* scratch_bytes, int32_t* lds_bytes);
/* Replaces new TopSim_singleSample(g, sample, step).compute() +
 * Print.printByOrder's per-row FixedMaxPQ (TopSim_singleSample.java:35-54,
 * Print.java:25-53) for the given sources: out_ids_dev[nsrc*topk],
 * out_scores_dev[nsrc*topk], rows sorted by score desc then id asc, padded
 * with (-1, 0.0).  Scores are NOT divided by sample for SINGLE_SAMPLE /
 * ENUMERATE (as the reference); SINGLE_RW divides (SingleRandomWalk.java:89).
 * C: decay (MyConfiguration.C = 0.6).  stats_dev (optional, 4 x int64):
 * gw_topsim_stats_t accumulated on the device.                              */
int gw_topsim(gw_graph* g, int variant, int sample, int step, double C,
              uint64_t seed, const int32_t* sources_dev, int64_t nsrc, int topk,
              int32_t* out_ids_dev, double* out_scores_dev, int64_t* stats_dev,
              void* stream);
/* Dense rows for small graphs (getResult(), TopSim_singleSample.java:235):
 * out_rows_dev[nsrc*n] doubles, row r = sim[sources[r]][*], diagonal 0.     */
int gw_topsim_dense(gw_graph* g, int variant, int sample, int step, double C,
                    uint64_t seed, const int32_t* sources_dev, int64_t nsrc,
                    double* out_rows_dev, int64_t* stats_dev, void* stream);

/* Sparse rows, the input of the Java-exact writer at any V (Print.java:25-53
 * needs every nonzero score of a row, not only its top k): per source r its
 * nonzero entries sim[sources[r]][id] > 0, in no particular order, at
 * out_ids_dev / out_scores_dev[row_begin_dev[r] .. + row_len_dev[r]).  Rows
 * are packed at offsets claimed in completion order, up to `capacity`
 * entries; *used_dev (one int64, zeroed by the call) ends as the room ALL rows
 * needed.  A row that did not fit gets row_begin = row_len = -1 and the call
 * returns GW_ERR_CAPACITY (re-run with capacity >= *used).  Same walks, sums
 * and stats as gw_topsim; synchronises the stream.                          */
int gw_topsim_sparse(gw_graph* g, int variant, int sample, int step, double C,
                     uint64_t seed, const int32_t* sources_dev, int64_t nsrc,
                     int64_t capacity, int64_t* row_begin_dev,
                     int32_t* row_len_dev, int32_t* out_ids_dev,
                     double* out_scores_dev, int64_t* used_dev,
                     int64_t* stats_dev, void* stream);
/* new TopSim_singleSample(g, sample, step).compute() followed by
 * Print.printByOrder(sim, path, topk, ...) (TopSim_singleSample.java:47-54,
 * Print.java:25-53) for the given sources (host array), Java-exact at any V:
 * batches of sparse rows replayed through FixedMaxPQ on the host, rows
 * written in source order.  Writes path and path+".sim.txt" (sep, %.<decimals>f);
 * stats[4] optional.                                                        */
int gw_topsim_write_text(gw_graph* g, int variant, int sample, int step,
                         double C, uint64_t seed, const int32_t* sources,
                         int64_t nsrc, int topk, const char* path,
                         const char* sep, int decimals, int64_t* stats);

/* Host-buffer form of gw_topsim / gw_topsim_dense for JNI and C++ callers:
 * sources[nsrc] on the host; either out_rows[nsrc*n] (dense, getResult())
 * or out_ids/out_scores[nsrc*topk] (top-k); stats[4] optional.            */
int gw_topsim_host(gw_graph* g, int variant, int sample, int step, double C,
                   uint64_t seed, const int32_t* sources, int64_t nsrc,
                   int topk, int32_t* out_ids, double* out_scores,
                   double* out_rows, int64_t* stats);

/* ---- bounded-memory variants with FixedCacheMap (§8f-3) -------------------- */
/* Replaces new TopSim_singleSample_M(g, M, sample).compute() (variant
 * GW_TOPSIM_SINGLE_SAMPLE; TopSim_singleSample_M.java:33-239, the reference
 * fixes STEP = 5) and new SingleRandomWalk_M(g, M, sample).compute()
 * (GW_TOPSIM_SINGLE_RW; SingleRandomWalk_M.java:24-92): every pair update
 * (float)(... / SAMPLE) is put() into a lxctools.FixedCacheMap(capacity =
 * TOPK*M) in the reference's order (FixedCacheMap.java:32-50: add to a
 * present key, insert while not full, else replace the minimum when larger).
 * Per source r the map is then iterated (delMin, ascending) into
 * out_keys_dev/out_vals_dev[r*capacity + i], i < out_size_dev[r] (-1 / 0
 * padded).  Same Philox walks as gw_topsim.  capacity <= 4096.             */
int gw_topsim_m(gw_graph* g, int variant, int capacity, int sample, int step,
                double C, uint64_t seed, const int32_t* sources_dev, int64_t nsrc,
                int32_t* out_keys_dev, float* out_vals_dev, int32_t* out_size_dev,
                int64_t* stats_dev, void* stream);
/* Host-buffer form (synchronous).                                           */
int gw_topsim_m_host(gw_graph* g, int variant, int capacity, int sample,
                     int step, double C, uint64_t seed, const int32_t* sources,
                     int64_t nsrc, int32_t* out_keys, float* out_vals,
                     int32_t* out_size, int64_t* stats);

/* ---- double-walk variants (§8f-4) ------------------------------------------ */
/* kinds for gw_double_sim_host                                              */
#define GW_DOUBLE_SAMPLE 0      /* TopSim_doubleSample */
#define GW_DOUBLE_DEV 1         /* TopSim_Dev          */
#define GW_DOUBLE_RANDOM_WALK 2 /* DoubleRandomWalk    */
/* Replaces new TopSim_doubleSample(g, sample, step).compute() + getResult()
 * (TopSim_doubleSample.java:30-197): per vertex the TopSim BFS over `step`
 * levels, paths[src][target][s] = mass of the LAST queued path reaching
 * target at level s; sim[i][j] = sum_x sum_s C^s P[i][x][s] P[j][x][s]
 * (i < j, mirrored, diag 0).  sim_dev[n*n]; Philox keys as gw_topsim.       */
int gw_topsim_double(gw_graph* g, int sample, int step, double C,
                     uint64_t seed, double* sim_dev, void* stream);
/* Replaces new TopSim_Dev(g, sample, step, topK, singleStep).compute(cand)
 * (TopSim_Dev.java:31-95): SAMPLE = (int)((step-singleStep)*sample*2 /
 * (step*(topK+1))); for every i its candidates cand_dev[i*topK + r] (as
 * gw_select_fixed_max_pq gives them, -1 padded) are each freshly sampled
 * (Philox call 1 + i*topK + r) and sim[i][j] = getSim; other entries 0.    */
int gw_topsim_dev(gw_graph* g, int sample, int step, int topK, int singleStep,
                  double C, uint64_t seed, const int32_t* cand_dev,
                  double* sim_dev, void* stream);
/* Replaces new DoubleRandomWalk(g, sample, step).compute()
 * (DoubleRandomWalk.java:25-91): `sample` uniform walks of `step` steps per
 * vertex, sim[v][w] = sum over walk pairs of C^(t+1) at their first meeting
 * step t, / sample^2 (v < w, mirrored, diag 0).                            */
int gw_double_random_walk(gw_graph* g, int sample, int step, double C,
                          uint64_t seed, double* sim_dev, void* stream);
/* Host-buffer form of the three (kind = GW_DOUBLE_*): sim[n*n] on the host,
 * cand[n*topK] on the host for GW_DOUBLE_DEV (ignored otherwise).           */
int gw_double_sim_host(gw_graph* g, int kind, int sample, int step, int topK,
                       int singleStep, double C, uint64_t seed,
                       const int32_t* cand, double* sim);
/* TopSim_Dev's candidate choice (TopSim_Dev.java:64-71): per row a
 * FixedMaxPQ(k) offered every (j, rows[r][j] >= min_score) in j order, then
 * sortedElement() -> out_ids[r*k + i] (-1 padded).  Host code.             */
int gw_select_fixed_max_pq(const double* rows, int64_t nrows, int64_t n, int k,
                           double min_score, int32_t* out_ids);
/* Java's Double.toString of v (string concatenation "" + v), as
 * Eval.precision writes its scores (Eval.java:118, :128): shortest round-trip
 * digits, plain for 1e-3 <= |v| < 1e7 (at least one fraction digit), else
 * "d.dddE[-]n".  NUL-terminated into buf[buflen]; GW_ERR_RANGE if too small. */
int gw_format_java_double(double v, char* buf, int64_t buflen);

/* ---- naive SimRank (TopSim ground truth) ------------------------------------ */
/* Replaces new SimRank(g).compute() + getResult() (SimRank.java:21-57, 79):
 * S := I; `iters` rounds (the reference's STEP = 3) of
 *   S'[v][w] = C * sum_{a in N(v), b in N(w)} S[a][b] / (deg(v)*deg(w)),
 * S'[v][v] = 1, 0 for isolated v or w; then diag := 0 (postProcess, :62-65).
 * sim_dev: n*n doubles row-major on the graph's device (symmetric).  Needs an
 * undirected graph (Java multigraph: duplicate entries count).  The n*n fp64
 * workspace is kept in the handle.  fp64 result equals the reference up to
 * summation order (tested at rtol 1e-12).                                   */
int gw_simrank_naive(gw_graph* g, double C, int iters, double* sim_dev,
                     void* stream);
/* Host-buffer form (synchronous): sim[n*n].                                 */
int gw_simrank_naive_host(gw_graph* g, double C, int iters, double* sim);

/* ---- output writers (host) ------------------------------------------------ */
/* DeepSim save_list format (DeepSim/src/main.py:237-243): one walk per line,
 * every label followed by '\t', then '\n'.  walks: dense ids (-1 padded).   */
int gw_write_walks_text(const gw_graph* g, const char* path,
                        const int32_t* walks, const int32_t* lens,
                        int64_t nwalks, int walk_len);
/* Print.printByOrder format (Print.java:25-53): per row "v,id,id,...\r\n" to
 * path and "v,id:%.6f,...\r\n" to path+".sim.txt".  Rows come from dense
 * score rows (java_exact: emulate FixedMaxPQ/PriorityQueue tie order and
 * Java's HALF_UP %.6f exactly) given as [nrows][n] host doubles.            */
int gw_write_sim_text_dense(const char* path, const double* rows,
                            const int32_t* row_ids, int64_t nrows, int64_t n,
                            int topk, const char* sep, int decimals);
/* Same format from sparse rows (gw_topsim_sparse, copied to the host): row r
 * = sim[row_ids[r]][*] with the listed nonzero entries and 0.0 elsewhere
 * (n columns).  FixedMaxPQ(topk) is replayed exactly — the first min(topk, n)
 * ids fill the heap (zero scores included), later offers enter only when
 * strictly larger than the heap minimum — and written in sortedElement()
 * order: min(topk, n) entries per row, byte-identical to
 * gw_write_sim_text_dense on the same rows.                                */
int gw_write_sim_text_sparse(const char* path, const int64_t* row_begin,
                             const int32_t* row_len, const int32_t* ids,
                             const double* scores, const int32_t* row_ids,
                             int64_t nrows, int64_t n, int topk,
                             const char* sep, int decimals);
/* Same format from top-k rows as produced by gw_topsim (score desc, id asc,
 * -1 padding dropped).  NOT Java-exact: a top-k row carries neither the
 * zero-score ids FixedMaxPQ keeps when a row has fewer than topk nonzeros
 * nor the heap history that orders ties; use gw_write_sim_text_sparse /
 * gw_topsim_write_text for the reference's bytes.                          */
int gw_write_sim_text_topk(const char* path, const int32_t* ids,
                           const double* scores, const int32_t* row_ids,
                           int64_t nrows, int topk, const char* sep,
                           int decimals);

/* Print.printByOrder(FixedCacheMap[] sim, outPath, topk) (Print.java:94-124):
 * per row the last `topk` entries of the ascending iteration, "%.6f" of the
 * float values; rows as produced by gw_topsim_m.                            */
int gw_write_sim_text_cachemap(const char* path, const int32_t* keys,
                               const float* vals, const int32_t* sizes,
                               const int32_t* row_ids, int64_t nrows,
                               int capacity, int topk, const char* sep);

/* ---- multi-GPU exchange (RCCL over xGMI) ---------------------------------- */
/* the graph is replicated and units (walks, TopSim sources) are
 * sharded by global index with no data-path collective; the only exchange is
 * an all-gather of emitted blocks for hosts that need every walk on every
 * rank.  One process (or thread) per GPU; RCCL (librccl.so.1) is loaded on
 * first use, so the library itself carries no link-time RCCL dependency.
 * Rank 0 calls gw_comm_unique_id and hands the GW_COMM_ID_BYTES bytes to the
 * other ranks out of band (MPI, a file, torch.distributed, ...).            */
#define GW_COMM_ID_BYTES 128
#define GW_DTYPE_I32 0
#define GW_DTYPE_F64 1
typedef struct gw_comm gw_comm;
int gw_comm_unique_id(uint8_t* id);
int gw_comm_init(const uint8_t* id, int nranks, int rank, int device, gw_comm** out);
/* recv_dev[nranks * count] = concatenation of every rank's send_dev[count]
 * in rank order (ncclAllGather); asynchronous on `stream` (NULL = default). */
int gw_comm_allgather(gw_comm* c, const void* send_dev, void* recv_dev, int64_t count, int dtype, void* stream);
int gw_comm_free(gw_comm* c);
const char* gw_comm_last_error(const gw_comm* c);

#ifdef __cplusplus
}
#endif
#endif /* GRAPHWALK_H */
