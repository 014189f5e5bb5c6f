/*
 * oracle.c — CPU restatement of the reference algorithms on the hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so; nothing on the product
 * path (graph-embedding_amd/) links or calls it.
 *
 * Each function names the reference lines it restates (paths relative to the
 * reference checkout).  Pinning (see DESIGN.md "Oracle"):
 *   - or_alias_setup / or_alias_nodes / or_alias_edges / or_walks_replay are
 *     checked bit-for-bit against golden vectors produced by importing the
 *     reference node2vec.py (oracle/gen_goldens.py -> tests/golden/).
 *   - or_simrank_naive is checked against the reference's committed naive
 *     SimRank output IsoMap_LE/data/0_333_5038_simrank_navie_top10.txt.sim.txt.
 *   - or_topsim (deterministic regime) is checked against or_simrank_naive
 *     truncated at STEP iterations (exact KAT).  In the random
 *     regime the reference's RNG is an unseeded java.util.Random, so the
 *     Philox-keyed restatement here is the GPU's parity target and
 *     or_topsim_java (java.util.Random stream) is used statistically.
 *   - or_walks_scale restates the scale-mode sampling design (rejection
 *     sampling of the node2vec.py:61-81 bias, and for unweighted undirected
 *     graphs at q > 1 its exact mixture form); its distribution is checked
 *     against exact per-edge probabilities in tests.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../graph-embedding_amd/csrc/gw_philox.h"

/* ------------------------------------------------------------------------ */
/* node2vec.py:116-147 alias_setup                                           */
/* ------------------------------------------------------------------------ */
void or_alias_setup(const double* probs, int64_t K, int64_t* J, double* q) {
  int64_t* smaller = (int64_t*)malloc(sizeof(int64_t) * (K + 1));
  int64_t* larger = (int64_t*)malloc(sizeof(int64_t) * (K + 1));
  int64_t ns = 0, nl = 0;
  for (int64_t kk = 0; kk < K; ++kk) { /* :127-132 */
    J[kk] = 0;
    q[kk] = (double)K * probs[kk];
    if (q[kk] < 1.0)
      smaller[ns++] = kk;
    else
      larger[nl++] = kk;
  }
  while (ns > 0 && nl > 0) { /* :134-143 */
    int64_t small = smaller[--ns];
    int64_t large = larger[--nl];
    J[small] = large;
    q[large] = q[large] + q[small] - 1.0;
    if (q[large] < 1.0)
      smaller[ns++] = large;
    else
      larger[nl++] = large;
  }
  free(smaller);
  free(larger);
}

/* node2vec.py:91-97: per node, probs = w / sum(w) over sorted neighbours */
void or_alias_nodes(int64_t n, const int64_t* off, const double* w, int64_t* J, double* q) {
  for (int64_t v = 0; v < n; ++v) {
    int64_t b = off[v], K = off[v + 1] - off[v];
    if (!K) continue;
    double norm = 0.0;
    for (int64_t k = 0; k < K; ++k) norm += w ? w[b + k] : 1.0;
    double* pr = (double*)malloc(sizeof(double) * K);
    for (int64_t k = 0; k < K; ++k) pr[k] = (w ? w[b + k] : 1.0) / norm;
    or_alias_setup(pr, K, J + b, q + b);
    free(pr);
  }
}

static int has_edge(const int64_t* off, const int32_t* nbrs, int32_t a, int32_t b) {
  int64_t lo = off[a], hi = off[a + 1];
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (nbrs[mid] < b)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < off[a + 1] && nbrs[lo] == b;
}

/* sizes of the per-edge tables: slot e = (u -> v) holds a table over N(v) */
int64_t or_alias_edges_offsets(int64_t n, const int64_t* off, const int32_t* nbrs, int64_t* eoff) {
  int64_t acc = 0, e = 0;
  for (int64_t u = 0; u < n; ++u)
    for (int64_t k = off[u]; k < off[u + 1]; ++k, ++e) {
      eoff[e] = acc;
      acc += off[nbrs[k] + 1] - off[nbrs[k]];
    }
  eoff[e] = acc;
  return acc;
}

/* node2vec.py:61-81 get_alias_edge for every slot (src=u, dst=v) */
void or_alias_edges(int64_t n, const int64_t* off, const int32_t* nbrs, const double* w, double p,
                    double q, const int64_t* eoff, int64_t* J, double* qq) {
  int64_t e = 0;
  for (int64_t src = 0; src < n; ++src)
    for (int64_t k = off[src]; k < off[src + 1]; ++k, ++e) {
      int32_t dst = nbrs[k];
      int64_t db = off[dst], K = off[dst + 1] - off[dst];
      if (!K) continue;
      double* un = (double*)malloc(sizeof(double) * K);
      double norm = 0.0;
      for (int64_t j = 0; j < K; ++j) {
        int32_t x = nbrs[db + j];
        double wx = w ? w[db + j] : 1.0;
        if (x == src)
          un[j] = wx / p;
        else if (has_edge(off, nbrs, x, (int32_t)src))
          un[j] = wx;
        else
          un[j] = wx / q;
        norm += un[j];
      }
      for (int64_t j = 0; j < K; ++j) un[j] = un[j] / norm;
      or_alias_setup(un, K, J + eoff[e], qq + eoff[e]);
      free(un);
    }
}

/* ------------------------------------------------------------------------ */
/* node2vec.py:13-59 walks with a caller-supplied uniform stream (exact)     */
/* sequential: walk w consumes its draws right after walk w-1                */
/* ------------------------------------------------------------------------ */
int64_t or_walks_replay(int64_t n, const int64_t* off, const int32_t* nbrs, const int64_t* nJ,
                        const double* nq, const int64_t* eoff, const int64_t* eJ, const double* eq,
                        int L, int64_t nwalks, const int32_t* starts, const double* U, int64_t nU,
                        int32_t* out, int32_t* lens) {
  (void)n;
  int64_t o = 0;
  for (int64_t w = 0; w < nwalks; ++w) {
    int32_t* row = out + w * (int64_t)L;
    int32_t cur = starts[w];
    int len = 1;
    int64_t slot = -1;
    row[0] = cur;
    while (len < L) { /* :23-38 */
      int64_t b = off[cur], d = off[cur + 1] - off[cur];
      if (d == 0) break;
      if (o + 2 > nU) return -1;
      double u1 = U[o++], u2 = U[o++];
      int64_t kk = (int64_t)floor(u1 * (double)d); /* alias_draw :156 */
      const int64_t* J;
      const double* q;
      if (len == 1) {
        J = nJ + b;
        q = nq + b;
      } else {
        J = eJ + eoff[slot];
        q = eq + eoff[slot];
      }
      int64_t idx = (u2 < q[kk]) ? kk : J[kk]; /* :157-160 */
      slot = b + idx;
      cur = nbrs[slot];
      row[len++] = cur;
    }
    for (int t = len; t < L; ++t) row[t] = -1;
    lens[w] = len;
  }
  return o;
}

/* ------------------------------------------------------------------------ */
/* scale mode (Philox): restatement of the sampling design used on the GPU:  */
/* first-order proposal from the node distribution, exact second-order bias  */
/* of node2vec.py:61-81 by rejection with the return edge as an outlier.     */
/* ------------------------------------------------------------------------ */
static int64_t find_slot(const int64_t* off, const int32_t* nbrs, int32_t row, int32_t key) {
  int64_t lo = off[row], hi = off[row + 1];
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (nbrs[mid] < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < off[row + 1] && nbrs[lo] == key) ? lo : -1;
}

void or_walks_scale(int64_t n, const int64_t* off, const int32_t* nbrs, const double* w,
                    const double* wsum, const int32_t* nJ, const double* nq, const int32_t* order,
                    int directed, double p, double q, uint64_t seed, int L, int64_t walk_begin,
                    int64_t walk_count, int shuffle, int32_t* out, int32_t* lens, uint64_t* counters,
                    int nthreads) {
  const int first_order = (p == 1.0 && q == 1.0);
  const double a_p = 1.0 / p, a_q = 1.0 / q;
  const double M = a_q > 1.0 ? a_q : 1.0;
  const double lo = a_q < 1.0 ? a_q : 1.0;
  const double extra = a_p > M ? a_p - M : 0.0;
  const double h_prev = a_p < M ? a_p : M;
  /* mixture proposal for unweighted undirected graphs at q > 1 (w = 1/q on
   * N(cur) + (1 - 1/q) on N(prev) + the return outlier), taken by a step
   * iff deg(prev) < deg(cur): see k_walk_scale (gw_n2v.hip) */
  const int mix = !w && !directed && a_q < 1.0;
  const double mix_o = a_p - a_q > 0.0 ? a_p - a_q : 0.0;
  const double mix_p = 1.0 - a_q;
  const double mix_prev = a_p / a_q < 1.0 ? a_p / a_q : 1.0;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_STEP;
  const uint32_t pk0 = (uint32_t)seed, pk1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_PERM;
  uint64_t tot_steps = 0, tot_trials = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : tot_steps, tot_trials)
#endif
  for (int64_t i = 0; i < walk_count; ++i) {
    const int64_t wi = walk_begin + i;
    const uint64_t it = (uint64_t)wi / (uint64_t)n, pos = (uint64_t)wi % (uint64_t)n;
    const uint64_t sp = shuffle ? gw_feistel_perm(pos, (uint64_t)n, pk0, pk1, (uint32_t)it) : pos;
    int32_t cur = order[sp], prev = -1;
    double w_back = 1.0;
    int back_ok = 0;
    int32_t* row = out + i * (int64_t)L;
    row[0] = cur;
    int len = 1;
    const uint32_t c0 = (uint32_t)wi, c1 = (uint32_t)((uint64_t)wi >> 32);
    while (len < L) {
      const int64_t b = off[cur], d = off[cur + 1] - b;
      if (d == 0) break;
      int64_t slot;
      int32_t next;
      if (first_order || len == 1) {
        struct gw_u4 u = gw_philox(c0, c1, (uint32_t)len, 0u, k0, k1);
        ++tot_trials;
        int64_t kk = gw_index(u.x, u.z, (uint32_t)d);
        if (w) kk = (gw_u01(u.y) < nq[b + kk]) ? kk : nJ[b + kk];
        slot = b + kk;
        next = nbrs[slot];
      } else if (mix && off[prev + 1] - off[prev] < d) {
        const int64_t pb = off[prev], dp = off[prev + 1] - pb;
        const double Ac = (double)d * a_q;
        const double H = mix_o + Ac + (double)dp * mix_p;
        uint32_t trial = 0;
        for (;;) {
          struct gw_u4 u = gw_philox(c0, c1, (uint32_t)len, trial, k0, k1);
          ++trial;
          const double r = gw_u01(u.z) * H;
          if (r < mix_o) { /* return-edge outlier */
            slot = -1;
            next = prev;
            break;
          }
          const int from_cur = r < mix_o + Ac;
          const int64_t s = (from_cur ? b : pb) + (int64_t)gw_index(u.x, u.y, (uint32_t)(from_cur ? d : dp));
          const int32_t x = nbrs[s];
          int acc;
          if (from_cur)
            acc = x != prev || gw_u01(u.w) < mix_prev;
          else
            acc = x != prev && find_slot(off, nbrs, cur, x) >= 0; /* x in N(cur) */
          if (trial >= (1u << 24) && from_cur) acc = 1;
          if (acc) {
            slot = s;
            next = x;
            break;
          }
        }
        tot_trials += trial;
      } else {
        const double Wc = w ? wsum[cur] : (double)d;
        const double oa = (back_ok && extra > 0.0) ? extra * w_back : 0.0;
        const double A = M * Wc + oa;
        uint32_t trial = 0;
        for (;;) {
          struct gw_u4 u = gw_philox(c0, c1, (uint32_t)len, trial, k0, k1);
          ++trial;
          if (oa > 0.0 && gw_u01(u.z) * A < oa) {
            slot = -1;
            next = prev;
            break;
          }
          /* low word of the 64-bit index draw: u.y unweighted, else one more Philox block */
          const uint32_t ulo = w ? gw_philox(c0, c1, (uint32_t)len, (trial - 1u) | 0x80000000u, k0, k1).x : u.y;
          int64_t kk = gw_index(u.x, ulo, (uint32_t)d);
          if (w) kk = (gw_u01(u.y) < nq[b + kk]) ? kk : nJ[b + kk];
          const int64_t s = b + kk;
          const int32_t x = nbrs[s];
          const double t = gw_u01(u.w) * M;
          int acc;
          if (x == prev)
            acc = t < h_prev;
          else if (t < lo)
            acc = 1;
          else {
            int adj = directed ? (find_slot(off, nbrs, x, prev) >= 0)
                               : (find_slot(off, nbrs, prev, x) >= 0);
            acc = t < (adj ? 1.0 : a_q);
          }
          if (acc || trial >= (1u << 24)) {
            slot = s;
            next = x;
            break;
          }
        }
        tot_trials += trial;
      }
      if (directed) {
        if (!first_order && extra > 0.0) {
          int64_t bs = find_slot(off, nbrs, next, cur);
          back_ok = bs >= 0;
          w_back = (back_ok && w) ? w[bs] : 1.0;
        }
      } else if (slot >= 0) {
        back_ok = 1;
        w_back = w ? w[slot] : 1.0;
      }
      prev = cur;
      cur = next;
      row[len++] = cur;
    }
    for (int t = len; t < L; ++t) row[t] = -1;
    if (lens) lens[i] = len;
    tot_steps += (uint64_t)(len - 1);
  }
  if (counters) {
    counters[0] += tot_steps;
    counters[1] += tot_trials;
  }
}

/* ------------------------------------------------------------------------ */
/* java.util.Random (JDK 8): LCG48, next(bits), nextInt(bound)               */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint64_t seed;
} jrand;
void or_jrand_init(jrand* r, int64_t s) { r->seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
static int32_t jrand_next(jrand* r, int bits) {
  r->seed = (r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(int64_t)(r->seed >> (48 - bits));
}
int32_t or_jrand_next_int(jrand* r, int32_t bound) {
  if ((bound & -bound) == bound) return (int32_t)(((int64_t)bound * (int64_t)jrand_next(r, 31)) >> 31);
  int32_t bits, val;
  do {
    bits = jrand_next(r, 31);
    val = bits % bound;
  } while (bits - val + (bound - 1) < 0);
  return val;
}
/* exposed for tests: first k nextInt(bound) values from new Random(seed) */
void or_jrand_sequence(int64_t seed, int32_t bound, int64_t k, int32_t* out) {
  jrand r;
  or_jrand_init(&r, seed);
  for (int64_t i = 0; i < k; ++i) out[i] = or_jrand_next_int(&r, bound);
}

/* ------------------------------------------------------------------------ */
/* TopSim_singleSample.walk / computePathSim (TopSim_singleSample.java:62-203)
 * restated literally as a FIFO queue of paths, one source at a time.
 * variant 0: singleSample (:99 mass >= degree -> enumerate; else ceil(mass)
 *            random children), 1: Enumerate (TopSim_Enumerate.java:99
 *            always enumerate), 2: SingleRandomWalk (SingleRandomWalk.java).
 * rng 0: Philox keyed by (source, walker index, level) with walker indices
 *        assigned in queue order when a path first takes the random branch;
 * rng 1: java.util.Random stream (seeded with java_seed, shared across
 *        sources in source order, as Graph.rand is static).               */
/* ------------------------------------------------------------------------ */
typedef struct {
  int32_t* cur;    /* [cap][L+1] */
  double* mass;    /* [cap][L+1] */
  int64_t* walker; /* [cap]      */
  int64_t size, cap;
} pqueue;

static void pq_reserve(pqueue* q, int64_t need, int L) {
  if (need <= q->cap) return;
  int64_t nc = q->cap ? q->cap : 1024;
  while (nc < need) nc *= 2;
  q->cur = (int32_t*)realloc(q->cur, sizeof(int32_t) * nc * (L + 1));
  q->mass = (double*)realloc(q->mass, sizeof(double) * nc * (L + 1));
  q->walker = (int64_t*)realloc(q->walker, sizeof(int64_t) * nc);
  q->cap = nc;
}

static int first_meet(const int32_t* path, int dst) { /* isFirstMeet(path, 0, dst) :211-218 */
  int internal = dst / 2;
  for (int i = 0; i < internal; ++i)
    if (path[i] == path[dst - i]) return 0;
  return 1;
}

/* lxctools.FixedCacheMap (FixedCacheMap.java:14-110), literal: 1-based  */
/* min-heap on float values, key2Index map, sink/swim/exch as in Java.     */
typedef struct {
  int NMAX, N;
  int32_t* keys;
  float* vals;
  int32_t* hk; /* hash: key -> heap index (stands in for HashMap<Integer,Short>) */
  int32_t* hv;
  int hmask;
} fcm;

static void fcm_init(fcm* m, int nmax) {
  m->NMAX = nmax;
  m->N = 0;
  m->keys = (int32_t*)calloc((size_t)nmax + 1, sizeof(int32_t));
  m->vals = (float*)calloc((size_t)nmax + 1, sizeof(float));
  int hs = 4;
  while (hs < 4 * (nmax + 1)) hs <<= 1;
  m->hmask = hs - 1;
  m->hk = (int32_t*)malloc(sizeof(int32_t) * hs);
  m->hv = (int32_t*)malloc(sizeof(int32_t) * hs);
  for (int i = 0; i < hs; ++i) m->hk[i] = -1;
}
static void fcm_free(fcm* m) { free(m->keys); free(m->vals); free(m->hk); free(m->hv); }
static void fcm_clear(fcm* m) {
  m->N = 0;
  for (int i = 0; i <= m->hmask; ++i) m->hk[i] = -1;
}
static uint32_t fcm_h(int32_t k) { return (uint32_t)k * 0x9E3779B1u; }
static int fcm_get(const fcm* m, int32_t k) {
  for (uint32_t h = fcm_h(k) & m->hmask;; h = (h + 1) & m->hmask) {
    if (m->hk[h] == k) return m->hv[h];
    if (m->hk[h] == -1) return -1;
  }
}
static void fcm_hput(fcm* m, int32_t k, int v) {
  uint32_t h = fcm_h(k) & m->hmask;
  while (m->hk[h] != -1 && m->hk[h] != k) h = (h + 1) & m->hmask;
  m->hk[h] = k;
  m->hv[h] = v;
}
static void fcm_hdel(fcm* m, int32_t k) { /* linear probing, backward-shift delete */
  uint32_t h = fcm_h(k) & m->hmask;
  while (m->hk[h] != k) {
    if (m->hk[h] == -1) return;
    h = (h + 1) & m->hmask;
  }
  uint32_t i = h;
  for (;;) {
    m->hk[i] = -1;
    uint32_t j = i;
    for (;;) {
      j = (j + 1) & m->hmask;
      if (m->hk[j] == -1) return;
      uint32_t home = fcm_h(m->hk[j]) & m->hmask;
      /* move j back to i when home is not cyclically in (i, j] */
      int in = (i <= j) ? (home > i && home <= j) : (home > i || home <= j);
      if (!in) break;
    }
    m->hk[i] = m->hk[j];
    m->hv[i] = m->hv[j];
    i = j;
  }
}
static void fcm_exch(fcm* m, int a, int b) { /* :86-98 */
  fcm_hput(m, m->keys[a], b);
  fcm_hput(m, m->keys[b], a);
  int32_t tk = m->keys[a];
  m->keys[a] = m->keys[b];
  m->keys[b] = tk;
  float tv = m->vals[a];
  m->vals[a] = m->vals[b];
  m->vals[b] = tv;
}
static void fcm_sink(fcm* m, int i) { /* :61-69 */
  while (2 * i <= m->N) {
    int j = 2 * i;
    if (j < m->N && m->vals[j] > m->vals[j + 1]) j++;
    if (!(m->vals[i] > m->vals[j])) break;
    fcm_exch(m, i, j);
    i = j;
  }
}
static void fcm_swim(fcm* m, int i) { /* :73-78 */
  while (i > 1 && m->vals[i / 2] > m->vals[i]) {
    fcm_exch(m, i, i / 2);
    i = i / 2;
  }
}
static void fcm_put(fcm* m, int32_t key, float value) { /* :32-50 */
  int idx = fcm_get(m, key);
  if (idx >= 0) {
    m->vals[idx] += value;
    fcm_sink(m, idx);
  } else if (m->N < m->NMAX) {
    m->N++;
    m->keys[m->N] = key;
    m->vals[m->N] = value;
    fcm_hput(m, key, m->N);
    fcm_swim(m, m->N);
  } else if (value > m->vals[1]) {
    fcm_hdel(m, m->keys[1]);
    m->keys[1] = key;
    m->vals[1] = value;
    fcm_hput(m, key, 1);
    fcm_sink(m, 1);
  }
}
/* iteration = repeated delMin (:104-127): ascending order, empties the map */
static int fcm_drain(fcm* m, int32_t* ok, float* ov) {
  int c = 0;
  while (m->N > 0) {
    ok[c] = m->keys[1];
    ov[c] = m->vals[1];
    c++;
    fcm_hdel(m, m->keys[1]);
    fcm_exch(m, 1, m->N--);
    fcm_sink(m, 1);
  }
  return c;
}

typedef struct {
  int64_t ext, upd, maxf, walkers;
} tstats;

/* touched-target list of one source (top-k mode): every increment is > 0, so
   row[t] == 0 before an add means t enters the row for the first time */
typedef struct {
  int32_t* ids;
  int64_t size, cap;
} tlist;
static void row_add(double* row, tlist* tl, int32_t t, double v) {
  if (tl && row[t] == 0.0) {
    if (tl->size == tl->cap) {
      tl->cap = tl->cap ? 2 * tl->cap : 4096;
      tl->ids = (int32_t*)realloc(tl->ids, sizeof(int32_t) * tl->cap);
    }
    tl->ids[tl->size++] = t;
  }
  row[t] += v;
}

static void topsim_one(const int64_t* off, const int32_t* nbrs, int variant, int SAMPLE, int STEP,
                       const double* cache, uint32_t k0, uint32_t k1, int rng, jrand* jr, int32_t src,
                       double* row, pqueue* A, pqueue* B, tstats* st, fcm* map, tlist* tl) {
  const int L = 2 * STEP;
  if (variant == 2) { /* SingleRandomWalk.walk :53-72 + computePathSim :81-92 */
    int32_t* path = (int32_t*)malloc(sizeof(int32_t) * (L + 1));
    for (int64_t i = 0; i < SAMPLE; ++i) {
      int pathLen = 0;
      for (int t = 0; t <= L; ++t) path[t] = -1;
      path[0] = src;
      int32_t cur = src;
      while (pathLen < L) {
        int64_t d = off[cur + 1] - off[cur];
        if (d == 0) break;
        int64_t k;
        if (rng == 0) {
          struct gw_u4 u = gw_philox((uint32_t)src, (uint32_t)i, (uint32_t)(pathLen + 1), 0u, k0, k1);
          k = gw_index(u.x, u.y, (uint32_t)d);
        } else {
          k = or_jrand_next_int(jr, (int32_t)d);
        }
        cur = nbrs[off[cur] + k];
        path[++pathLen] = cur;
        st->ext++;
      }
      st->walkers++;
      if (pathLen == 0) continue;
      for (int ii = 1; ii <= STEP && 2 * ii <= pathLen; ++ii) {
        int32_t inter = path[ii], target = path[2 * ii];
        if (target == src) continue;
        if (first_meet(path, 2 * ii)) {
          double dm = (double)(off[inter + 1] - off[inter]), dt = (double)(off[target + 1] - off[target]);
          double incre = ((cache[ii] * dm) / dt) / (double)SAMPLE;
          if (map)
            fcm_put(map, target, (float)incre); /* SingleRandomWalk_M.java:computePathSim */
          else
            row_add(row, tl, target, incre);
          st->upd++;
        }
      }
    }
    free(path);
    return;
  }
  /* :65-74 */
  A->size = 0;
  pq_reserve(A, 1, L);
  for (int t = 0; t <= L; ++t) {
    A->cur[t] = -1;
    A->mass[t] = 0.0;
  }
  A->cur[0] = src;
  A->mass[0] = (double)SAMPLE;
  A->walker[0] = -1;
  A->size = 1;
  int64_t next_walker = 0;
  int pathLen = 0, TopSim = 1;
  for (;;) {
    if (pathLen >= L || pathLen / 2 == TopSim) {
      /* computePathSim(queue, pathLen, TopSim) :167-196 */
      if (pathLen > 0) {
        for (int64_t pi = 0; pi < A->size; ++pi) {
          const int32_t* path = A->cur + pi * (L + 1);
          const double* mass = A->mass + pi * (L + 1);
          int32_t source = path[0];
          for (int i = TopSim; i <= STEP && 2 * i <= pathLen; ++i) {
            int32_t inter = path[i], target = path[2 * i];
            if (target == source) continue;
            if (target == -1) continue;
            if (first_meet(path, 2 * i)) {
              double dm = (double)(off[inter + 1] - off[inter]);
              double dt = (double)(off[target + 1] - off[target]);
              if (map) /* TopSim_singleSample_M.java:224-225 */
                fcm_put(map, target, (float)((((mass[2 * i] * cache[i]) * dm) / dt) / (double)SAMPLE));
              else
                row_add(row, tl, target, ((mass[2 * i] * cache[i]) * dm) / dt); /* :189 */
              st->upd++;
            }
          }
        }
      }
      if (pathLen >= L) break;
      TopSim++;
    }
    if (A->size > st->maxf) st->maxf = A->size;
    /* expand every queued path by one level (:84-153) */
    B->size = 0;
    for (int64_t pi = 0; pi < A->size; ++pi) {
      const int32_t* path = A->cur + pi * (L + 1);
      const double* mass = A->mass + pi * (L + 1);
      int32_t cur = path[pathLen];
      double s = mass[pathLen];
      int64_t d = off[cur + 1] - off[cur];
      int det = (variant == 1) ? (d != 0) : (d != 0 && s >= (double)d);
      if (det) {
        double ns = s / (double)d; /* :104 */
        pq_reserve(B, B->size + d, L);
        for (int64_t j = 0; j < d; ++j) {
          int64_t c = B->size++;
          memcpy(B->cur + c * (L + 1), path, sizeof(int32_t) * (L + 1));
          memcpy(B->mass + c * (L + 1), mass, sizeof(double) * (L + 1));
          B->cur[c * (L + 1) + pathLen + 1] = nbrs[off[cur] + j];
          B->mass[c * (L + 1) + pathLen + 1] = ns;
          B->walker[c] = A->walker[pi];
          st->ext++;
        }
      } else {
        int number = (int)s; /* :131-135 */
        if ((double)number != s) number += 1;
        double ns = s / (double)number; /* :142 */
        for (int j = 0; j < number; ++j) {
          if (d == 0) break; /* randNeighbor == -1 -> break (:143-144) */
          int64_t wid = A->walker[pi] >= 0 ? A->walker[pi] : next_walker++;
          if (A->walker[pi] < 0) st->walkers++;
          int64_t k;
          if (rng == 0) {
            struct gw_u4 u = gw_philox((uint32_t)src, (uint32_t)wid, (uint32_t)(pathLen + 1), 0u, k0, k1);
            k = gw_index(u.x, u.y, (uint32_t)d);
          } else {
            k = or_jrand_next_int(jr, (int32_t)d);
          }
          pq_reserve(B, B->size + 1, L);
          int64_t c = B->size++;
          memcpy(B->cur + c * (L + 1), path, sizeof(int32_t) * (L + 1));
          memcpy(B->mass + c * (L + 1), mass, sizeof(double) * (L + 1));
          B->cur[c * (L + 1) + pathLen + 1] = nbrs[off[cur] + k];
          B->mass[c * (L + 1) + pathLen + 1] = ns;
          B->walker[c] = wid;
          st->ext++;
        }
      }
    }
    pqueue tmp = *A;
    *A = *B;
    *B = tmp;
    pathLen++;
  }
  if (row) row[src] = 0.0; /* sim[i][i] = 0 (:52) */
}

/* rows[r*n + t] = sim[sources[r]][t]; stats: ext, upd, maxf, walkers */
void or_topsim(int64_t n, const int64_t* off, const int32_t* nbrs, int variant, int sample, int step,
               double C, uint64_t seed, int rng, int64_t java_seed, const int32_t* sources, int64_t nsrc,
               double* rows, int64_t* stats, int nthreads) {
  double cache[32];
  for (int i = 0; i < 32; ++i) cache[i] = 0.0;
  for (int i = 1; i <= step && i < 32; ++i) cache[i] = pow(C, (double)i); /* :42-43 */
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  int64_t e = 0, u = 0, mf = 0, w = 0;
  memset(rows, 0, sizeof(double) * nsrc * n);
  if (rng == 1) { /* java stream: sequential over sources */
    jrand jr;
    or_jrand_init(&jr, java_seed);
    pqueue A = {0}, B = {0};
    tstats st = {0, 0, 0, 0};
    for (int64_t r = 0; r < nsrc; ++r)
      topsim_one(off, nbrs, variant, sample, step, cache, k0, k1, 1, &jr, sources[r], rows + r * n, &A, &B, &st, NULL, NULL);
    e = st.ext;
    u = st.upd;
    mf = st.maxf;
    w = st.walkers;
    free(A.cur); free(A.mass); free(A.walker);
    free(B.cur); free(B.mass); free(B.walker);
  } else {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : e, u, w) reduction(max : mf)
#endif
    {
      pqueue A = {0}, B = {0};
      tstats st = {0, 0, 0, 0};
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
      for (int64_t r = 0; r < nsrc; ++r)
        topsim_one(off, nbrs, variant, sample, step, cache, k0, k1, 0, NULL, sources[r], rows + r * n, &A, &B, &st, NULL, NULL);
      e += st.ext;
      u += st.upd;
      w += st.walkers;
      if (st.maxf > mf) mf = st.maxf;
      free(A.cur); free(A.mass); free(A.walker);
      free(B.cur); free(B.mass); free(B.walker);
    }
  }
  if (stats) {
    stats[0] = e;
    stats[1] = u;
    stats[2] = mf;
    stats[3] = w;
  }
}

/* TopSim_singleSample_M (variant 0) / SingleRandomWalk_M (variant 2): the  */
/* same walks as or_topsim (Philox keys), every pair update put() into a    */
/* FixedCacheMap(capacity) in the reference's order; per source the map is   */
/* drained ascending (its iteration order): out_keys/out_vals[r*cap + i],   */
/* out_size[r].                                                            */
typedef struct {
  double v;
  int32_t id;
} vid;
static int vid_cmp(const void* a, const void* b) { /* score desc, id asc (Print.printByOrder order) */
  const vid *x = (const vid*)a, *y = (const vid*)b;
  if (x->v != y->v) return x->v > y->v ? -1 : 1;
  return (x->id > y->id) - (x->id < y->id);
}

/* Per-source top-k of sim[source][*] (Print.printByOrder, Print.java:25-53):
   the same walks and sums as or_topsim, with one reused dense row per thread
   whose touched entries are ranked and re-zeroed (no n-wide memset per
   source, so large graphs cost what the walks cost).  ids/scores[r*topk ..]:
   score desc, id asc; rows with fewer than topk positive entries are padded
   with id -1, score 0 (the GPU's convention). */
void or_topsim_topk(int64_t n, const int64_t* off, const int32_t* nbrs, int variant, int sample, int step,
                    double C, uint64_t seed, const int32_t* sources, int64_t nsrc, int topk, int32_t* ids,
                    double* scores, int64_t* stats, int nthreads) {
  double cache[32];
  for (int i = 0; i < 32; ++i) cache[i] = 0.0;
  for (int i = 1; i <= step && i < 32; ++i) cache[i] = pow(C, (double)i); /* :42-43 */
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  int64_t e = 0, u = 0, mf = 0, w = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : e, u, w) reduction(max : mf)
#endif
  {
    pqueue A = {0}, B = {0};
    tstats st = {0, 0, 0, 0};
    tlist tl = {0};
    double* row = (double*)calloc((size_t)n, sizeof(double));
    vid* buf = NULL;
    int64_t bcap = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int64_t r = 0; r < nsrc; ++r) {
      tl.size = 0;
      topsim_one(off, nbrs, variant, sample, step, cache, k0, k1, 0, NULL, sources[r], row, &A, &B, &st, NULL, &tl);
      if (tl.size > bcap) {
        bcap = tl.size;
        buf = (vid*)realloc(buf, sizeof(vid) * bcap);
      }
      int64_t m = 0;
      for (int64_t i = 0; i < tl.size; ++i) {
        const int32_t t = tl.ids[i];
        if (row[t] > 0.0) {
          buf[m].v = row[t];
          buf[m].id = t;
          ++m;
        }
        row[t] = 0.0;
      }
      qsort(buf, (size_t)m, sizeof(vid), vid_cmp);
      for (int k = 0; k < topk; ++k) {
        ids[r * topk + k] = k < m ? buf[k].id : -1;
        scores[r * topk + k] = k < m ? buf[k].v : 0.0;
      }
    }
    e += st.ext;
    u += st.upd;
    w += st.walkers;
    if (st.maxf > mf) mf = st.maxf;
    free(A.cur); free(A.mass); free(A.walker);
    free(B.cur); free(B.mass); free(B.walker);
    free(tl.ids);
    free(buf);
    free(row);
  }
  if (stats) {
    stats[0] = e;
    stats[1] = u;
    stats[2] = mf;
    stats[3] = w;
  }
}

void or_topsim_m(int64_t n, const int64_t* off, const int32_t* nbrs, int variant, int sample, int step,
                 double C, uint64_t seed, int capacity, const int32_t* sources, int64_t nsrc, int32_t* out_keys,
                 float* out_vals, int32_t* out_size, int64_t* stats, int nthreads) {
  (void)n;
  double cache[32];
  for (int i = 0; i < 32; ++i) cache[i] = 0.0;
  for (int i = 1; i <= step && i < 32; ++i) cache[i] = pow(C, (double)i);
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  int64_t e = 0, u = 0, mf = 0, w = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : e, u, w) reduction(max : mf)
#endif
  {
    pqueue A = {0}, B = {0};
    tstats st = {0, 0, 0, 0};
    fcm m;
    fcm_init(&m, capacity);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int64_t r = 0; r < nsrc; ++r) {
      fcm_clear(&m);
      topsim_one(off, nbrs, variant, sample, step, cache, k0, k1, 0, NULL, sources[r], NULL, &A, &B, &st, &m, NULL);
      out_size[r] = fcm_drain(&m, out_keys + r * (int64_t)capacity, out_vals + r * (int64_t)capacity);
    }
    e += st.ext;
    u += st.upd;
    w += st.walkers;
    if (st.maxf > mf) mf = st.maxf;
    fcm_free(&m);
    free(A.cur); free(A.mass); free(A.walker);
    free(B.cur); free(B.mass); free(B.walker);
  }
  if (stats) {
    stats[0] = e;
    stats[1] = u;
    stats[2] = mf;
    stats[3] = w;
  }
}

/* TopSim_doubleSample.sample / TopSim_Dev.sample (TopSim_doubleSample.java */
/* :71-140, computePath :141-164): the BFS queue over STEP levels; at level  */
/* s every queued path with target path[s] != source assigns               */
/* paths[source][target][s] = path[s].sample in queue order (last wins).     */
/* Task t = (vertex tv[t], Philox call tc[t]); out[t][s-1][x], 0 = absent.  */
void or_topsim_levels(int64_t n, const int64_t* off, const int32_t* nbrs, int sample, int step, uint64_t seed,
                      const int32_t* tv, const int32_t* tc, int64_t ntask, double* out, int nthreads) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  const int L = step;
  memset(out, 0, sizeof(double) * ntask * step * n);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    pqueue A = {0}, B = {0};
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int64_t t = 0; t < ntask; ++t) {
      const int32_t src = tv[t];
      const uint32_t call = (uint32_t)tc[t];
      double* row = out + t * step * n;
      A.size = 0;
      pq_reserve(&A, 1, L);
      for (int q = 0; q <= L; ++q) {
        A.cur[q] = -1;
        A.mass[q] = 0.0;
      }
      A.cur[0] = src;
      A.mass[0] = (double)sample;
      A.walker[0] = -1;
      A.size = 1;
      int64_t next_walker = 0;
      for (int pathLen = 0;; ++pathLen) {
        if (pathLen >= 1) { /* computePath(queue, pathLen, TopSim = pathLen) */
          for (int64_t pi = 0; pi < A.size; ++pi) {
            int32_t target = A.cur[pi * (L + 1) + pathLen];
            if (target == src || target == -1) continue;
            row[(int64_t)(pathLen - 1) * n + target] = A.mass[pi * (L + 1) + pathLen];
          }
        }
        if (pathLen >= L) break;
        B.size = 0;
        for (int64_t pi = 0; pi < A.size; ++pi) {
          const int32_t* path = A.cur + pi * (L + 1);
          const double* mass = A.mass + pi * (L + 1);
          int32_t cur = path[pathLen];
          double sm = mass[pathLen];
          int64_t d = off[cur + 1] - off[cur];
          if (d != 0 && sm >= (double)d) {
            double ns = sm / (double)d;
            pq_reserve(&B, B.size + d, L);
            for (int64_t j = 0; j < d; ++j) {
              int64_t c = B.size++;
              memcpy(B.cur + c * (L + 1), path, sizeof(int32_t) * (L + 1));
              memcpy(B.mass + c * (L + 1), mass, sizeof(double) * (L + 1));
              B.cur[c * (L + 1) + pathLen + 1] = nbrs[off[cur] + j];
              B.mass[c * (L + 1) + pathLen + 1] = ns;
              B.walker[c] = A.walker[pi];
            }
          } else {
            int number = (int)sm;
            if ((double)number != sm) number += 1;
            double ns = sm / (double)number;
            for (int j = 0; j < number; ++j) {
              if (d == 0) break;
              int64_t wid = A.walker[pi] >= 0 ? A.walker[pi] : next_walker++;
              struct gw_u4 u = gw_philox((uint32_t)src, (uint32_t)wid, (uint32_t)(pathLen + 1), call, k0, k1);
              int64_t k = gw_index(u.x, u.y, (uint32_t)d);
              pq_reserve(&B, B.size + 1, L);
              int64_t c = B.size++;
              memcpy(B.cur + c * (L + 1), path, sizeof(int32_t) * (L + 1));
              memcpy(B.mass + c * (L + 1), mass, sizeof(double) * (L + 1));
              B.cur[c * (L + 1) + pathLen + 1] = nbrs[off[cur] + k];
              B.mass[c * (L + 1) + pathLen + 1] = ns;
              B.walker[c] = wid;
            }
          }
        }
        pqueue tmp = A;
        A = B;
        B = tmp;
      }
    }
    free(A.cur); free(A.mass); free(A.walker);
    free(B.cur); free(B.mass); free(B.walker);
  }
}

/* getSim(src, dst) of TopSim_doubleSample / TopSim_Dev (:181-193): the Java */
/* loop order over vertices i then steps, cache[s]*P[src]*P[dst].           */
static double levels_dot(const double* a, const double* b, int64_t n, int step, const double* cache) {
  double result = 0.0;
  for (int64_t i = 0; i < n; ++i)
    for (int s = 1; s <= step; ++s) {
      double pa = a[(int64_t)(s - 1) * n + i], pb = b[(int64_t)(s - 1) * n + i];
      if (pa > 0.0 && pb > 0.0) result += cache[s] * pa * pb;
    }
  return result;
}

/* TopSim_doubleSample.computeSims (:167-176): sim[i][j] = getSim(i, j) for  */
/* i < j, mirrored; diagonal 0.  M = or_topsim_levels over tasks (v, 0).    */
void or_topsim_double_sims(int64_t n, const double* M, int step, double C, double* sim, int nthreads) {
  double cache[32];
  for (int i = 0; i <= step && i < 32; ++i) cache[i] = pow(C, (double)i);
  memset(sim, 0, sizeof(double) * n * n);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = i + 1; j < n; ++j) {
      double v = levels_dot(M + i * step * n, M + j * step * n, n, step, cache);
      sim[i * n + j] = v;
      sim[j * n + i] = v;
    }
}

/* TopSim_Dev.compute (:57-95) given the candidate lists cand[i*K + r]       */
/* (FixedMaxPQ sortedElement order, -1 padded): sample(i) with call 0, each */
/* candidate j = cand[i*K+r] freshly sampled with call 1 + i*K + r;         */
/* sim[i][j] = getSim, sim[i][i] = 0.  `sample` is the derived SAMPLE.      */
void or_topsim_dev(int64_t n, const int64_t* off, const int32_t* nbrs, int sample, int step, double C, uint64_t seed,
                   const int32_t* cand, int K, double* sim, int nthreads) {
  double cache[32];
  for (int i = 0; i <= step && i < 32; ++i) cache[i] = pow(C, (double)i);
  memset(sim, 0, sizeof(double) * n * n);
  double* Mi = (double*)malloc(sizeof(double) * step * n);
  double* Mj = (double*)malloc(sizeof(double) * step * n);
  for (int64_t i = 0; i < n; ++i) {
    int32_t tv = (int32_t)i, tc = 0;
    or_topsim_levels(n, off, nbrs, sample, step, seed, &tv, &tc, 1, Mi, nthreads);
    for (int r = 0; r < K; ++r) {
      int32_t j = cand[i * K + r];
      if (j < 0) break;
      int32_t cv = j, cc = 1 + (int32_t)(i * K + r);
      or_topsim_levels(n, off, nbrs, sample, step, seed, &cv, &cc, 1, Mj, nthreads);
      sim[i * n + j] = levels_dot(Mi, Mj, n, step, cache);
    }
    sim[i * n + i] = 0.0;
  }
  free(Mi);
  free(Mj);
}

/* DoubleRandomWalk (DoubleRandomWalk.java:50-91): SAMPLE walks of STEP      */
/* steps per vertex (Philox (v, i, step+1)), then for every pair v < w the   */
/* first-meeting estimator sum cache[t+1] / SAMPLE^2, mirrored.             */
void or_double_random_walk(int64_t n, const int64_t* off, const int32_t* nbrs, int sample, int step, double C,
                           uint64_t seed, double* sim, int nthreads) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  double cache[32];
  for (int i = 0; i <= step && i < 32; ++i) cache[i] = pow(C, (double)i);
  int32_t* paths = (int32_t*)calloc((size_t)(n * sample * step), sizeof(int32_t));
  for (int64_t v = 0; v < n; ++v)
    for (int i = 0; i < sample; ++i) {
      int32_t cur = (int32_t)v;
      for (int t = 0; t < step; ++t) { /* sample(src) :56-65 */
        int64_t d = off[cur + 1] - off[cur];
        if (d == 0) {
          cur = -1;
        } else {
          struct gw_u4 u = gw_philox((uint32_t)v, (uint32_t)i, (uint32_t)(t + 1), 0u, k0, k1);
          cur = nbrs[off[cur] + gw_index(u.x, u.y, (uint32_t)d)];
        }
        paths[(v * sample + i) * step + t] = cur;
        if (cur == -1) break;
      }
    }
  memset(sim, 0, sizeof(double) * n * n);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t v = 0; v < n; ++v)
    for (int64_t w = v + 1; w < n; ++w) {
      double result = 0.0;
      for (int i = 0; i < sample; ++i)
        for (int j = 0; j < sample; ++j) {
          const int32_t* a = paths + (v * sample + i) * step;
          const int32_t* b = paths + (w * sample + j) * step;
          for (int t = 0; t < step && a[t] != -1 && b[t] != -1; ++t)
            if (a[t] == b[t]) {
              result += cache[t + 1];
              break;
            }
        }
      double val = result / ((double)sample * (double)sample);
      sim[v * n + w] = val;
      sim[w * n + v] = val;
    }
  free(paths);
}

/* FixedCacheMap.main (FixedCacheMap.java:134-148) as a known-answer check:  */
/* puts (key, value) in order into a map of capacity nmax, drains ascending. */
int or_fcm_run(int nmax, int64_t nput, const int32_t* keys, const float* vals, int32_t* ok, float* ov) {
  fcm m;
  fcm_init(&m, nmax);
  for (int64_t i = 0; i < nput; ++i) fcm_put(&m, keys[i], vals[i]);
  int c = fcm_drain(&m, ok, ov);
  fcm_free(&m);
  return c;
}

/* ------------------------------------------------------------------------ */
/* naive SimRank (SimRank.java:21-77): `iters` Jacobi sweeps over the upper  */
/* triangle, sim(v,v)=1 during the sweeps, 0 afterwards (postProcess :62-65) */
/* ------------------------------------------------------------------------ */
void or_simrank_naive(int64_t n, const int64_t* off, const int32_t* nbrs, double C, int iters,
                      double* sim, int nthreads) {
  double* tmp = (double*)calloc((size_t)(n * n), sizeof(double));
  memset(sim, 0, sizeof(double) * n * n);
  for (int64_t i = 0; i < n; ++i) sim[i * n + i] = tmp[i * n + i] = 1.0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  for (int r = 0; r < iters; ++r) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int64_t i = 0; i < n; ++i)
      for (int64_t j = i + 1; j < n; ++j) {
        double v = 0.0;
        int64_t di = off[i + 1] - off[i], dj = off[j + 1] - off[j];
        if (di != 0 && dj != 0) {
          double res = 0.0;
          for (int64_t a = off[i]; a < off[i + 1]; ++a)
            for (int64_t b = off[j]; b < off[j + 1]; ++b) res += sim[(int64_t)nbrs[a] * n + nbrs[b]];
          v = C * res / (double)(di * dj); /* :76 */
        }
        tmp[i * n + j] = v;
        tmp[j * n + i] = v;
      }
    memcpy(sim, tmp, sizeof(double) * n * n);
  }
  for (int64_t i = 0; i < n; ++i) sim[i * n + i] = 0.0;
  free(tmp);
}

/* One sweep of SimRank.java:42-47 for rows [rb, re) only (timing samples   */
/* for bench.py's CPU baseline): out[(i-rb)*n + j] = sim(i, j), j > i, from */
/* the matrix S.  Returns the number of neighbour pairs summed.             */
int64_t or_simrank_round_rows(int64_t n, const int64_t* off, const int32_t* nbrs, double C, const double* S,
                              int64_t rb, int64_t re, double* out, int nthreads) {
  int64_t pairs = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : pairs)
#endif
  for (int64_t i = rb; i < re; ++i)
    for (int64_t j = i + 1; j < n; ++j) {
      double v = 0.0;
      int64_t di = off[i + 1] - off[i], dj = off[j + 1] - off[j];
      if (di != 0 && dj != 0) {
        double res = 0.0;
        for (int64_t a = off[i]; a < off[i + 1]; ++a)
          for (int64_t b = off[j]; b < off[j + 1]; ++b) res += S[(int64_t)nbrs[a] * n + nbrs[b]];
        v = C * res / (double)(di * dj);
        pairs += di * dj;
      }
      out[(i - rb) * n + j] = v;
    }
  return pairs;
}

/* ------------------------------------------------------------------------ */
/* GW_N2V_BITSET restatement: the same 3-way exact mixture of the reference */
/* get_alias_edge weights (node2vec.py:61-81; unweighted, undirected), but   */
/* computing c and the common neighbours by explicit has_edge scans instead  */
/* of precomputed bitsets.  Philox usage: step 1: (u.x:u.z) -> uniform       */
/* neighbour (64-bit index draw); step >= 2: philox(w, step, 0).x ->        */
/* component, (.y:.z) -> first "other" candidate, philox(w, step, t) (.y:.z) */
/* -> retries t = 1, 2, ...                                                 */
/* ------------------------------------------------------------------------ */
void or_walks_bitset(int64_t n, const int64_t* off, const int32_t* nbrs, const int32_t* order, double p,
                     double q, uint64_t seed, int L, int64_t walk_begin, int64_t walk_count, int shuffle,
                     int32_t* out, int32_t* lens, uint64_t* counters, int nthreads) {
  const double a_p = 1.0 / p, a_q = 1.0 / q;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_STEP;
  const uint32_t pk0 = (uint32_t)seed, pk1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_PERM;
  uint64_t tot_steps = 0, tot_trials = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : tot_steps, tot_trials)
#endif
  for (int64_t i = 0; i < walk_count; ++i) {
    const int64_t wi = walk_begin + i;
    const uint64_t it = (uint64_t)wi / (uint64_t)n, pos = (uint64_t)wi % (uint64_t)n;
    const uint64_t sp = shuffle ? gw_feistel_perm(pos, (uint64_t)n, pk0, pk1, (uint32_t)it) : pos;
    int32_t cur = order[sp], prev = -1;
    int32_t* row = out + i * (int64_t)L;
    row[0] = cur;
    int len = 1;
    const uint32_t c0 = (uint32_t)wi, c1 = (uint32_t)((uint64_t)wi >> 32);
    while (len < L) {
      const int64_t b = off[cur], d = off[cur + 1] - b;
      if (d == 0) break;
      int64_t k = 0;
      uint32_t trial = 0;
      struct gw_u4 u = gw_philox(c0, c1, (uint32_t)len, 0u, k0, k1);
      ++trial;
      if (len == 1) {
        k = gw_index(u.x, u.z, (uint32_t)d);
      } else {
        int64_t kp = -1, c = 0;
        for (int64_t j = 0; j < d; ++j) {
          int32_t x = nbrs[b + j];
          if (x == prev) kp = j;
          else if (find_slot(off, nbrs, prev, x) >= 0) ++c;
        }
        const double Z = (a_p + (double)c) + (double)(d - 1 - c) * a_q;
        const double r = gw_u01(u.x) * Z;
        if (r < a_p) {
          k = kp;
        } else if (r - a_p < (double)c) {
          uint32_t jj = (uint32_t)(r - a_p);
          if (jj >= (uint32_t)c) jj = (uint32_t)c - 1;
          for (int64_t j = 0; j < d; ++j) {
            int32_t x = nbrs[b + j];
            if (x != prev && find_slot(off, nbrs, prev, x) >= 0) {
              if (jj == 0) {
                k = j;
                break;
              }
              --jj;
            }
          }
        } else {
          for (;;) {
            k = gw_index(u.y, u.z, (uint32_t)d);
            int32_t x = nbrs[b + k];
            int bit = (x != prev) && find_slot(off, nbrs, prev, x) >= 0;
            if ((k != kp && !bit) || trial >= (1u << 24)) break;
            u = gw_philox(c0, c1, (uint32_t)len, trial, k0, k1);
            ++trial;
          }
        }
      }
      tot_trials += trial;
      prev = cur;
      cur = nbrs[b + k];
      row[len++] = cur;
    }
    for (int t = len; t < L; ++t) row[t] = -1;
    if (lens) lens[i] = len;
    tot_steps += (uint64_t)(len - 1);
  }
  if (counters) {
    counters[0] += tot_steps;
    counters[1] += tot_trials;
  }
}
