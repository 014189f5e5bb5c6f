// Host-side graph construction for libgraphwalk.
//
//  * NX_SIMPLE: the graph `read_graph` builds (node2vec/src/main.py:76-89):
//    nx.read_edgelist into a DiGraph (duplicate (u,v) -> last weight wins),
//    optional G.to_undirected() (reciprocal pair -> the directed edge whose
//    source comes later in node order wins, because networkx 3.x
//    `to_undirected` walks `_adj` in node order and `update`s one shared
//    datadict), node order = first appearance, draw order = sorted labels
//    (node2vec.py:25,67,94 `sorted(G.neighbors(...))`).
//  * JAVA_MULTI: structures.Graph(path, V) (Graph.java:28-57): each line
//    appends b to adj[a] and a to adj[b], duplicates kept, insertion order.
//
// Dense ids for NX_SIMPLE are the rank of the label in sorted label order, so
// "sorted by label" == "sorted by dense id" and has_edge is a binary search
// on dense ids.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <numeric>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#include <parallel/algorithm>
#endif

#include "gw_internal.h"
#include "gw_philox.h"

template <class It, class Cmp>
static void par_sort(It b, It e, Cmp c) {
#ifdef _OPENMP
  if (e - b > (1 << 16)) {
    __gnu_parallel::sort(b, e, c);
    return;
  }
#endif
  std::sort(b, e, c);
}

// ------------------------------------------------------------------------
// NX_SIMPLE builder
// ------------------------------------------------------------------------
int gw_build_nx_simple(gw_graph* g, int64_t m, const int64_t* src,
                       const int64_t* dst, const double* w, int directed) {
  g->semantics = GW_SEM_NX_SIMPLE;
  g->directed = directed ? 1 : 0;
  g->weighted = w ? 1 : 0;
  // 1. labels -> dense rank; first-appearance node order (u then v per line:
  //    DiGraph.add_edge adds u before v).
  std::vector<int64_t> lab(2 * m);
  for (int64_t i = 0; i < m; ++i) {
    lab[2 * i] = src[i];
    lab[2 * i + 1] = dst[i];
  }
  std::vector<int64_t> uniq(lab);
  par_sort(uniq.begin(), uniq.end(), std::less<int64_t>());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  const int64_t n = (int64_t)uniq.size();
  auto rank = [&](int64_t x) -> int32_t {
    return (int32_t)(std::lower_bound(uniq.begin(), uniq.end(), x) - uniq.begin());
  };
  if (n >= (int64_t)INT32_MAX) return gw_fail(g, GW_ERR_UNSUPPORTED, "too many vertices (%lld)", (long long)n);
  std::vector<int32_t> u(m), v(m);
  std::vector<int64_t> first(n, INT64_MAX);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < m; ++i) {
    u[i] = rank(src[i]);
    v[i] = rank(dst[i]);
  }
  for (int64_t i = 0; i < m; ++i) {  // sequential: first appearance
    if (first[u[i]] == INT64_MAX) first[u[i]] = 2 * i;
    if (first[v[i]] == INT64_MAX) first[v[i]] = 2 * i + 1;
  }
  std::vector<int32_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  par_sort(order.begin(), order.end(),
           [&](int32_t a, int32_t b) { return first[a] < first[b]; });
  std::vector<int64_t> pos(n);  // node-order position
  for (int64_t i = 0; i < n; ++i) pos[order[i]] = i;

  // 2. DiGraph: duplicate (u,v) -> last line's weight.  Entries carry the
  //    line index so a stable "last wins" survives the sort.
  struct E {
    int32_t a, b;
    int64_t prio;  // line index (step 2) / winner priority (step 3)
    double w;
  };
  std::vector<E> es(m);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < m; ++i) es[i] = E{u[i], v[i], i, w ? w[i] : 1.0};
  auto by_ab_prio = [](const E& x, const E& y) {
    if (x.a != y.a) return x.a < y.a;
    if (x.b != y.b) return x.b < y.b;
    return x.prio < y.prio;
  };
  par_sort(es.begin(), es.end(), by_ab_prio);
  {
    int64_t k = 0;
    for (int64_t i = 0; i < m; ++i) {
      if (i + 1 < m && es[i + 1].a == es[i].a && es[i + 1].b == es[i].b) continue;  // keep last
      es[k++] = es[i];
    }
    es.resize(k);
  }
  // 3. to_undirected: for a reciprocal pair the edge whose source is later in
  //    node order is processed later and its data wins.
  if (!directed) {
    const int64_t k = (int64_t)es.size();
    std::vector<E> und;
    und.reserve(2 * k);
    for (int64_t i = 0; i < k; ++i) {
      const E& e = es[i];
      int64_t pr = pos[e.a];
      und.push_back(E{e.a, e.b, pr, e.w});
      if (e.a != e.b) und.push_back(E{e.b, e.a, pr, e.w});
    }
    par_sort(und.begin(), und.end(), by_ab_prio);
    int64_t j = 0;
    for (int64_t i = 0; i < (int64_t)und.size(); ++i) {
      if (i + 1 < (int64_t)und.size() && und[i + 1].a == und[i].a && und[i + 1].b == und[i].b) continue;
      und[j++] = und[i];
    }
    und.resize(j);
    es.swap(und);
  }
  // 4. CSR, rows sorted by dense id (== by label)
  g->n = n;
  g->nnz = (int64_t)es.size();
  g->offsets.assign(n + 1, 0);
  for (const E& e : es) g->offsets[e.a + 1]++;
  for (int64_t i = 0; i < n; ++i) g->offsets[i + 1] += g->offsets[i];
  g->nbrs.resize(g->nnz);
  if (w) g->weights.resize(g->nnz);
  for (int64_t i = 0; i < g->nnz; ++i) {  // es sorted by (a,b): already in place
    g->nbrs[i] = es[i].b;
    if (w) g->weights[i] = es[i].w;
  }
  g->labels = uniq;
  g->order = order;
  g->max_degree = 0;
  for (int64_t i = 0; i < n; ++i)
    g->max_degree = std::max(g->max_degree, g->offsets[i + 1] - g->offsets[i]);
  return GW_OK;
}

// ------------------------------------------------------------------------
// JAVA_MULTI builder (Graph.java:28-57)
// ------------------------------------------------------------------------
int gw_build_java_multi(gw_graph* g, int64_t m, const int64_t* src,
                        const int64_t* dst, int64_t vcount) {
  g->semantics = GW_SEM_JAVA_MULTI;
  g->directed = 0;
  g->weighted = 0;
  if (vcount < 0) return gw_fail(g, GW_ERR_INVALID, "JAVA_MULTI needs vcount >= 0");
  if (vcount >= (int64_t)INT32_MAX) return gw_fail(g, GW_ERR_UNSUPPORTED, "vcount too large");
  for (int64_t i = 0; i < m; ++i) {
    if (src[i] < 0 || src[i] >= vcount || dst[i] < 0 || dst[i] >= vcount)
      return gw_fail(g, GW_ERR_RANGE, "edge %lld (%lld,%lld) outside [0,%lld) (Graph.java:54 adjs[from])",
                     (long long)i, (long long)src[i], (long long)dst[i], (long long)vcount);
  }
  g->n = vcount;
  g->nnz = 2 * m;
  g->offsets.assign(vcount + 1, 0);
  for (int64_t i = 0; i < m; ++i) {
    g->offsets[src[i] + 1]++;
    g->offsets[dst[i] + 1]++;
  }
  for (int64_t i = 0; i < vcount; ++i) g->offsets[i + 1] += g->offsets[i];
  std::vector<int64_t> fill(g->offsets.begin(), g->offsets.end() - 1);
  g->nbrs.resize(g->nnz);
  for (int64_t i = 0; i < m; ++i) {  // insertion order: adjs[a].add(b); adjs[b].add(a)
    g->nbrs[fill[src[i]]++] = (int32_t)dst[i];
    g->nbrs[fill[dst[i]]++] = (int32_t)src[i];
  }
  g->labels.resize(vcount);
  std::iota(g->labels.begin(), g->labels.end(), 0);
  g->order.resize(vcount);
  std::iota(g->order.begin(), g->order.end(), 0);
  g->max_degree = 0;
  for (int64_t i = 0; i < vcount; ++i)
    g->max_degree = std::max(g->max_degree, g->offsets[i + 1] - g->offsets[i]);
  return GW_OK;
}

// ------------------------------------------------------------------------
// edgelist parsing
// ------------------------------------------------------------------------
static bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// Python int(): optional surrounding whitespace, sign, digits (underscores
// between digits are accepted by Python; accepted here too).  Labels must fit
// int64 (Python's ints are unbounded: larger labels are refused as a parse error).
static bool parse_py_int(const char* b, const char* e, int64_t* out) {
  while (b < e && is_space(*b)) ++b;
  while (e > b && is_space(e[-1])) --e;
  if (b == e) return false;
  bool neg = false;
  if (*b == '+' || *b == '-') {
    neg = (*b == '-');
    ++b;
  }
  if (b == e) return false;
  int64_t v = 0;
  bool last_digit = false;
  for (const char* p = b; p < e; ++p) {
    if (*p >= '0' && *p <= '9') {
      if (v > (INT64_MAX - (*p - '0')) / 10) return false;  // beyond int64
      v = v * 10 + (*p - '0');
      last_digit = true;
    } else if (*p == '_' && last_digit && p + 1 < e && p[1] >= '0' && p[1] <= '9') {
      last_digit = false;
    } else {
      return false;
    }
  }
  *out = neg ? -v : v;
  return true;
}

// Java Integer.valueOf: no whitespace, optional sign, digits, int32 range.
static bool parse_java_int(const char* b, const char* e, int64_t* out) {
  if (b == e) return false;
  bool neg = false;
  if (*b == '+' || *b == '-') {
    neg = (*b == '-');
    ++b;
  }
  if (b == e) return false;
  int64_t v = 0;
  for (const char* p = b; p < e; ++p) {
    if (*p < '0' || *p > '9') return false;
    v = v * 10 + (*p - '0');
    if (v > (int64_t)2147483648LL) return false;
  }
  if (neg) v = -v;
  if (v > INT32_MAX || v < INT32_MIN) return false;
  *out = v;
  return true;
}

static bool parse_py_float(const char* b, const char* e, double* out) {
  while (b < e && is_space(*b)) ++b;
  while (e > b && is_space(e[-1])) --e;
  if (b == e) return false;
  std::string s(b, e);
  char* end = nullptr;
  errno = 0;
  double v = strtod(s.c_str(), &end);
  if (end != s.c_str() + s.size()) return false;
  *out = v;
  return true;
}

// split [b,e) by delim (empty delim: whitespace runs, Python str.split())
static void split_tokens(const char* b, const char* e, const std::string& delim,
                         std::vector<std::pair<const char*, const char*>>& toks) {
  toks.clear();
  if (delim.empty()) {
    const char* p = b;
    while (p < e) {
      while (p < e && is_space(*p)) ++p;
      if (p >= e) break;
      const char* s = p;
      while (p < e && !is_space(*p)) ++p;
      toks.emplace_back(s, p);
    }
    return;
  }
  const char* s = b;
  const size_t dl = delim.size();
  for (const char* p = b; p + dl <= e;) {
    if (memcmp(p, delim.data(), dl) == 0) {
      toks.emplace_back(s, p);
      p += dl;
      s = p;
    } else {
      ++p;
    }
  }
  toks.emplace_back(s, e);
}

static int read_file(const char* path, std::string* buf) {
  FILE* f = fopen(path, "rb");
  if (!f) return GW_ERR_IO;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  buf->resize(sz > 0 ? (size_t)sz : 0);
  size_t got = sz > 0 ? fread(&(*buf)[0], 1, (size_t)sz, f) : 0;
  fclose(f);
  return got == buf->size() ? GW_OK : GW_ERR_IO;
}

int gw_load_edgelist_impl(gw_graph* g, const char* path, const char* delim,
                          int semantics, int directed, int weighted,
                          int64_t vcount) {
  std::string buf;
  if (read_file(path, &buf) != GW_OK) return gw_fail(g, GW_ERR_IO, "cannot read '%s'", path);
  std::string d = delim ? std::string(delim) : std::string();
  std::vector<int64_t> src, dst;
  std::vector<double> wts;
  std::vector<std::pair<const char*, const char*>> toks;
  const char* p = buf.data();
  const char* end = p + buf.size();
  int64_t lineno = 0;
  while (p < end) {
    const char* nl = (const char*)memchr(p, '\n', end - p);
    const char* le = nl ? nl : end;
    const char* lb = p;
    p = nl ? nl + 1 : end;
    ++lineno;
    if (semantics == GW_SEM_NX_SIMPLE) {
      // networkx 3.x parse_edgelist: cut at '#' (skip if nothing is left),
      // then line.rstrip("\n").split(delimiter) -- no other stripping.
      const char* c = (const char*)memchr(lb, '#', le - lb);
      const char* ce = c ? c : le;
      if (c == lb) continue;
      split_tokens(lb, ce, d, toks);
      if (toks.size() < 2) continue;
      int64_t a, b;
      if (!parse_py_int(toks[0].first, toks[0].second, &a) || !parse_py_int(toks[1].first, toks[1].second, &b))
        return gw_fail(g, GW_ERR_PARSE, "%s:%lld: failed to convert nodes to int (networkx parse_edgelist)", path, (long long)lineno);
      if (weighted) {
        if (toks.size() != 3)
          return gw_fail(g, GW_ERR_PARSE, "%s:%lld: edge data and data_keys not the same length", path, (long long)lineno);
        double wv;
        if (!parse_py_float(toks[2].first, toks[2].second, &wv))
          return gw_fail(g, GW_ERR_PARSE, "%s:%lld: failed to convert weight to float", path, (long long)lineno);
        wts.push_back(wv);
      } else if (toks.size() > 2) {
        return gw_fail(g, GW_ERR_PARSE, "%s:%lld: extra edge data on an unweighted edgelist (networkx data=True expects a dict)", path, (long long)lineno);
      }
      src.push_back(a);
      dst.push_back(b);
    } else {
      // Java BufferedReader.readLine strips "\n" / "\r\n"; String.split(sep)
      const char* se = le;
      if (se > lb && se[-1] == '\r') --se;
      if (lb == end) break;
      split_tokens(lb, se, d.empty() ? std::string(",") : d, toks);
      while (!toks.empty() && toks.back().first == toks.back().second) toks.pop_back();  // trailing empties dropped
      if (toks.size() < 2)
        return gw_fail(g, GW_ERR_PARSE, "%s:%lld: ArrayIndexOutOfBoundsException: line has < 2 fields for separator '%s' (Graph.java:38-39)", path, (long long)lineno, d.c_str());
      int64_t a, b;
      if (!parse_java_int(toks[0].first, toks[0].second, &a) || !parse_java_int(toks[1].first, toks[1].second, &b))
        return gw_fail(g, GW_ERR_PARSE, "%s:%lld: NumberFormatException (Graph.java:39)", path, (long long)lineno);
      src.push_back(a);
      dst.push_back(b);
    }
  }
  if (semantics == GW_SEM_NX_SIMPLE)
    return gw_build_nx_simple(g, (int64_t)src.size(), src.data(), dst.data(), weighted ? wts.data() : nullptr, directed);
  if (semantics == GW_SEM_JAVA_MULTI)
    return gw_build_java_multi(g, (int64_t)src.size(), src.data(), dst.data(), vcount);
  return gw_fail(g, GW_ERR_INVALID, "unknown semantics %d", semantics);
}

// ------------------------------------------------------------------------
// Graph500 R-MAT generator (bench input)
// ------------------------------------------------------------------------
int gw_rmat_impl(gw_graph* g, int scale, int edge_factor, double a, double b,
                 double c, uint64_t seed) {
  if (scale < 1 || scale > 30 || edge_factor < 1) return gw_fail(g, GW_ERR_INVALID, "bad rmat scale/edge_factor");
  if (!(a > 0 && b >= 0 && c >= 0 && a + b + c < 1.0)) return gw_fail(g, GW_ERR_INVALID, "bad rmat probabilities");
  const uint64_t N = 1ull << scale;
  const int64_t M = (int64_t)edge_factor << scale;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_RMAT;
  const double ab = a + b, abc = a + b + c;
  // undirected pairs, packed (u << 32 | v), both directions
  std::vector<uint64_t> pairs((size_t)2 * M);
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < M; ++e) {
    uint64_t u = 0, v = 0;
    for (int l = 0; l < scale; l += 4) {
      gw_u4 r = gw_philox((uint32_t)e, (uint32_t)((uint64_t)e >> 32), (uint32_t)l, 0u, k0, k1);
      uint32_t rr[4] = {r.x, r.y, r.z, r.w};
      for (int j = 0; j < 4 && l + j < scale; ++j) {
        double x = gw_u01(rr[j]);
        uint64_t bu = 0, bv = 0;
        if (x < a) {
        } else if (x < ab) {
          bv = 1;
        } else if (x < abc) {
          bu = 1;
        } else {
          bu = 1;
          bv = 1;
        }
        u = (u << 1) | bu;
        v = (v << 1) | bv;
      }
    }
    // Graph500 scrambles vertex labels with a random permutation
    u = gw_feistel_perm(u, N, k0 ^ 0x5bd1e995u, k1, 0xFFFFFFFFu);
    v = gw_feistel_perm(v, N, k0 ^ 0x5bd1e995u, k1, 0xFFFFFFFFu);
    if (u == v) {
      pairs[2 * e] = pairs[2 * e + 1] = UINT64_MAX;  // self-loop dropped
    } else {
      pairs[2 * e] = (u << 32) | v;
      pairs[2 * e + 1] = (v << 32) | u;
    }
  }
  par_sort(pairs.begin(), pairs.end(), std::less<uint64_t>());
  pairs.erase(std::unique(pairs.begin(), pairs.end()), pairs.end());
  if (!pairs.empty() && pairs.back() == UINT64_MAX) pairs.pop_back();
  // compact non-isolated vertices; dense id = rank of label
  std::vector<uint8_t> present(N, 0);
  for (uint64_t pr : pairs) present[pr >> 32] = 1;
  std::vector<int64_t> dense(N, -1);
  int64_t n = 0;
  g->labels.clear();
  for (uint64_t i = 0; i < N; ++i)
    if (present[i]) {
      dense[i] = n++;
      g->labels.push_back((int64_t)i);
    }
  g->semantics = GW_SEM_NX_SIMPLE;
  g->directed = 0;
  g->weighted = 0;
  g->n = n;
  g->nnz = (int64_t)pairs.size();
  g->offsets.assign(n + 1, 0);
  g->nbrs.resize(g->nnz);
  for (int64_t i = 0; i < g->nnz; ++i) {
    g->offsets[dense[pairs[i] >> 32] + 1]++;
    g->nbrs[i] = (int32_t)dense[pairs[i] & 0xFFFFFFFFull];
  }
  for (int64_t i = 0; i < n; ++i) g->offsets[i + 1] += g->offsets[i];
  g->order.resize(n);
  std::iota(g->order.begin(), g->order.end(), 0);  // synthetic: label order
  g->max_degree = 0;
  for (int64_t i = 0; i < n; ++i) g->max_degree = std::max(g->max_degree, g->offsets[i + 1] - g->offsets[i]);
  return GW_OK;
}

// ------------------------------------------------------------------------
// R-MAT with an arbitrary vertex count, Java multigraph semantics (TopSim
// synthetic input): the quadrant recursion of the
// reference generator (RMATGraphGenerator.java:119-145, halving
// [st, en] ranges until both are singletons), one Philox uniform per level in
// place of Random.nextDouble(); every generated line (col_st, row_st) is
// added both ways as structures.Graph.addEdge does (duplicates and self
// loops kept, Graph.java:53-57).
// ------------------------------------------------------------------------
int gw_rmat_java_impl(gw_graph* g, int64_t n, int64_t m, double a, double b, double c,
                      uint64_t seed) {
  if (n < 1 || n >= (int64_t)INT32_MAX || m < 0) return gw_fail(g, GW_ERR_INVALID, "bad rmat n/m");
  if (!(a > 0 && b >= 0 && c >= 0 && a + b + c < 1.0)) return gw_fail(g, GW_ERR_INVALID, "bad rmat probabilities");
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_RMAT ^ 0x4A415641u;  // "JAVA"
  const double cumA = a, cumB = a + b, cumC = a + b + c;
  std::vector<int64_t> src(m), dst(m);
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m; ++e) {
    int64_t col_st = 0, col_en = n - 1, row_st = 0, row_en = n - 1;
    uint32_t lvl = 0;
    gw_u4 r{0, 0, 0, 0};
    while (col_st != col_en || row_st != row_en) {
      if ((lvl & 3) == 0) r = gw_philox((uint32_t)e, (uint32_t)((uint64_t)e >> 32), lvl >> 2, 1u, k0, k1);
      const uint32_t rr = (lvl & 3) == 0 ? r.x : (lvl & 3) == 1 ? r.y : (lvl & 3) == 2 ? r.z : r.w;
      ++lvl;
      const double x = gw_u01(rr);
      if (x < cumA) {  // top-left
        col_en = col_st + (col_en - col_st) / 2;
        row_en = row_st + (row_en - row_st) / 2;
      } else if (x < cumB) {  // top-right
        col_st = col_en - (col_en - col_st) / 2;
        row_en = row_st + (row_en - row_st) / 2;
      } else if (x < cumC) {  // bottom-left
        col_en = col_st + (col_en - col_st) / 2;
        row_st = row_en - (row_en - row_st) / 2;
      } else {  // bottom-right
        col_st = col_en - (col_en - col_st) / 2;
        row_st = row_en - (row_en - row_st) / 2;
      }
    }
    src[e] = col_st;
    dst[e] = row_st;
  }
  return gw_build_java_multi(g, m, src.data(), dst.data(), n);
}

// ------------------------------------------------------------------------
// writers
// ------------------------------------------------------------------------
int gw_write_walks_impl(const gw_graph* g, const char* path, const int32_t* walks,
                        const int32_t* lens, int64_t nwalks, int walk_len,
                        std::string* err) {
  // Every label's decimal text once (a flat table), then walks are formatted
  // by copying those strings: chunks of walks in parallel, each into its own
  // buffer, written in order and overlapped with formatting the next batch.
  const int64_t n = g->n;
  std::vector<uint64_t> loff((size_t)n + 1, 0);
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < n; ++v) {
    char tmp[32];
    auto r = std::to_chars(tmp, tmp + sizeof tmp, (long long)g->labels[v]);
    loff[v + 1] = (uint64_t)(r.ptr - tmp) + 1;  // + '\t'
  }
  for (int64_t v = 0; v < n; ++v) loff[v + 1] += loff[v];
  std::vector<char> ltxt(loff[n]);
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < n; ++v) {
    auto r = std::to_chars(ltxt.data() + loff[v], ltxt.data() + loff[v + 1], (long long)g->labels[v]);
    *r.ptr = '\t';
  }
  FILE* f = fopen(path, "wb");
  if (!f) {
    *err = std::string("cannot open '") + path + "'";
    return GW_ERR_IO;
  }
  const int64_t chunk = 1 << 13;
  const int64_t nchunks = (nwalks + chunk - 1) / chunk;
  const int64_t batch = 256;  // chunks formatted per round
  std::vector<std::vector<char>> buf[2];
  int rc = GW_OK;
  int bad = 0;
  for (int64_t b0 = 0, round = 0; b0 < nchunks && rc == GW_OK; b0 += batch, ++round) {
    auto& cur = buf[round & 1];
    const int64_t nb = std::min(batch, nchunks - b0);
    cur.resize((size_t)nb);
    auto& prev = buf[(round + 1) & 1];
    const int64_t nprev = round > 0 ? (int64_t)prev.size() : 0;
#pragma omp parallel
    {
#pragma omp single nowait
      {  // one thread writes the previous round while the others format this one
        for (int64_t k = 0; k < nprev; ++k)
          if (fwrite(prev[k].data(), 1, prev[k].size(), f) != prev[k].size()) rc = GW_ERR_IO;
      }
#pragma omp for schedule(dynamic)
      for (int64_t bi = 0; bi < nb; ++bi) {
        std::vector<char>& out = cur[bi];
        const int64_t w0 = (b0 + bi) * chunk, w1 = std::min(nwalks, w0 + chunk);
        size_t sz = 0;
        for (int64_t wi = w0; wi < w1; ++wi) {
          const int32_t* w = walks + wi * (int64_t)walk_len;
          const int L = lens ? lens[wi] : walk_len;
          for (int t = 0; t < L && w[t] >= 0; ++t) {
            if (w[t] >= n) {
              bad = 1;
              break;
            }
            sz += loff[w[t] + 1] - loff[w[t]];
          }
          ++sz;
        }
        out.resize(sz);
        char* o = out.data();
        for (int64_t wi = w0; wi < w1; ++wi) {
          const int32_t* w = walks + wi * (int64_t)walk_len;
          const int L = lens ? lens[wi] : walk_len;
          for (int t = 0; t < L && w[t] >= 0 && w[t] < n; ++t) {
            const uint64_t a = loff[w[t]], e = loff[w[t] + 1];
            memcpy(o, ltxt.data() + a, e - a);
            o += e - a;
          }
          *o++ = '\n';
        }
        out.resize((size_t)(o - out.data()));
      }
    }
    prev.clear();
    if (bad) break;
  }
  if (!bad && rc == GW_OK) {
    auto& last = buf[(((nchunks + batch - 1) / batch) - 1) & 1];
    if (nchunks > 0)
      for (auto& c : last)
        if (fwrite(c.data(), 1, c.size(), f) != c.size()) rc = GW_ERR_IO;
  }
  if (fclose(f) != 0 && rc == GW_OK) rc = GW_ERR_IO;
  if (bad) {
    *err = "walk entry outside the graph";
    return GW_ERR_RANGE;
  }
  if (rc != GW_OK) *err = "write failed";
  return rc;
}

// --- Java emulation for Print.printByOrder ------------------------------------
// Double.compare (Double.java): numeric order with -0.0 < 0.0 and NaN largest.
static int java_double_compare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x, y;
  double aa = std::isnan(a) ? NAN : a, bb = std::isnan(b) ? NAN : b;
  memcpy(&x, &aa, 8);
  memcpy(&y, &bb, 8);
  return x == y ? 0 : (x < y ? -1 : 1);
}

struct JPair {
  int32_t key;
  double value;
};

// java.util.PriorityQueue (JDK 8) with Pair.compareTo (by value, Pair.java:77-80)
struct JavaPQ {
  std::vector<JPair> q;
  static int cmp(const JPair& a, const JPair& b) { return java_double_compare(a.value, b.value); }
  void offer(JPair e) {
    int k = (int)q.size();
    q.push_back(e);
    while (k > 0) {  // siftUpComparable
      int parent = (k - 1) >> 1;
      if (cmp(e, q[parent]) >= 0) break;
      q[k] = q[parent];
      k = parent;
    }
    q[k] = e;
  }
  void poll() {
    int n = (int)q.size() - 1;
    JPair x = q[n];
    q.pop_back();
    if (n == 0) return;
    int k = 0, half = n >> 1;  // siftDownComparable
    while (k < half) {
      int child = 2 * k + 1;
      JPair c = q[child];
      int right = child + 1;
      if (right < n && cmp(c, q[right]) > 0) c = q[child = right];
      if (cmp(x, c) <= 0) break;
      q[k] = c;
      k = child;
    }
    q[k] = x;
  }
};

// Double.toString / string concatenation of a double (Java): shortest
// round-trip digits; plain notation with at least one fraction digit for
// 1e-3 <= |v| < 1e7, else computerized scientific "d.dddE[-]n" (JLS
// Double.toString).  Eval.precision writes its scores this way (Eval.java:118).
// Assumes JDK 19+ (JDK-4511638 fixed): JDK 8-18 print a few values with more
// digits than the shortest repr; the reference commits no Eval output that
// would pin the JDK it ran on.
void gw_java_double_to_string(double v, std::string* out) {
  if (std::isnan(v)) {
    *out += "NaN";
    return;
  }
  if (std::isinf(v)) {
    *out += v > 0 ? "Infinity" : "-Infinity";
    return;
  }
  if (v == 0.0) {
    *out += std::signbit(v) ? "-0.0" : "0.0";
    return;
  }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  std::string s(buf, r.ptr);  // [-]d[.ddd]e[+-]xx  (shortest round-trip)
  size_t i = 0;
  if (s[0] == '-') {
    *out += '-';
    i = 1;
  }
  const size_t epos = s.find('e');
  std::string digits;
  for (size_t k = i; k < epos; ++k)
    if (s[k] != '.') digits.push_back(s[k]);
  const int e = atoi(s.c_str() + epos + 1);  // value = d1.d2d3... * 10^e
  const double a = std::fabs(v);
  if (a >= 1e-3 && a < 1e7) {
    if (e >= 0) {
      std::string ip = digits.substr(0, std::min(digits.size(), (size_t)e + 1));
      if ((int)ip.size() < e + 1) ip += std::string((size_t)e + 1 - ip.size(), '0');
      std::string fp = digits.size() > (size_t)e + 1 ? digits.substr((size_t)e + 1) : std::string("0");
      *out += ip + "." + fp;
    } else {
      *out += "0." + std::string((size_t)(-e - 1), '0') + digits;
    }
  } else {
    *out += digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : std::string("0")) + "E" +
            std::to_string(e);
  }
}

// String.format("%.Nf") in Java 8: FloatingDecimal digits, HALF_UP rounding.
void gw_java_format_fixed(double v, int decimals, std::string* out) {
  if (std::isnan(v)) {
    *out += "NaN";
    return;
  }
  if (std::isinf(v)) {
    *out += v > 0 ? "Infinity" : "-Infinity";
    return;
  }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  std::string s(buf, r.ptr);  // [-]d[.ddd]e[+-]xx  (shortest round-trip)
  bool neg = false;
  size_t i = 0;
  if (s[0] == '-') {
    neg = true;
    i = 1;
  }
  size_t epos = s.find('e');
  std::string digits;
  for (size_t k = i; k < epos; ++k)
    if (s[k] != '.') digits.push_back(s[k]);
  int exp10 = atoi(s.c_str() + epos + 1);  // value = 0.d1d2.. * 10^(exp10+1)
  int point = exp10 + 1;                    // digits before the decimal point
  // integer part and fraction digits as a digit string with implicit point
  std::string all;
  int intlen;
  if (point <= 0) {
    all = std::string((size_t)(-point), '0') + digits;
    intlen = 0;
  } else {
    all = digits;
    if ((int)all.size() < point) all += std::string(point - all.size(), '0');
    intlen = point;
  }
  // round HALF_UP at intlen + decimals
  int cut = intlen + decimals;
  if ((int)all.size() > cut) {
    bool up = all[cut] >= '5';
    all.resize(cut);
    if (up) {
      int k = cut - 1;
      while (k >= 0 && all[k] == '9') all[k--] = '0';
      if (k >= 0)
        all[k]++;
      else {
        all.insert(all.begin(), '1');
        intlen++;
      }
    }
  }
  if ((int)all.size() < intlen + decimals) all += std::string(intlen + decimals - all.size(), '0');
  std::string ip = intlen > 0 ? all.substr(0, intlen) : std::string("0");
  std::string fp = all.substr(intlen, decimals);
  bool zero = true;
  for (char ch : all)
    if (ch != '0') zero = false;
  if (neg && !zero) *out += '-';
  else if (neg && zero) *out += '-';  // Java prints -0.000000 for negative values rounding to 0
  *out += ip;
  if (decimals > 0) {
    *out += '.';
    *out += fp;
  }
}

static void emit_row(std::string& o, std::string& os, int64_t v, const std::vector<JPair>& row,
                     const std::string& sep, int decimals) {
  char tmp[32];
  auto r = std::to_chars(tmp, tmp + sizeof tmp, (long long)v);
  o.append(tmp, r.ptr);
  os.append(tmp, r.ptr);
  for (const JPair& p : row) {
    r = std::to_chars(tmp, tmp + sizeof tmp, (long long)p.key);
    o += sep;
    o.append(tmp, r.ptr);
    os += sep;
    os.append(tmp, r.ptr);
    os += ':';
    gw_java_format_fixed(p.value, decimals, &os);
  }
  o += "\r\n";
  os += "\r\n";
}

// Print.printByOrder (Print.java:25-53) over dense rows, exact Java order.
int gw_write_sim_dense_impl(const char* path, const double* rows, const int32_t* row_ids,
                            int64_t nrows, int64_t n, int topk, const std::string& sep,
                            int decimals, std::string* err) {
  std::string p2 = std::string(path) + ".sim.txt";
  FILE* f1 = fopen(path, "wb");
  FILE* f2 = fopen(p2.c_str(), "wb");
  if (!f1 || !f2) {
    if (f1) fclose(f1);
    if (f2) fclose(f2);
    *err = std::string("cannot open '") + path + "'";
    return GW_ERR_IO;
  }
  std::vector<std::string> o(nrows), os(nrows);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t r = 0; r < nrows; ++r) {
    const double* row = rows + r * n;
    JavaPQ pq;
    pq.q.reserve(topk + 1);
    for (int64_t i = 0; i < n; ++i) {  // FixedMaxPQ.offer (FixedMaxPQ.java:30-39)
      JPair e{(int32_t)i, row[i]};
      if ((int64_t)pq.q.size() < topk) {
        pq.offer(e);
      } else if (topk > 0 && JavaPQ::cmp(pq.q[0], e) < 0) {
        pq.poll();
        pq.offer(e);
      }
    }
    std::vector<JPair> sorted(pq.q);  // new ArrayList<E>(pq): heap array order
    std::stable_sort(sorted.begin(), sorted.end(), [](const JPair& a, const JPair& b) {
      return JavaPQ::cmp(a, b) > 0;  // Collections.sort(reverseOrder()): stable
    });
    emit_row(o[r], os[r], row_ids ? row_ids[r] : r, sorted, sep, decimals);
  }
  int rc = GW_OK;
  for (int64_t r = 0; r < nrows; ++r) {
    if (fwrite(o[r].data(), 1, o[r].size(), f1) != o[r].size()) rc = GW_ERR_IO;
    if (fwrite(os[r].data(), 1, os[r].size(), f2) != os[r].size()) rc = GW_ERR_IO;
  }
  if (fclose(f1) != 0) rc = GW_ERR_IO;
  if (fclose(f2) != 0) rc = GW_ERR_IO;
  if (rc != GW_OK) *err = "write failed";
  return rc;
}

int gw_write_sim_topk_impl(const char* path, const int32_t* ids, const double* scores,
                           const int32_t* row_ids, int64_t nrows, int topk,
                           const std::string& sep, int decimals, std::string* err) {
  std::string p2 = std::string(path) + ".sim.txt";
  FILE* f1 = fopen(path, "wb");
  FILE* f2 = fopen(p2.c_str(), "wb");
  if (!f1 || !f2) {
    if (f1) fclose(f1);
    if (f2) fclose(f2);
    *err = std::string("cannot open '") + path + "'";
    return GW_ERR_IO;
  }
  std::vector<std::string> o(nrows), os(nrows);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t r = 0; r < nrows; ++r) {
    std::vector<JPair> row;
    for (int k = 0; k < topk; ++k) {
      int32_t id = ids[r * (int64_t)topk + k];
      if (id < 0) break;
      row.push_back(JPair{id, scores[r * (int64_t)topk + k]});
    }
    emit_row(o[r], os[r], row_ids ? row_ids[r] : r, row, sep, decimals);
  }
  int rc = GW_OK;
  for (int64_t r = 0; r < nrows; ++r) {
    if (fwrite(o[r].data(), 1, o[r].size(), f1) != o[r].size()) rc = GW_ERR_IO;
    if (fwrite(os[r].data(), 1, os[r].size(), f2) != os[r].size()) rc = GW_ERR_IO;
  }
  if (fclose(f1) != 0) rc = GW_ERR_IO;
  if (fclose(f2) != 0) rc = GW_ERR_IO;
  if (rc != GW_OK) *err = "write failed";
  return rc;
}

// Print.printByOrder (Print.java:25-53) from sparse rows: row r lists its
// nonzero entries (any order); every other column is 0.0.  FixedMaxPQ(topk)
// is offered (i, sim[v][i]) for i = 0..n-1 (FixedMaxPQ.java:30-39).  The
// first min(topk, n) offers fill the heap whatever their value (zeros
// included); after that an offer enters only when the heap minimum compares
// below it, which a 0.0 never does (scores are >= +0.0), so only the listed
// nonzero entries past the fill need replaying, in id order.  The heap array
// is then stably sorted in reverse (sortedElement(), FixedMaxPQ.java:72-76):
// byte-identical to the dense writer on the same rows.
int gw_sparse_rows_text(const int64_t* begin, const int32_t* len, const int32_t* ids, const double* scores,
                        const int32_t* row_ids, int64_t nrows, int64_t n, int topk, const std::string& sep,
                        int decimals, std::vector<std::string>* o, std::vector<std::string>* os, std::string* err) {
  o->assign(nrows, std::string());
  os->assign(nrows, std::string());
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t r = 0; r < nrows; ++r) {
    std::vector<JPair> ent;
    const int32_t m = len[r];
    if (m < 0) {
      bad = 1;
      continue;
    }
    ent.reserve((size_t)m);
    for (int32_t t = 0; t < m; ++t) ent.push_back(JPair{ids[begin[r] + t], scores[begin[r] + t]});
    std::sort(ent.begin(), ent.end(), [](const JPair& a, const JPair& b) { return a.key < b.key; });
    bool ok = true;
    for (size_t t = 0; t < ent.size(); ++t)
      if (ent[t].key < 0 || ent[t].key >= n || (t > 0 && ent[t].key == ent[t - 1].key) || !(ent[t].value > 0.0))
        ok = false;
    if (!ok) {
      bad = 2;
      continue;
    }
    JavaPQ pq;
    const int64_t fill = std::min<int64_t>(topk, n);
    pq.q.reserve((size_t)fill + 1);
    size_t p = 0;
    for (int64_t i = 0; i < fill; ++i) {
      double v = 0.0;
      if (p < ent.size() && ent[p].key == i) v = ent[p++].value;
      pq.offer(JPair{(int32_t)i, v});
    }
    for (; p < ent.size() && fill > 0; ++p) {
      if (JavaPQ::cmp(pq.q[0], ent[p]) < 0) {
        pq.poll();
        pq.offer(ent[p]);
      }
    }
    std::vector<JPair> sorted(pq.q);
    std::stable_sort(sorted.begin(), sorted.end(), [](const JPair& a, const JPair& b) { return JavaPQ::cmp(a, b) > 0; });
    emit_row((*o)[r], (*os)[r], row_ids ? row_ids[r] : r, sorted, sep, decimals);
  }
  if (bad) {
    *err = bad == 1 ? "a sparse row has length -1 (it did not fit the device output)"
                    : "sparse row entries must be distinct ids in [0, n) with scores > 0";
    return bad == 1 ? GW_ERR_INVALID : GW_ERR_RANGE;
  }
  return GW_OK;
}

int gw_write_sim_sparse_impl(const char* path, const int64_t* begin, const int32_t* len, const int32_t* ids,
                             const double* scores, const int32_t* row_ids, int64_t nrows, int64_t n, int topk,
                             const std::string& sep, int decimals, bool append, std::string* err) {
  std::vector<std::string> o, os;
  int rc = gw_sparse_rows_text(begin, len, ids, scores, row_ids, nrows, n, topk, sep, decimals, &o, &os, err);
  if (rc != GW_OK) return rc;
  std::string p2 = std::string(path) + ".sim.txt";
  FILE* f1 = fopen(path, append ? "ab" : "wb");
  FILE* f2 = fopen(p2.c_str(), append ? "ab" : "wb");
  if (!f1 || !f2) {
    if (f1) fclose(f1);
    if (f2) fclose(f2);
    *err = std::string("cannot open '") + path + "'";
    return GW_ERR_IO;
  }
  for (int64_t r = 0; r < nrows; ++r) {
    if (fwrite(o[r].data(), 1, o[r].size(), f1) != o[r].size()) rc = GW_ERR_IO;
    if (fwrite(os[r].data(), 1, os[r].size(), f2) != os[r].size()) rc = GW_ERR_IO;
  }
  if (fclose(f1) != 0) rc = GW_ERR_IO;
  if (fclose(f2) != 0) rc = GW_ERR_IO;
  if (rc != GW_OK) *err = "write failed";
  return rc;
}

// Print.printByOrder(FixedCacheMap[] sim, outPath, topk) (Print.java:94-124):
// each row iterates its map ascending and prints the last `topk` entries,
// "%.6f" of the float value (Formatter widens the float to double).
int gw_write_sim_cachemap_impl(const char* path, const int32_t* keys, const float* vals, const int32_t* sizes,
                               const int32_t* row_ids, int64_t nrows, int capacity, int topk,
                               const std::string& sep, std::string* err) {
  std::string p2 = std::string(path) + ".sim.txt";
  FILE* f1 = fopen(path, "wb");
  FILE* f2 = fopen(p2.c_str(), "wb");
  if (!f1 || !f2) {
    if (f1) fclose(f1);
    if (f2) fclose(f2);
    *err = std::string("cannot open '") + path + "'";
    return GW_ERR_IO;
  }
  std::vector<std::string> o(nrows), os(nrows);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t r = 0; r < nrows; ++r) {
    std::vector<JPair> row;
    const int size = sizes[r];
    for (int i = std::max(0, size - topk); i < size; ++i)
      row.push_back(JPair{keys[r * (int64_t)capacity + i], (double)vals[r * (int64_t)capacity + i]});
    emit_row(o[r], os[r], row_ids ? row_ids[r] : r, row, sep, 6);
  }
  int rc = GW_OK;
  for (int64_t r = 0; r < nrows; ++r) {
    if (fwrite(o[r].data(), 1, o[r].size(), f1) != o[r].size()) rc = GW_ERR_IO;
    if (fwrite(os[r].data(), 1, os[r].size(), f2) != os[r].size()) rc = GW_ERR_IO;
  }
  if (fclose(f1) != 0) rc = GW_ERR_IO;
  if (fclose(f2) != 0) rc = GW_ERR_IO;
  if (rc != GW_OK) *err = "write failed";
  return rc;
}

// TopSim_Dev.compute (TopSim_Dev.java:64-71): FixedMaxPQ(k) offered every
// (j, rows[i][j]) with rows[i][j] >= min_score in j order, then
// sortedElement(); out_ids[i*k + r] (-1 padded).
void gw_select_fixed_max_pq_impl(const double* rows, int64_t nrows, int64_t n, int k, double min_score,
                                 int32_t* out_ids) {
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t r = 0; r < nrows; ++r) {
    const double* row = rows + r * n;
    JavaPQ pq;
    pq.q.reserve(k + 1);
    for (int64_t i = 0; i < n; ++i) {
      if (!(row[i] >= min_score)) continue;
      JPair e{(int32_t)i, row[i]};
      if ((int64_t)pq.q.size() < k) {
        pq.offer(e);
      } else if (k > 0 && JavaPQ::cmp(pq.q[0], e) < 0) {
        pq.poll();
        pq.offer(e);
      }
    }
    std::vector<JPair> sorted(pq.q);
    std::stable_sort(sorted.begin(), sorted.end(), [](const JPair& a, const JPair& b) {
      return JavaPQ::cmp(a, b) > 0;
    });
    for (int q = 0; q < k; ++q) out_ids[r * (int64_t)k + q] = q < (int)sorted.size() ? sorted[(size_t)q].key : -1;
  }
}
