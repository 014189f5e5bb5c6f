// C ABI of libgraphwalk (include/graphwalk.h): argument validation, error
// reporting and dispatch to the host builders / HIP entry points.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "gw_internal.h"

// host implementations (gw_graph_host.cpp)
int gw_load_edgelist_impl(gw_graph* g, const char* path, const char* delim, int semantics,
                          int directed, int weighted, int64_t vcount);
int gw_rmat_impl(gw_graph* g, int scale, int edge_factor, double a, double b, double c,
                 uint64_t seed);
int gw_rmat_java_impl(gw_graph* g, int64_t n, int64_t m, double a, double b, double c, uint64_t seed);
int gw_write_walks_impl(const gw_graph* g, const char* path, const int32_t* walks,
                        const int32_t* lens, int64_t nwalks, int walk_len, std::string* err);
int gw_write_sim_dense_impl(const char* path, const double* rows, const int32_t* row_ids,
                            int64_t nrows, int64_t n, int topk, const std::string& sep,
                            int decimals, std::string* err);
int gw_write_sim_topk_impl(const char* path, const int32_t* ids, const double* scores,
                           const int32_t* row_ids, int64_t nrows, int topk,
                           const std::string& sep, int decimals, std::string* err);
void gw_java_double_to_string(double v, std::string* out);
int gw_write_sim_cachemap_impl(const char* path, const int32_t* keys, const float* vals, const int32_t* sizes,
                               const int32_t* row_ids, int64_t nrows, int capacity, int topk,
                               const std::string& sep, std::string* err);
void gw_select_fixed_max_pq_impl(const double* rows, int64_t nrows, int64_t n, int k, double min_score,
                                 int32_t* out_ids);
int gw_hip_device_count(int* count);

static thread_local std::string tls_err;

void gw_set_tls_error(const std::string& s) { tls_err = s; }

int gw_fail(gw_graph* g, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (g) g->err = buf;
  tls_err = buf;
  return code;
}

// propagate a handle error to the thread-local slot too
static int ret(gw_graph* g, int rc) {
  if (rc != GW_OK && g) tls_err = g->err;
  return rc;
}

extern "C" {

const char* gw_version(void) { return "graphwalk 0.1.0 (gfx950)"; }

const char* gw_last_error(const gw_graph* g) {
  if (g) return g->err.c_str();
  return tls_err.c_str();
}

const char* gw_strerror(int code) {
  switch (code) {
    case GW_OK: return "ok";
    case GW_ERR_INVALID: return "invalid argument";
    case GW_ERR_IO: return "I/O error";
    case GW_ERR_PARSE: return "parse error";
    case GW_ERR_NOMEM: return "out of memory";
    case GW_ERR_DEVICE: return "HIP device error";
    case GW_ERR_STATE: return "invalid call order";
    case GW_ERR_UNSUPPORTED: return "unsupported";
    case GW_ERR_RANGE: return "id out of range";
    case GW_ERR_KEY: return "missing key";
    case GW_ERR_ZERODIV: return "division by zero";
    case GW_ERR_CAPACITY: return "capacity exceeded";
    default: return "unknown error";
  }
}

gw_device_guard::gw_device_guard(int dev) {
  if (dev < 0) return;  // host-only handle: nothing to select
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) {
    ok = false;
    return;
  }
  if (cur == dev) return;
  if (hipSetDevice(dev) != hipSuccess) {
    ok = false;
    return;
  }
  prev = cur;
}
gw_device_guard::~gw_device_guard() {
  if (prev >= 0) (void)hipSetDevice(prev);
}

int gw_device_count(int* count) {
  if (!count) return gw_fail(nullptr, GW_ERR_INVALID, "count is NULL");
  int rc = gw_hip_device_count(count);
  if (rc != GW_OK) return gw_fail(nullptr, rc, "no HIP device visible");
  return GW_OK;
}

int gw_graph_load_edgelist(const char* path, const char* delim, int semantics, int directed,
                           int weighted, int64_t vcount, gw_graph** out) {
  if (!path || !out) return gw_fail(nullptr, GW_ERR_INVALID, "path/out is NULL");
  *out = nullptr;
  if (semantics == GW_SEM_JAVA_MULTI && (weighted || directed))
    return gw_fail(nullptr, GW_ERR_UNSUPPORTED, "JAVA_MULTI graphs are undirected and unweighted (Graph.java:12)");
  gw_graph* g = new gw_graph();
  int rc = gw_load_edgelist_impl(g, path, delim, semantics, directed, weighted, vcount);
  if (rc != GW_OK) {
    tls_err = g->err;
    delete g;
    return rc;
  }
  *out = g;
  return GW_OK;
}

int gw_graph_from_edges(int64_t m, const int64_t* src, const int64_t* dst, const double* w,
                        int semantics, int directed, int64_t vcount, gw_graph** out) {
  if (!out || m < 0 || (m > 0 && (!src || !dst))) return gw_fail(nullptr, GW_ERR_INVALID, "bad edge arrays");
  *out = nullptr;
  gw_graph* g = new gw_graph();
  int rc;
  if (semantics == GW_SEM_NX_SIMPLE)
    rc = gw_build_nx_simple(g, m, src, dst, w, directed);
  else if (semantics == GW_SEM_JAVA_MULTI)
    rc = (w || directed) ? gw_fail(g, GW_ERR_UNSUPPORTED, "JAVA_MULTI graphs are undirected and unweighted")
                         : gw_build_java_multi(g, m, src, dst, vcount);
  else
    rc = gw_fail(g, GW_ERR_INVALID, "unknown semantics %d", semantics);
  if (rc != GW_OK) {
    tls_err = g->err;
    delete g;
    return rc;
  }
  *out = g;
  return GW_OK;
}

int gw_graph_from_csr(int64_t n, const int64_t* offsets, const int32_t* nbrs, const double* weights,
                      const int64_t* labels, const int32_t* node_order, int semantics, int directed,
                      gw_graph** out) {
  if (!out || n < 0 || !offsets) return gw_fail(nullptr, GW_ERR_INVALID, "bad CSR arguments");
  *out = nullptr;
  if (semantics != GW_SEM_NX_SIMPLE && semantics != GW_SEM_JAVA_MULTI)
    return gw_fail(nullptr, GW_ERR_INVALID, "unknown semantics %d", semantics);
  if (n >= (int64_t)INT32_MAX) return gw_fail(nullptr, GW_ERR_UNSUPPORTED, "too many vertices");
  if (offsets[0] != 0) return gw_fail(nullptr, GW_ERR_INVALID, "offsets[0] != 0");
  for (int64_t v = 0; v < n; ++v)
    if (offsets[v + 1] < offsets[v]) return gw_fail(nullptr, GW_ERR_INVALID, "offsets not monotone at %lld", (long long)v);
  const int64_t nnz = offsets[n];
  if (nnz > 0 && !nbrs) return gw_fail(nullptr, GW_ERR_INVALID, "nbrs is NULL");
  for (int64_t v = 0; v < n; ++v)
    for (int64_t k = offsets[v]; k < offsets[v + 1]; ++k) {
      if (nbrs[k] < 0 || nbrs[k] >= n) return gw_fail(nullptr, GW_ERR_RANGE, "neighbour id %d out of range", nbrs[k]);
      if (semantics == GW_SEM_NX_SIMPLE && k > offsets[v] && nbrs[k] <= nbrs[k - 1])
        return gw_fail(nullptr, GW_ERR_INVALID, "NX_SIMPLE rows must be strictly increasing (row %lld)", (long long)v);
    }
  gw_graph* g = new gw_graph();
  g->semantics = semantics;
  g->directed = directed ? 1 : 0;
  g->weighted = weights ? 1 : 0;
  g->n = n;
  g->nnz = nnz;
  g->offsets.assign(offsets, offsets + n + 1);
  g->nbrs.assign(nbrs, nbrs + nnz);
  if (weights) g->weights.assign(weights, weights + nnz);
  g->labels.resize(n);
  g->order.resize(n);
  std::vector<char> seen(n, 0);
  for (int64_t v = 0; v < n; ++v) {
    g->labels[v] = labels ? labels[v] : v;
    int32_t o = node_order ? node_order[v] : (int32_t)v;
    if (o < 0 || o >= n || seen[o]) {
      delete g;
      return gw_fail(nullptr, GW_ERR_INVALID, "node_order is not a permutation of [0,n)");
    }
    seen[o] = 1;
    g->order[v] = o;
  }
  g->max_degree = 0;
  for (int64_t v = 0; v < n; ++v) g->max_degree = std::max<int64_t>(g->max_degree, offsets[v + 1] - offsets[v]);
  *out = g;
  return GW_OK;
}

int gw_graph_rmat(int scale, int edge_factor, double a, double b, double c, uint64_t seed,
                  gw_graph** out) {
  if (!out) return gw_fail(nullptr, GW_ERR_INVALID, "out is NULL");
  *out = nullptr;
  gw_graph* g = new gw_graph();
  int rc = gw_rmat_impl(g, scale, edge_factor, a, b, c, seed);
  if (rc != GW_OK) {
    tls_err = g->err;
    delete g;
    return rc;
  }
  *out = g;
  return GW_OK;
}

int gw_graph_rmat_java(int64_t n, int64_t m, double a, double b, double c, uint64_t seed, gw_graph** out) {
  if (!out) return gw_fail(nullptr, GW_ERR_INVALID, "out is NULL");
  *out = nullptr;
  gw_graph* g = new gw_graph();
  int rc = gw_rmat_java_impl(g, n, m, a, b, c, seed);
  if (rc != GW_OK) {
    tls_err = g->err;
    delete g;
    return rc;
  }
  *out = g;
  return GW_OK;
}

int gw_graph_info(const gw_graph* g, gw_graph_info_t* info) {
  if (!g || !info) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle/info");
  info->n = g->n;
  info->nnz = g->nnz;
  info->max_degree = g->max_degree;
  info->edge_alias_entries = g->edge_alias_entries;
  info->semantics = g->semantics;
  info->directed = g->directed;
  info->weighted = g->weighted;
  info->device = g->device;
  info->sampler_bytes = (g->d.bs_nbr ? g->bitset_words * 4 + g->nnz * (int64_t)sizeof(gw_bs_nbr) : 0) +
                        (g->d.sent ? g->nnz * (int64_t)sizeof(gw_ts_ent) : 0) +
                        (g->d.eh ? 4 * g->nnz * (int64_t)sizeof(int32_t) : 0);
  info->n2v_mode = g->n2v_prepared ? g->n2v_mode : -1;
  info->listed = (g->n2v_prepared && g->n2v_mode == GW_N2V_REJECTION && g->d.bs_nbr) ? 1 : 0;
  return GW_OK;
}

int gw_graph_export_csr(const gw_graph* g, int64_t* offsets, int32_t* nbrs, double* weights,
                        int64_t* labels, int32_t* node_order) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  if (offsets) memcpy(offsets, g->offsets.data(), sizeof(int64_t) * (g->n + 1));
  if (nbrs && g->nnz) memcpy(nbrs, g->nbrs.data(), sizeof(int32_t) * g->nnz);
  if (weights && g->nnz) {
    if (g->weighted)
      memcpy(weights, g->weights.data(), sizeof(double) * g->nnz);
    else
      for (int64_t i = 0; i < g->nnz; ++i) weights[i] = 1.0;
  }
  if (labels && g->n) memcpy(labels, g->labels.data(), sizeof(int64_t) * g->n);
  if (node_order && g->n) memcpy(node_order, g->order.data(), sizeof(int32_t) * g->n);
  return GW_OK;
}

int gw_graph_free(gw_graph* g) {
  if (!g) return GW_OK;
  {
    gw_device_guard dg(g->device);  // best effort: release even if the switch failed
    gw_dev_release(g);
  }
  delete g;
  return GW_OK;
}

int gw_graph_set_options(gw_graph* g, const gw_options_t* opt) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  if (!opt) {
    g->opt = gw_options_t{0, 0, -1, 0, 0, 0, 0};
    return GW_OK;
  }
  if (opt->table_budget_bytes < 0 || opt->expected_steps < 0 || opt->listed < -1 || opt->listed > 1 ||
      opt->simrank_hbm_row < 0 || opt->simrank_hbm_row > 1 || opt->host_chunk_bytes < 0 ||
      opt->topsim_part_shrink < 0 || opt->topsim_part_shrink > 8 || opt->reserved0 != 0)
    return gw_fail(g, GW_ERR_INVALID, "option out of range");
  g->opt = *opt;
  return GW_OK;
}

int gw_graph_get_options(const gw_graph* g, gw_options_t* opt) {
  if (!g || !opt) return gw_fail(nullptr, GW_ERR_INVALID, "NULL argument");
  *opt = g->opt;
  return GW_OK;
}

int gw_graph_to_device(gw_graph* g, int device) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, device);
  return ret(g, gw_dev_upload(g, device));
}

int gw_n2v_prepare(gw_graph* g, double p, double q, int mode) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (!(p > 0) || !(q > 0)) return ret(g, gw_fail(g, GW_ERR_ZERODIV, "p and q must be > 0 (node2vec.py:70-76 divides by them)"));
  if (mode != GW_N2V_REPLAY && mode != GW_N2V_REJECTION && mode != GW_N2V_BITSET && mode != GW_N2V_AUTO)
    return ret(g, gw_fail(g, GW_ERR_INVALID, "unknown mode %d", mode));
  if (mode == GW_N2V_BITSET && (g->weighted || g->directed || g->semantics != GW_SEM_NX_SIMPLE))
    return ret(g, gw_fail(g, GW_ERR_UNSUPPORTED, "GW_N2V_BITSET needs an unweighted undirected NX_SIMPLE graph"));
  if (g->semantics != GW_SEM_NX_SIMPLE && !(p == 1.0 && q == 1.0))
    return ret(g, gw_fail(g, GW_ERR_UNSUPPORTED, "biased walks need NX_SIMPLE semantics (sorted rows)"));
  if (g->weighted) {
    for (int64_t v = 0; v < g->n; ++v) {
      double s = 0;
      for (int64_t k = g->offsets[v]; k < g->offsets[v + 1]; ++k) s += g->weights[k];
      if (g->offsets[v + 1] > g->offsets[v] && s == 0.0)
        return ret(g, gw_fail(g, GW_ERR_ZERODIV, "weights of vertex %lld sum to 0 (node2vec.py:95)", (long long)g->labels[v]));
    }
  }
  return ret(g, gw_dev_n2v_prepare(g, p, q, mode));
}

int gw_n2v_export_alias(const gw_graph* g_, int32_t* node_J, double* node_q, int64_t* edge_off,
                        int32_t* edge_J, double* edge_q);

int gw_alias_setup(int device, const double* probs, int64_t K, int64_t* J, double* q) {
  if (K < 0 || (K > 0 && (!probs || !J || !q))) return gw_fail(nullptr, GW_ERR_INVALID, "bad arrays");
  std::string err;
  GW_GUARD_DEVICE(nullptr, device);
  int rc = gw_dev_alias_setup(device, probs, K, J, q, &err);
  if (rc != GW_OK) return gw_fail(nullptr, rc, "%s", err.c_str());
  return GW_OK;
}

int gw_n2v_walks_replay(gw_graph* g, int walk_len, int64_t nwalks, const int32_t* starts,
                        const double* uniforms, int64_t n_uniforms, int32_t* out_walks,
                        int32_t* out_len, int64_t* uniforms_used) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (!g->n2v_prepared || g->n2v_mode != GW_N2V_REPLAY)
    return ret(g, gw_fail(g, GW_ERR_STATE, "call gw_n2v_prepare(..., GW_N2V_REPLAY) first"));
  if (walk_len < 1 || nwalks < 0 || (nwalks > 0 && (!starts || !out_walks || !out_len)) ||
      n_uniforms < 0 || (n_uniforms > 0 && !uniforms))
    return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  for (int64_t w = 0; w < nwalks; ++w)
    if (starts[w] < 0 || starts[w] >= g->n) return ret(g, gw_fail(g, GW_ERR_KEY, "start vertex %d not in graph", starts[w]));
  if (nwalks == 0) {
    if (uniforms_used) *uniforms_used = 0;
    return GW_OK;
  }
  return ret(g, gw_dev_n2v_walks_replay(g, walk_len, nwalks, starts, uniforms, n_uniforms, out_walks,
                                        out_len, uniforms_used));
}

int gw_n2v_walks(gw_graph* g, int walk_len, uint64_t seed, int64_t walk_begin, int64_t walk_count,
                 int shuffle, int32_t* out_walks_dev, int32_t* out_len_dev, uint64_t* counters_dev,
                 void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (!g->n2v_prepared) return ret(g, gw_fail(g, GW_ERR_STATE, "call gw_n2v_prepare first"));
  if (walk_len < 1 || walk_begin < 0 || walk_count < 0 || (walk_count > 0 && !out_walks_dev))
    return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  if (g->n == 0) return walk_count == 0 ? GW_OK : ret(g, gw_fail(g, GW_ERR_INVALID, "empty graph"));
  return ret(g, gw_dev_n2v_walks(g, walk_len, seed, walk_begin, walk_count, shuffle, out_walks_dev,
                                 out_len_dev, counters_dev, stream));
}

int gw_topsim_prepare(gw_graph* g, int variant, int sample, int step, int topk) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  return ret(g, gw_dev_topsim_prepare(g, variant, sample, step, topk));
}

int gw_topsim(gw_graph* g, int variant, int sample, int step, double C, uint64_t seed,
              const int32_t* sources_dev, int64_t nsrc, int topk, int32_t* out_ids_dev,
              double* out_scores_dev, int64_t* stats_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->device < 0) return ret(g, gw_fail(g, GW_ERR_STATE, "graph is not on a device"));
  if (nsrc < 0 || (nsrc > 0 && (!sources_dev || !out_ids_dev || !out_scores_dev)) || topk < 0)
    return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  return ret(g, gw_dev_topsim(g, variant, sample, step, C, seed, sources_dev, nsrc, topk, out_ids_dev,
                              out_scores_dev, nullptr, stats_dev, stream));
}

int gw_topsim_dense(gw_graph* g, int variant, int sample, int step, double C, uint64_t seed,
                    const int32_t* sources_dev, int64_t nsrc, double* out_rows_dev,
                    int64_t* stats_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->device < 0) return ret(g, gw_fail(g, GW_ERR_STATE, "graph is not on a device"));
  if (nsrc < 0 || (nsrc > 0 && (!sources_dev || !out_rows_dev)))
    return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  return ret(g, gw_dev_topsim(g, variant, sample, step, C, seed, sources_dev, nsrc, 0, nullptr, nullptr,
                              out_rows_dev, stats_dev, stream));
}

int gw_topsim_sparse(gw_graph* g, int variant, int sample, int step, double C, uint64_t seed,
                     const int32_t* sources_dev, int64_t nsrc, int64_t capacity, int64_t* row_begin_dev,
                     int32_t* row_len_dev, int32_t* out_ids_dev, double* out_scores_dev, int64_t* used_dev,
                     int64_t* stats_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->device < 0) return ret(g, gw_fail(g, GW_ERR_STATE, "graph is not on a device"));
  if (nsrc < 0 || capacity < 0 || !used_dev ||
      (nsrc > 0 && (!sources_dev || !row_begin_dev || !row_len_dev || (capacity > 0 && (!out_ids_dev || !out_scores_dev)))))
    return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  if (hipMemsetAsync(used_dev, 0, sizeof(int64_t), (hipStream_t)stream) != hipSuccess)
    return ret(g, gw_fail(g, GW_ERR_DEVICE, "hipMemsetAsync(used_dev) failed"));
  gw_ts_sparse sp;
  sp.cap = capacity;
  sp.begin = row_begin_dev;
  sp.len = row_len_dev;
  sp.ids = out_ids_dev;
  sp.scores = out_scores_dev;
  sp.cursor = reinterpret_cast<unsigned long long*>(used_dev);
  return ret(g, gw_dev_topsim(g, variant, sample, step, C, seed, sources_dev, nsrc, 0, nullptr, nullptr, nullptr,
                              stats_dev, stream, &sp));
}

int gw_topsim_m(gw_graph* g, int variant, int capacity, int sample, int step, double C, uint64_t seed,
                const int32_t* sources_dev, int64_t nsrc, int32_t* out_keys_dev, float* out_vals_dev,
                int32_t* out_size_dev, int64_t* stats_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->device < 0) return ret(g, gw_fail(g, GW_ERR_STATE, "graph is not on a device"));
  if (nsrc < 0 || capacity < 1 || (nsrc > 0 && (!sources_dev || !out_keys_dev || !out_vals_dev || !out_size_dev)))
    return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  return ret(g, gw_dev_topsim_m(g, variant, capacity, sample, step, C, seed, sources_dev, nsrc, out_keys_dev,
                                out_vals_dev, out_size_dev, stats_dev, stream));
}

int gw_topsim_double(gw_graph* g, int sample, int step, double C, uint64_t seed, double* sim_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->n > 0 && !sim_dev) return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  return ret(g, gw_dev_topsim_double(g, sample, step, C, seed, sim_dev, stream));
}

int gw_topsim_dev(gw_graph* g, int sample, int step, int topK, int singleStep, double C, uint64_t seed,
                  const int32_t* cand_dev, double* sim_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->n > 0 && (!sim_dev || (topK > 0 && !cand_dev))) return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  return ret(g, gw_dev_topsim_dev(g, sample, step, topK, singleStep, C, seed, cand_dev, sim_dev, stream));
}

int gw_double_random_walk(gw_graph* g, int sample, int step, double C, uint64_t seed, double* sim_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->n > 0 && !sim_dev) return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  return ret(g, gw_dev_double_random_walk(g, sample, step, C, seed, sim_dev, stream));
}

int gw_simrank_naive(gw_graph* g, double C, int iters, double* sim_dev, void* stream) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->device < 0) return ret(g, gw_fail(g, GW_ERR_STATE, "graph is not on a device"));
  if (g->directed) return ret(g, gw_fail(g, GW_ERR_UNSUPPORTED, "naive SimRank needs an undirected graph"));
  if (iters < 0 || (g->n > 0 && !sim_dev)) return ret(g, gw_fail(g, GW_ERR_INVALID, "bad arguments"));
  return ret(g, gw_dev_simrank_naive(g, C, iters, sim_dev, stream));
}

int gw_write_walks_text(const gw_graph* g, const char* path, const int32_t* walks,
                        const int32_t* lens, int64_t nwalks, int walk_len) {
  if (!g || !path || (nwalks > 0 && !walks) || walk_len < 1)
    return gw_fail(nullptr, GW_ERR_INVALID, "bad arguments");
  std::string err;  // (entries >= n are refused inside the parallel writer: GW_ERR_RANGE)
  int rc = gw_write_walks_impl(g, path, walks, lens, nwalks, walk_len, &err);
  if (rc != GW_OK) return gw_fail(nullptr, rc, "%s", err.c_str());
  return GW_OK;
}

int gw_write_sim_text_dense(const char* path, const double* rows, const int32_t* row_ids,
                            int64_t nrows, int64_t n, int topk, const char* sep, int decimals) {
  if (!path || (nrows > 0 && !rows) || n < 0 || topk < 0 || decimals < 0 || decimals > 30)
    return gw_fail(nullptr, GW_ERR_INVALID, "bad arguments");
  std::string err;
  int rc = gw_write_sim_dense_impl(path, rows, row_ids, nrows, n, topk, sep ? sep : ",", decimals, &err);
  if (rc != GW_OK) return gw_fail(nullptr, rc, "%s", err.c_str());
  return GW_OK;
}

int gw_write_sim_text_topk(const char* path, const int32_t* ids, const double* scores,
                           const int32_t* row_ids, int64_t nrows, int topk, const char* sep,
                           int decimals) {
  if (!path || (nrows > 0 && (!ids || !scores)) || topk < 0 || decimals < 0 || decimals > 30)
    return gw_fail(nullptr, GW_ERR_INVALID, "bad arguments");
  std::string err;
  int rc = gw_write_sim_topk_impl(path, ids, scores, row_ids, nrows, topk, sep ? sep : ",", decimals, &err);
  if (rc != GW_OK) return gw_fail(nullptr, rc, "%s", err.c_str());
  return GW_OK;
}

int gw_write_sim_text_sparse(const char* path, const int64_t* row_begin, const int32_t* row_len, const int32_t* ids,
                             const double* scores, const int32_t* row_ids, int64_t nrows, int64_t n, int topk,
                             const char* sep, int decimals) {
  if (!path || n < 0 || topk < 0 || decimals < 0 || decimals > 30 || nrows < 0 ||
      (nrows > 0 && (!row_begin || !row_len)))
    return gw_fail(nullptr, GW_ERR_INVALID, "bad arguments");
  for (int64_t r = 0; r < nrows; ++r)
    if (row_len[r] > 0 && (!ids || !scores || row_begin[r] < 0))
      return gw_fail(nullptr, GW_ERR_INVALID, "bad arguments");
  std::string err;
  int rc = gw_write_sim_sparse_impl(path, row_begin, row_len, ids, scores, row_ids, nrows, n, topk, sep ? sep : ",",
                                    decimals, false, &err);
  if (rc != GW_OK) return gw_fail(nullptr, rc, "%s", err.c_str());
  return GW_OK;
}

int gw_select_fixed_max_pq(const double* rows, int64_t nrows, int64_t n, int k, double min_score, int32_t* out_ids) {
  if ((nrows > 0 && (!rows || !out_ids)) || n < 0 || k < 0) return gw_fail(nullptr, GW_ERR_INVALID, "bad arguments");
  gw_select_fixed_max_pq_impl(rows, nrows, n, k, min_score, out_ids);
  return GW_OK;
}

int gw_write_sim_text_cachemap(const char* path, const int32_t* keys, const float* vals, const int32_t* sizes,
                               const int32_t* row_ids, int64_t nrows, int capacity, int topk, const char* sep) {
  if (!path || (nrows > 0 && (!keys || !vals || !sizes)) || capacity < 1 || topk < 0)
    return gw_fail(nullptr, GW_ERR_INVALID, "bad arguments");
  for (int64_t r = 0; r < nrows; ++r)
    if (sizes[r] < 0 || sizes[r] > capacity) return gw_fail(nullptr, GW_ERR_INVALID, "row size outside [0, capacity]");
  std::string err;
  int rc = gw_write_sim_cachemap_impl(path, keys, vals, sizes, row_ids, nrows, capacity, topk, sep ? sep : ",", &err);
  if (rc != GW_OK) return gw_fail(nullptr, rc, "%s", err.c_str());
  return GW_OK;
}

int gw_format_java_double(double v, char* buf, int64_t buflen) {
  std::string s;
  gw_java_double_to_string(v, &s);
  if (!buf || buflen < (int64_t)s.size() + 1) return gw_fail(nullptr, GW_ERR_RANGE, "buffer too small (%lld B needed)",
                                                             (long long)s.size() + 1);
  memcpy(buf, s.c_str(), s.size() + 1);
  return GW_OK;
}

}  // extern "C"

