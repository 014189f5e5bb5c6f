// Internal definitions shared by the host translation units and the HIP
// translation units of libgraphwalk.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/graphwalk.h"

// Diagnostic A/B knobs (timing experiments; some of them return wrong walks on
// purpose) exist only in libraries built with -DGW_DIAG (build.py --diag writes
// gwamd/libgraphwalk_diag.so, loaded with GW_LIB=...): the release library
// neither reads the GW_DIAG_* variables nor carries their code paths.
#ifdef GW_DIAG
#include <cstdlib>
constexpr bool kGwDiag = true;
#define GW_DIAG_ENV(name) std::getenv(name)
#else
constexpr bool kGwDiag = false;
#define GW_DIAG_ENV(name) ((const char*)nullptr)
#endif

// Device-side mirror of the CSR (all pointers are HBM allocations owned by
// the handle).  Layout (SoA, one array per field so each gather touches only
// the bytes it needs):
//   offsets  int64[n+1]   row bounds (16 B per step: offsets[v], offsets[v+1])
//   nbrs     int32[nnz]   neighbour dense ids, row order = draw order
//   weights  f64[nnz]     (weighted graphs only)
//   wsum     f64[n]       per-row weight sums (weighted graphs only)
//   order    int32[n]     reference G.nodes() order (walk start order)
//   deg      int32[n]     row lengths (TopSim reads deg(mid), deg(target))
//   node_J/q int32/f64[nnz] per-node alias tables (weighted or REPLAY)
//   edge_off int64[nnz+1], edge_J/q per-edge alias tables (REPLAY only)
//   bitmap   u32[16*nnz/32] has_edge membership pre-filter (BITSET build; REJECTION when eh does not fit)
//   eh       int32[4*nnz] per-row bucketed neighbour sets (REJECTION, p/q != 1): deg(v) 16 B buckets at 4*offsets[v]
//   bs_*     per-edge common-neighbour bitsets (BITSET mode, sum(deg^2) bits)
constexpr uint32_t GW_BS_PACK_D = 65536;  // deg(x) below this: kp and c share one word
struct gw_bs_nbr {  // GW_N2V_BITSET: one 64 B entry (one HBM sector) per adjacency slot (u -> x)
  uint32_t x, d;                 // neighbour, deg(x)
  uint32_t off;                  // offsets[x] (this mode needs < 2^32 adjacency entries)
  uint32_t meta;                 // payload mode | Elias-Fano l << 2 | U << 7 | region dir blocks << 16
  uint32_t r[12];                // d < 65536: r[0] = kp | c << 16, r[1..11] = payload (352 bits);
                                 // else r[0] = kp, r[1] = c, r[2..11] = payload (320 bits).
                                 // kp = position of u in N(x), c = #common neighbours.  Payload,
                                 // by (c, d): c <= 22 && d < 65536: positions of the common
                                 // neighbours (u16, ascending, 0xFFFF padded); else d <= 352:
                                 // the bitset itself; else Elias-Fano positions when they fit;
                                 // else w[0] = region block index, directory, draw filter.
                                 // (The build keeps r[0] = kp, r[1] = c until pass 2 packs.)
};
#if defined(__HIPCC__)
#define GW_BS_HD __host__ __device__
#else
#define GW_BS_HD
#endif
GW_BS_HD inline uint32_t gw_bs_pw(uint32_t d) { return d < GW_BS_PACK_D ? 11u : 10u; }  // payload words
GW_BS_HD inline uint32_t gw_bs_bits(uint32_t d) { return 32u * gw_bs_pw(d); }            // payload bits
GW_BS_HD inline bool gw_bs_is_list(uint32_t c, uint32_t d) { return c <= 22u && d < GW_BS_PACK_D; }
GW_BS_HD inline bool gw_bs_is_inline(uint32_t d) { return d <= gw_bs_bits(d); }
// Elias-Fano payload (neither list nor inline bitset): the unary high parts
// (U = c + ((d-1)>>l) + 1 bits) first, then l low bits per position; fits
// when U + c*l <= the payload bits.  l = floor(log2(d / c)).
GW_BS_HD inline int gw_bs_ef_l(uint32_t c, uint32_t d) { return 31 - __builtin_clz(d / c); }
GW_BS_HD inline bool gw_bs_is_ef(uint32_t c, uint32_t d) {
  if (gw_bs_is_list(c, d) || gw_bs_is_inline(d) || c == 0) return false;
  const int l = gw_bs_ef_l(c, d);
  return (uint64_t)c * l + c + ((d - 1) >> l) + 1 <= (uint64_t)gw_bs_bits(d);  // U + c*l
}
static_assert(sizeof(gw_bs_nbr) == 64, "bitset entry must be one 64 B sector");

struct alignas(16) gw_ts_ent {  // adjacency slot (u -> x): everything a walker's next step needs
  int32_t x, d;      // neighbour, deg(x)
  int64_t off;       // offsets[x]
};

struct gw_dev_graph {
  int64_t n = 0, nnz = 0;
  int64_t* offsets = nullptr;
  int32_t* nbrs = nullptr;
  double* weights = nullptr;
  double* wsum = nullptr;
  int32_t* order = nullptr;
  int32_t* deg = nullptr;
  int32_t* node_J = nullptr;
  double* node_q = nullptr;
  int64_t* edge_off = nullptr;
  int32_t* edge_J = nullptr;
  double* edge_q = nullptr;
  uint32_t* bitmap = nullptr;  // has_edge pre-filter, 16 bits per entry
  int32_t* eh = nullptr;       // REJECTION mode: exact has_edge hash, deg(v) buckets of 4 int32 slots at 4*offsets[v]
  uint32_t* bs_region = nullptr;  // GW_N2V_BITSET per-edge regions (gw_n2v_bitset.hip)
  gw_bs_nbr* bs_nbr = nullptr;    // [nnz] neighbour + region offset
  gw_ts_ent* sent = nullptr;      // [nnz] REJECTION mode: {x, deg(x), offsets[x]} per slot
};



struct gw_topsim_ws {
  int variant = -1, sample = 0, step = 0, topk = 0;
  int blocks = 0;               // persistent workgroups
  int64_t level_cap = 0;        // records per level per workgroup
  int64_t spawn_cap = 0;        // spawner records per workgroup
  int64_t touch_cap = 0;        // distinct targets per workgroup
  int lds_row = 0;              // accumulator: 0 dense LDS row, 1 LDS hash (8192 slots)
  size_t lds_bytes = 0;         // dynamic LDS per workgroup
  int32_t* lvl_vertex = nullptr;  // [blocks][levels][level_cap]
  int32_t* lvl_parent = nullptr;  // [blocks][levels][level_cap]
  int32_t* lvl_deg = nullptr;     // [blocks][levels][level_cap] deg(vertex)
  int64_t* lvl_off = nullptr;     // [blocks][levels][level_cap] offsets[vertex]
  gw_ts_ent* ent = nullptr;       // [nnz] slot entries (built once per graph)
  double* lvl_mass = nullptr;     // [blocks][2][level_cap] (current/next)
  int32_t* child_off = nullptr;   // [blocks][level_cap+1] expansion scan
  int32_t* spawn_node = nullptr;  // [blocks][spawn_cap] index into its level
  int32_t* spawn_level = nullptr; // [blocks][spawn_cap]
  int32_t* spawn_first = nullptr; // [blocks][spawn_cap+1] walker prefix
  double* spawn_mass = nullptr;   // [blocks][spawn_cap] child mass m/ceil(m)
  double* acc_row = nullptr;      // [blocks][touch_cap] overflow hash, 16 B slots {int32 key (-1 empty), pad, f64 value}
  double* ov_list = nullptr;      // [blocks][touch_cap] compacted overflow values of a source (hash mode)
  int32_t* touched = nullptr;     // [blocks][touch_cap] claimed overflow slots
  int64_t app_cap = 0;            // pipelined hash mode: appended pair updates per source (heavy sources)
  double* app = nullptr;          // [blocks][2 app_cap] 16 B entries {int32 key, pad, f64 value}: a heavy source's partitions
  int32_t* claim = nullptr;       // [blocks][touch_cap] a heavy source's claimed overflow-hash slots
  long long* redo = nullptr;      // [5] the caller's stats / sparse cursor before a launch that may be re-run
  int pipe = 0;                   // pipelined kernel (levels of the next source built by wave 0 during
                                  // the walkers): level / spawner scratch doubled per workgroup
  int diag_pipe = -1;             // -DGW_DIAG builds: the GW_DIAG_TS_PIPE_MAX override the workspace was made for
  int64_t enum_cap = 0;           // enumerated-node pair updates per source (pipelined kernel)
  int32_t* enum_tgt = nullptr;    // [blocks][2][enum_cap]
  double* enum_val = nullptr;     // [blocks][2][enum_cap]
  int32_t* dsel_id = nullptr;     // [blocks][TOPK_MAX] pipelined kernel: selected entries awaiting order
  double* dsel_val = nullptr;
  unsigned int* src_counter = nullptr;  // work queue head
  int* error_flag = nullptr;      // capacity overflow
  char kernel[32] = {0};          // the kernel this workspace launches (gw_topsim_kernel)
};

// TopSim sparse rows (gw_topsim_sparse): per source r, row_len[r] nonzero
// (id, score) entries at ids/scores[begin[r] ..], packed at offsets claimed
// from *cursor (a row past `cap` gets begin = len = -1); on when cursor != nullptr
struct gw_ts_sparse {
  int64_t cap = 0;
  int64_t* begin = nullptr;
  int32_t* len = nullptr;
  int32_t* ids = nullptr;
  double* scores = nullptr;
  unsigned long long* cursor = nullptr;
};

struct gw_graph {
  gw_options_t opt{0, 0, -1, 0, 0, 0, 0};  // per-handle tuning (gw_graph_set_options)
  // host CSR
  int semantics = 0;
  int directed = 0;
  int weighted = 0;
  int64_t n = 0, nnz = 0, max_degree = 0;
  std::vector<int64_t> offsets;  // n+1
  std::vector<int32_t> nbrs;     // nnz
  std::vector<double> weights;   // nnz (empty if unweighted)
  std::vector<int64_t> labels;   // n (dense id -> original label)
  std::vector<int32_t> order;    // n (G.nodes() order as dense ids)
  // device state
  int device = -1;
  gw_dev_graph d;
  // node2vec state
  int n2v_prepared = 0;
  int n2v_mode = -1;
  double p = 1.0, q = 1.0;
  int64_t edge_alias_entries = 0;
  int64_t bitset_words = 0;
  double bs_model_s = -1.0;     // gw_bitset_build_model_s of the resident graph (cached; -1: not computed)
  // TopSim state
  gw_topsim_ws ts;
  // naive SimRank workspace (gw_simrank.hip)
  double* sr_work = nullptr;   // m*m doubles (U = A S), m = non-isolated vertices
  double* sr_x = nullptr;      // m*m compact S when m < n (else the output is used)
  uint32_t* sr_ent = nullptr;    // [nnz + pad] byte offset of the compact neighbour
  uint16_t* sr_heads = nullptr;  // [(nnz + pad) / 16] head-of-row bits
  int64_t* sr_off = nullptr;   // [m+1] compact offsets
  int64_t* sr_poff = nullptr;  // [m+1] offsets of the row-padded stream (rows start on 16-entry chunks)
  int32_t* sr_rows = nullptr;  // [m] compact id -> vertex
  int64_t sr_n = 0, sr_m = 0;
  std::string err;
};

// Scoped device selection for every C-ABI entry point that touches a device:
// selects `dev` (the graph's device) for the call and restores the caller's
// current device on return, so a call never changes the caller's (or torch's)
// current device and a NULL stream launches on the graph's own device.
struct gw_device_guard {
  int prev = -1;
  bool ok = true;  // false: the graph's device could not be selected (the call must fail)
  explicit gw_device_guard(int dev);
  ~gw_device_guard();
  gw_device_guard(const gw_device_guard&) = delete;
  gw_device_guard& operator=(const gw_device_guard&) = delete;
};

// every device-touching entry point: select the graph's device or fail with
// GW_ERR_DEVICE (never run silently on the caller's current device)
#define GW_GUARD_DEVICE(g, dev)                                                              \
  gw_device_guard gw_dg_(dev);                                                               \
  if (!gw_dg_.ok) return gw_fail((g), GW_ERR_DEVICE, "cannot select HIP device %d", (int)(dev))

// Java-exact Print.printByOrder from sparse rows (gw_graph_host.cpp)
int gw_write_sim_sparse_impl(const char* path, const int64_t* begin, const int32_t* len, const int32_t* ids,
                             const double* scores, const int32_t* row_ids, int64_t nrows, int64_t n, int topk,
                             const std::string& sep, int decimals, bool append, std::string* err);

// error helpers (gw_capi.cpp)
int gw_fail(gw_graph* g, int code, const char* fmt, ...);
void gw_set_tls_error(const std::string& s);

// host graph builders (gw_graph_host.cpp)
int gw_build_nx_simple(gw_graph* g, int64_t m, const int64_t* src,
                       const int64_t* dst, const double* w, int directed);
int gw_build_java_multi(gw_graph* g, int64_t m, const int64_t* src,
                        const int64_t* dst, int64_t vcount);

// device code entry points (gw_*.hip), all return GW_* codes
int gw_dev_upload(gw_graph* g, int device);
void gw_dev_release(gw_graph* g);
int gw_dev_n2v_prepare(gw_graph* g, double p, double q, int mode);
int gw_dev_alias_setup(int device, const double* probs, int64_t K, int64_t* J,
                       double* q, std::string* err);
int gw_dev_n2v_walks_replay(gw_graph* g, int walk_len, int64_t nwalks,
                            const int32_t* starts, const double* uniforms,
                            int64_t n_uniforms, int32_t* out_walks,
                            int32_t* out_len, int64_t* uniforms_used);
void gw_dev_bitset_release(gw_graph* g);
void gw_dev_simrank_release(gw_graph* g);
int gw_dev_topsim_double(gw_graph* g, int sample, int step, double C, uint64_t seed, double* sim_dev, void* stream);
int gw_dev_topsim_dev(gw_graph* g, int sample_total, int step, int topK, int singleStep, double C, uint64_t seed,
                      const int32_t* cand_dev, double* sim_dev, void* stream);
int gw_dev_double_random_walk(gw_graph* g, int sample, int step, double C, uint64_t seed, double* sim_dev,
                              void* stream);
int gw_dev_topsim_m(gw_graph* g, int variant, int capacity, int sample, int step, double C, uint64_t seed,
                    const int32_t* sources_dev, int64_t nsrc, int32_t* out_keys_dev, float* out_vals_dev,
                    int32_t* out_size_dev, int64_t* stats_dev, void* stream);
int gw_dev_simrank_naive(gw_graph* g, double C, int iters, double* sim_dev, void* stream);
int gw_dev_bitset_build(gw_graph* g, int64_t budget_bytes, bool lists_only = false);
double gw_bitset_build_model_s(gw_graph* g);
int gw_dev_walk_bitset_launch(gw_graph* g, int L, uint64_t seed, int64_t walk_begin, int64_t walk_count,
                              int shuffle, int32_t* out_dev, int32_t* len_dev, uint64_t* counters_dev,
                              void* stream);
int gw_dev_walk_listed_launch(gw_graph* g, int L, uint64_t seed, int64_t walk_begin, int64_t walk_count,
                              int shuffle, int32_t* out_dev, int32_t* len_dev, uint64_t* counters_dev,
                              void* stream);
int gw_dev_n2v_walks(gw_graph* g, int walk_len, uint64_t seed,
                     int64_t walk_begin, int64_t walk_count, int shuffle,
                     int32_t* out_walks_dev, int32_t* out_len_dev,
                     uint64_t* counters_dev, void* stream);
int gw_dev_topsim_prepare(gw_graph* g, int variant, int sample, int step,
                          int topk);
int gw_dev_topsim(gw_graph* g, int variant, int sample, int step, double C,
                  uint64_t seed, const int32_t* sources_dev, int64_t nsrc,
                  int topk, int32_t* out_ids_dev, double* out_scores_dev,
                  double* out_rows_dev, int64_t* stats_dev, void* stream,
                  const gw_ts_sparse* sparse = nullptr);
