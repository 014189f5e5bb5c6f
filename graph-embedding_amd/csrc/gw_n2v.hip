// node2vec walk generation on gfx950 (H1).
//
// Reference: node2vec/src/node2vec.py
//   preprocess_transition_probs :83-113   -> k_alias_nodes, k_alias_edges
//   get_alias_edge               :61-81    -> k_alias_edges (bias per dst_nbr)
//   alias_setup                  :116-147  -> gw_alias_build (device)
//   alias_draw                   :150-160  -> replay kernel draw
//   node2vec_walk / simulate_walks :13-59  -> k_walk_replay / k_walk_scale
//
// Work decomposition: one lane per walk.  A walk is a dependent chain of
// gathers (row bounds -> candidate -> [has_edge probe] -> next row), so the
// kernel is latency/gather bound: occupancy (waves in flight per CU) and
// bytes per step are the levers, MFMA is irrelevant.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "gw_device_common.h"

namespace {

constexpr int kBlock = 256;

inline unsigned grid_for(int64_t n, int block = kBlock) {
  int64_t g = (n + block - 1) / block;
  return (unsigned)std::max<int64_t>(1, g);
}

template <typename T>
int dev_alloc(gw_graph* g, T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) return GW_OK;
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (size_t)count);
  if (e != hipSuccess) {
    g->err = std::string("hipMalloc(") + std::to_string(sizeof(T) * (size_t)count) + " B): " + hipGetErrorString(e);
    *p = nullptr;
    return GW_ERR_NOMEM;
  }
  return GW_OK;
}

template <typename T>
void dev_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// ---------------------------------------------------------------------------
// preprocessing kernels
// ---------------------------------------------------------------------------
__global__ void k_degree_wsum(int64_t n, const int64_t* __restrict__ off,
                              const double* __restrict__ w, int32_t* __restrict__ deg,
                              double* __restrict__ wsum) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  int64_t b = off[v], e = off[v + 1];
  deg[v] = (int32_t)(e - b);
  if (w) {
    double s = 0.0;  // sequential left-to-right sum, as Python sum()
    for (int64_t k = b; k < e; ++k) s += w[k];
    wsum[v] = s;
  }
}

// alias_nodes (node2vec.py:91-97): probs = w / sum(w) over the sorted row.
__global__ void k_alias_nodes(int64_t n, const int64_t* __restrict__ off,
                              const double* __restrict__ w, int32_t* __restrict__ J,
                              double* __restrict__ q, int32_t* __restrict__ stack) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  int64_t b = off[v], e = off[v + 1];
  int64_t K = e - b;
  if (K == 0) return;
  double norm = 0.0;
  if (w) {
    for (int64_t k = b; k < e; ++k) norm += w[k];
  } else {
    norm = (double)K;  // sum of int 1 weights (main.py:84-85)
  }
  for (int64_t k = 0; k < K; ++k) q[b + k] = (w ? w[b + k] : 1.0) / norm;
  gw_alias_build<int32_t>(q + b, J + b, stack + b, K);
}

// per-slot table sizes for alias_edges: size(e) = deg(nbrs[e])
__global__ void k_edge_sizes(int64_t nnz, const int32_t* __restrict__ nbrs,
                             const int32_t* __restrict__ deg, int64_t* __restrict__ sz) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  sz[e] = deg[nbrs[e]];
}

// alias_edges (node2vec.py:61-81, :102-108): for slot e = (src -> dst), the
// table over sorted N(dst): dst_nbr == src -> w/p ; elif has_edge(dst_nbr,
// src) -> w ; else w/q ; normalised by the sequential sum.
__global__ void k_alias_edges(int64_t n, int64_t nnz, const int64_t* __restrict__ off,
                              const int32_t* __restrict__ nbrs, const double* __restrict__ w,
                              double p, double q, const int64_t* __restrict__ eoff,
                              int32_t* __restrict__ eJ, double* __restrict__ eq,
                              int32_t* __restrict__ stack) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  // src = row containing slot e (upper_bound over offsets)
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (off[mid + 1] <= e)
      lo = mid + 1;
    else
      hi = mid;
  }
  const int32_t src = (int32_t)lo;
  const int32_t dst = nbrs[e];
  const int64_t db = off[dst], de = off[dst + 1];
  const int64_t K = de - db;
  if (K == 0) return;
  double* qt = eq + eoff[e];
  double norm = 0.0;
  for (int64_t k = 0; k < K; ++k) {
    const int32_t x = nbrs[db + k];
    const double wx = w ? w[db + k] : 1.0;
    double u;
    if (x == src) {
      u = wx / p;
    } else if (gw_row_find(nbrs, off[x], off[x + 1], src) >= 0) {  // G.has_edge(x, src)
      u = wx;
    } else {
      u = wx / q;
    }
    qt[k] = u;
    norm += u;
  }
  for (int64_t k = 0; k < K; ++k) qt[k] = qt[k] / norm;
  gw_alias_build<int32_t>(qt, eJ + eoff[e], stack + eoff[e], K);
}

__global__ void k_alias_single(const double* __restrict__ probs, int64_t K,
                               int64_t* __restrict__ J, double* __restrict__ q,
                               int32_t* __restrict__ stack) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (int64_t k = 0; k < K; ++k) q[k] = probs[k];
  gw_alias_build<int64_t>(q, J, stack, K);
}

// ---------------------------------------------------------------------------
// exact replay walk (node2vec.py:13-39 with alias_draw :150-160)
// ---------------------------------------------------------------------------
__global__ void k_walk_replay(gw_dev_graph G, int L, int64_t nwalks,
                              const int32_t* __restrict__ starts,
                              const double* __restrict__ U, int64_t nU,
                              const int64_t* __restrict__ uoff,
                              int32_t* __restrict__ out, int32_t* __restrict__ lens,
                              int* __restrict__ overrun) {
  int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwalks) return;
  int32_t* row = out + w * (int64_t)L;
  int32_t cur = starts[w];
  row[0] = cur;
  int len = 1;
  int64_t o = uoff[w];
  int64_t slot = -1;
  while (len < L) {
    const int64_t b = G.offsets[cur], e = G.offsets[cur + 1];
    const int64_t d = e - b;
    if (d == 0) break;  // directed sink (node2vec.py:36-37)
    if (o + 2 > nU) {   // caller supplied too few uniforms
      atomicOr(overrun, 1);
      break;
    }
    const double u1 = U[o], u2 = U[o + 1];
    o += 2;
    int64_t kk = (int64_t)floor(u1 * (double)d);  // int(np.floor(rand()*K))
    if (kk >= d) kk = d - 1;
    const int32_t* J;
    const double* q;
    if (len == 1) {
      J = G.node_J + b;
      q = G.node_q + b;
    } else {
      const int64_t t0 = G.edge_off[slot];
      J = G.edge_J + t0;
      q = G.edge_q + t0;
    }
    const int64_t idx = (u2 < q[kk]) ? kk : (int64_t)J[kk];
    slot = b + idx;
    cur = G.nbrs[slot];
    row[len++] = cur;
  }
  for (int t = len; t < L; ++t) row[t] = -1;
  lens[w] = len;
}

// ---------------------------------------------------------------------------
// scale walk: Philox4x32-10, per-node alias (weighted) or uniform
// (unweighted) proposal, exact second-order bias by rejection with the return
// edge as an outlier (KnightKing-style envelope).
// ---------------------------------------------------------------------------
struct N2VParams {
  double a_p, a_q;   // 1/p, 1/q
  double M;          // envelope height for non-return candidates = max(1, 1/q)
  double lo;         // min(1, 1/q): accept without probing below this
  double extra;      // outlier height for the return edge = max(0, 1/p - M)
  double h_prev;     // min(1/p, M): in-envelope height of the return edge
  uint32_t k0, k1;   // step key
  uint32_t pk0, pk1; // permutation key
  uint32_t diag;     // timing experiments only (GW_DIAG_NO_STORE=1: no walk output stores)
  // mixture proposal (unweighted undirected, q > 1; see k_walk_scale)
  double mix_o;       // outlier mass of the return edge: max(0, 1/p - 1/q)
  double mix_p;       // mass per vertex of the prev branch: 1 - 1/q
  double mix_prev;    // acceptance of prev drawn by the cur branch: min(1, (1/p) / (1/q))
};

template <bool WEIGHTED>
__device__ __forceinline__ int64_t draw_first_order(const gw_dev_graph& G, int64_t b,
                                                    int64_t d, uint32_t ux, uint32_t ulo, uint32_t uy) {
  int64_t kk = (int64_t)gw_index(ux, ulo, (uint32_t)d);  // 64-bit draw (ux:ulo)
  if (!WEIGHTED) return kk;
  return (gw_u01(uy) < G.node_q[b + kk]) ? kk : (int64_t)G.node_J[b + kk];
}

// Membership pre-filter for has_edge: every row r owns 16 bits per adjacency
// entry at bit offset 16*offsets[r]; neighbour x sets bit h(x) of its row.
// A clear bit proves x is not a neighbour (one cache line instead of a
// log2(deg)-probe binary search); a set bit (true hit or ~6% false positive)
// falls through to the exact search, so results never change.
__device__ __forceinline__ uint64_t gw_bm_bit(int64_t rowb, int64_t deg, int32_t key) {
  const uint32_t h = (uint32_t)key * 0x9E3779B1u;
  return 16ull * (uint64_t)rowb + (((uint64_t)h * (uint64_t)(16 * deg)) >> 32);
}

// Exact neighbour sets (gw_eh_has, gw_device_common.h) when built, else the
// membership bitmap + binary search.
__device__ __forceinline__ bool gw_has_edge(const gw_dev_graph& G, int64_t rb, int64_t re,
                                            int32_t key) {
  if (G.eh) return gw_eh_has(G.eh, rb, re, key);
  if (G.bitmap) {
    const uint64_t bit = gw_bm_bit(rb, re - rb, key);
    if (!((G.bitmap[bit >> 5] >> (bit & 31)) & 1u)) return false;
  }
  return gw_row_find(G.nbrs, rb, re, key) >= 0;
}

__global__ void k_scale_ent(gw_dev_graph G, gw_ts_ent* __restrict__ ent) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= G.nnz) return;
  const int32_t x = G.nbrs[e];
  gw_ts_ent v;
  v.x = x;
  v.off = G.offsets[x];
  v.d = (int32_t)(G.offsets[x + 1] - v.off);
  ent[e] = v;
}

// one thread per adjacency slot: insert nbrs[e] into its row's set (the
// first free slot of its bucket, else of the next bucket: a bucket's slots
// fill in order, see gw_eh_has)
__global__ void k_build_ehash(gw_dev_graph G, int32_t* __restrict__ eh) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= G.nnz) return;
  int64_t lo = 0, hi = G.n;  // row of slot e
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (G.offsets[mid + 1] <= e)
      lo = mid + 1;
    else
      hi = mid;
  }
  const int64_t rb = G.offsets[lo];
  const uint32_t nbk = (uint32_t)(G.offsets[lo + 1] - rb);
  const int32_t key = G.nbrs[e];
  int32_t* t = eh + 4 * rb;
  uint32_t h = gw_eh_slot(key, nbk);
  for (uint32_t i = 0; i < nbk; ++i) {
    for (int j = 0; j < 4; ++j) {
      const int32_t old = atomicCAS(&t[4 * h + j], -1, key);
      if (old == -1 || old == key) return;
    }
    h = h + 1 == nbk ? 0u : h + 1;
  }
}

__global__ void k_build_bitmap(int64_t n, const int64_t* __restrict__ off,
                               const int32_t* __restrict__ nbrs, uint32_t* __restrict__ bm) {
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int64_t b = off[v], e = off[v + 1];
  for (int64_t k = b; k < e; ++k) {
    const uint64_t bit = gw_bm_bit(b, e - b, nbrs[k]);
    atomicOr(&bm[bit >> 5], 1u << (bit & 31));
  }
}

// One lane per walk.  The loop is flattened to ONE rejection trial per
// iteration: a lane that accepts advances to its next step while the others
// retry, so a wave is not held at every step by its unluckiest lane (the
// expected maximum of 64 geometric trial counts is ~4x their mean).
// Output: each lane stages its positions in a private LDS column and writes
// them back 16 at a time (64 contiguous bytes per lane) instead of one
// 4-byte store per step at a 4*L-byte lane stride.
constexpr int kStage = 16;

// ENT: G.sent (16 B slot entries) exists.  A compile-time switch, not a
// runtime test: with both paths in one body the compiler merges the two
// neighbour-id loads into one dword load after the entry's dwordx3, which
// serialises two dependent requests per step.
//
// MIX (unweighted, undirected, q > 1): the target weights over x in N(cur)
// (node2vec.py:61-81) are w(prev) = 1/p, w(x) = 1 for x in N(prev), 1/q
// otherwise, i.e.  w = 1/q * [x in N(cur)] + (1 - 1/q) * [x in N(prev)]
// (+ the return edge's own weight).  Sampling that mixture directly needs no
// envelope: with mass d_cur/q pick x uniformly from N(cur) and accept it (no
// has_edge probe), with mass (1 - 1/q) * d_prev pick x uniformly from N(prev)
// and accept it iff x is in N(cur) (one probe of cur's neighbour set; x ==
// prev, a self-loop of prev, is rejected), with mass max(0, 1/p - 1/q) return
// to prev (an outlier; when 1/p < 1/q a prev drawn from N(cur) is accepted
// with probability q/p).  Every x then has accepted mass exactly w(x).  Per
// step it costs (d_cur/q + 2 (1 - 1/q) d_prev) / Z requests against
// d_cur (2 - 1/q) / Z for the uniform-proposal rejection below (Z = sum of
// w), so a step takes the mixture iff d_prev < d_cur — known before the first
// draw, so the choice is a pure function of the walk (oracle: or_walks_scale).
template <bool FIRST_ORDER, bool WEIGHTED, bool DIRECTED, bool ENT, bool MIX = false>
__global__ void __launch_bounds__(kBlock)
k_walk_scale(gw_dev_graph G, N2VParams P, int L, int64_t walk_begin, int64_t walk_count,
             int shuffle, int32_t* __restrict__ out, int32_t* __restrict__ lens,
             unsigned long long* __restrict__ counters) {
  __shared__ int32_t s_stage[kBlock / 64][kStage][64];
  __shared__ int32_t s_ids[kBlock / 64][64];  // flush: lanes of the ready walkers, by rank
  const int lane = threadIdx.x & 63;
  int32_t* stage = &s_stage[threadIdx.x >> 6][0][lane];  // slot j at stage[64*j]
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < walk_count;
  unsigned long long my_steps = 0, my_trials = 0;
  const int64_t w = walk_begin + (valid ? i : 0);
  int32_t cur = -1;
  int32_t prev = -1;
  int64_t pb = 0, pe = 0;  // prev row bounds (undirected has_edge probes)
  double w_back = 1.0;     // weight of edge cur<->prev (outlier area)
  bool back_ok = false;    // cur -> prev exists (always true undirected)
  const bool vec_ok = (L & 3) == 0;
  int len = L;  // lanes past walk_count take no step
  uint32_t trial = 0;
  const uint32_t c0 = (uint32_t)w, c1 = (uint32_t)((uint64_t)w >> 32);
  int64_t b = 0, e = 0;
  int64_t nb = 0;  // candidate's row (slot entries)
  int32_t nd = 0;
  double Wcur = 0.0;
  if (valid) {
    const uint64_t it = (uint64_t)w / (uint64_t)G.n;
    const uint64_t pos = (uint64_t)w % (uint64_t)G.n;
    const uint64_t sp = shuffle ? gw_feistel_perm(pos, (uint64_t)G.n, P.pk0, P.pk1, (uint32_t)it) : pos;
    cur = G.order[sp];
    len = 1;
    b = G.offsets[cur];
    e = G.offsets[cur + 1];
    Wcur = WEIGHTED ? G.wsum[cur] : (double)(e - b);
  }
  stage[0] = cur;
  // wave-uniform loop: the stage flush below is cooperative
  for (;;) {
    const bool active = len < L && e != b;  // e == b: directed sink (node2vec.py:36-37)
    if (__ballot(active) == 0ull) break;
    bool ready = false;  // this lane completed 16 staged positions (flen-15 .. flen)
    int flen = 0;
    if (active) {
      const int64_t d = e - b;
      bool acc;
      int64_t slot;
      int32_t next;
      if (FIRST_ORDER || len == 1) {
        gw_u4 u = gw_philox(c0, c1, (uint32_t)len, 0u, P.k0, P.k1);
        trial = 1;
        slot = b + draw_first_order<WEIGHTED>(G, b, d, u.x, u.z, u.y);
        if (FIRST_ORDER && ENT) {  // the slot entry carries the next row
          const gw_ts_ent en = gw_ts_load(G.sent + slot);
          next = en.x;
          nb = en.off;
          nd = en.d;
        } else {
          next = G.nbrs[slot];
        }
        acc = true;
      } else if (MIX && pe - pb < d) {  // mixture proposal (see above)
        const gw_u4 u = gw_philox(c0, c1, (uint32_t)len, trial, P.k0, P.k1);
        ++trial;
        const int64_t dp = pe - pb;
        const double Ac = (double)d * P.a_q;
        const double H = P.mix_o + Ac + (double)dp * P.mix_p;
        const double r = gw_u01(u.z) * H;
        if (r < P.mix_o) {  // return-edge outlier
          slot = -1;
          next = prev;
          acc = true;
        } else {
          const bool from_cur = r < P.mix_o + Ac;
          slot = (from_cur ? b : pb) + (int64_t)gw_index(u.x, u.y, (uint32_t)(from_cur ? d : dp));
          if (ENT) {  // the slot entry (of cur's or prev's row) carries the candidate's row
            const gw_ts_ent en = gw_ts_load(G.sent + slot);
            next = en.x;
            nb = en.off;
            nd = en.d;
          } else {
            next = G.nbrs[slot];
          }
          if (from_cur)
            acc = next != prev || gw_u01(u.w) < P.mix_prev;
          else
            acc = next != prev && gw_has_edge(G, b, e, next);  // x in N(cur)
          if (trial >= (1u << 24) && from_cur) acc = true;
        }
      } else {
        const gw_u4 u = gw_philox(c0, c1, (uint32_t)len, trial, P.k0, P.k1);
        ++trial;
        const double out_area = (back_ok && P.extra > 0.0) ? P.extra * w_back : 0.0;
        const double A = P.M * Wcur + out_area;
        if (out_area > 0.0 && gw_u01(u.z) * A < out_area) {  // return-edge outlier
          slot = -1;
          next = prev;
          acc = true;
        } else {
          // low word of the index draw: u.y (unweighted), else one more Philox block
          // (u.y is the weighted node-alias accept, u.z / u.w are taken)
          const uint32_t ulo =
              WEIGHTED ? gw_philox(c0, c1, (uint32_t)len, (trial - 1u) | 0x80000000u, P.k0, P.k1).x : u.y;
          slot = b + draw_first_order<WEIGHTED>(G, b, d, u.x, ulo, u.y);
          if (ENT) {  // the slot entry carries the candidate's row for the next step
            const gw_ts_ent en = gw_ts_load(G.sent + slot);
            next = en.x;
            nb = en.off;
            nd = en.d;
          } else {
            next = G.nbrs[slot];
          }
          const double t = gw_u01(u.w) * P.M;
          if (next == prev) {
            acc = t < P.h_prev;
          } else if (t < P.lo) {
            acc = true;
          } else {
            bool adj;
            if (DIRECTED)
              adj = ENT ? gw_has_edge(G, nb, nb + nd, prev)
                           : gw_has_edge(G, G.offsets[next], G.offsets[next + 1], prev);  // edge x -> prev
            else
              adj = gw_has_edge(G, pb, pe, next);  // x in N(prev)
            acc = t < (adj ? 1.0 : P.a_q);
          }
          if (trial >= (1u << 24)) acc = true;
        }
      }
      if (acc) {
        my_trials += trial;
        trial = 0;
        // carry state for the next step: existence/weight of edge next -> cur
        if (DIRECTED) {
          if (!FIRST_ORDER && P.extra > 0.0) {  // probe once per step
            const int64_t bs = gw_row_find(G.nbrs, G.offsets[next], G.offsets[next + 1], cur);
            back_ok = bs >= 0;
            w_back = (back_ok && WEIGHTED) ? G.weights[bs] : 1.0;
          }
        } else if (slot >= 0) {
          back_ok = true;
          w_back = WEIGHTED ? G.weights[slot] : 1.0;
        }  // undirected return over the same edge: w_back unchanged
        const int64_t ob = pb, oe = pe;  // row of the old prev (= next on a return)
        prev = cur;
        pb = b;
        pe = e;
        cur = next;
        stage[64 * (len & (kStage - 1))] = cur;
        ready = (len & (kStage - 1)) == kStage - 1;
        flen = len;
        ++len;
        if (FIRST_ORDER && ENT) {
          b = nb;
          e = nb + nd;
        } else if (ENT && !FIRST_ORDER && len > 2) {  // row of cur known: from its slot entry, or prev's row
          if (slot >= 0) {
            b = nb;
            e = nb + nd;
          } else {
            b = ob;
            e = oe;
          }
        } else {
          b = G.offsets[cur];
          e = G.offsets[cur + 1];
        }
        if (WEIGHTED) Wcur = G.wsum[cur];
        else Wcur = (double)(e - b);
      }
    }
    // flush: 64 contiguous bytes per ready walker.  Cooperative (like the
    // bitset kernel's loads): in round j lanes 4m..4m+3 store the four 16 B
    // pieces of the chunk of the (16j+m)-th ready walker, so an instruction
    // writes 16 whole sectors instead of a 16 B piece of 64 (per-lane stores
    // cost up to 22% of a launch: GW_DIAG_NO_STORE A/B), and the ready
    // walkers are compacted first: ceil(ready / 16) rounds, not 4
    const unsigned long long rm = __ballot(ready);
    if (rm && !(kGwDiag && P.diag)) {
      if (vec_ok) {
        const int nready = __popcll(rm);
        int32_t* ids = s_ids[threadIdx.x >> 6];
        __builtin_amdgcn_wave_barrier();
        if (ready)
          ids[__builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u))] = lane;
        __builtin_amdgcn_wave_barrier();
        const int32_t* sw = &s_stage[threadIdx.x >> 6][0][0];
        for (int j = 0; 16 * j < nready; ++j) {
          const int q = 16 * j + (lane >> 2), p4 = 4 * (lane & 3);
          const int r = ids[q < nready ? q : nready - 1];
          const int lr = __shfl(flen, r, 64);
          const int64_t ir = ((int64_t)__shfl((int)(i >> 32), r, 64) << 32) | (uint32_t)__shfl((int)i, r, 64);
          if (q < nready) {
            const int4 v = make_int4(sw[64 * p4 + r], sw[64 * (p4 + 1) + r], sw[64 * (p4 + 2) + r], sw[64 * (p4 + 3) + r]);
            *reinterpret_cast<int4*>(out + ir * (int64_t)L + (lr - (kStage - 1)) + p4) = v;
          }
        }
        __builtin_amdgcn_wave_barrier();
      } else if (ready) {
        int32_t* dst = out + i * (int64_t)L + (flen - (kStage - 1));
        for (int j = 0; j < kStage; ++j) dst[j] = stage[64 * j];
      }
    }
  }
  if (valid) {
    // tail: staged positions [len & ~15, len) then -1 padding up to L
    int32_t* row = out + i * (int64_t)L;
    const int base = len & ~(kStage - 1);
    for (int t = base; t < len; ++t) row[t] = stage[64 * (t - base)];
    for (int t = len; t < L; ++t) row[t] = -1;
    if (lens) lens[i] = len;
    my_steps = (unsigned long long)(len - 1);
  }
  if (counters) {
    // wave-level reduction, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
      my_steps += __shfl_down(my_steps, off, 64);
      my_trials += __shfl_down(my_trials, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&counters[0], my_steps);
      atomicAdd(&counters[1], my_trials);
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host entry points
// ---------------------------------------------------------------------------
void gw_dev_release(gw_graph* g) {
  if (g->device < 0) return;
  (void)hipSetDevice(g->device);
  gw_dev_graph& d = g->d;
  dev_free(d.offsets);
  dev_free(d.nbrs);
  dev_free(d.weights);
  dev_free(d.wsum);
  dev_free(d.order);
  dev_free(d.deg);
  dev_free(d.node_J);
  dev_free(d.node_q);
  dev_free(d.edge_off);
  dev_free(d.edge_J);
  dev_free(d.edge_q);
  dev_free(d.bitmap);
  dev_free(d.eh);
  dev_free(d.sent);
  gw_dev_bitset_release(g);
  gw_dev_simrank_release(g);
  gw_topsim_ws& t = g->ts;
  dev_free(t.lvl_vertex);
  dev_free(t.lvl_parent);
  dev_free(t.lvl_deg);
  dev_free(t.lvl_off);
  dev_free(t.ent);
  dev_free(t.lvl_mass);
  dev_free(t.child_off);
  dev_free(t.spawn_node);
  dev_free(t.spawn_mass);
  dev_free(t.spawn_level);
  dev_free(t.spawn_first);
  dev_free(t.acc_row);
  dev_free(t.ov_list);
  dev_free(t.touched);
  dev_free(t.app);
  dev_free(t.enum_tgt);
  dev_free(t.enum_val);
  dev_free(t.dsel_id);
  dev_free(t.dsel_val);
  dev_free(t.src_counter);
  dev_free(t.error_flag);
  t = gw_topsim_ws();
  g->n2v_prepared = 0;
  g->bs_model_s = -1.0;
  g->device = -1;
}

int gw_dev_upload(gw_graph* g, int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    g->err = "no HIP device visible (libgraphwalk has no CPU fallback)";
    return GW_ERR_DEVICE;
  }
  if (device < 0 || device >= count) {
    g->err = "device ordinal out of range";
    return GW_ERR_INVALID;
  }
  if (g->device >= 0) gw_dev_release(g);
  GW_HIP_TRY(hipSetDevice(device));
  g->device = device;
  gw_dev_graph& d = g->d;
  d.n = g->n;
  d.nnz = g->nnz;
  int rc;
  if ((rc = dev_alloc(g, &d.offsets, g->n + 1)) || (rc = dev_alloc(g, &d.nbrs, g->nnz)) ||
      (rc = dev_alloc(g, &d.order, g->n)) || (rc = dev_alloc(g, &d.deg, g->n))) {
    gw_dev_release(g);
    return rc;
  }
  GW_HIP_TRY(hipMemcpy(d.offsets, g->offsets.data(), sizeof(int64_t) * (g->n + 1), hipMemcpyHostToDevice));
  if (g->nnz) GW_HIP_TRY(hipMemcpy(d.nbrs, g->nbrs.data(), sizeof(int32_t) * g->nnz, hipMemcpyHostToDevice));
  if (g->n) GW_HIP_TRY(hipMemcpy(d.order, g->order.data(), sizeof(int32_t) * g->n, hipMemcpyHostToDevice));
  if (g->weighted) {
    if ((rc = dev_alloc(g, &d.weights, g->nnz)) || (rc = dev_alloc(g, &d.wsum, g->n))) {
      gw_dev_release(g);
      return rc;
    }
    if (g->nnz) GW_HIP_TRY(hipMemcpy(d.weights, g->weights.data(), sizeof(double) * g->nnz, hipMemcpyHostToDevice));
  }
  if (g->n) {
    k_degree_wsum<<<grid_for(g->n), kBlock>>>(g->n, d.offsets, d.weights, d.deg, d.wsum);
    GW_HIP_TRY(hipGetLastError());
  }
  GW_HIP_TRY(hipDeviceSynchronize());
  return GW_OK;
}

// per-slot sampler tables may take this much HBM (the handle's option, else
// half of the free HBM)
static int64_t table_budget(gw_graph* g) {
  size_t fr = 0, tot = 0;
  int64_t budget = hipMemGetInfo(&fr, &tot) == hipSuccess ? (int64_t)(fr / 2) : 0;
  if (g->opt.table_budget_bytes > 0) budget = std::min(budget, g->opt.table_budget_bytes);
  return budget;
}

// GW_N2V_REJECTION on an unweighted undirected graph: build the 64 B listed
// entries?  They save ~0.46 fabric requests per second-order step (config 4:
// 1.60 -> 1.14 requests/step at ~4.9e10 requests/s) but cost an
// edge-centric common-neighbour build; with expected_steps known, build them
// only when the modelled build time is paid back.
static bool listed_pays(gw_graph* g, double q) {
  // the payload answers the lazy has_edge probes of the q < 1 envelope; with
  // q > 1 k_walk_scale's mixture proposal needs no such probe (and with
  // q = 1 no probe happens at all), so listed entries are built for q < 1
  // only, whatever the option says (the walks never depend on options)
  if (q >= 1.0) return false;
  if (g->opt.listed == 0) return false;
  if (g->opt.listed == 1 || g->opt.expected_steps <= 0) return true;
  const double save_s = (double)g->opt.expected_steps * (0.46 / 4.9e10);
  const double build_s = gw_bitset_build_model_s(g);
  if (build_s < 0) {  // the model run failed on the device: keep the plain entries
    (void)hipGetLastError();
    return false;
  }
  return save_s > build_s;
}

// bitset walk time per step (R-MAT-20 headline 3.2e10 walk-steps/s) and the
// rejection sampler's time per trial (see n2v_prepare_auto)
constexpr double kBitsetStepSeconds = 1.0 / 3.2e10;
constexpr double kRejTrialSeconds = 3.0e-11;  // round 5 (bucketed neighbour hash); round 4: 4.0e-11

// GW_N2V_AUTO: see include/graphwalk.h
static int n2v_prepare_auto(gw_graph* g, double p, double q) {
  const bool bs_ok = !g->weighted && !g->directed && g->semantics == GW_SEM_NX_SIMPLE && !(p == 1.0 && q == 1.0) &&
                     g->nnz > 0 && g->nnz < (int64_t)0xFFFFFFFF;
  auto bitset_or_rejection = [&]() {
    int rc = gw_dev_n2v_prepare(g, p, q, GW_N2V_BITSET);
    if (rc == GW_ERR_CAPACITY || rc == GW_ERR_NOMEM || rc == GW_ERR_UNSUPPORTED) {
      (void)hipGetLastError();
      g->err.clear();
      rc = gw_dev_n2v_prepare(g, p, q, GW_N2V_REJECTION);
    }
    return rc;
  };
  if (!bs_ok) return gw_dev_n2v_prepare(g, p, q, GW_N2V_REJECTION);
  const int64_t steps = g->opt.expected_steps;
  if (steps <= 0) return bitset_or_rejection();
  // the pilot needs the plain rejection sampler only: its trial count does
  // not depend on listed entries, so their build is deferred until rejection
  // is the final choice (and then only when listed_pays)
  const int32_t listed_opt = g->opt.listed;
  g->opt.listed = 0;
  int rc = gw_dev_n2v_prepare(g, p, q, GW_N2V_REJECTION);
  g->opt.listed = listed_opt;
  if (rc != GW_OK) return rc;
  auto keep_rejection = [&]() {
    if (listed_opt != 0 && listed_pays(g, q)) return gw_dev_n2v_prepare(g, p, q, GW_N2V_REJECTION);
    return GW_OK;
  };
  // pilot: the rejection sampler's own walks (65,536 walks of length 80 from
  // iteration 0's shuffled starts, a fixed internal seed) counting its trials
  // per step; the modelled time per trial is measured (round 5, bucketed
  // neighbour hash: R-MAT-20 p = 0.25 q = 4: 1.98 trials/step, 28.3 ms per
  // 5.1e8 steps = 2.8e-11 s per trial; R-MAT-24 ef 16 p = 1 q = 0.5: 1.045,
  // 25.8 ms per 7.0e8 = 3.5e-11).  Counting, not timing, keeps the choice
  // (and so the walks) a function of the inputs.
  const int64_t pw = std::min<int64_t>(65536, std::max<int64_t>(g->n, 1));
  const int L = 80;
  int32_t* buf = nullptr;
  uint64_t* cnt = nullptr;
  double t_rej = -1.0;
  if (dev_alloc(g, &buf, pw * L) == GW_OK && dev_alloc(g, &cnt, 2) == GW_OK) {
    uint64_t h[2] = {0, 0};
    const bool ok = hipMemset(cnt, 0, 2 * sizeof(uint64_t)) == hipSuccess &&
                    gw_dev_n2v_walks(g, L, 0x5eedull, 0, pw, 1, buf, nullptr, cnt, nullptr) == GW_OK &&
                    hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost) == hipSuccess;
    if (ok && h[0] > 0) t_rej = (double)h[1] / (double)h[0] * kRejTrialSeconds;
  }
  dev_free(buf);
  dev_free(cnt);
  (void)hipGetLastError();
  if (t_rej < 0) return keep_rejection();  // no pilot: keep the rejection sampler
  const double build = gw_bitset_build_model_s(g);
  (void)hipGetLastError();
  const double bitset_s = build + (double)steps * kBitsetStepSeconds;
  const double rejection_s = (double)steps * t_rej;
  if (build < 0 || bitset_s >= rejection_s) return keep_rejection();
  return bitset_or_rejection();
}

int gw_dev_n2v_prepare(gw_graph* g, double p, double q, int mode) {
  if (mode == GW_N2V_AUTO) return n2v_prepare_auto(g, p, q);
  if (g->device < 0) {
    g->err = "graph is not on a device (call gw_graph_to_device)";
    return GW_ERR_STATE;
  }
  GW_HIP_TRY(hipSetDevice(g->device));
  gw_dev_graph& d = g->d;
  dev_free(d.node_J);
  dev_free(d.node_q);
  dev_free(d.edge_off);
  dev_free(d.edge_J);
  dev_free(d.edge_q);
  g->edge_alias_entries = 0;
  g->n2v_prepared = 0;
  const bool need_node_alias = g->weighted || mode == GW_N2V_REPLAY;
  int rc;
  int32_t* stack = nullptr;
  if (need_node_alias && g->nnz) {
    if ((rc = dev_alloc(g, &d.node_J, g->nnz)) || (rc = dev_alloc(g, &d.node_q, g->nnz)) ||
        (rc = dev_alloc(g, &stack, g->nnz)))
      return rc;
    k_alias_nodes<<<grid_for(g->n), kBlock>>>(g->n, d.offsets, d.weights, d.node_J, d.node_q, stack);
    GW_HIP_TRY(hipGetLastError());
    GW_HIP_TRY(hipDeviceSynchronize());
    dev_free(stack);
  }
  if (mode == GW_N2V_REPLAY && g->nnz) {
    int64_t* sz = nullptr;
    if ((rc = dev_alloc(g, &d.edge_off, g->nnz + 1)) || (rc = dev_alloc(g, &sz, g->nnz + 1))) return rc;
    k_edge_sizes<<<grid_for(g->nnz), kBlock>>>(g->nnz, d.nbrs, d.deg, sz);
    GW_HIP_TRY(hipMemset(sz + g->nnz, 0, sizeof(int64_t)));
    size_t tmp_bytes = 0;
    GW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, sz, d.edge_off, g->nnz + 1));
    void* tmp = nullptr;
    if ((rc = dev_alloc(g, (char**)&tmp, (int64_t)tmp_bytes + 1))) return rc;
    GW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, sz, d.edge_off, g->nnz + 1));
    GW_HIP_TRY(hipDeviceSynchronize());
    dev_free(tmp);
    dev_free(sz);
    int64_t total = 0;
    GW_HIP_TRY(hipMemcpy(&total, d.edge_off + g->nnz, sizeof(int64_t), hipMemcpyDeviceToHost));
    // sum(deg^2) tables: refuse beyond ~16 GB of tables
    if (total > (int64_t)1 << 30) {
      dev_free(d.edge_off);
      g->err = "per-edge alias tables need " + std::to_string(total) +
               " entries (sum of deg^2); use GW_N2V_REJECTION at this scale";
      return GW_ERR_CAPACITY;
    }
    if ((rc = dev_alloc(g, &d.edge_J, total)) || (rc = dev_alloc(g, &d.edge_q, total)) ||
        (rc = dev_alloc(g, &stack, total)))
      return rc;
    k_alias_edges<<<grid_for(g->nnz), kBlock>>>(g->n, g->nnz, d.offsets, d.nbrs, d.weights, p, q,
                                                d.edge_off, d.edge_J, d.edge_q, stack);
    GW_HIP_TRY(hipGetLastError());
    GW_HIP_TRY(hipDeviceSynchronize());
    dev_free(stack);
    g->edge_alias_entries = total;
  }
  dev_free(d.bitmap);
  dev_free(d.eh);
  gw_dev_bitset_release(g);
  g->bitset_words = 0;
  const char* nobm = GW_DIAG_ENV("GW_DIAG_NO_BITMAP");  // diagnostic A/B knob only
  const char* noeh = GW_DIAG_ENV("GW_DIAG_NO_EHASH");   // diagnostic A/B knob only
  if (mode == GW_N2V_REJECTION && !(p == 1.0 && q == 1.0) && g->nnz && g->semantics == GW_SEM_NX_SIMPLE &&
      !(noeh && noeh[0] == '1')) {
    size_t fr = 0, tot = 0;
    const int64_t slots = 4 * g->nnz;  // deg(v) buckets of 4 int32 per row
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && (int64_t)fr / 2 > slots * 4) {
      if (dev_alloc(g, &d.eh, slots) == GW_OK) {
        GW_HIP_TRY(hipMemset(d.eh, 0xFF, sizeof(int32_t) * (size_t)slots));
        k_build_ehash<<<grid_for(g->nnz), kBlock>>>(d, d.eh);
        GW_HIP_TRY(hipGetLastError());
        GW_HIP_TRY(hipDeviceSynchronize());
      } else {
        d.eh = nullptr;
        (void)hipGetLastError();
      }
    }
  }
  // membership pre-filter for has_edge probes of the rejection sampler when
  // the exact hash does not fit (the bitset build intersects rows directly)
  if (mode == GW_N2V_REJECTION && !(p == 1.0 && q == 1.0) && !d.eh && g->nnz && !(nobm && nobm[0] == '1')) {
    const int64_t words = (16 * g->nnz + 31) / 32 + 1;
    if ((rc = dev_alloc(g, &d.bitmap, words))) return rc;
    GW_HIP_TRY(hipMemset(d.bitmap, 0, sizeof(uint32_t) * words));
    k_build_bitmap<<<grid_for(g->n), kBlock>>>(g->n, d.offsets, d.nbrs, d.bitmap);
    GW_HIP_TRY(hipGetLastError());
    GW_HIP_TRY(hipDeviceSynchronize());
  }
  dev_free(d.sent);
  const bool fo = (p == 1.0 && q == 1.0);
  // rejection sampling on an unweighted undirected simple graph: 64 B listed
  // entries (k_walk_listed) answer most has_edge(x, prev) probes from the
  // payload of the entry that led to cur; when they do not fit (half the free
  // HBM, < 2^32 slots) the 16 B slot entries below serve k_walk_scale
  bool listed = false;
  if (mode == GW_N2V_REJECTION && !fo && g->nnz && !g->weighted && !g->directed &&
      g->semantics == GW_SEM_NX_SIMPLE && !GW_DIAG_ENV("GW_DIAG_NO_LISTS") && listed_pays(g, q)) {
    rc = gw_dev_bitset_build(g, table_budget(g), true);
    if (rc == GW_OK) {
      listed = true;
    } else if (rc == GW_ERR_CAPACITY || rc == GW_ERR_NOMEM || rc == GW_ERR_UNSUPPORTED) {
      gw_dev_bitset_release(g);
      (void)hipGetLastError();
      g->err.clear();
    } else {
      return rc;
    }
  }
  const char* nosent = GW_DIAG_ENV("GW_DIAG_NO_SENT");  // diagnostic A/B knob only
  if ((mode == GW_N2V_REJECTION || fo) && !listed && g->nnz && !(nosent && nosent[0] == '1')) {
    // slot entries (16 B per slot, one dwordx4 per step) spare the candidate's
    // offsets[] read: +14% on R-MAT-24 ef 16 (p=1, q=0.5; 8.3 GB of entries),
    // so they are built whenever they fit the table budget
    const int64_t ent_bytes = g->nnz * (int64_t)sizeof(gw_ts_ent);
    if (ent_bytes <= table_budget(g)) {
      if (dev_alloc(g, &d.sent, g->nnz) == GW_OK) {
        k_scale_ent<<<grid_for(g->nnz), kBlock>>>(d, d.sent);
        GW_HIP_TRY(hipGetLastError());
        GW_HIP_TRY(hipDeviceSynchronize());
      } else {
        d.sent = nullptr;
        (void)hipGetLastError();
      }
    }
  }
  if (mode == GW_N2V_BITSET && !(p == 1.0 && q == 1.0)) {
    if ((rc = gw_dev_bitset_build(g, table_budget(g)))) return rc;
  }
  g->p = p;
  g->q = q;
  g->n2v_mode = mode;
  g->n2v_prepared = 1;
  return GW_OK;
}

int gw_dev_alias_setup(int device, const double* probs, int64_t K, int64_t* J,
                       double* q, std::string* err) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    *err = "no HIP device visible (libgraphwalk has no CPU fallback)";
    return GW_ERR_DEVICE;
  }
  if (K <= 0) return GW_OK;
  if (hipSetDevice(device) != hipSuccess) {
    *err = "hipSetDevice failed";
    return GW_ERR_DEVICE;
  }
  double *dp = nullptr, *dq = nullptr;
  int64_t* dJ = nullptr;
  int32_t* st = nullptr;
  hipError_t e = hipMalloc((void**)&dp, K * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&dq, K * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&dJ, K * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc((void**)&st, K * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemcpy(dp, probs, K * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    k_alias_single<<<1, 64>>>(dp, K, dJ, dq, st);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(J, dJ, K * sizeof(int64_t), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(q, dq, K * sizeof(double), hipMemcpyDeviceToHost);
  if (dp) (void)hipFree(dp);
  if (dq) (void)hipFree(dq);
  if (dJ) (void)hipFree(dJ);
  if (st) (void)hipFree(st);
  if (e != hipSuccess) {
    *err = hipGetErrorString(e);
    return GW_ERR_DEVICE;
  }
  return GW_OK;
}

int gw_dev_n2v_walks_replay(gw_graph* g, int L, int64_t nwalks, const int32_t* starts,
                            const double* uniforms, int64_t nU, int32_t* out_walks,
                            int32_t* out_len, int64_t* used) {
  GW_HIP_TRY(hipSetDevice(g->device));
  int rc;
  int32_t *d_starts = nullptr, *d_out = nullptr, *d_len = nullptr;
  double* d_U = nullptr;
  int64_t* d_uoff = nullptr;
  int* d_over = nullptr;
  auto cleanup = [&]() {
    dev_free(d_starts);
    dev_free(d_out);
    dev_free(d_len);
    dev_free(d_U);
    dev_free(d_uoff);
    dev_free(d_over);
  };
  if ((rc = dev_alloc(g, &d_starts, nwalks)) || (rc = dev_alloc(g, &d_out, nwalks * (int64_t)L)) ||
      (rc = dev_alloc(g, &d_len, nwalks)) || (rc = dev_alloc(g, &d_U, std::max<int64_t>(nU, 1))) ||
      (rc = dev_alloc(g, &d_uoff, nwalks)) || (rc = dev_alloc(g, &d_over, 1))) {
    cleanup();
    return rc;
  }
  GW_HIP_TRY(hipMemcpy(d_starts, starts, nwalks * sizeof(int32_t), hipMemcpyHostToDevice));
  if (nU) GW_HIP_TRY(hipMemcpy(d_U, uniforms, nU * sizeof(double), hipMemcpyHostToDevice));
  GW_HIP_TRY(hipMemset(d_over, 0, sizeof(int)));
  // Offsets into the uniform stream: walk w starts after all draws of walks
  // < w (2 per step).  Assume full-length walks; a walk that stops early at a
  // sink shifts every later walk, so re-run from the first walk whose length
  // differs until the lengths are a fixed point (each pass finalises at
  // least one more walk; undirected graphs converge in one pass).
  std::vector<int64_t> uoff(nwalks);
  std::vector<int32_t> lens(nwalks, L);
  for (int64_t w = 0; w < nwalks; ++w) {
    // a start with no neighbours draws nothing
    int64_t s = starts[w];
    if (g->offsets[s + 1] == g->offsets[s]) lens[w] = 1;
  }
  std::vector<int32_t> got(nwalks);
  int64_t first_unsettled = 0;
  for (int pass = 0;; ++pass) {
    int64_t acc = 0;
    for (int64_t w = 0; w < nwalks; ++w) {
      uoff[w] = acc;
      acc += 2 * (int64_t)(lens[w] - 1);
    }
    GW_HIP_TRY(hipMemcpy(d_uoff, uoff.data(), nwalks * sizeof(int64_t), hipMemcpyHostToDevice));
    GW_HIP_TRY(hipMemset(d_over, 0, sizeof(int)));  // speculative passes may overrun
    const int64_t todo = nwalks - first_unsettled;
    k_walk_replay<<<grid_for(todo), kBlock>>>(g->d, L, todo, d_starts + first_unsettled, d_U, nU,
                                              d_uoff + first_unsettled, d_out + first_unsettled * (int64_t)L,
                                              d_len + first_unsettled, d_over);
    GW_HIP_TRY(hipGetLastError());
    GW_HIP_TRY(hipMemcpy(got.data(), d_len, nwalks * sizeof(int32_t), hipMemcpyDeviceToHost));
    int64_t mism = -1;
    for (int64_t w = first_unsettled; w < nwalks; ++w)
      if (got[w] != lens[w]) {
        mism = w;
        break;
      }
    if (mism < 0) {
      int over = 0;
      GW_HIP_TRY(hipMemcpy(&over, d_over, sizeof(int), hipMemcpyDeviceToHost));
      if (over) {
        cleanup();
        g->err = "uniform stream exhausted (supply 2*(walk_len-1) uniforms per walk)";
        return GW_ERR_INVALID;
      }
      if (used) *used = acc;
      break;
    }
    // walks before mism used correct offsets; mism's own offset was correct
    // too, so its length is final.  Every later walk takes this pass's length
    // as its next guess (not the full length again): a sink-heavy directed
    // graph then converges in a few passes instead of one pass per walk that
    // stops early, and the settled prefix still grows by >= 1 per pass.
    for (int64_t w = first_unsettled; w < nwalks; ++w) lens[w] = got[w];
    first_unsettled = mism + 1;
    if (first_unsettled >= nwalks) {
      int64_t a2 = 0;
      for (int64_t w = 0; w < nwalks; ++w) a2 += 2 * (int64_t)(lens[w] - 1);
      if (used) *used = a2;
      break;
    }
  }
  GW_HIP_TRY(hipMemcpy(out_walks, d_out, nwalks * (int64_t)L * sizeof(int32_t), hipMemcpyDeviceToHost));
  GW_HIP_TRY(hipMemcpy(out_len, d_len, nwalks * sizeof(int32_t), hipMemcpyDeviceToHost));
  cleanup();
  return GW_OK;
}

int gw_dev_n2v_walks(gw_graph* g, int L, uint64_t seed, int64_t walk_begin, int64_t walk_count,
                     int shuffle, int32_t* out_dev, int32_t* len_dev, uint64_t* counters_dev,
                     void* stream) {
  if (walk_count <= 0) return GW_OK;
  // one thread per walk and a launch's work-items must stay below 2^32:
  // split larger requests (walks are a pure function of the global index)
  constexpr int64_t kMaxLaunch = (int64_t)1 << 31;
  if (walk_count > kMaxLaunch) {
    for (int64_t o = 0; o < walk_count; o += kMaxLaunch) {
      const int rc = gw_dev_n2v_walks(g, L, seed, walk_begin + o, std::min(kMaxLaunch, walk_count - o), shuffle,
                                      out_dev + o * (int64_t)L, len_dev ? len_dev + o : nullptr, counters_dev,
                                      stream);
      if (rc != GW_OK) return rc;
    }
    return GW_OK;
  }
  const bool first_order = (g->p == 1.0 && g->q == 1.0);
  if (!first_order && g->semantics != GW_SEM_NX_SIMPLE) {
    g->err = "second-order walks need sorted rows (NX_SIMPLE semantics)";
    return GW_ERR_UNSUPPORTED;
  }
  N2VParams P;
  P.a_p = 1.0 / g->p;
  P.a_q = 1.0 / g->q;
  P.M = std::max(1.0, P.a_q);
  P.lo = std::min(1.0, P.a_q);
  P.extra = P.a_p > P.M ? P.a_p - P.M : 0.0;
  P.h_prev = std::min(P.a_p, P.M);
  P.mix_o = std::max(0.0, P.a_p - P.a_q);
  P.mix_p = 1.0 - P.a_q;
  P.mix_prev = std::min(1.0, P.a_p / P.a_q);
  P.k0 = (uint32_t)seed;
  P.k1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_STEP;
  P.pk0 = (uint32_t)seed;
  P.pk1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_PERM;
  {
    const char* ns = GW_DIAG_ENV("GW_DIAG_NO_STORE");
    P.diag = (ns && ns[0] == '1') ? 1u : 0u;
  }
  if (g->n2v_mode == GW_N2V_BITSET && !first_order)
    return gw_dev_walk_bitset_launch(g, L, seed, walk_begin, walk_count, shuffle, out_dev, len_dev, counters_dev,
                                     stream);
  if (g->n2v_mode == GW_N2V_REJECTION && !first_order && g->d.bs_nbr)
    return gw_dev_walk_listed_launch(g, L, seed, walk_begin, walk_count, shuffle, out_dev, len_dev, counters_dev,
                                     stream);
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = grid_for(walk_count);
  unsigned long long* C = (unsigned long long*)counters_dev;
#define GW_LAUNCH_MIX(FO, WT, DI, MX)                                                                              \
  do {                                                                                                             \
    if (g->d.sent)                                                                                                 \
      k_walk_scale<FO, WT, DI, true, MX><<<grid, kBlock, 0, s>>>(g->d, P, L, walk_begin, walk_count, shuffle,      \
                                                                 out_dev, len_dev, C);                             \
    else                                                                                                           \
      k_walk_scale<FO, WT, DI, false, MX><<<grid, kBlock, 0, s>>>(g->d, P, L, walk_begin, walk_count, shuffle,     \
                                                                  out_dev, len_dev, C);                            \
  } while (0)
#define GW_LAUNCH(FO, WT, DI) GW_LAUNCH_MIX(FO, WT, DI, false)
  const bool wt = g->weighted != 0, di = g->directed != 0;
  if (first_order) {
    if (wt) GW_LAUNCH(true, true, false);
    else GW_LAUNCH(true, false, false);
  } else if (wt) {
    if (di) GW_LAUNCH(false, true, true);
    else GW_LAUNCH(false, true, false);
  } else {
    if (di) GW_LAUNCH(false, false, true);
    else if (P.a_q < 1.0) GW_LAUNCH_MIX(false, false, false, true);  // q > 1: mixture proposal
    else GW_LAUNCH(false, false, false);
  }
#undef GW_LAUNCH
#undef GW_LAUNCH_MIX
  GW_HIP_TRY(hipGetLastError());
  return GW_OK;
}

__global__ void k_philox(const uint32_t* __restrict__ in, int64_t n, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* a = in + 6 * i;
  const gw_u4 r = gw_philox(a[0], a[1], a[2], a[3], a[4], a[5]);
  uint32_t* o = out + 4 * i;
  o[0] = r.x;
  o[1] = r.y;
  o[2] = r.z;
  o[3] = r.w;
}

extern "C" int gw_philox4x32(int device, const uint32_t* in, int64_t n, uint32_t* out) {
  if (n < 0 || (n > 0 && (!in || !out))) return gw_fail(nullptr, GW_ERR_INVALID, "bad arrays");
  if (n == 0) return GW_OK;
  if (device < 0) {  // host evaluation of the same header
    for (int64_t i = 0; i < n; ++i) {
      const uint32_t* a = in + 6 * i;
      const gw_u4 r = gw_philox(a[0], a[1], a[2], a[3], a[4], a[5]);
      out[4 * i] = r.x;
      out[4 * i + 1] = r.y;
      out[4 * i + 2] = r.z;
      out[4 * i + 3] = r.w;
    }
    return GW_OK;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
    return gw_fail(nullptr, GW_ERR_DEVICE, "no HIP device visible (libgraphwalk has no CPU fallback)");
  if (device >= count) return gw_fail(nullptr, GW_ERR_INVALID, "device ordinal out of range");
  GW_GUARD_DEVICE(nullptr, device);
  uint32_t *d_in = nullptr, *d_out = nullptr;
  hipError_t e = hipMalloc((void**)&d_in, sizeof(uint32_t) * 6 * (size_t)n);
  if (e == hipSuccess) e = hipMalloc((void**)&d_out, sizeof(uint32_t) * 4 * (size_t)n);
  if (e == hipSuccess) e = hipMemcpy(d_in, in, sizeof(uint32_t) * 6 * (size_t)n, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    k_philox<<<grid_for(n), kBlock>>>(d_in, n, d_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, d_out, sizeof(uint32_t) * 4 * (size_t)n, hipMemcpyDeviceToHost);
  if (d_in) (void)hipFree(d_in);
  if (d_out) (void)hipFree(d_out);
  if (e != hipSuccess) return gw_fail(nullptr, GW_ERR_DEVICE, "%s", hipGetErrorString(e));
  return GW_OK;
}

int gw_hip_device_count(int* count) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *count = c;
  return c > 0 ? GW_OK : GW_ERR_DEVICE;
}

extern "C" int gw_n2v_export_alias(const gw_graph* gc, int32_t* node_J, double* node_q,
                                   int64_t* edge_off, int32_t* edge_J, double* edge_q) {
  gw_graph* g = const_cast<gw_graph*>(gc);
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);  // restores the caller's current device on return
  if (!g->n2v_prepared) return gw_fail(g, GW_ERR_STATE, "call gw_n2v_prepare first");
  GW_HIP_TRY(hipSetDevice(g->device));
  const gw_dev_graph& d = g->d;
  if ((node_J || node_q) && !d.node_J)
    return gw_fail(g, GW_ERR_STATE, "no per-node alias tables (unweighted REJECTION mode draws uniformly)");
  if (node_J && g->nnz) GW_HIP_TRY(hipMemcpy(node_J, d.node_J, sizeof(int32_t) * g->nnz, hipMemcpyDeviceToHost));
  if (node_q && g->nnz) GW_HIP_TRY(hipMemcpy(node_q, d.node_q, sizeof(double) * g->nnz, hipMemcpyDeviceToHost));
  if (edge_off || edge_J || edge_q) {
    if (g->n2v_mode != GW_N2V_REPLAY) return gw_fail(g, GW_ERR_STATE, "per-edge tables exist only in GW_N2V_REPLAY mode");
    if (edge_off) GW_HIP_TRY(hipMemcpy(edge_off, d.edge_off, sizeof(int64_t) * (g->nnz + 1), hipMemcpyDeviceToHost));
    if (edge_J && g->edge_alias_entries)
      GW_HIP_TRY(hipMemcpy(edge_J, d.edge_J, sizeof(int32_t) * g->edge_alias_entries, hipMemcpyDeviceToHost));
    if (edge_q && g->edge_alias_entries)
      GW_HIP_TRY(hipMemcpy(edge_q, d.edge_q, sizeof(double) * g->edge_alias_entries, hipMemcpyDeviceToHost));
  }
  return GW_OK;
}

extern "C" int gw_n2v_walks_host(gw_graph* g, int walk_len, uint64_t seed, int64_t walk_begin,
                                 int64_t walk_count, int shuffle, int32_t* out_walks, int32_t* out_len,
                                 uint64_t* counters) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);  // restores the caller's current device on return
  if (!g->n2v_prepared) return gw_fail(g, GW_ERR_STATE, "call gw_n2v_prepare first");
  if (walk_len < 1 || walk_begin < 0 || walk_count < 0 || (walk_count > 0 && !out_walks))
    return gw_fail(g, GW_ERR_INVALID, "bad arguments");
  if (walk_count == 0) return GW_OK;
  GW_HIP_TRY(hipSetDevice(g->device));
  // Chunks of ~256 MB of walks, double-buffered: chunk k+1 is walked on one
  // stream while chunk k is copied out on another (a pageable copy blocks
  // the host, so the next kernel is enqueued before it).
  const int64_t chunk_bytes = g->opt.host_chunk_bytes > 0 ? g->opt.host_chunk_bytes : (int64_t)256 << 20;
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(walk_count, chunk_bytes / (4 * (int64_t)walk_len)));
  const int64_t nch = (walk_count + chunk - 1) / chunk;
  int32_t *d_out[2] = {nullptr, nullptr}, *d_len[2] = {nullptr, nullptr};
  uint64_t* d_cnt = nullptr;
  hipStream_t sc = nullptr, sx = nullptr;
  hipEvent_t done[2] = {nullptr, nullptr};
  auto release = [&]() {
    for (int b = 0; b < 2; ++b) {
      dev_free(d_out[b]);
      dev_free(d_len[b]);
      if (done[b]) (void)hipEventDestroy(done[b]);
    }
    dev_free(d_cnt);
    if (sc) (void)hipStreamDestroy(sc);
    if (sx) (void)hipStreamDestroy(sx);
  };
  int rc = GW_OK;
  const int nb = nch > 1 ? 2 : 1;
  for (int b = 0; b < nb && rc == GW_OK; ++b)
    if ((rc = dev_alloc(g, &d_out[b], chunk * (int64_t)walk_len)) == GW_OK) rc = dev_alloc(g, &d_len[b], chunk);
  if (rc == GW_OK) rc = dev_alloc(g, &d_cnt, 2);
  if (rc != GW_OK) {
    release();
    return rc;
  }
  hipError_t e = hipStreamCreateWithFlags(&sc, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&sx, hipStreamNonBlocking);
  for (int b = 0; b < nb && e == hipSuccess; ++b) e = hipEventCreateWithFlags(&done[b], hipEventDisableTiming);
  if (e == hipSuccess) e = hipMemsetAsync(d_cnt, 0, 2 * sizeof(uint64_t), sc);
  auto launch = [&](int64_t k) -> int {
    const int64_t c0 = k * chunk, cn = std::min(chunk, walk_count - c0);
    const int b = (int)(k & 1);
    int r = gw_dev_n2v_walks(g, walk_len, seed, walk_begin + c0, cn, shuffle, d_out[b], d_len[b], d_cnt, sc);
    if (r == GW_OK && hipEventRecord(done[b], sc) != hipSuccess) r = GW_ERR_DEVICE;
    return r;
  };
  if (e == hipSuccess) rc = launch(0);
  for (int64_t k = 0; k < nch && e == hipSuccess && rc == GW_OK; ++k) {
    // buffer (k+1)&1 was last read by the copy of chunk k-1, finished below
    if (k + 1 < nch && (rc = launch(k + 1)) != GW_OK) break;
    const int64_t c0 = k * chunk, cn = std::min(chunk, walk_count - c0);
    const int b = (int)(k & 1);
    e = hipStreamWaitEvent(sx, done[b], 0);
    if (e == hipSuccess)
      e = hipMemcpyAsync(out_walks + c0 * walk_len, d_out[b], cn * walk_len * sizeof(int32_t),
                         hipMemcpyDeviceToHost, sx);
    if (e == hipSuccess && out_len)
      e = hipMemcpyAsync(out_len + c0, d_len[b], cn * sizeof(int32_t), hipMemcpyDeviceToHost, sx);
    if (e == hipSuccess) e = hipStreamSynchronize(sx);
  }
  if (rc == GW_OK && e == hipSuccess) e = hipStreamSynchronize(sc);
  if (rc == GW_OK && e == hipSuccess && counters)
    e = hipMemcpy(counters, d_cnt, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost);
  release();
  if (rc != GW_OK) return rc;
  if (e != hipSuccess) return gw_fail(g, GW_ERR_DEVICE, "%s", hipGetErrorString(e));
  return GW_OK;
}
