// Double-walk SimRank variants (§8f-4): TopSim_doubleSample, TopSim_Dev,
// DoubleRandomWalk.
//
// Reference: DeepSim/TopSimAll/src/simrank/
//   TopSim_doubleSample.java  sample :71-140 — the TopSim BFS queue over STEP
//       levels; computePath :141-164 assigns paths[src][target][s] =
//       path[s].sample for every queued path in queue order (the LAST path
//       reaching `target` at level s wins); computeSims/getSim :167-193 —
//       sim[i][j] = sum_x sum_s C^s * P[i][x][s] * P[j][x][s] (i < j,
//       mirrored, diagonal 0).
//   TopSim_Dev.java  :31-95 — SAMPLE = (int)((step-singleStep)*sample*2 /
//       (step*(topK+1))); for every i: sample(i), then for each of i's top
//       `topK` candidates j (FixedMaxPQ over candidate[i][*] >= MIN) a fresh
//       sample(j) and sim[i][j] = getSim.
//   DoubleRandomWalk.java :50-91 — SAMPLE uniform walks of STEP steps per
//       vertex; sim[v][w] = sum over walk pairs of C^(t+1) at their first
//       meeting step t, / SAMPLE^2.
//
// GPU decomposition:
//   * k_topsim_levels: one workgroup per task (vertex, Philox call); the queue
//     is materialised level by level in Java queue order (as k_topsim_m) and
//     "last wins" is an atomicMax of queue positions per target, then the
//     winners write the level's mass row M[task][s-1][x] (dense, 0 = absent);
//   * k_levels_syrk: sim = M_c M^T with M_c = C^s-scaled rows (the product
//     (C^s * a) * b of getSim), a dense fp64 MFMA kernel
//     (v_mfma_f64_16x16x4f64, 64x64 tiles, upper triangle, mirrored);
//   * k_levels_dot: TopSim_Dev's per-candidate dot products (wave per pair);
//   * DoubleRandomWalk: walks keyed by (v, i, t); per step the walks are
//     radix-sorted by position and every bucket's walk pairs from different
//     sources with no earlier meeting add C^(t+1) (fp64 atomics).
// Sums are reassociated relative to the Java loops (rtol 1e-12 in tests).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "gw_device_common.h"

namespace {

constexpr int TD_BLOCK = 256;
constexpr int TD_WAVES = TD_BLOCK / 64;

__device__ __forceinline__ int td_excl_scan(int v, int* s_wave, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wave[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < TD_WAVES; ++w) {
      int t = s_wave[w];
      s_wave[w] = acc;
      acc += t;
    }
    s_wave[TD_WAVES] = acc;
  }
  __syncthreads();
  int r = s_wave[wid] + x - v;
  *total = s_wave[TD_WAVES];
  __syncthreads();
  return r;
}

__device__ __forceinline__ int td_upper_bound(const int32_t* a, int n, int x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (a[mid] <= x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

struct LvArgs {
  gw_dev_graph G;
  double sampled;
  uint32_t k0, k1;
  const int32_t* tv;  // task vertex
  const int32_t* tc;  // task Philox call
  int64_t ntask;
  double* out;        // [ntask][STEP][n]
  int64_t cap;
  int32_t* qv;        // [blocks][cap] current level vertex
  int32_t* qw;        // [blocks][cap] walker id
  double* qm;         // [blocks][cap] mass
  int32_t* nv;        // [blocks][cap] next level (ping-pong)
  int32_t* nwk;
  double* nm;
  int32_t* co;        // [blocks][cap+1]
  int32_t* nwo;       // [blocks][cap+1]
  int32_t* pos;       // [blocks][n] last position per target (-1)
  unsigned int* counter;
  int* error_flag;
};

template <int STEP>
__global__ void __launch_bounds__(TD_BLOCK) k_topsim_levels(LvArgs A) {
  __shared__ int s_wave[TD_WAVES + 1];
  __shared__ int s_task, s_size, s_abort;
  const int tid = threadIdx.x;
  const int64_t blk = blockIdx.x;
  const gw_dev_graph& G = A.G;
  const int64_t n = G.n, cap = A.cap;
  int32_t* V = A.qv + blk * cap;
  int32_t* W = A.qw + blk * cap;
  double* M = A.qm + blk * cap;
  int32_t* Vn = A.nv + blk * cap;
  int32_t* Wn = A.nwk + blk * cap;
  double* Mn = A.nm + blk * cap;
  int32_t* CO = A.co + blk * (cap + 1);
  int32_t* NW = A.nwo + blk * (cap + 1);
  int32_t* POS = A.pos + blk * n;
  for (;;) {
    if (tid == 0) {
      s_task = (int)atomicAdd(A.counter, 1u);
      s_abort = 0;
    }
    __syncthreads();
    const int64_t t = s_task;
    if (t >= A.ntask) break;
    const int32_t s = A.tv[t];
    const uint32_t call = (uint32_t)A.tc[t];
    double* out = A.out + t * (int64_t)STEP * n;
    if (tid == 0) {
      V[0] = s;
      W[0] = -1;
      M[0] = A.sampled;  // path[0].sample = SAMPLE (:76)
      s_size = 1;
    }
    __syncthreads();
    int walker_base = 0;
    for (int l = 0; l < STEP; ++l) {
      const int sz = s_size;
      // child counts and new walker ids in queue order (:88-134)
      int total_children = 0, total_new = 0;
      for (int base = 0; base < sz; base += TD_BLOCK) {
        const int j = base + tid;
        int cnt = 0, nwk = 0;
        if (j < sz) {
          const int d = G.deg[V[j]];
          const double m = M[j];
          if (d != 0 && m >= (double)d) {
            cnt = d;
          } else if (d != 0) {
            int c = (int)m;
            if ((double)c != m) c += 1;
            cnt = c;
            if (W[j] < 0) nwk = c;
          }
        }
        int tc, tn;
        const int ec = td_excl_scan(cnt, s_wave, &tc);
        const int en = td_excl_scan(nwk, s_wave, &tn);
        if (j < sz) {
          CO[j] = total_children + ec;
          NW[j] = total_new + en;
        }
        total_children += tc;
        total_new += tn;
        if ((int64_t)total_children > cap) total_children = (int)cap + 1;
      }
      if (tid == 0) {
        CO[sz] = total_children;
        if ((int64_t)total_children > cap) {
          atomicOr(A.error_flag, 1);
          s_abort = 1;
        }
      }
      __syncthreads();
      if (s_abort) break;
      for (int c = tid; c < total_children; c += TD_BLOCK) {
        const int j = td_upper_bound(CO, sz + 1, c) - 1;
        const int32_t v = V[j];
        const int k = c - CO[j];
        const int number = CO[j + 1] - CO[j];
        const int d = G.deg[v];
        const double m = M[j];
        int32_t x, wid;
        double nmass;
        if (m >= (double)d) {
          x = G.nbrs[G.offsets[v] + k];
          nmass = m / (double)d;
          wid = W[j];
        } else {
          const int g = W[j] >= 0 ? W[j] : walker_base + NW[j] + k;
          const gw_u4 u = gw_philox((uint32_t)s, (uint32_t)g, (uint32_t)(l + 1), call, A.k0, A.k1);
          x = G.nbrs[G.offsets[v] + gw_index(u.x, u.y, (uint32_t)d)];
          nmass = m / (double)number;
          wid = g;
        }
        Vn[c] = x;
        Wn[c] = wid;
        Mn[c] = nmass;
        if (x != s) atomicMax(&POS[x], c);  // computePath: last path in queue order wins (:157)
      }
      walker_base += total_new;
      __syncthreads();
      double* row = out + (int64_t)l * n;
      for (int c = tid; c < total_children; c += TD_BLOCK) {
        const int32_t x = Vn[c];
        if (x != s && POS[x] == c) row[x] = Mn[c];
      }
      __syncthreads();
      for (int c = tid; c < total_children; c += TD_BLOCK) {
        const int32_t x = Vn[c];
        if (x != s) POS[x] = -1;
      }
      // next level becomes current
      for (int c = tid; c < total_children; c += TD_BLOCK) {
        V[c] = Vn[c];
        W[c] = Wn[c];
        M[c] = Mn[c];
      }
      if (tid == 0) s_size = total_children;
      __syncthreads();
    }
  }
}

// sim[i][j] = sum_k (cache[k/n + 1] * M[i][k]) * M[j][k], K = STEP*n, for the
// 64x64 tiles with ti <= tj; i < j written to [i][j] and [j][i], i == j -> 0.
// Wave w of the tile owns rows 32*(w>>1).., cols 32*(w&1)..: 2x2 16x16 MFMAs.
constexpr int SY_T = 64, SY_K = 16;
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_levels_syrk(int64_t n, int step, const double* __restrict__ M,
                                                     const double* __restrict__ cache, double* __restrict__ sim,
                                                     const int32_t* __restrict__ tile_i, const int32_t* __restrict__ tile_j) {
  __shared__ double sa[SY_T][SY_K + 1];
  __shared__ double sb[SY_T][SY_K + 1];
  const int64_t K = (int64_t)step * n;
  const int64_t i0 = (int64_t)tile_i[blockIdx.x] * SY_T, j0 = (int64_t)tile_j[blockIdx.x] * SY_T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = 32 * (wave >> 1), wc = 32 * (wave & 1);
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  for (int64_t k0 = 0; k0 < K; k0 += SY_K) {
    // stage 64x16 of scaled A rows and B rows (coalesced 128 B segments)
    for (int e = tid; e < SY_T * SY_K; e += 256) {
      const int r = e / SY_K, c = e % SY_K;
      const int64_t k = k0 + c;
      const int64_t ia = i0 + r, jb = j0 + r;
      double av = 0.0, bv = 0.0;
      if (k < K) {
        const double sc = cache[k / n + 1];
        if (ia < n) av = sc * M[ia * K + k];  // (cache[step] * P[src]) as getSim (:187)
        if (jb < n) bv = M[jb * K + k];
      }
      sa[r][c] = av;
      sb[r][c] = bv;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < SY_K; kk += 4) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const double av = sa[wr + 16 * a + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const double bv = sb[wc + 16 * b + (lane & 15)][kk + (lane >> 4)];
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[a][b], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = i0 + wr + 16 * a + (lane >> 4) + 4 * r;
        const int64_t j = j0 + wc + 16 * b + (lane & 15);
        if (i < n && j < n && i < j) {
          const double v = acc[a][b][r];
          sim[i * n + j] = v;
          sim[j * n + i] = v;
        } else if (i < n && i == j) {
          sim[i * n + i] = 0.0;
        }
      }
}

// TopSim_Dev: sim[i][j] for each (i, rank) pair: dot of task rows
__global__ void k_levels_dot(int64_t n, int step, const double* __restrict__ M, const double* __restrict__ cache,
                             const int32_t* __restrict__ pr_src, const int32_t* __restrict__ pr_row_a,
                             const int32_t* __restrict__ pr_row_b, const int32_t* __restrict__ pr_dst, int64_t npairs,
                             double* __restrict__ sim) {
  const int lane = threadIdx.x & 63;
  const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (p >= npairs) return;
  const int64_t K = (int64_t)step * n;
  const double* a = M + (int64_t)pr_row_a[p] * K;
  const double* b = M + (int64_t)pr_row_b[p] * K;
  double acc = 0.0;
  for (int64_t k = lane; k < K; k += 64) {
    const double x = a[k], y = b[k];
    if (x > 0.0 && y > 0.0) acc += (cache[k / n + 1] * x) * y;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if (lane == 0) sim[(int64_t)pr_src[p] * n + pr_dst[p]] = acc;
}

// ---- DoubleRandomWalk ------------------------------------------------------
__global__ void k_drw_walks(gw_dev_graph G, int sample, int step, uint32_t k0, uint32_t k1,
                            int32_t* __restrict__ paths) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= G.n * (int64_t)sample) return;
  const int32_t v = (int32_t)(w / sample);
  const int i = (int)(w % sample);
  int32_t cur = v;
  for (int t = 0; t < step; ++t) {  // sample(src) :56-65
    if (cur >= 0) {
      const int d = G.deg[cur];
      if (d == 0) {
        cur = -1;
      } else {
        const gw_u4 u = gw_philox((uint32_t)v, (uint32_t)i, (uint32_t)(t + 1), 0u, k0, k1);
        cur = G.nbrs[G.offsets[cur] + gw_index(u.x, u.y, (uint32_t)d)];
      }
    }
    paths[w * step + t] = cur;  // -1 after a dead end (the Java loop stops there)
  }
}

__global__ void k_drw_keys(int64_t nw, int step, int t, const int32_t* __restrict__ paths, uint32_t* __restrict__ key,
                           int32_t* __restrict__ val) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  const int32_t p = paths[w * step + t];
  key[w] = p < 0 ? 0xFFFFFFFFu : (uint32_t)p;
  val[w] = (int32_t)w;
}

// every walk a in sorted order pairs with the later walks b of its bucket
__global__ void k_drw_pairs(int64_t nw, int sample, int step, int t, const int32_t* __restrict__ paths,
                            const uint32_t* __restrict__ skey, const int32_t* __restrict__ sval, double inc,
                            int64_t n, double* __restrict__ sim) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nw) return;
  const uint32_t key = skey[p];
  if (key == 0xFFFFFFFFu) return;
  const int32_t a = sval[p];
  const int64_t va = a / sample;
  const int32_t* pa = paths + (int64_t)a * step;
  for (int64_t q = p + 1; q < nw && skey[q] == key; ++q) {
    const int32_t b = sval[q];
    const int64_t vb = b / sample;
    if (vb == va) continue;  // getSim(v, w) is for v != w
    const int32_t* pb = paths + (int64_t)b * step;
    bool earlier = false;
    for (int u = 0; u < t; ++u) earlier |= pa[u] == pb[u];
    if (earlier) continue;  // met first at an earlier step (:81-87 break)
    const int64_t lo = va < vb ? va : vb, hi = va < vb ? vb : va;
    atomicAdd(&sim[lo * n + hi], inc);
  }
}

__global__ void k_drw_finish(int64_t n, double denom, double* __restrict__ sim) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * n) return;
  const int64_t i = e / n, j = e % n;
  if (i < j) {
    const double v = sim[e] / denom;  // result / (SAMPLE * SAMPLE) (:90)
    sim[e] = v;
    sim[j * n + i] = v;
  } else if (i == j) {
    sim[e] = 0.0;
  }
}

template <typename T>
int td_alloc(gw_graph* g, T** p, int64_t count) {
  *p = nullptr;
  if (count < 1) count = 1;
  if (hipMalloc((void**)p, sizeof(T) * (size_t)count) != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    g->err = "double-walk workspace allocation failed";
    return GW_ERR_NOMEM;
  }
  return GW_OK;
}

template <typename T>
void td_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

template <int STEP>
hipError_t launch_levels(const LvArgs& A, int blocks, hipStream_t s) {
  k_topsim_levels<STEP><<<blocks, TD_BLOCK, 0, s>>>(A);
  return hipGetLastError();
}

// level rows M[task][STEP][n] for tasks (tv, tc) on the device
int levels_run(gw_graph* g, int sample, int step, uint64_t seed, const int32_t* tv_dev, const int32_t* tc_dev,
               int64_t ntask, double* out_dev, hipStream_t s) {
  const int64_t n = g->n;
  // queue entries per level <= SAMPLE*(1 + 2*STEP) (see gw_topsim_m.hip) + a degree of slack
  const int64_t cap = std::max<int64_t>((int64_t)sample * (1 + 2 * step) + 16, g->max_degree + 16);
  int dev_cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, g->device) == hipSuccess) dev_cus = prop.multiProcessorCount;
  const int64_t per_block = cap * (4 + 4 + 8) * 2 + 2 * (cap + 1) * 4 + n * 4;
  const int64_t budget = (int64_t)8 << 30;
  int64_t blocks = std::min<int64_t>({(int64_t)2 * dev_cus, budget / std::max<int64_t>(per_block, 1), ntask});
  if (blocks < 1) {
    g->err = "double-walk level workspace exceeds the budget";
    return GW_ERR_CAPACITY;
  }
  LvArgs A{};
  A.G = g->d;
  A.sampled = (double)sample;
  A.k0 = (uint32_t)seed;
  A.k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  A.tv = tv_dev;
  A.tc = tc_dev;
  A.ntask = ntask;
  A.out = out_dev;
  A.cap = cap;
  int rc;
  if ((rc = td_alloc(g, &A.qv, blocks * cap)) || (rc = td_alloc(g, &A.qw, blocks * cap)) ||
      (rc = td_alloc(g, &A.qm, blocks * cap)) || (rc = td_alloc(g, &A.nv, blocks * cap)) ||
      (rc = td_alloc(g, &A.nwk, blocks * cap)) || (rc = td_alloc(g, &A.nm, blocks * cap)) ||
      (rc = td_alloc(g, &A.co, blocks * (cap + 1))) || (rc = td_alloc(g, &A.nwo, blocks * (cap + 1))) ||
      (rc = td_alloc(g, &A.pos, blocks * n)) || (rc = td_alloc(g, &A.counter, 1)) ||
      (rc = td_alloc(g, &A.error_flag, 1))) {
    td_free(A.qv); td_free(A.qw); td_free(A.qm); td_free(A.nv); td_free(A.nwk); td_free(A.nm);
    td_free(A.co); td_free(A.nwo); td_free(A.pos); td_free(A.counter); td_free(A.error_flag);
    return rc;
  }
  hipError_t e = hipMemsetAsync(out_dev, 0, sizeof(double) * (size_t)(ntask * step * n), s);
  if (e == hipSuccess) e = hipMemsetAsync(A.pos, 0xFF, sizeof(int32_t) * (size_t)(blocks * n), s);
  if (e == hipSuccess) e = hipMemsetAsync(A.counter, 0, sizeof(unsigned int), s);
  if (e == hipSuccess) e = hipMemsetAsync(A.error_flag, 0, sizeof(int), s);
  if (e == hipSuccess) {
    switch (step) {
      case 1: e = launch_levels<1>(A, (int)blocks, s); break;
      case 2: e = launch_levels<2>(A, (int)blocks, s); break;
      case 3: e = launch_levels<3>(A, (int)blocks, s); break;
      case 4: e = launch_levels<4>(A, (int)blocks, s); break;
      case 5: e = launch_levels<5>(A, (int)blocks, s); break;
      case 6: e = launch_levels<6>(A, (int)blocks, s); break;
      case 7: e = launch_levels<7>(A, (int)blocks, s); break;
      default: e = launch_levels<8>(A, (int)blocks, s); break;
    }
  }
  int flag = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&flag, A.error_flag, sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  td_free(A.qv); td_free(A.qw); td_free(A.qm); td_free(A.nv); td_free(A.nwk); td_free(A.nm);
  td_free(A.co); td_free(A.nwo); td_free(A.pos); td_free(A.counter); td_free(A.error_flag);
  GW_HIP_TRY(e);
  if (flag) {
    g->err = "double-walk sample(): a BFS level exceeded its queue capacity";
    return GW_ERR_CAPACITY;
  }
  return GW_OK;
}

int check_common(gw_graph* g, int sample, int step) {
  if (g->device < 0) {
    g->err = "graph is not on a device";
    return GW_ERR_STATE;
  }
  if (g->directed) {
    g->err = "double-walk SimRank variants need an undirected graph";
    return GW_ERR_UNSUPPORTED;
  }
  if (step < 1 || step > 8) {
    g->err = "step must be in [1, 8]";
    return GW_ERR_UNSUPPORTED;
  }
  if (sample < 0) {
    g->err = "sample must be >= 0";
    return GW_ERR_INVALID;
  }
  return GW_OK;
}

int upload_cache(gw_graph* g, int step, double C, double** cache_dev) {
  std::vector<double> cache((size_t)step + 2, 0.0);
  for (int i = 0; i <= step; ++i) cache[(size_t)i] = std::pow(C, (double)i);  // Math.pow (:37)
  int rc = td_alloc(g, cache_dev, step + 2);
  if (rc) return rc;
  GW_HIP_TRY(hipMemcpy(*cache_dev, cache.data(), sizeof(double) * (step + 2), hipMemcpyHostToDevice));
  return GW_OK;
}

}  // namespace

// TopSim_doubleSample(g, sample, step).compute(): sim_dev[n*n]
int gw_dev_topsim_double(gw_graph* g, int sample, int step, double C, uint64_t seed, double* sim_dev, void* stream) {
  int rc = check_common(g, sample, step);
  if (rc) return rc;
  GW_HIP_TRY(hipSetDevice(g->device));
  const int64_t n = g->n;
  if (n == 0) return GW_OK;
  hipStream_t s = (hipStream_t)stream;
  double* M = nullptr;
  double* cache = nullptr;
  int32_t *tv = nullptr, *tc = nullptr, *ti = nullptr, *tj = nullptr;
  const int64_t nt = (n + SY_T - 1) / SY_T;
  std::vector<int32_t> hv((size_t)n), hti, htj;
  for (int64_t v = 0; v < n; ++v) hv[(size_t)v] = (int32_t)v;
  for (int64_t a = 0; a < nt; ++a)
    for (int64_t b = a; b < nt; ++b) {
      hti.push_back((int32_t)a);
      htj.push_back((int32_t)b);
    }
  if ((rc = td_alloc(g, &M, n * step * n)) || (rc = td_alloc(g, &tv, n)) || (rc = td_alloc(g, &tc, n)) ||
      (rc = td_alloc(g, &ti, (int64_t)hti.size())) || (rc = td_alloc(g, &tj, (int64_t)htj.size())) ||
      (rc = upload_cache(g, step, C, &cache))) {
    td_free(M); td_free(tv); td_free(tc); td_free(ti); td_free(tj); td_free(cache);
    if (rc == GW_ERR_NOMEM) g->err = "TopSim_doubleSample needs STEP*n*n doubles of level rows";
    return rc;
  }
  hipError_t e = hipMemcpy(tv, hv.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(tc, 0, sizeof(int32_t) * n);
  if (e == hipSuccess) e = hipMemcpy(ti, hti.data(), sizeof(int32_t) * hti.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(tj, htj.data(), sizeof(int32_t) * htj.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    rc = levels_run(g, sample, step, seed, tv, tc, n, M, s);
    if (rc == GW_OK) {
      k_levels_syrk<<<(unsigned)hti.size(), 256, 0, s>>>(n, step, M, cache, sim_dev, ti, tj);
      e = hipGetLastError();
      if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
  }
  td_free(M); td_free(tv); td_free(tc); td_free(ti); td_free(tj); td_free(cache);
  if (rc != GW_OK) return rc;
  GW_HIP_TRY(e);
  return GW_OK;
}

// TopSim_Dev(g, sample, step, topK, singleStep).compute(candidate) given the
// candidate lists cand_dev[n*topK] (FixedMaxPQ order, -1 padded)
int gw_dev_topsim_dev(gw_graph* g, int sample_total, int step, int topK, int singleStep, double C, uint64_t seed,
                      const int32_t* cand_dev, double* sim_dev, void* stream) {
  // SAMPLE = (int)(((step-singleStep)*sample*2.0)/((double)step*(topK+1.0))) (TopSim_Dev.java:33)
  const int SAMPLE = (int)((((double)(step - singleStep) * (double)sample_total) * 2.0) /
                           ((double)step * ((double)topK + 1.0)));
  int rc = check_common(g, std::max(SAMPLE, 0), step);
  if (rc) return rc;
  if (topK < 0) {
    g->err = "topK must be >= 0";
    return GW_ERR_INVALID;
  }
  GW_HIP_TRY(hipSetDevice(g->device));
  const int64_t n = g->n;
  if (n == 0) return GW_OK;
  hipStream_t s = (hipStream_t)stream;
  GW_HIP_TRY(hipMemsetAsync(sim_dev, 0, sizeof(double) * (size_t)(n * n), s));
  if (topK == 0 || SAMPLE <= 0) return hipStreamSynchronize(s) == hipSuccess ? GW_OK : GW_ERR_DEVICE;
  std::vector<int32_t> cand((size_t)(n * topK));
  GW_HIP_TRY(hipMemcpy(cand.data(), cand_dev, sizeof(int32_t) * cand.size(), hipMemcpyDeviceToHost));
  // batches of sources: tasks (i, call 0) + (cand, call 1 + i*topK + r)
  const int64_t per_task = (int64_t)step * n * 8;
  const int64_t bsrc = std::max<int64_t>(1, std::min<int64_t>(n, ((int64_t)1 << 30) / (per_task * (1 + topK))));
  double* M = nullptr;
  double* cache = nullptr;
  int32_t *tv = nullptr, *tc = nullptr, *ps = nullptr, *pa = nullptr, *pb = nullptr, *pd = nullptr;
  const int64_t maxt = bsrc * (1 + topK);
  if ((rc = td_alloc(g, &M, maxt * step * n)) || (rc = td_alloc(g, &tv, maxt)) || (rc = td_alloc(g, &tc, maxt)) ||
      (rc = td_alloc(g, &ps, maxt)) || (rc = td_alloc(g, &pa, maxt)) || (rc = td_alloc(g, &pb, maxt)) ||
      (rc = td_alloc(g, &pd, maxt)) || (rc = upload_cache(g, step, C, &cache))) {
    td_free(M); td_free(tv); td_free(tc); td_free(ps); td_free(pa); td_free(pb); td_free(pd); td_free(cache);
    return rc;
  }
  hipError_t e = hipSuccess;
  for (int64_t i0 = 0; i0 < n && rc == GW_OK && e == hipSuccess; i0 += bsrc) {
    const int64_t i1 = std::min(n, i0 + bsrc);
    std::vector<int32_t> htv, htc, hs, ha, hb, hd;
    for (int64_t i = i0; i < i1; ++i) {
      const int32_t self = (int32_t)htv.size();
      htv.push_back((int32_t)i);
      htc.push_back(0);
      for (int r = 0; r < topK; ++r) {
        const int32_t j = cand[(size_t)(i * topK + r)];
        if (j < 0) break;
        hs.push_back((int32_t)i);
        ha.push_back(self);
        hb.push_back((int32_t)htv.size());
        hd.push_back(j);
        htv.push_back(j);
        htc.push_back(1 + (int32_t)(i * topK + r));
      }
    }
    e = hipMemcpy(tv, htv.data(), sizeof(int32_t) * htv.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(tc, htc.data(), sizeof(int32_t) * htc.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && !hs.empty()) {
      e = hipMemcpy(ps, hs.data(), sizeof(int32_t) * hs.size(), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(pa, ha.data(), sizeof(int32_t) * ha.size(), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(pb, hb.data(), sizeof(int32_t) * hb.size(), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(pd, hd.data(), sizeof(int32_t) * hd.size(), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) break;
    rc = levels_run(g, SAMPLE, step, seed, tv, tc, (int64_t)htv.size(), M, s);
    if (rc != GW_OK || hs.empty()) continue;
    const int64_t np = (int64_t)hs.size();
    k_levels_dot<<<(unsigned)((np * 64 + 255) / 256), 256, 0, s>>>(n, step, M, cache, ps, pa, pb, pd, np, sim_dev);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
  }
  td_free(M); td_free(tv); td_free(tc); td_free(ps); td_free(pa); td_free(pb); td_free(pd); td_free(cache);
  if (rc != GW_OK) return rc;
  GW_HIP_TRY(e);
  return GW_OK;
}

// DoubleRandomWalk(g, sample, step).compute(): sim_dev[n*n]
int gw_dev_double_random_walk(gw_graph* g, int sample, int step, double C, uint64_t seed, double* sim_dev,
                              void* stream) {
  int rc = check_common(g, sample, step);
  if (rc) return rc;
  if (sample < 1) {
    g->err = "sample must be >= 1";
    return GW_ERR_INVALID;
  }
  GW_HIP_TRY(hipSetDevice(g->device));
  const int64_t n = g->n;
  if (n == 0) return GW_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nw = n * (int64_t)sample;
  if (nw >= ((int64_t)1 << 31)) {
    g->err = "DoubleRandomWalk: n*SAMPLE walks must stay below 2^31";
    return GW_ERR_UNSUPPORTED;
  }
  int32_t *paths = nullptr, *val = nullptr, *sval = nullptr;
  uint32_t *key = nullptr, *skey = nullptr;
  void* tmp = nullptr;
  size_t tmpb = 0;
  GW_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmpb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                (const int32_t*)nullptr, (int32_t*)nullptr, (int)nw, 0, 32, s));
  if ((rc = td_alloc(g, &paths, nw * step)) || (rc = td_alloc(g, &key, nw)) || (rc = td_alloc(g, &skey, nw)) ||
      (rc = td_alloc(g, &val, nw)) || (rc = td_alloc(g, &sval, nw)) || (rc = td_alloc(g, (char**)&tmp, (int64_t)tmpb))) {
    td_free(paths); td_free(key); td_free(skey); td_free(val); td_free(sval); td_free(tmp);
    return rc;
  }
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  hipError_t e = hipMemsetAsync(sim_dev, 0, sizeof(double) * (size_t)(n * n), s);
  const unsigned gb = (unsigned)((nw + 255) / 256);
  if (e == hipSuccess) {
    k_drw_walks<<<gb, 256, 0, s>>>(g->d, sample, step, k0, k1, paths);
    e = hipGetLastError();
  }
  for (int t = 0; t < step && e == hipSuccess; ++t) {
    k_drw_keys<<<gb, 256, 0, s>>>(nw, step, t, paths, key, val);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, key, skey, val, sval, (int)nw, 0, 32, s);
    if (e == hipSuccess) {
      const double inc = std::pow(C, (double)(t + 1));  // cache[step+1] (:84)
      k_drw_pairs<<<gb, 256, 0, s>>>(nw, sample, step, t, paths, skey, sval, inc, n, sim_dev);
      e = hipGetLastError();
    }
  }
  if (e == hipSuccess) {
    k_drw_finish<<<(unsigned)((n * n + 255) / 256), 256, 0, s>>>(n, (double)(sample * sample), sim_dev);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  td_free(paths); td_free(key); td_free(skey); td_free(val); td_free(sval); td_free(tmp);
  GW_HIP_TRY(e);
  return GW_OK;
}

extern "C" int gw_double_sim_host(gw_graph* g, int kind, int sample, int step, int topK, int singleStep, double C,
                       uint64_t seed, const int32_t* cand, double* sim) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);  // restores the caller's current device on return
  if (g->device < 0) return gw_fail(g, GW_ERR_STATE, "graph is not on a device");
  if (g->n > 0 && !sim) return gw_fail(g, GW_ERR_INVALID, "bad arguments");
  if (kind == GW_DOUBLE_DEV && topK > 0 && !cand) return gw_fail(g, GW_ERR_INVALID, "candidates required");
  const int64_t n = g->n;
  if (n == 0) return GW_OK;
  double* d_sim = nullptr;
  int32_t* d_cand = nullptr;
  if (hipMalloc((void**)&d_sim, sizeof(double) * (size_t)(n * n)) != hipSuccess) {
    (void)hipGetLastError();
    return gw_fail(g, GW_ERR_NOMEM, "n*n result does not fit in device memory");
  }
  int rc = GW_OK;
  if (kind == GW_DOUBLE_DEV && topK > 0) {
    if (hipMalloc((void**)&d_cand, sizeof(int32_t) * (size_t)(n * topK)) != hipSuccess ||
        hipMemcpy(d_cand, cand, sizeof(int32_t) * (size_t)(n * topK), hipMemcpyHostToDevice) != hipSuccess)
      rc = gw_fail(g, GW_ERR_DEVICE, "candidate upload failed");
  }
  if (rc == GW_OK) {
    if (kind == GW_DOUBLE_SAMPLE)
      rc = gw_dev_topsim_double(g, sample, step, C, seed, d_sim, nullptr);
    else if (kind == GW_DOUBLE_DEV)
      rc = gw_dev_topsim_dev(g, sample, step, topK, singleStep, C, seed, d_cand, d_sim, nullptr);
    else if (kind == GW_DOUBLE_RANDOM_WALK)
      rc = gw_dev_double_random_walk(g, sample, step, C, seed, d_sim, nullptr);
    else
      rc = gw_fail(g, GW_ERR_INVALID, "unknown double-walk kind %d", kind);
  }
  if (rc == GW_OK && hipMemcpy(sim, d_sim, sizeof(double) * (size_t)(n * n), hipMemcpyDeviceToHost) != hipSuccess)
    rc = gw_fail(g, GW_ERR_DEVICE, "result copy failed");
  if (d_sim) (void)hipFree(d_sim);
  if (d_cand) (void)hipFree(d_cand);
  return rc;
}

