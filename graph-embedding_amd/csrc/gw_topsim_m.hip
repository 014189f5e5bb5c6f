// Bounded-memory TopSim variants with the reference's FixedCacheMap (§8f-3).
//
// Reference: DeepSim/TopSimAll/src/simrank/TopSim_singleSample_M.java
//   walk            :62-174  the same BFS queue of weighted paths as
//                            TopSim_singleSample (mass >= degree -> all
//                            neighbours with mass/d; else ceil(mass) random
//                            children with mass/ceil(mass))
//   computePathSim  :202-239 at pathLen = 2i, in queue order, every path with
//                            target != source and isFirstMeet puts
//                            (float)(mass*C^i*deg(mid)/deg(target)/SAMPLE)
// SingleRandomWalk_M.java:47-92: SAMPLE independent walks of 2*STEP steps,
//   each walk's updates (levels 1..STEP) put in walk order.
// lxctools/FixedCacheMap.java:14-127: float min-heap of `capacity` entries,
//   put() adds to a present key, inserts while not full, else replaces the
//   minimum when the new value is larger; iteration drains ascending.
//
// The put() sequence is order dependent (eviction), so the BFS queue is
// materialised level by level in queue order — enumerated paths and random
// walkers interleaved exactly as the Java LinkedList holds them (parent
// index per entry, walker ids in queue order so the Philox draws equal
// gw_topsim.hip's) — every level's updates are produced in parallel into a
// queue-ordered buffer, and one lane replays them into an LDS FixedCacheMap
// (heap + open-addressing key index), literally as Java does.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "gw_device_common.h"

namespace {

constexpr int TM_BLOCK = 256;
constexpr int TM_WAVES = TM_BLOCK / 64;
constexpr int TM_CAP_MAX = 4096;  // FixedCacheMap capacity held in LDS (Java's Short index allows 32767)

struct TmArgs {
  gw_dev_graph G;
  int variant;
  int sample;
  double sampled;
  double cache[16];
  uint32_t k0, k1;
  const int32_t* sources;
  int64_t nsrc;
  int capacity;
  int hash_slots;
  int32_t* out_keys;
  float* out_vals;
  int32_t* out_size;
  long long* stats;
  int64_t cap;  // queue entries per level (or SAMPLE*STEP updates)
  int32_t* qv;  // [blocks][L+1][cap] vertex
  int32_t* qp;  // [blocks][L+1][cap] parent index
  int32_t* qw;  // [blocks][L+1][cap] walker id (-1: enumerated)
  double* qm;   // [blocks][2][cap] mass (current / next level)
  int32_t* co;  // [blocks][cap+1] child offsets
  int32_t* nw;  // [blocks][cap+1] new-walker offsets
  int32_t* uk;  // [blocks][cap] update keys (-1: none), queue order
  float* uvv;   // [blocks][cap] update values
  unsigned int* src_counter;
  int* error_flag;
};

__device__ __forceinline__ int tm_excl_scan(int v, int* s_wave, int* total) {
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
    for (int w = 0; w < TM_WAVES; ++w) {
      int t = s_wave[w];
      s_wave[w] = acc;
      acc += t;
    }
    s_wave[TM_WAVES] = acc;
  }
  __syncthreads();
  int r = s_wave[wid] + x - v;
  *total = s_wave[TM_WAVES];
  __syncthreads();
  return r;
}

__device__ __forceinline__ int tm_upper_bound(const int32_t* a, int n, int x) {
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

// ---- FixedCacheMap in LDS, single lane (FixedCacheMap.java) -----------------
struct Fcm {
  int N, NMAX, hmask;
  int32_t* keys;  // [NMAX+1], 1-based heap
  float* vals;    // [NMAX+1]
  int32_t* hk;    // [hmask+1] key (-1 empty)
  int32_t* hv;    // [hmask+1] heap index
};

__device__ __forceinline__ uint32_t fcm_h(int32_t k) { return (uint32_t)k * 0x9E3779B1u; }

__device__ int fcm_get(const Fcm& m, int32_t k) {
  for (uint32_t h = fcm_h(k) & m.hmask;; h = (h + 1) & m.hmask) {
    const int32_t x = m.hk[h];
    if (x == k) return m.hv[h];
    if (x == -1) return -1;
  }
}
__device__ void fcm_hput(Fcm& m, int32_t k, int v) {
  uint32_t h = fcm_h(k) & m.hmask;
  while (m.hk[h] != -1 && m.hk[h] != k) h = (h + 1) & m.hmask;
  m.hk[h] = k;
  m.hv[h] = v;
}
__device__ void fcm_hdel(Fcm& m, int32_t k) {  // backward-shift deletion
  uint32_t h = fcm_h(k) & m.hmask;
  while (m.hk[h] != k) {
    if (m.hk[h] == -1) return;
    h = (h + 1) & m.hmask;
  }
  uint32_t i = h;
  for (;;) {
    m.hk[i] = -1;
    uint32_t j = i;
    for (;;) {
      j = (j + 1) & m.hmask;
      if (m.hk[j] == -1) return;
      const uint32_t home = fcm_h(m.hk[j]) & m.hmask;
      const bool in = (i <= j) ? (home > i && home <= j) : (home > i || home <= j);
      if (!in) break;
    }
    m.hk[i] = m.hk[j];
    m.hv[i] = m.hv[j];
    i = j;
  }
}
__device__ void fcm_exch(Fcm& m, int a, int b) {  // :86-98
  fcm_hput(m, m.keys[a], b);
  fcm_hput(m, m.keys[b], a);
  const int32_t tk = m.keys[a];
  m.keys[a] = m.keys[b];
  m.keys[b] = tk;
  const float tv = m.vals[a];
  m.vals[a] = m.vals[b];
  m.vals[b] = tv;
}
__device__ void fcm_sink(Fcm& m, int i) {  // :61-69
  while (2 * i <= m.N) {
    int j = 2 * i;
    if (j < m.N && m.vals[j] > m.vals[j + 1]) j++;
    if (!(m.vals[i] > m.vals[j])) break;
    fcm_exch(m, i, j);
    i = j;
  }
}
__device__ void fcm_swim(Fcm& m, int i) {  // :73-78
  while (i > 1 && m.vals[i / 2] > m.vals[i]) {
    fcm_exch(m, i, i / 2);
    i = i / 2;
  }
}
__device__ void fcm_put(Fcm& m, int32_t key, float value) {  // :32-50
  const int idx = fcm_get(m, key);
  if (idx >= 0) {
    m.vals[idx] += value;
    fcm_sink(m, idx);
  } else if (m.N < m.NMAX) {
    m.N++;
    m.keys[m.N] = key;
    m.vals[m.N] = value;
    fcm_hput(m, key, m.N);
    fcm_swim(m, m.N);
  } else if (value > m.vals[1]) {
    fcm_hdel(m, m.keys[1]);
    m.keys[1] = key;
    m.vals[1] = value;
    fcm_hput(m, key, 1);
    fcm_sink(m, 1);
  }
}

template <int STEP>
__global__ void __launch_bounds__(TM_BLOCK) k_topsim_m(TmArgs A) {
  constexpr int L = 2 * STEP;
  extern __shared__ int32_t s_dyn[];
  __shared__ int s_wave[TM_WAVES + 1];
  __shared__ int s_size[L + 2];
  __shared__ int s_src, s_abort;
  __shared__ long long s_st[4];

  const int tid = threadIdx.x;
  const int64_t blk = blockIdx.x;
  const gw_dev_graph& G = A.G;
  const int64_t cap = A.cap;
  int32_t* V = A.qv + blk * (int64_t)(L + 1) * cap;
  int32_t* P = A.qp + blk * (int64_t)(L + 1) * cap;
  int32_t* W = A.qw + blk * (int64_t)(L + 1) * cap;
  double* M = A.qm + blk * 2 * cap;
  int32_t* CO = A.co + blk * (cap + 1);
  int32_t* NW = A.nw + blk * (cap + 1);
  int32_t* UK = A.uk + blk * cap;
  float* UV = A.uvv + blk * cap;
  Fcm fm;
  fm.NMAX = A.capacity;
  fm.hmask = A.hash_slots - 1;
  fm.keys = s_dyn;
  fm.hk = s_dyn + (A.capacity + 1);
  fm.hv = fm.hk + A.hash_slots;
  fm.vals = reinterpret_cast<float*>(fm.hv + A.hash_slots);
  const bool rw = A.variant == GW_TOPSIM_SINGLE_RW;
  if (tid == 0) s_st[0] = s_st[1] = s_st[2] = s_st[3] = 0;

  // one update (or none) of path `path[0..2i]` with mass `mass`
  auto update = [&](const int32_t* path, int i, int32_t source, double mass, int32_t* key, float* val) {
    *key = -1;
    const int32_t target = path[2 * i];
    if (target == source) return;
#pragma unroll
    for (int j = 0; j < STEP; ++j)  // isFirstMeet (:251-258)
      if (j < i && path[j] == path[2 * i - j]) return;
    const double dm = (double)G.deg[path[i]];
    const double dt = (double)G.deg[target];
    double incre;
    if (rw)  // SingleRandomWalk_M.java: cache[i]*deg/deg/SAMPLE
      incre = ((A.cache[i] * dm) / dt) / A.sampled;
    else     // TopSim_singleSample_M.java:224
      incre = (((mass * A.cache[i]) * dm) / dt) / A.sampled;
    *key = target;
    *val = (float)incre;
  };

  for (;;) {
    if (tid == 0) {
      s_src = (int)atomicAdd(A.src_counter, 1u);
      s_abort = 0;
      fm.N = 0;
    }
    for (int h = tid; h < A.hash_slots; h += TM_BLOCK) fm.hk[h] = -1;
    __syncthreads();
    const int64_t r = s_src;
    if (r >= A.nsrc) break;
    const int32_t s = A.sources[r];
    long long my_ext = 0, my_upd = 0, my_walk = 0;

    if (rw) {
      // SAMPLE walks; walk w's updates at UK[w*STEP + i-1] (walk-major order)
      const int ds = G.deg[s];
      for (int w = tid; w < A.sample; w += TM_BLOCK) {
        int32_t path[L + 1];
        path[0] = s;
        int32_t cur = s;
        int len = 0;
#pragma unroll
        for (int t = 1; t <= L; ++t) {
          if (len == t - 1) {
            const int d = G.deg[cur];
            if (d != 0) {
              const gw_u4 u = gw_philox((uint32_t)s, (uint32_t)w, (uint32_t)t, 0u, A.k0, A.k1);
              cur = G.nbrs[G.offsets[cur] + gw_index(u.x, u.y, (uint32_t)d)];
              path[t] = cur;
              len = t;
              ++my_ext;
            }
          }
        }
#pragma unroll
        for (int i = 1; i <= STEP; ++i) {
          int32_t k = -1;
          float v = 0.f;
          if (2 * i <= len) update(path, i, s, 0.0, &k, &v);
          UK[(int64_t)w * STEP + (i - 1)] = k;
          UV[(int64_t)w * STEP + (i - 1)] = v;
          if (k >= 0) ++my_upd;
        }
        ++my_walk;
      }
      (void)ds;
      __syncthreads();
      if (tid == 0) {
        const int64_t nu = (int64_t)A.sample * STEP;
        for (int64_t q = 0; q < nu; ++q)
          if (UK[q] >= 0) fcm_put(fm, UK[q], UV[q]);
      }
      __syncthreads();
    } else {
      if (tid == 0) {
        V[0] = s;
        P[0] = -1;
        W[0] = -1;
        M[0] = A.sampled;  // path[0].sample = SAMPLE (:89)
        s_size[0] = 1;
      }
      __syncthreads();
      int walker_base = 0;
      for (int l = 0; l <= L; ++l) {
        const int sz = s_size[l];
        const int32_t* Vl = V + (int64_t)l * cap;
        const int32_t* Wl = W + (int64_t)l * cap;
        const double* Ml = M + (int64_t)(l & 1) * cap;
        if (tid == 0 && l < L && sz > s_st[2]) s_st[2] = sz;
        // computePathSim at pathLen = 2i (:96-99, :173), queue order
        if ((l & 1) == 0 && l >= 2) {
          for (int j = tid; j < sz; j += TM_BLOCK) {
            int32_t path[L + 1];
            int p = j;
#pragma unroll
            for (int t = L; t >= 1; --t) {
              if (t <= l) {
                path[t] = V[(int64_t)t * cap + p];
                p = P[(int64_t)t * cap + p];
              }
            }
            path[0] = s;
            int32_t k = -1;
            float v = 0.f;
#pragma unroll
            for (int t = 2; t <= L; t += 2)
              if (t == l) update(path, t / 2, s, Ml[j], &k, &v);
            UK[j] = k;
            UV[j] = v;
            if (k >= 0) ++my_upd;
          }
          __syncthreads();
          if (tid == 0)
            for (int j = 0; j < sz; ++j)
              if (UK[j] >= 0) fcm_put(fm, UK[j], UV[j]);
          __syncthreads();
        }
        if (l == L) break;
        // child counts (:110-165) and new walker ids, in queue order
        int total_children = 0, total_new = 0;
        for (int base = 0; base < sz; base += TM_BLOCK) {
          const int j = base + tid;
          int cnt = 0, nwk = 0;
          if (j < sz) {
            const int d = G.deg[Vl[j]];
            const double m = Ml[j];
            if (d != 0 && m >= (double)d) {
              cnt = d;
            } else if (d != 0) {
              int c = (int)m;  // number = (int)s == s ? (int)s : (int)s + 1 (:147-151)
              if ((double)c != m) c += 1;
              cnt = c;
              if (Wl[j] < 0) nwk = c;
            }
          }
          int tc, tn;
          const int ec = tm_excl_scan(cnt, s_wave, &tc);
          const int en = tm_excl_scan(nwk, s_wave, &tn);
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
        int32_t* Vn = V + (int64_t)(l + 1) * cap;
        int32_t* Pn = P + (int64_t)(l + 1) * cap;
        int32_t* Wn = W + (int64_t)(l + 1) * cap;
        double* Mn = M + (int64_t)((l + 1) & 1) * cap;
        for (int c = tid; c < total_children; c += TM_BLOCK) {
          const int j = tm_upper_bound(CO, sz + 1, c) - 1;
          const int32_t v = Vl[j];
          const int k = c - CO[j];
          const int number = CO[j + 1] - CO[j];
          const int d = G.deg[v];
          const double m = Ml[j];
          int32_t x, wid;
          double nm;
          if (m >= (double)d) {  // all neighbours, insertion order (:118-131)
            x = G.nbrs[G.offsets[v] + k];
            nm = m / (double)d;
            wid = Wl[j];
          } else {  // number random children (:153-164)
            const int g = Wl[j] >= 0 ? Wl[j] : walker_base + NW[j] + k;
            const gw_u4 u = gw_philox((uint32_t)s, (uint32_t)g, (uint32_t)(l + 1), 0u, A.k0, A.k1);
            x = G.nbrs[G.offsets[v] + gw_index(u.x, u.y, (uint32_t)d)];
            nm = m / (double)number;
            wid = g;
          }
          Vn[c] = x;
          Pn[c] = j;
          Wn[c] = wid;
          Mn[c] = nm;
        }
        my_ext += (tid == 0) ? total_children : 0;
        my_walk += (tid == 0) ? total_new : 0;
        walker_base += total_new;
        if (tid == 0) s_size[l + 1] = total_children;
        __syncthreads();
      }
    }
    // drain ascending (FixedCacheMap iteration: repeated delMin, :104-127)
    if (tid == 0) {
      int c = 0;
      int32_t* ok = A.out_keys + r * (int64_t)A.capacity;
      float* ov = A.out_vals + r * (int64_t)A.capacity;
      if (!s_abort) {
        while (fm.N > 0) {
          ok[c] = fm.keys[1];
          ov[c] = fm.vals[1];
          ++c;
          fcm_hdel(fm, fm.keys[1]);
          fcm_exch(fm, 1, fm.N--);
          fcm_sink(fm, 1);
        }
      }
      for (int q = c; q < A.capacity; ++q) {
        ok[q] = -1;
        ov[q] = 0.f;
      }
      A.out_size[r] = c;
    }
    // stats
    atomicAdd((unsigned long long*)&s_st[0], (unsigned long long)my_ext);
    atomicAdd((unsigned long long*)&s_st[1], (unsigned long long)my_upd);
    atomicAdd((unsigned long long*)&s_st[3], (unsigned long long)my_walk);
    __syncthreads();
  }
  if (tid == 0 && A.stats) {
    atomicAdd((unsigned long long*)&A.stats[0], (unsigned long long)s_st[0]);
    atomicAdd((unsigned long long*)&A.stats[1], (unsigned long long)s_st[1]);
    atomicMax(&A.stats[2], s_st[2]);
    atomicAdd((unsigned long long*)&A.stats[3], (unsigned long long)s_st[3]);
  }
}

template <int STEP>
hipError_t launch_m(const TmArgs& A, int blocks, size_t lds, hipStream_t s) {
  hipError_t e = hipFuncSetAttribute((const void*)k_topsim_m<STEP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  k_topsim_m<STEP><<<blocks, TM_BLOCK, lds, s>>>(A);
  return hipGetLastError();
}

template <typename T>
int tm_alloc(gw_graph* g, T** p, int64_t count) {
  *p = nullptr;
  if (count < 1) count = 1;
  if (hipMalloc((void**)p, sizeof(T) * (size_t)count) != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    g->err = "TopSim_M workspace allocation failed";
    return GW_ERR_NOMEM;
  }
  return GW_OK;
}

template <typename T>
void tm_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

}  // namespace

// Device-pointer form; allocates its own per-call workspace (synchronous).
int gw_dev_topsim_m(gw_graph* g, int variant, int capacity, int sample, int step, double C, uint64_t seed,
                    const int32_t* sources_dev, int64_t nsrc, int32_t* out_keys_dev, float* out_vals_dev,
                    int32_t* out_size_dev, int64_t* stats_dev, void* stream) {
  if (variant != GW_TOPSIM_SINGLE_SAMPLE && variant != GW_TOPSIM_SINGLE_RW) {
    g->err = "TopSim_M variants: GW_TOPSIM_SINGLE_SAMPLE (TopSim_singleSample_M) or GW_TOPSIM_SINGLE_RW "
             "(SingleRandomWalk_M)";
    return GW_ERR_UNSUPPORTED;
  }
  if (step < 1 || step > 8) {
    g->err = "step must be in [1, 8]";
    return GW_ERR_UNSUPPORTED;
  }
  if (sample < 1 || capacity < 1) {
    g->err = "sample and capacity must be >= 1";
    return GW_ERR_INVALID;
  }
  if (capacity > TM_CAP_MAX) {
    g->err = "FixedCacheMap capacity above 4096 (LDS-resident map) is not supported";
    return GW_ERR_UNSUPPORTED;
  }
  if (nsrc == 0) return GW_OK;
  GW_HIP_TRY(hipSetDevice(g->device));
  hipStream_t s = (hipStream_t)stream;
  const int L = 2 * step;
  // queue entries per level: <= SAMPLE enumerated (mass >= 1) + 2*SAMPLE new
  // walkers per level, walkers persist -> SAMPLE*(1 + 2L)
  int64_t cap = variant == GW_TOPSIM_SINGLE_RW ? (int64_t)sample * step : (int64_t)sample * (1 + 2 * L) + 16;
  int dev_cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, g->device) == hipSuccess) dev_cus = prop.multiProcessorCount;
  const int64_t per_block = variant == GW_TOPSIM_SINGLE_RW ? cap * 8
                                                            : (int64_t)(L + 1) * cap * 12 + 2 * cap * 8 +
                                                                  2 * (cap + 1) * 4 + cap * 8;
  const int64_t budget = (int64_t)16 << 30;
  int64_t blocks = std::min<int64_t>({(int64_t)2 * dev_cus, budget / std::max<int64_t>(per_block, 1), nsrc});
  if (blocks < 1) {
    g->err = "TopSim_M workspace exceeds the 16 GB budget";
    return GW_ERR_CAPACITY;
  }
  int hash_slots = 4;
  while (hash_slots < 2 * (capacity + 1)) hash_slots <<= 1;
  const size_t lds = (size_t)(capacity + 1) * 8 + (size_t)hash_slots * 8;
  TmArgs A{};
  A.G = g->d;
  A.variant = variant;
  A.sample = sample;
  A.sampled = (double)sample;
  for (int i = 0; i < 16; ++i) A.cache[i] = 0.0;
  for (int i = 1; i <= step; ++i) A.cache[i] = std::pow(C, (double)i);  // Math.pow (:44-45)
  A.k0 = (uint32_t)seed;
  A.k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  A.sources = sources_dev;
  A.nsrc = nsrc;
  A.capacity = capacity;
  A.hash_slots = hash_slots;
  A.out_keys = out_keys_dev;
  A.out_vals = out_vals_dev;
  A.out_size = out_size_dev;
  A.stats = (long long*)stats_dev;
  A.cap = cap;
  int rc = GW_OK;
  const bool q = variant != GW_TOPSIM_SINGLE_RW;
  const int64_t lv = q ? blocks * (L + 1) * cap : 1;
  if ((rc = tm_alloc(g, &A.qv, lv)) || (rc = tm_alloc(g, &A.qp, lv)) || (rc = tm_alloc(g, &A.qw, lv)) ||
      (rc = tm_alloc(g, &A.qm, q ? blocks * 2 * cap : 1)) || (rc = tm_alloc(g, &A.co, q ? blocks * (cap + 1) : 1)) ||
      (rc = tm_alloc(g, &A.nw, q ? blocks * (cap + 1) : 1)) || (rc = tm_alloc(g, &A.uk, blocks * cap)) ||
      (rc = tm_alloc(g, &A.uvv, blocks * cap)) || (rc = tm_alloc(g, &A.src_counter, 1)) ||
      (rc = tm_alloc(g, &A.error_flag, 1))) {
    tm_free(A.qv); tm_free(A.qp); tm_free(A.qw); tm_free(A.qm); tm_free(A.co); tm_free(A.nw);
    tm_free(A.uk); tm_free(A.uvv); tm_free(A.src_counter); tm_free(A.error_flag);
    return rc;
  }
  hipError_t e = hipMemsetAsync(A.src_counter, 0, sizeof(unsigned int), s);
  if (e == hipSuccess) e = hipMemsetAsync(A.error_flag, 0, sizeof(int), s);
  if (e == hipSuccess) {
    switch (step) {
      case 1: e = launch_m<1>(A, (int)blocks, lds, s); break;
      case 2: e = launch_m<2>(A, (int)blocks, lds, s); break;
      case 3: e = launch_m<3>(A, (int)blocks, lds, s); break;
      case 4: e = launch_m<4>(A, (int)blocks, lds, s); break;
      case 5: e = launch_m<5>(A, (int)blocks, lds, s); break;
      case 6: e = launch_m<6>(A, (int)blocks, lds, s); break;
      case 7: e = launch_m<7>(A, (int)blocks, lds, s); break;
      default: e = launch_m<8>(A, (int)blocks, lds, s); break;
    }
  }
  int flag = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&flag, A.error_flag, sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  tm_free(A.qv); tm_free(A.qp); tm_free(A.qw); tm_free(A.qm); tm_free(A.co); tm_free(A.nw);
  tm_free(A.uk); tm_free(A.uvv); tm_free(A.src_counter); tm_free(A.error_flag);
  GW_HIP_TRY(e);
  if (flag) {
    g->err = "TopSim_M: a BFS level exceeded its queue capacity";
    return GW_ERR_CAPACITY;
  }
  return GW_OK;
}

extern "C" int gw_topsim_m_host(gw_graph* g, int variant, int capacity, int sample, int step, double C,
                                uint64_t seed, const int32_t* sources, int64_t nsrc, int32_t* out_keys,
                                float* out_vals, int32_t* out_size, int64_t* stats) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);  // restores the caller's current device on return
  if (g->device < 0) return gw_fail(g, GW_ERR_STATE, "graph is not on a device");
  if (nsrc < 0 || (nsrc > 0 && (!sources || !out_keys || !out_vals || !out_size)) || capacity < 1)
    return gw_fail(g, GW_ERR_INVALID, "bad arguments");
  for (int64_t i = 0; i < nsrc; ++i)
    if (sources[i] < 0 || sources[i] >= g->n) return gw_fail(g, GW_ERR_RANGE, "source %d out of [0,V)", sources[i]);
  if (nsrc == 0) return GW_OK;
  GW_HIP_TRY(hipSetDevice(g->device));
  int32_t *d_src = nullptr, *d_k = nullptr, *d_sz = nullptr;
  float* d_v = nullptr;
  int64_t* d_st = nullptr;
  int rc;
  if ((rc = tm_alloc(g, &d_src, nsrc)) || (rc = tm_alloc(g, &d_k, nsrc * (int64_t)capacity)) ||
      (rc = tm_alloc(g, &d_v, nsrc * (int64_t)capacity)) || (rc = tm_alloc(g, &d_sz, nsrc)) ||
      (rc = tm_alloc(g, &d_st, 4))) {
    tm_free(d_src); tm_free(d_k); tm_free(d_v); tm_free(d_sz); tm_free(d_st);
    return rc;
  }
  hipError_t e = hipMemcpy(d_src, sources, nsrc * sizeof(int32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(d_st, 0, 4 * sizeof(int64_t));
  if (e == hipSuccess) {
    rc = gw_dev_topsim_m(g, variant, capacity, sample, step, C, seed, d_src, nsrc, d_k, d_v, d_sz, d_st, nullptr);
    if (rc == GW_OK) {
      e = hipMemcpy(out_keys, d_k, nsrc * (size_t)capacity * sizeof(int32_t), hipMemcpyDeviceToHost);
      if (e == hipSuccess) e = hipMemcpy(out_vals, d_v, nsrc * (size_t)capacity * sizeof(float), hipMemcpyDeviceToHost);
      if (e == hipSuccess) e = hipMemcpy(out_size, d_sz, nsrc * sizeof(int32_t), hipMemcpyDeviceToHost);
      if (e == hipSuccess && stats) e = hipMemcpy(stats, d_st, 4 * sizeof(int64_t), hipMemcpyDeviceToHost);
    }
  }
  tm_free(d_src); tm_free(d_k); tm_free(d_v); tm_free(d_sz); tm_free(d_st);
  if (rc != GW_OK) return rc;
  if (e != hipSuccess) return gw_fail(g, GW_ERR_DEVICE, "%s", hipGetErrorString(e));
  return GW_OK;
}
