// TopSim random-walk SimRank on gfx950 (H2).
//
// Reference: DeepSim/TopSimAll/src/simrank/TopSim_singleSample.java
//   ctor/compute   :35-54   cache[i] = C^i, one walk() per source, sim[i][i]=0
//   walk           :62-158  level-synchronous expansion of weighted paths:
//                           mass >= degree  -> enumerate all neighbours, mass/d
//                           else            -> ceil(mass) random children,
//                                              mass/ceil(mass) each
//   computePathSim :167-203 at pathLen = 2i, every path with target != source
//                           and isFirstMeet (:211-218) adds
//                           ((mass * C^i) * deg(mid)) / deg(target)
// plus TopSim_Enumerate.java:61-136 (always enumerate) and
// SingleRandomWalk.java:53-92 (SAMPLE independent walks, score / SAMPLE),
// and Print.printByOrder's per-row top-k (Print.java:25-53).
//
// Decomposition (one persistent workgroup per query source at a time):
//   * the deterministic part of the path tree (nodes created by enumeration)
//     is expanded level by level with workgroup scans; level arrays hold
//     (vertex, parent) so any path is rebuilt by walking parents;
//   * a node with mass < degree spawns ceil(mass) random children; each such
//     child and all its descendants have mass <= 1 and exactly ONE child per
//     level (mass stays m/ceil(m)), i.e. it is an independent random walk.
//     Those walkers run one per lane with the path in registers, Philox keyed
//     by (source, walker index, level), the walker index being the position
//     in the reference's BFS queue order (level-major, queue order, child j);
//   * pair updates accumulate in a dense fp64 row of the workgroup (LDS when
//     n*8 fits, HBM otherwise with a touched list), then a radix select picks
//     the top-k (score desc, id asc) and the row is re-zeroed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "gw_device_common.h"

namespace {

constexpr int TS_BLOCK = 512;
constexpr int TS_WAVES = TS_BLOCK / 64;
constexpr int TOPK_MAX = 256;
constexpr int TS_CO_LDS = 1792;  // child / spawner offsets kept in LDS up to this many entries
constexpr int64_t LDS_ROW_MAX_BYTES = 96 * 1024;
constexpr int kPipeMaxSample = 2048;  // k_topsim_pipe for SAMPLE up to this (above: pipe_pays_large_sample)
constexpr int kTsProbeCap = 16;       // LDS-hash slots a key may probe before it overflows to HBM

struct TsArgs {
  gw_dev_graph G;
  int variant;
  int diag;  // GW_DIAG_TS (timing experiments only, wrong results): 1 = walkers skip computePathSim, 2 = cheap RNG,
             // 4 / 8 = walker reads confined to the first 2^26 / 2^27 slot entries;
             // A/B knobs (same results): 32 = no deferred ordering, 8192 = counter-free LDS-hash insert (4-wide
             // probes, kTsProbeCap), 1024 = a walker's pair update before its next entry load (round 4),
             // 2048 = a walker's last pair update not carried into the lane's next walker,
             // 4096 = top-k selection from the compacted LDS table (no register-held values),
             // 16384 = overflow compaction always through `touched`, 32768 = no append-and-reduce path
  int sample;
  double sampled;
  double cache[16];
  uint32_t k0, k1;
  const int32_t* sources;
  int64_t nsrc;
  int topk;
  int32_t* out_ids;
  double* out_scores;
  double* out_rows;
  gw_ts_sparse sp;  // sparse rows (sp.cursor != nullptr): nonzero (id, score) entries per source
  long long* stats;
  int64_t level_cap, spawn_cap, touch_cap;
  int32_t* lvl_vertex;
  int32_t* lvl_parent;
  int32_t* lvl_deg;
  int64_t* lvl_off;
  const gw_ts_ent* ent;
  double* lvl_mass;
  int32_t* child_off;
  int32_t* spawn_node;
  int32_t* spawn_level;
  int32_t* spawn_first;
  double* spawn_mass;
  double* ov_vals;
  double* ov_list;  // [blocks][touch_cap] the compacted overflow values of a source (keys in `touched`)
  int32_t* enum_tgt;  // pipelined kernel: enumerated-node pair updates of a source, [blocks][2][enum_cap]
  double* enum_val;
  int64_t enum_cap;
  int32_t* dsel_id;  // pipelined kernel, top-k rows: a source's selected entries awaiting order, [blocks][TOPK_MAX]
  double* dsel_val;
  int32_t* touched;
  double* app;         // pipelined hash mode: [blocks][2 app_cap] 16 B entries: a heavy source's key-hash partitions
  int64_t app_cap;     // 0: no append-and-reduce path
  int64_t heavy_min;   // a source appends past the LDS table when its pair-update bound exceeds this
  int32_t* claim;      // [blocks][touch_cap] a heavy source's claimed overflow-hash slots
  int part_entries;    // a heavy source gets the power of two of partitions that keeps its bound <= this each
  int pcap_shrink;     // gw_options_t.topsim_part_shrink: partitions get 2^-k of their room (tests flag 8's re-run)
  unsigned int* src_counter;
  int* error_flag;
  unsigned long long* phase;  // diagnostics (GW_DIAG_TS_PHASES): cycles per phase, thread 0 of each block
};

template <int NW = TS_WAVES, typename T = int>
__device__ __forceinline__ T block_excl_scan(T v, T* s_wave, T* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wave[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T acc = 0;
    for (int w = 0; w < NW; ++w) {
      T t = s_wave[w];
      s_wave[w] = acc;
      acc += t;
    }
    s_wave[NW] = acc;
  }
  __syncthreads();
  T r = s_wave[wid] + x - v;
  *total = s_wave[NW];
  __syncthreads();
  return r;
}

template <typename T, int NW = TS_WAVES>
__device__ __forceinline__ T block_sum(T v, T* s_red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  T r = 0;
  for (int w = 0; w < NW; ++w) r += s_red[w];
  __syncthreads();
  return r;
}

// first index i in [0, n) with a[i] > x  (a non-decreasing)
__device__ __forceinline__ int upper_bound_i32(const int32_t* a, int n, int x) {
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

// one wave: the radix bin holding the need-th key, scanning the 256 bins
// from the top (desc) or from the bottom (asc); 4 bins per lane and one wave
// scan instead of a serial 256-step loop.  Every lane gets (bin, keys in the
// bins scanned before it, keys in all bins).
__device__ __forceinline__ void select_bin_w(const unsigned* hist, int need, bool desc, int& bin, int& before,
                                             int& total) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));  // its bin addresses formed per call, not held across the kernel
  int c[4], loc = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int o = 4 * lane + q;
    c[q] = (int)hist[desc ? 255 - o : o];
    loc += c[q];
  }
  int inc = loc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  int run = inc - loc, first = -1, cum_at = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (first < 0 && run + c[q] >= need) {
      first = 4 * lane + q;
      cum_at = run;
    }
    run += c[q];
  }
  const unsigned long long m = __ballot(first >= 0);
  const int src = m ? __ffsll(m) - 1 : 63;
  const int o = __shfl(first >= 0 ? first : 255, src, 64);
  before = __shfl(first >= 0 ? cum_at : run - c[3], src, 64);
  total = __shfl(inc, 63, 64);
  bin = desc ? 255 - o : o;
}

// the same, lane 0 storing the results (wave 0 for the whole workgroup)
__device__ __forceinline__ void select_bin(const unsigned* hist, int need, bool desc, int* bin, int* before,
                                           int* total = nullptr) {
  int b, cb, tot;
  select_bin_w(hist, need, desc, b, cb, tot);
  if ((threadIdx.x & 63) == 0) {
    *bin = b;
    *before = cb;
    if (total) *total = tot;
  }
}

__device__ __forceinline__ unsigned long long dkey(double v) {
  return (unsigned long long)__double_as_longlong(v);  // v >= 0: bit order == value order
}

// One wave, no workgroup barrier: the cnt (<= TOPK_MAX) selected (id, value)
// entries sid / sval ranked (value desc, id asc — the FixedMaxPQ /
// Print.printByOrder order, FixedMaxPQ.java:30-39), ranks < K written to
// oid / osc, -1 / 0 padded.  The pipelined kernel's deferred ordering: the
// workgroup selects source s's top entries, and one wave ranks them while
// the others walk source s + 1.
__device__ __forceinline__ void ts_wave_rank(const int32_t* sid, const double* sval, int cnt, int K, int32_t* oid,
                                             double* osc) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));  // per-lane addresses formed here, not hoisted out of the source loop
  constexpr int Q = TOPK_MAX / 64;
  int32_t mi[Q];
  double mv[Q];
  int rk[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int idx = q * 64 + lane;
    mi[q] = idx < cnt ? sid[idx] : 0x7fffffff;
    mv[q] = idx < cnt ? sval[idx] : -1.0;
    rk[q] = 0;
  }
  // rank = entries before it in (value desc, id asc); sources broadcast by readlane
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    if (q * 64 < cnt) {
      const int m = min(64, cnt - q * 64);
      const long long mvb = __double_as_longlong(mv[q]);
      for (int src = 0; src < m; ++src) {
        const int lo = __builtin_amdgcn_readlane((int)mvb, src);
        const int hi = __builtin_amdgcn_readlane((int)(mvb >> 32), src);
        const double vj = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
        const int32_t ij = __builtin_amdgcn_readlane(mi[q], src);
#pragma unroll
        for (int qq = 0; qq < Q; ++qq)
          if (qq * 64 < cnt) rk[qq] += (vj > mv[qq]) || (vj == mv[qq] && ij < mi[qq]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (q * 64 + lane < cnt && rk[q] < K) {
      oid[rk[q]] = mi[q];
      osc[rk[q]] = mv[q];
    }
  for (int k = min(cnt, K) + lane; k < K; k += 64) {
    oid[k] = -1;
    osc[k] = 0.0;
  }
}

// MODE 0: dense LDS row; 1: LDS hash of 8192 slots (96 KB, one workgroup per
// CU); 2: LDS hash of 6144 slots (72 KB, two workgroups per CU)
template <int MODE>
struct TsHash {
  static constexpr int SLOTS = MODE == 2 ? 6144 : 8192;
  static constexpr int LIMIT = SLOTS * 3 / 4;  // load limit before overflowing to HBM
  __device__ static __forceinline__ uint32_t slot(int32_t key) {
    return (uint32_t)(((uint64_t)((uint32_t)key * 0x9E3779B1u) * (uint64_t)SLOTS) >> 32);
  }
  __device__ static __forceinline__ uint32_t next(uint32_t h) { return h + 1 == (uint32_t)SLOTS ? 0u : h + 1; }
};

// per-buffer state of the pipelined kernel (PIPE): the source whose levels
// wave 0 built into that buffer
struct TsPipeMeta {
  long long r;  // index into A.sources
  int s, ds;
  int nspawn, nwalk, ncontrib;
  uint32_t ovmask;  // slots - 1 of the source's overflow hash (hash mode)
  int heavy;        // append-and-reduce past the LDS table (hash mode)
  int plg;          // log2 of its key-hash partitions
  int valid;
};

struct TsLevelStats {
  long long ext, upd, maxf;
};

// ---- PIPE: wave 0 builds the levels of sources[r] into buffer b ---------
// Same queue order, records and pair updates as the workgroup version in
// the source loop below; control flow is wave-uniform, lanes exchange
// through shuffles (child -> parent by a binary search over the chunk's
// inclusive child counts held one per lane).  The chain of dependent
// memory round trips is kept short, since the walkers of the previous
// source saturate the memory system meanwhile: the
// level-2 pair updates (i = 1: target = child, mid = its parent, both at
// hand) are computed while the level is filled; deeper even levels rebuild
// their paths from the level arrays after a fence.
template <int STEP>
__device__ __forceinline__ TsLevelStats ts_wave_levels(const TsArgs& A, int b, int64_t r, TsPipeMeta* s_pm) {
  constexpr int L = 2 * STEP;
  TsLevelStats st{0, 0, 0};
  long long& my_ext = st.ext;
  long long& my_upd = st.upd;
  long long& my_maxf = st.maxf;
  const int tid = threadIdx.x;
  const int64_t blk = blockIdx.x;
  const gw_dev_graph& G = A.G;
  const int64_t cap = A.level_cap;
  const int64_t lvl_stride = (int64_t)(L + 1) * cap;
  int32_t* V = A.lvl_vertex + blk * 2 * lvl_stride;
  int32_t* P = A.lvl_parent + blk * 2 * lvl_stride;
  int32_t* D = A.lvl_deg + blk * 2 * lvl_stride;
  int64_t* O = A.lvl_off + blk * 2 * lvl_stride;
  double* M = A.lvl_mass + blk * 2 * cap;
  int32_t* SN = A.spawn_node + blk * 2 * A.spawn_cap;
  int32_t* SL = A.spawn_level + blk * 2 * A.spawn_cap;
  int32_t* SF = A.spawn_first + blk * 2 * (A.spawn_cap + 1);
  double* SM = A.spawn_mass + blk * 2 * A.spawn_cap;
  {
    // opaque per source: the per-lane array addresses below are then formed
    // here, not hoisted out of the kernel's source loop as 64-bit VGPR pairs
    // held across the walkers (one of them spilled at the 128-VGPR cap)
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    int32_t* Vb = V + b * lvl_stride;
    int32_t* Pb = P + b * lvl_stride;
    int32_t* Db = D + b * lvl_stride;
    int64_t* Ob = O + b * lvl_stride;
    int32_t* SNb = SN + b * A.spawn_cap;
    int32_t* SLb = SL + b * A.spawn_cap;
    int32_t* SFb = SF + b * (A.spawn_cap + 1);
    double* SMb = SM + b * A.spawn_cap;
    int32_t* ETb = A.enum_tgt + (blk * 2 + b) * A.enum_cap;
    double* EVb = A.enum_val + (blk * 2 + b) * A.enum_cap;
    const int32_t s = A.sources[r];
    const int ds = G.deg[s];
    const int64_t os = G.offsets[s];
    if (lane == 0) {
      Vb[0] = s;
      Db[0] = ds;
      Ob[0] = os;
      Pb[0] = -1;
      // path[0].sample = SAMPLE (:73); converted here, not hoisted out of the
      // source loop (a loop-invariant double held across the kernel spills)
      int smp = A.sample;
      asm volatile("" : "+v"(smp));
      M[0] = (double)smp;
    }
    __threadfence_block();
    int sz = 1, nsp = 0, nwk = 0, nct = 0;
    bool abort = false;
    // record a pair update (target, val) of lanes with tgt >= 0, queue order irrelevant (a sum)
    auto emit = [&](int32_t tgt, double val) {
      const unsigned long long em = __ballot(tgt >= 0);
      const int k = nct + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
      if (tgt >= 0 && k < A.enum_cap) {
        ETb[k] = tgt;
        EVb[k] = val;
      }
      nct += __popcll(em);
    };
    for (int l = 0; l <= L && sz > 0; ++l) {
      if (lane == 0 && sz > my_maxf) my_maxf = sz;
      const double* Ml = M + (int64_t)(l & 1) * cap;
      if ((l & 1) == 0 && l >= 4) {  // computePathSim at pathLen = 2i (:80-83, :157), i >= 2: recorded
        for (int j0 = 0; j0 < sz; j0 += 64) {
          const int j = j0 + lane;
          int32_t tgt = -1;
          double val = 0.0;
          if (j < sz) {
            int32_t path[L + 1], dpath[L + 1];
            int p = j;
#pragma unroll
            for (int t = L; t >= 1; --t) {
              if (t <= l) {
                path[t] = Vb[(int64_t)t * cap + p];
                dpath[t] = Db[(int64_t)t * cap + p];
                p = Pb[(int64_t)t * cap + p];
              }
            }
            path[0] = s;
            dpath[0] = ds;
#pragma unroll
            for (int t = 4; t <= L; t += 2) {
              if (t == l) {
                const int i = t / 2;
                bool meet = path[t] != s;  // :183
#pragma unroll
                for (int q = 0; q < STEP; ++q)  // isFirstMeet (:211-218)
                  if (q < i && path[q] == path[t - q]) meet = false;
                if (meet) {
                  tgt = path[t];
                  val = ((Ml[j] * A.cache[i]) * (double)dpath[i]) / (double)dpath[t];  // :189
                  ++my_upd;
                }
              }
            }
          }
          emit(tgt, val);
        }
        if (nct > A.enum_cap) abort = true;
      }
      if (l == L || abort) break;
      int32_t* Vn = Vb + (int64_t)(l + 1) * cap;
      int32_t* Pn = Pb + (int64_t)(l + 1) * cap;
      int32_t* Dn = Db + (int64_t)(l + 1) * cap;
      int64_t* On = Ob + (int64_t)(l + 1) * cap;
      double* Mn = M + (int64_t)((l + 1) & 1) * cap;
      const int32_t* Dl = Db + (int64_t)l * cap;
      const int64_t* Ol = Ob + (int64_t)l * cap;
      const bool level2 = l + 1 == 2;  // the children are level 2: record their pair updates now
      int tot = 0;
      for (int j0 = 0; j0 < sz; j0 += 64) {
        const int j = j0 + lane;
        int cnt = 0, c = 0, d = 0;
        double m = 0.0;
        int64_t o = 0;
        if (j < sz) {
          d = Dl[j];
          m = Ml[j];
          o = Ol[j];
        }
        if (d != 0 && m >= (double)d) {  // enumerate (:99)
          cnt = d;
        } else if (d != 0) {  // d == 0: randNeighbor() == -1 -> no child (:143-144)
          c = (int)m;         // number = (int)s == s ? (int)s : (int)s + 1 (:131-135)
          if ((double)c != m) c += 1;
        }
        int ic = cnt, iw = c;  // inclusive wave scans: children, walkers
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
          const int a = __shfl_up(ic, dd, 64), w = __shfl_up(iw, dd, 64);
          if (lane >= dd) {
            ic += a;
            iw += w;
          }
        }
        const int ctot = __shfl(ic, 63, 64), wtot = __shfl(iw, 63, 64);
        const unsigned long long spm = __ballot(c > 0);
        const int ksp = nsp + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(spm >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)spm, 0u));
        if (c > 0 && ksp < A.spawn_cap) {
          SLb[ksp] = l;
          SNb[ksp] = j;
          SFb[ksp] = nwk + iw - c;        // first walker of this spawner (queue order)
          SMb[ksp] = m / (double)c;      // (double)cur.sample/(double)number (:142)
        }
        nsp += __popcll(spm);
        nwk += wtot;
        if (nsp > A.spawn_cap || (int64_t)tot + ctot > cap) {
          abort = true;
          break;
        }
        // the chunk's children, BFS queue order (edges.get(k), insertion order :103-110)
        for (int c0 = 0; c0 < ctot; c0 += 64) {
          const int cc = c0 + lane;
          int pl = 0;  // parent lane: the first lane whose inclusive count exceeds cc
#pragma unroll
          for (int st = 32; st >= 1; st >>= 1)
            if (__shfl(ic, pl + st - 1, 64) <= cc) pl += st;
          const int pd = __shfl(cnt, pl, 64);
          const int pex = __shfl(ic, pl, 64) - pd;
          const int64_t po = ((int64_t)__shfl((int)(o >> 32), pl, 64) << 32) | (uint32_t)__shfl((int)o, pl, 64);
          const double pm = __shfl(m, pl, 64);
          int32_t tgt = -1;
          double val = 0.0;
          if (cc < ctot) {
            const gw_ts_ent e = gw_ts_load(A.ent + po + (cc - pex));
            const int ci = tot + cc;
            const double cm = pm / (double)pd;  // newSample = cur.sample / degree (:104)
            Vn[ci] = e.x;
            Dn[ci] = e.d;
            On[ci] = e.off;
            Pn[ci] = j0 + pl;
            Mn[ci] = cm;
            if (level2 && e.x != s) {  // i = 1: ((mass * C) * deg(mid)) / deg(target) (:183-189)
              tgt = e.x;
              val = ((cm * A.cache[1]) * (double)pd) / (double)e.d;
              ++my_upd;
            }
          }
          if (level2) emit(tgt, val);
        }
        tot += ctot;
      }
      if (level2 && nct > A.enum_cap) abort = true;
      if (abort) break;
      if (lane == 0) my_ext += tot;
      sz = tot;
      __threadfence_block();  // the next level is read back from the level arrays
    }
    if (abort && lane == 0) atomicOr(A.error_flag, 1);
    if (lane == 0) {
      SFb[abort ? 0 : nsp] = abort ? 0 : nwk;
      s_pm[b].r = r;
      s_pm[b].s = s;
      s_pm[b].ds = ds;
      s_pm[b].nspawn = abort ? 0 : nsp;
      s_pm[b].nwalk = abort ? 0 : nwk;
      s_pm[b].ncontrib = abort ? 0 : min(nct, (int)A.enum_cap);
      // the source's overflow hash (hash mode): pair updates it can make are
      // STEP per walker + the enumerated ones, so no more distinct overflow
      // keys; the power of two above 9/8 of that bound (<= touch_cap)
      // Distinct keys are also <= n, but appended pair updates repeat keys:
      // the append-and-reduce choice uses the uncapped pair-update bound
      // (a small graph at a large SAMPLE can make more updates than app_cap
      // holds while n <= app_cap; such a source keeps the HBM hash)
      const int64_t pairs = abort ? 0 : (int64_t)nwk * STEP + min(nct, (int)A.enum_cap);
      const int64_t ub = min((int64_t)G.n, pairs);
      int64_t t = 64;
      while (t < ub + ub / 8 + 1 && t < A.touch_cap) t <<= 1;
      s_pm[b].ovmask = (uint32_t)(t - 1);
      s_pm[b].heavy = A.app_cap > 0 && pairs > A.heavy_min && pairs <= A.app_cap && !(kGwDiag && (A.diag & (32768 | 8192)));
      int lg = 0;
      while (((int64_t)A.part_entries << lg) < pairs && lg < 6) ++lg;
      s_pm[b].plg = lg;
      s_pm[b].valid = 1;
    }
  }
  return st;
}


// PIPE (TopSim_singleSample, hash accumulator): the deterministic levels of
// source s+1 are built by wave 0 alone (wave scans and lane shuffles, no
// workgroup barrier) into the second half of double-buffered level /
// spawner scratch while the other waves run the walkers of source s; wave 0
// then joins them.  Walkers and the enumerated nodes' pair updates (wave 0
// records them as (target, value) lists instead of adding them while the
// accumulator belongs to source s) are dealt out 64 at a time from an LDS
// counter, so the workgroup's barrier-bound level phase (28% of its cycles
// at P10M) overlaps its walkers instead of stalling every wave.
template <int STEP, int MODE, int BLOCK = TS_BLOCK, bool PIPE = false>
__device__ __forceinline__ void topsim_body(const TsArgs& A) {
  constexpr int NW = BLOCK / 64;
  constexpr int NB = PIPE ? 2 : 1;  // level / spawner scratch buffers per workgroup
  // pipelined kernel: a source's top-k ordered by one wave during the next
  // source's walkers (deferred ordering)
  constexpr bool DEFER = PIPE;
  constexpr int CO_LDS = TS_CO_LDS;
  constexpr bool LDS_ROW = MODE == 0;
  using H = TsHash<MODE>;
  constexpr int HASH_SLOTS = H::SLOTS;
  constexpr int HASH_LIMIT = H::LIMIT;
  constexpr int L = 2 * STEP;
  extern __shared__ double s_row[];  // LDS row (LDS_ROW) or hash values+keys
  __shared__ int s_wave[NW + 1];
  __shared__ long long s_red[NW];
  __shared__ int s_size[L + 2];
  __shared__ int s_src, s_nspawn, s_nwalk, s_ntouch, s_cnt, s_need, s_abort, s_hcount, s_bin, s_cum, s_exact, s_total,
      s_ncomp, s_all, s_novc;
  __shared__ uint32_t s_ovmask;  // the slots (minus 1) of this source's overflow hash
  __shared__ int s_heavy, s_plg;  // append-and-reduce source; log2 of its key-hash partitions
  __shared__ int s_pinfo;          // s_plg | log2(entries per partition) << 8
  __shared__ int s_hdone;          // LDS-table reservations whose CAS has completed (the key set is final at HASH_LIMIT)
  __shared__ int s_pcur[64];       // its partitions' fill counts
  __shared__ unsigned long long s_prefix, s_mask, s_spbase;
  // the output phase's selection arrays share LDS with the levels' child
  // offsets / the walkers' spawner offsets (binary-searched per child / walker)
  __shared__ union {
    struct {
      double sel_val[TOPK_MAX];
      int32_t sel_id[TOPK_MAX];
      unsigned hist[256];
      unsigned hist2[256];  // radix passes alternate histograms: one is cleared while the other fills
    } out;
    int32_t co[CO_LDS];
  } s_u;
  int32_t* const s_sel_id = s_u.out.sel_id;
  double* const s_sel_val = s_u.out.sel_val;
  unsigned* const s_hist = s_u.out.hist;
  unsigned* const s_hist2 = s_u.out.hist2;
  int32_t* const s_co = s_u.co;

  const int tid = threadIdx.x;
  const int64_t blk = blockIdx.x;
  const gw_dev_graph& G = A.G;
  const int n = (int)G.n;
  const int64_t cap = A.level_cap;
  // level / spawner scratch of buffer b (PIPE: two, the source being walked
  // and the next one; otherwise one)
  const int64_t lvl_stride = (int64_t)(L + 1) * cap;
  int32_t* V = A.lvl_vertex + blk * NB * lvl_stride;
  int32_t* P = A.lvl_parent + blk * NB * lvl_stride;
  int32_t* D = A.lvl_deg + blk * NB * lvl_stride;
  int64_t* O = A.lvl_off + blk * NB * lvl_stride;
  double* M = A.lvl_mass + blk * 2 * cap;
  int32_t* CO = A.child_off + blk * (cap + 1);
  int32_t* SN = A.spawn_node + blk * NB * A.spawn_cap;
  int32_t* SL = A.spawn_level + blk * NB * A.spawn_cap;
  int32_t* SF = A.spawn_first + blk * NB * (A.spawn_cap + 1);
  double* SM = A.spawn_mass + blk * NB * A.spawn_cap;
  __shared__ TsPipeMeta s_pm[2];
  __shared__ unsigned s_wnext;
  // accumulator: dense LDS row (small n) or LDS open-addressing hash with a
  // per-workgroup HBM overflow hash (large n)
  double* s_hval = s_row;                                   // [HASH_SLOTS]
  int32_t* s_hkey = reinterpret_cast<int32_t*>(s_row + HASH_SLOTS);  // [HASH_SLOTS]
  // overflow hash slots are 16 B {int32 key, pad, f64 value}: the CAS on the
  // key and the add to the value touch ONE cache line (round 5; two separate
  // arrays before); key of slot h at ov_key[4h], value at ov_val[2h + 1]
  int32_t* ov_key = LDS_ROW ? nullptr : reinterpret_cast<int32_t*>(A.ov_vals + 2 * blk * A.touch_cap);
  double* ov_val = LDS_ROW ? nullptr : (A.ov_vals + 2 * blk * A.touch_cap);
  double* ov_list = LDS_ROW ? nullptr : (A.ov_list + blk * A.touch_cap);
  int32_t* touched = LDS_ROW ? nullptr : (A.touched + blk * A.touch_cap);
  // append-and-reduce (PIPE, hash mode): pair updates appended past the LDS
  // table, then partitioned by key hash into the second buffer
  // (the block's base offset passes through an empty asm at each use, so it
  // is recomputed there instead of held in registers through the walkers)
  // Instantiated for STEP >= 4 only: at STEP 3 (P10M) the pipelined kernel
  // measured 0.7-1.2% slower with this code present and no source using it
  // (register allocation), and a STEP-3 source over the LDS table keeps the
  // HBM hash (profiles/r05/tsab_r05s*, tsab_r05t*).
  constexpr bool APPEND = PIPE && STEP >= 4;
  auto app_base = [&]() -> double* {  // [2 app_cap] 16 B entries: partition p at entries [p cap_p, (p+1) cap_p)
    int64_t o = 4 * blk * A.app_cap;
    asm volatile("" : "+s"(o));
    return A.app + o;
  };
  auto claim_base = [&]() -> int32_t* {
    int64_t o = blk * A.touch_cap;
    asm volatile("" : "+s"(o));
    return A.claim + o;
  };
  // key-hash partition of a heavy source's key (lg = log2 of its partitions)
  auto part_of = [](int32_t key, int lg) -> int {
    return lg ? (int)(((uint32_t)key * 0x85EBCA77u) >> (32 - lg)) : 0;
  };
  // the slots a source's overflow hash uses: all touch_cap of them, or (PIPE)
  // the power of two above the source's own bound on distinct overflow keys,
  // so that a heavy source's compaction can scan its slots in order
  // (read from LDS where used: no register held through the walker phase)
  const bool rw = !PIPE && (A.variant == GW_TOPSIM_SINGLE_RW);  // PIPE: TopSim_singleSample only
  const bool enumerate_all = !PIPE && (A.variant == GW_TOPSIM_ENUMERATE);

  long long my_ext = 0, my_upd = 0, my_walk = 0, my_maxf = 0;
  unsigned long long w1_t = 0, w1_walk = 0, w1_wait = 0;  // diagnostics: wave 1's walker phase
  // deferred ordering of the top-k rows (the dense / sparse row writers keep the in-place phase)
  const bool defer = DEFER && A.out_ids && !(kGwDiag && (A.diag & 32));
  int64_t pend_r = -1;  // the source whose selected entries await ranking
  int pend_n = 0;
  auto deferred_topk = [&]() {
    const int K = A.topk;
    ts_wave_rank(A.dsel_id + blk * TOPK_MAX, A.dsel_val + blk * TOPK_MAX, pend_n, K,
                 A.out_ids + pend_r * (int64_t)K, A.out_scores + pend_r * (int64_t)K);
  };

  if (LDS_ROW) {
    for (int j = tid; j < n; j += BLOCK) s_row[j] = 0.0;
  } else {
    for (int j = tid; j < HASH_SLOTS; j += BLOCK) {
      s_hval[j] = 0.0;
      s_hkey[j] = -1;
    }
  }
  if (tid == 0) {
    s_ntouch = 0;
    s_hcount = 0;
    s_ovmask = (uint32_t)(A.touch_cap - 1);
    s_heavy = 0;
    s_plg = 0;
    s_pinfo = 0;
    s_hdone = 0;
  }
  if (tid < 64) s_pcur[tid] = 0;
  __syncthreads();

  // overflow insert into the workgroup's HBM hash (slots claimed by CAS; the
  // claimed slot is recorded for selection and cleanup)
  auto ov_add = [&](int32_t target, double val) {
    // the product's high bits (Fibonacci hashing): clz(mask) = 32 - log2(slots)
    const uint32_t ov_mask = s_ovmask;  // a power of two >= 2^6, minus 1
    uint32_t h = ((uint32_t)target * 0x9E3779B1u) >> __builtin_clz(ov_mask);
    for (int64_t probe = 0; probe <= (int64_t)ov_mask; ++probe) {
      const int32_t old = atomicCAS(&ov_key[4 * h], -1, target);
      if (old == -1 || old == target) {
        if (old == -1) {
          const int k = atomicAdd(&s_ntouch, 1);
          if ((int64_t)k >= A.touch_cap * 3 / 4) atomicOr(A.error_flag, 2);
          else if (APPEND && s_heavy) claim_base()[k] = (int32_t)h;  // (heavy: merged and compacted from the claims)
          else touched[k] = (int32_t)h;
        }
        atomicAdd(&ov_val[2 * h + 1], val);
        return;
      }
      h = (h + 1) & ov_mask;
    }
    atomicOr(A.error_flag, 2);
  };

  // counter-free LDS-hash insert: a CAS on the key's first empty slot, keys
  // read four at a time, at most kTsProbeCap slots (false: no room)
  auto cf_insert = [&](int32_t target, double val) -> bool {
    uint32_t h = H::slot(target);
    int probed = 0;
    while (probed < kTsProbeCap) {
      const uint32_t g0 = h & ~3u;
      const int4 kv = *reinterpret_cast<const int4*>(&s_hkey[g0]);
      const int32_t ks[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if ((uint32_t)j < (h & 3u) || probed >= kTsProbeCap) continue;
        ++probed;
        const uint32_t sl = g0 + (uint32_t)j;
        int32_t k = ks[j];
        if (k == -1) {  // claim it; a lost race leaves the winner's key
          const int32_t old = atomicCAS(&s_hkey[sl], -1, target);
          k = old == -1 ? target : old;
        }
        if (k == target) {
          atomicAdd(&s_hval[sl], val);
          return true;
        }
      }
      h = g0 + 4u == (uint32_t)HASH_SLOTS ? 0u : g0 + 4u;
    }
    return false;
  };

  // accumulate one pair update
  auto add = [&](int32_t target, double val) {
    if (LDS_ROW) {
      atomicAdd(&s_row[target], val);
      return;
    }
    uint32_t h = H::slot(target);
    // Linear probing from the key's slot; a new key first reserves an entry on
    // the workgroup's load counter, so the table stays below HASH_LIMIT (75%)
    // and every chain ends at an empty slot within a few probes; past the
    // limit new keys go to the HBM overflow hash.  Measured against it in one
    // library (round 5, profiles/r05/tsab_r05e_knobs.jsonl, diag bit 8192): a
    // counter-free insert (a CAS on the empty slot, keys read four at a time,
    // at most kTsProbeCap slots) is +1.2% on P10M and +6.8% on arxiv at SAMPLE
    // 10000, whose tables fill; with an approximate limit (a plain counter
    // read and a non-returning add) +3.7% / +7.4%.  (Round 4 measured the
    // counter-free insert at -2.4% before the fold and output changes.)
    if (kGwDiag && (A.diag & 8192)) {
      if (!cf_insert(target, val)) ov_add(target, val);
      return;
    }
    if (PIPE) {
      // the same probe, four keys per ds_read_b128: once the table is full
      // (every heavy source's walk) an unsuccessful search runs to the end of
      // its cluster — ~8.5 slots on average at 75% load and several times
      // that for the slowest lane of a wave, which the whole wave waits for.
      // Stretch -3.9%, P10M -1.1%; the unpipelined kernel (arxiv, SAMPLE >=
      // 2500) +4%: not there (profiles/r06/tsab_r06n.jsonl, tsab_r06o.jsonl)
      for (int probed = 0; probed < HASH_SLOTS;) {
        const uint32_t g0 = h & ~3u;
        const int4 kv = *reinterpret_cast<const int4*>(&s_hkey[g0]);
        const int32_t ks[4] = {kv.x, kv.y, kv.z, kv.w};
        int at = 4;  // the first slot at or after h holding the key or empty
        bool hit = false;
#pragma unroll
        for (int j = 3; j >= 0; --j)
          if ((uint32_t)j >= (h & 3u) && (ks[j] == target || ks[j] == -1)) {
            at = j;
            hit = ks[j] == target;
          }
        if (at < 4) {
          h = g0 + (uint32_t)at;
          if (hit) {
            atomicAdd(&s_hval[h], val);
            return;
          }
          // (APPEND: a full table is seen without the atomic — every
          // overflowing key would otherwise take a returning atomic on this
          // one LDS address)
          if ((APPEND && s_hcount >= HASH_LIMIT) || atomicAdd(&s_hcount, 1) >= HASH_LIMIT) break;
          const int32_t old = atomicCAS(&s_hkey[h], -1, target);
          const bool mine = old == -1 || old == target;
          if (APPEND) atomicAdd(&s_hdone, 1);  // (after the CAS has returned: device ISA checked)
          if (mine) {
            atomicAdd(&s_hval[h], val);
            return;
          }
          h = H::next(h);  // another key took the slot: go on after it
          ++probed;
          continue;
        }
        probed += 4 - (int)(h & 3u);
        h = g0 + 4u == (uint32_t)HASH_SLOTS ? 0u : g0 + 4u;
      }
    } else {
      for (int probe = 0; probe < HASH_SLOTS; ++probe) {
        const int32_t k = s_hkey[h];
        if (k == target) {
          atomicAdd(&s_hval[h], val);
          return;
        }
        if (k == -1) {
          // reserve an LDS entry first; past the load limit new keys overflow
          if (atomicAdd(&s_hcount, 1) >= HASH_LIMIT) break;
          const int32_t old = atomicCAS(&s_hkey[h], -1, target);
          if (old == -1 || old == target) {
            atomicAdd(&s_hval[h], val);
            return;
          }
        }
        h = H::next(h);
      }
    }
    // (order: a lane's count follows its CAS — the compiler waits for the CAS
    // before issuing the add — and the slot re-read below is control-dependent
    // on this check; both checked in the gfx950 assembly.  Explicit fences or
    // compiler barriers here cost 16 B more scratch per lane.)
    if (APPEND && s_heavy && s_hdone >= HASH_LIMIT) {
      // append-and-reduce source whose LDS table is final (every reserved
      // insert has landed).  Slots never empty and keys never change, so the
      // key, if an insert racing this probe placed it, sits at or after the
      // empty slot the probe stopped at (an insert takes its chain's first
      // empty slot): finish the check there — one LDS read unless that slot
      // filled meanwhile.
      for (int probe = 0; probe < HASH_SLOTS; ++probe) {
        const int32_t k = s_hkey[h];
        if (k == target) {
          atomicAdd(&s_hval[h], val);
          return;
        }
        if (k == -1) break;
        h = H::next(h);
      }
      // not in the table: appended to its key-hash partition, reduced per
      // partition in the output phase
      // (32-bit: 2 app_cap = touch_cap entries, a power of two; partition p
      // holds 2^cs of them from entry p 2^cs)
      const int pi = s_pinfo;
      const int lg = pi & 255, cs = pi >> 8;
      const uint32_t p = lg ? ((uint32_t)target * 0x85EBCA77u) >> (32 - lg) : 0u;
      const int k = atomicAdd(&s_pcur[p], 1);
      if (k < (1 << cs)) {
        double* ab = app_base();
        const uint32_t e = (p << cs) + (uint32_t)k;
        reinterpret_cast<int32_t*>(ab)[4 * e] = target;
        ab[2 * e + 1] = val;
      } else {
        // a partition past 2x its share (one key with thousands of updates
        // that missed the table): the host re-runs the launch without the
        // append path (flag 8)
        atomicOr(A.error_flag, 8);
      }
      return;
    }
    // (heavy: an update made before the table's last inserts landed goes to
    // the HBM hash; the output phase merges its keys with the tables)
    ov_add(target, val);
  };

  // computePathSim for the path node at depth 2i with mass `mass`
  // (degrees travel with the path: dpath[t] = deg(path[t]))
  // the pair update of a path node at depth 2i: false when computePathSim
  // skips it (target == source, or not a first meeting)
  auto contrib_val = [&](const int32_t* path, const int32_t* dpath, int i, int32_t source, double mass,
                         int32_t* target, double* val) -> bool {
    *target = path[2 * i];
    if (*target == source) return false;  // TopSim_singleSample.java:183
#pragma unroll
    for (int j = 0; j < STEP; ++j)  // isFirstMeet (:211-218)
      if (j < i && path[j] == path[2 * i - j]) return false;
    const double dm = (double)dpath[i];
    const double dt = (double)dpath[2 * i];
    if (rw)  // SingleRandomWalk.java:89: cache[i]*deg/deg/SAMPLE
      *val = ((A.cache[i] * dm) / dt) / A.sampled;
    else     // TopSim_singleSample.java:189
      *val = ((mass * A.cache[i]) * dm) / dt;
    ++my_upd;
    return true;
  };
  auto contrib = [&](const int32_t* path, const int32_t* dpath, int i, int32_t source, double mass) {
    int32_t target;
    double val;
    if (contrib_val(path, dpath, i, source, mass, &target, &val)) add(target, val);
  };

  // PIPE: wave 0 claims the next source and builds its levels into buffer b
  auto claim_and_build = [&](int b) {
    long long r = 0;
    if (tid == 0) r = (long long)atomicAdd(A.src_counter, 1u);
    r = ((long long)__shfl((int)(r >> 32), 0, 64) << 32) | (uint32_t)__shfl((int)r, 0, 64);
    if (r < A.nsrc) {
      const TsLevelStats ls = ts_wave_levels<STEP>(A, b, (int64_t)r, s_pm);
      my_ext += ls.ext;
      my_upd += ls.upd;
      if (ls.maxf > my_maxf) my_maxf = ls.maxf;
    } else if (tid == 0) {
      s_pm[b].valid = 0;
    }
  };

  __shared__ unsigned long long s_ph[16];  // diagnostics only: [15] = last timestamp
  if (tid == 0)
    for (int k = 0; k < 16; ++k) s_ph[k] = 0;
  auto mark = [&](int k) {
    if (kGwDiag && A.phase && tid == 0) {
      const unsigned long long now = __builtin_readcyclecounter();
      if (k >= 0) s_ph[k] += now - s_ph[15];
      s_ph[15] = now;
    }
  };
  // one walker (index g in the reference's BFS queue order) of source s from
  // the level / spawner records of buffer b
  // (pt, pv): a pair update carried from the lane's previous walker — the one
  // of its last step (2*STEP), added after this walker's first entry load is
  // issued, so it too leaves the chain of dependent loads (pt < 0: none)
  auto run_walker = [&](int g, int b, int32_t s, int ds, int ns, int32_t& pt, double& pv) {
    const int32_t* Vb = V + b * lvl_stride;
    const int32_t* Db = D + b * lvl_stride;
    const int32_t* Pb = P + b * lvl_stride;
    const int64_t* Ob = O + b * lvl_stride;
    const int32_t* SFb = SF + b * (A.spawn_cap + 1);
    const int sp = upper_bound_i32(ns + 1 <= CO_LDS ? s_co : SFb, ns + 1, g) - 1;
    const int l0 = SL[b * A.spawn_cap + sp];
    const double mw = SM[b * A.spawn_cap + sp];
    int32_t path[L + 1], dpath[L + 1];
    int p = SN[b * A.spawn_cap + sp];
    int32_t dcur = ds;
    int64_t ocur = rw ? G.offsets[s] : (l0 == 0 ? Ob[0] : Ob[(int64_t)l0 * cap + p]);
#pragma unroll
    for (int t = L; t >= 1; --t) {
      if (t <= l0) {
        path[t] = Vb[(int64_t)t * cap + p];
        dpath[t] = Db[(int64_t)t * cap + p];
        p = Pb[(int64_t)t * cap + p];
      }
    }
    path[0] = s;
    dpath[0] = ds;
#pragma unroll
    for (int t = 0; t <= L; ++t)
      if (t == l0) dcur = dpath[t];
    bool alive = true;
    // The draw of step t depends on (s, g, t) only, so step t+1's Philox block
    // is computed while step t's entry load is in flight, and step t+1's
    // entry load is issued BEFORE step t's computePathSim: the LDS-hash probe /
    // insert of a pair update runs while the next random read is in flight
    // instead of on the walker's chain of dependent loads.
    const bool early = !(kGwDiag && (A.diag & 1024));  // diag bit 1024: contrib before the next load (A/B)
    auto slot_of = [&](const gw_u4& u, int t) -> uint64_t {
      uint32_t ux = u.x, uy = u.y;
      if (kGwDiag && (A.diag & 2)) {  // timing only: cheap hash instead of Philox
        ux = ((uint32_t)s * 0x9E3779B1u) ^ ((uint32_t)g * 0x85EBCA6Bu) ^ ((uint32_t)t * 0xC2B2AE35u);
        ux ^= ux >> 15;
        ux *= 0x2C1B3C6Du;
        uy = 0u;
      }
      uint64_t ei = (uint64_t)ocur + gw_index(ux, uy, (uint32_t)dcur);
      if (kGwDiag && (A.diag & 12))  // timing only: walker reads confined to 1 GB / 2 GB of the table
        ei &= (A.diag & 4) ? ((1ull << 26) - 1) : ((1ull << 27) - 1);
      return ei;
    };
    gw_u4 un = gw_philox((uint32_t)s, (uint32_t)g, (uint32_t)(l0 + 1), 0u, A.k0, A.k1);
    gw_ts_ent en = {0, 0, 0};  // step t's entry, requested during step t-1
    bool inflight = false;
#pragma unroll
    for (int t = 1; t <= L; ++t) {
      if (t > l0 && alive) {
        if (!inflight && dcur == 0) {
          alive = false;
        } else {
          if (!inflight) {  // the walker's first step
            en = gw_ts_load(A.ent + slot_of(un, t));  // randNeighbor
            if (t < L) un = gw_philox((uint32_t)s, (uint32_t)g, (uint32_t)(t + 1), 0u, A.k0, A.k1);
            if (pt >= 0) {  // the previous walker's last pair update
              add(pt, pv);
              pt = -1;
            }
          }
          const gw_ts_ent e = en;
          inflight = false;
          path[t] = e.x;
          dpath[t] = e.d;
          dcur = e.d;
          ocur = e.off;
          ++my_ext;
          if (early && t < L && dcur != 0) {  // step t+1's read, then step t's pair update
            en = gw_ts_load(A.ent + slot_of(un, t + 1));
            inflight = true;
            if (t + 1 < L) un = gw_philox((uint32_t)s, (uint32_t)g, (uint32_t)(t + 2), 0u, A.k0, A.k1);
          }
          if ((t & 1) == 0 && !(kGwDiag && (A.diag & 1))) {
            if (PIPE && t == L && early && !(kGwDiag && (A.diag & 2048))) {  // carried to the next walker
              if (pt >= 0) add(pt, pv);  // (not flushed: this walker issued no first load)
              if (!contrib_val(path, dpath, t / 2, s, mw, &pt, &pv)) pt = -1;
            } else {
              contrib(path, dpath, t / 2, s, mw);
            }
          }
        }
      }
    }
    ++my_walk;
  };

  int cur = 0;  // PIPE: buffer of the source being walked
  if (PIPE) {
    if (tid < 64) claim_and_build(0);
    __syncthreads();
  }
  for (;;) {
    mark(-1);
    int64_t r;
    int32_t s;
    int ds;
    int p_ns = 0, p_nw = 0, p_ne = 0;
    if (PIPE) {
      // hand-over: the source whose levels wave 0 built during the last walker phase
      if (!s_pm[cur].valid) break;
      r = s_pm[cur].r;
      s = s_pm[cur].s;
      ds = s_pm[cur].ds;
      p_ns = s_pm[cur].nspawn;
      p_nw = s_pm[cur].nwalk;
      p_ne = s_pm[cur].ncontrib;
      if (p_ns + 1 <= CO_LDS) {
        const int32_t* SFb = SF + cur * (A.spawn_cap + 1);
        for (int k = tid; k <= p_ns; k += BLOCK) s_co[k] = SFb[k];
      }
      if (tid == 0) {
        s_wnext = 0u;
        s_ncomp = 0;
        s_novc = 0;
        if (!LDS_ROW) s_ovmask = s_pm[cur].ovmask;
        s_heavy = (APPEND && !LDS_ROW) ? s_pm[cur].heavy : 0;
        s_plg = s_pm[cur].plg;
        s_pinfo = s_plg | ((31 - __builtin_clz((uint32_t)A.touch_cap) - s_plg - A.pcap_shrink) << 8);
      }
      __syncthreads();
    } else {
    if (tid == 0) {
      s_src = (int)atomicAdd(A.src_counter, 1u);
      s_abort = 0;
      s_ncomp = 0;
      s_novc = 0;
    }
    __syncthreads();
    r = s_src;
    if (r >= A.nsrc) break;
    s = A.sources[r];
    ds = G.deg[s];

    if (rw) {
      if (tid == 0) {
        s_nspawn = 0;
        s_nwalk = 0;
        if (ds > 0) {  // root spawns SAMPLE walks (SingleRandomWalk.java:55)
          SL[0] = 0;
          SN[0] = 0;
          SM[0] = 1.0;
          s_co[0] = 0;
          s_co[1] = A.sample;
          s_nspawn = 1;
          s_nwalk = A.sample;
        }
      }
      __syncthreads();
    } else {
      if (tid == 0) {
        V[0] = s;
        D[0] = ds;
        O[0] = G.offsets[s];
        P[0] = -1;
        M[0] = A.sampled;  // path[0].sample = SAMPLE (:73)
        s_size[0] = 1;
        s_nspawn = 0;
      }
      __syncthreads();
      for (int l = 0; l <= L; ++l) {
        const int sz = s_size[l];
        if (sz == 0) break;  // every later level is empty too: skip their barriers
        const int32_t* Vl = V + (int64_t)l * cap;
        const double* Ml = M + (int64_t)(l & 1) * cap;
        if (tid == 0 && sz > my_maxf) my_maxf = sz;
        // computePathSim at pathLen = 2i (:80-83, :157) for enumerated nodes
        if ((l & 1) == 0 && l >= 2) {
          for (int j = tid; j < sz; j += BLOCK) {
            int32_t path[L + 1], dpath[L + 1];
            int p = j;
#pragma unroll
            for (int t = L; t >= 1; --t) {
              if (t <= l) {
                path[t] = V[(int64_t)t * cap + p];
                dpath[t] = D[(int64_t)t * cap + p];
                p = P[(int64_t)t * cap + p];
              }
            }
            path[0] = s;
            dpath[0] = ds;
#pragma unroll
            for (int t = 2; t <= L; t += 2)
              if (t == l) contrib(path, dpath, t / 2, s, Ml[j]);
          }
        }
        if (l == L) break;
        // expansion: child counts (enumerated) and spawners (random branch)
        int32_t* const COx = sz + 1 <= CO_LDS ? s_co : CO;
        int total_children = 0;
        int spawn_base = s_nspawn;
        for (int base = 0; base < sz; base += BLOCK) {
          const int j = base + tid;
          int cnt = 0, sp = 0;
          double m = 0.0;
          if (j < sz) {
            const int d = D[(int64_t)l * cap + j];
            m = Ml[j];
            const bool det = enumerate_all ? (d != 0) : (d != 0 && m >= (double)d);  // :99
            if (det)
              cnt = d;
            else if (d != 0)
              sp = 1;  // d == 0: randNeighbor() == -1 -> no child (:143-144)
          }
          int tot_c, tot_s;
          const int ex_c = block_excl_scan<NW>(cnt, s_wave, &tot_c);
          const int ex_s = block_excl_scan<NW>(sp, s_wave, &tot_s);
          if (j < sz) COx[j] = total_children + ex_c;
          if (sp) {
            const int k = spawn_base + ex_s;
            if (k < A.spawn_cap) {
              int c = (int)m;  // number = (int)s == s ? (int)s : (int)s + 1 (:131-135)
              if ((double)c != m) c += 1;
              SL[k] = l;
              SN[k] = j;
              SF[k] = c;
              SM[k] = m / (double)c;  // (double)cur.sample/(double)number (:142)
            } else {
              atomicOr(A.error_flag, 1);
              s_abort = 1;
            }
          }
          total_children += tot_c;
          spawn_base += tot_s;
          if ((int64_t)total_children > cap) total_children = (int)cap + 1;  // saturate
        }
        if (tid == 0) {
          COx[sz] = total_children;
          s_nspawn = spawn_base;
          if ((int64_t)total_children > cap) {
            atomicOr(A.error_flag, 1);
            s_abort = 1;
          }
        }
        __syncthreads();
        if (s_abort) break;
        // load-balanced fill of level l+1 (BFS queue order)
        int32_t* Vn = V + (int64_t)(l + 1) * cap;
        int32_t* Pn = P + (int64_t)(l + 1) * cap;
        double* Mn = M + (int64_t)((l + 1) & 1) * cap;
        int32_t* Dn = D + (int64_t)(l + 1) * cap;
        int64_t* On = O + (int64_t)(l + 1) * cap;
        const int64_t* Ol = O + (int64_t)l * cap;
        for (int c = tid; c < total_children; c += BLOCK) {
          const int j = upper_bound_i32(COx, sz + 1, c) - 1;
          const int k = c - COx[j];
          const int d = COx[j + 1] - COx[j];
          const gw_ts_ent e = gw_ts_load(A.ent + Ol[j] + k);  // edges.get(j), insertion order (:103-110)
          Vn[c] = e.x;
          Dn[c] = e.d;
          On[c] = e.off;
          Pn[c] = j;
          Mn[c] = Ml[j] / (double)d;         // newSample = cur.sample / degree (:104)
        }
        if (tid == 0) {
          my_ext += total_children;
          s_size[l + 1] = total_children;
        }
        __syncthreads();
      }
      mark(0);
      // walker index prefix over spawners (queue order)
      const int ns = s_abort ? 0 : s_nspawn;
      int32_t* const SFx = ns + 1 <= CO_LDS ? s_co : SF;
      int run = 0;
      for (int base = 0; base < ns; base += BLOCK) {
        const int k = base + tid;
        const int c = (k < ns) ? SF[k] : 0;
        int tot;
        const int ex = block_excl_scan<NW>(c, s_wave, &tot);
        if (k < ns) SFx[k] = run + ex;
        run += tot;
      }
      if (tid == 0) {
        SFx[ns] = run;
        s_nspawn = ns;
        s_nwalk = run;
      }
      __syncthreads();
    }

    }  // !PIPE: levels built by the whole workgroup

    mark(1);
    // random walkers: one lane each, path in registers
    if (PIPE) {
      // wave 0 first builds the next source's levels into the other buffer
      if (tid < 64)
        claim_and_build(cur ^ 1);
      else if (defer && pend_r >= 0 && tid >= BLOCK - 64)
        deferred_topk();  // the last wave ranks the previous source meanwhile
      mark(0);  // diagnostics: wave 0's level build (the rest of its walker phase goes to "walkers")
      // walkers g < p_nw, then the enumerated nodes' recorded pair updates,
      // dealt out 64 at a time
      const int lane = tid & 63;
      const int32_t* ETb = A.enum_tgt + (blk * 2 + cur) * A.enum_cap;
      const double* EVb = A.enum_val + (blk * 2 + cur) * A.enum_cap;
      int32_t pt = -1;
      double pv = 0.0;
      if (kGwDiag && A.phase && tid == 64) w1_t = __builtin_readcyclecounter();
      for (;;) {
        unsigned base = 0u;
        if (lane == 0) base = atomicAdd(&s_wnext, 64u);
        base = (unsigned)__shfl((int)base, 0, 64);
        if ((int)base >= p_nw + p_ne) break;
        const int g = (int)base + lane;
        if (g < p_nw)
          run_walker(g, cur, s, ds, p_ns, pt, pv);
        else if (g < p_nw + p_ne)
          add(ETb[g - p_nw], EVb[g - p_nw]);
      }
      if (pt >= 0) add(pt, pv);
      if (kGwDiag && A.phase && tid == 64) {  // diagnostics: a walker wave's walk / wait at the barrier
        const unsigned long long now = __builtin_readcyclecounter();
        w1_walk += now - w1_t;
        w1_t = now;
      }
    } else {
      const int W = s_nwalk;
      const int ns = s_nspawn;
      int32_t pt = -1;
      double pv = 0.0;
      for (int g = tid; g < W; g += BLOCK) run_walker(g, 0, s, ds, ns, pt, pv);
      if (pt >= 0) add(pt, pv);
    }
    __syncthreads();
    if (PIPE && kGwDiag && A.phase && tid == 64) w1_wait += __builtin_readcyclecounter() - w1_t;

    mark(2);
    // ---- output ------------------------------------------------------------
    // hash mode: the overflow entries leave the HBM hash for a compact
    // per-workgroup list — key in touched[k] (which held its slot), value in
    // ov_list[k] — so the selection passes read them coalesced instead of
    // through two dependent reads per entry and pass, and their slots are
    // cleared right here for the next source.  A key that also reached the
    // LDS table (a racing load-limit read lets it into both) is folded into
    // its LDS entry first; it sits in its first kTsProbeCap slots there.
    int nov = LDS_ROW ? 0 : min((int64_t)s_ntouch, A.touch_cap * 3 / 4);
    // (counter-limited table: the chain ends at an empty slot; diag 8192: within kTsProbeCap slots)
    const int fold_cap = (kGwDiag && (A.diag & 8192)) ? kTsProbeCap : HASH_SLOTS;
    // the key's LDS chain, four keys per ds_read_b128, up to its first empty slot
    auto fold_lds = [&](int32_t key, double& v, int cap) {
      uint32_t h = H::slot(key);
      bool done = false;
      for (int probed = 0; probed < cap && !done;) {
        const uint32_t g0 = h & ~3u;
        const int4 kv = *reinterpret_cast<const int4*>(&s_hkey[g0]);
        const int32_t ks[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (done || (uint32_t)j < (h & 3u) || probed >= cap) continue;
          ++probed;
          if (ks[j] == -1) {
            done = true;
          } else if (ks[j] == key) {
            atomicAdd(&s_hval[g0 + (uint32_t)j], v);
            v = 0.0;
            done = true;
          }
        }
        h = g0 + 4u == (uint32_t)HASH_SLOTS ? 0u : g0 + 4u;
      }
    };
    // this thread's LDS-table slots -> the candidate list (touched / ov_list
    // from s_novc on), cleared; keys placed by a wave scan + one LDS atomic
    // (entries whose key is below tl cannot reach the source's top k: dropped)
    auto dump_lds = [&](unsigned long long tl) {
      constexpr int SPT_D = HASH_SLOTS / BLOCK;
      int32_t kk[SPT_D];
      int mine = 0;
#pragma unroll
      for (int i = 0; i < SPT_D; ++i) {
        kk[i] = s_hkey[tid + i * BLOCK];
        if (kk[i] != -1 && tl != 0ull && dkey(s_hval[tid + i * BLOCK]) < tl) {
          s_hkey[tid + i * BLOCK] = -1;  // below the bound: cleared, not listed
          s_hval[tid + i * BLOCK] = 0.0;
          kk[i] = -1;
        }
        mine += kk[i] != -1;
      }
      // (lane made opaque: its compare masks are not hoisted into scalar
      // registers held through the whole kernel)
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      int incl = mine;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      int wbase = 0;
      if (lane == 63 && incl > 0) wbase = atomicAdd(&s_novc, incl);
      int o = __shfl(wbase, 63, 64) + incl - mine;
      const int cap34 = (int)(A.touch_cap * 3 / 4);
#pragma unroll
      for (int i = 0; i < SPT_D; ++i)
        if (kk[i] != -1) {
          const double v = s_hval[tid + i * BLOCK];
          s_hkey[tid + i * BLOCK] = -1;
          s_hval[tid + i * BLOCK] = 0.0;
          if (o < cap34) {
            __hip_atomic_store(&touched[o], kk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ov_list[o], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            atomicOr(A.error_flag, 2);
          }
          ++o;
        }
    };
    // append-and-reduce source (PIPE, hash mode; wave 0's level build bounds its
    // pair updates above heavy_min): an update whose key is not in the full
    // LDS table was appended, during the walk, to its key-hash partition
    // (16 B, no random CAS line in the HBM hash).  Updates that raced the
    // table's last inserts (the key may have landed in it) and those of a
    // full partition went to the HBM hash, whose claimed slots are listed.
    // Here: (0) those HBM keys the LDS table holds are folded into it; the
    // table moves to the candidate list; (1) each partition is reduced in the
    // emptied LDS table (counter-free insert: a key without room within
    // kTsProbeCap slots goes to the HBM hash), the HBM keys of that partition
    // are folded into it, and it moves to the candidate list; (2) the HBM
    // keys left are compacted into the list.  A key thus ends in exactly one
    // candidate entry; the selection reads the list only.
    const bool heavy = APPEND && !LDS_ROW && s_heavy;
    if (heavy) {
      const int lg = s_plg;
      const int NP = 1 << lg;
      const int64_t cap_p = (int64_t)1 << (s_pinfo >> 8);  // == 2 app_cap >> lg
      const int32_t* bkey = reinterpret_cast<const int32_t*>(app_base());
      const double* bval = app_base();
      int32_t* cl = claim_base();
      const int cap34 = (int)(A.touch_cap * 3 / 4);
      mark(13);
      // top-k rows only: a lower bound on the source's K-th largest score from
      // the final values of the LDS table (every key left there is final:
      // its other updates were folded in below), by two radix passes over
      // its slots — the key's bin lower edge with >= K table entries at or
      // above it.  Partition and HBM candidates below it cannot make the top
      // k and are never listed (the list was ~36k entries per stretch source,
      // re-read by every selection pass).
      const bool prune = A.out_ids && !A.out_rows && !A.sp.cursor && A.topk > 0 && !(kGwDiag && (A.diag & 65536));
      unsigned long long tlb = 0ull;
      // (0) claimed HBM keys held by the LDS table (a folded entry keeps its key
      // for the probe chains; value 0 marks it: pair updates are > 0)
      int nt = min(s_ntouch, cap34);
      for (int k = tid; k < nt; k += BLOCK) {
        const int32_t slot = cl[k];
        const int32_t key = __hip_atomic_load(&ov_key[4 * slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        double v = __hip_atomic_load(&ov_val[2 * slot + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fold_lds(key, v, fold_cap);
        if (v == 0.0) __hip_atomic_store(&ov_val[2 * slot + 1], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (prune) {
        for (int b = tid; b < 256; b += BLOCK) {
          s_hist[b] = 0;
          s_hist2[b] = 0;
        }
        if (tid == 0) {
          s_prefix = 0;
          s_mask = 0;
          s_need = A.topk;
          s_all = 0;
        }
      }
      __syncthreads();
      if (prune) {
        for (int pass = 0; pass < 2; ++pass) {
          const int shift = 56 - 8 * pass;
          unsigned* const Hh = pass ? s_hist2 : s_hist;
          const unsigned long long pre = s_prefix, msk = s_mask;
#pragma unroll
          for (int i = 0; i < HASH_SLOTS / BLOCK; ++i)
            if (s_hkey[tid + i * BLOCK] != -1) {
              const unsigned long long k = dkey(s_hval[tid + i * BLOCK]);
              if ((k & msk) == pre) atomicAdd(&Hh[(k >> shift) & 255], 1u);
            }
          __syncthreads();
          if (tid < 64) {
            int bin, before, tot;
            select_bin_w(Hh, s_need, true, bin, before, tot);
            if (tid == 0) {
              if (pass == 0 && tot < A.topk) {
                s_all = 1;  // fewer than K table entries: no bound
              } else {
                s_need -= before;
                s_prefix = pre | ((unsigned long long)bin << shift);
                s_mask = msk | (255ull << shift);
              }
            }
          }
          __syncthreads();
          if (s_all) break;
        }
        tlb = s_all ? 0ull : (unsigned long long)s_prefix;
      }
      dump_lds(tlb);
      __syncthreads();
      mark(10);  // diagnostics: claims folded into the table + table dump
      for (int p = 0; p < NP; ++p) {  // (1)
        const int np = (int)min((int64_t)s_pcur[p], cap_p);
        const int64_t e0 = (int64_t)p * cap_p;
        constexpr int U = 8;  // eight entries per thread and round: their reads issued together
        for (int k0 = tid; k0 < np; k0 += U * BLOCK) {
          int32_t key[U];
          double v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = k0 + u * BLOCK;
            key[u] = k < np ? bkey[4 * (e0 + k)] : -1;
            v[u] = k < np ? bval[2 * (e0 + k) + 1] : 0.0;
          }
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (key[u] != -1 && !cf_insert(key[u], v[u])) ov_add(key[u], v[u]);
        }
        __syncthreads();
        nt = min(s_ntouch, cap34);
        if (nt > 0) {  // this partition's claimed HBM keys held by its table
          for (int k = tid; k < nt; k += BLOCK) {
            const int32_t slot = cl[k];
            const int32_t key = __hip_atomic_load(&ov_key[4 * slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (part_of(key, lg) != p) continue;
            double v = __hip_atomic_load(&ov_val[2 * slot + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v == 0.0) continue;
            fold_lds(key, v, kTsProbeCap);  // (counter-free table: a key sits within its first kTsProbeCap slots)
            if (v == 0.0) __hip_atomic_store(&ov_val[2 * slot + 1], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          __syncthreads();
        }
        dump_lds(tlb);
        __syncthreads();
      }
      mark(11);  // diagnostics: partition reduces
      // (2) the claimed HBM keys no table held -> the candidate list; every claimed slot cleared
      nt = min(s_ntouch, cap34);
      const int lane = tid & 63;
      const unsigned long long below = (1ull << lane) - 1ull;
      for (int k0 = 0; k0 < nt; k0 += BLOCK) {
        const int k = k0 + tid;
        int32_t key = -1;
        double v = 0.0;
        if (k < nt) {
          const int32_t slot = cl[k];
          key = __hip_atomic_load(&ov_key[4 * slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v = __hip_atomic_load(&ov_val[2 * slot + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ov_key[4 * slot], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ov_val[2 * slot + 1], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const bool keep = v != 0.0 && dkey(v) >= tlb;
        const unsigned long long m = __ballot(keep);
        int wbase = 0;
        if (lane == 0 && m) wbase = atomicAdd(&s_novc, __popcll(m));
        wbase = __shfl(wbase, 0, 64);
        if (keep) {
          const int o = wbase + __popcll(m & below);
          if (o < cap34) {
            __hip_atomic_store(&touched[o], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ov_list[o], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            atomicOr(A.error_flag, 2);
          }
        }
      }
      __syncthreads();
      nov = min(s_novc, cap34);
      if (tid == 0) s_hcount = 0;
      mark(12);  // diagnostics: claims compaction
    }
    // a source with many overflow keys for its table (>= 1/8 of the slots)
    // compacts by scanning the slots in order: coalesced reads and clears
    // instead of two random line accesses per key through `touched` (an
    // append-and-reduce source always: its list is the candidate list)
    const uint32_t ov_mask = s_ovmask;
    const bool ov_scan = !LDS_ROW && !heavy && s_ntouch > 0 &&
                         (int64_t)s_ntouch * 8 >= (int64_t)ov_mask + 1 &&
                         !(kGwDiag && (A.diag & 16384));  // diag bit 16384: always through `touched` (A/B)
    if (ov_scan) {
      const int T = (int)ov_mask + 1;
      const int cap34 = (int)(A.touch_cap * 3 / 4);
      const int lane = tid & 63;
      const unsigned long long below = (1ull << lane) - 1ull;
      constexpr int U = 4;
      int ti = tid;  // (opaque: the slot addresses are formed here, not hoisted out of the source loop)
      asm volatile("" : "+v"(ti));
      for (int b0 = 0; b0 < T; b0 += U * BLOCK) {
        int32_t key[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = b0 + u * BLOCK + ti;
          key[u] = -1;
          v[u] = 0.0;
          if (i < T) {
            key[u] = __hip_atomic_load(&ov_key[4 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[u] = __hip_atomic_load(&ov_val[2 * i + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        int cnt[U], pre[U], tot = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const unsigned long long m = __ballot(key[u] != -1);
          pre[u] = tot + __popcll(m & below);
          cnt[u] = __popcll(m);
          tot += cnt[u];
        }
        int wbase = 0;
        if (lane == 0 && tot > 0) wbase = atomicAdd(&s_novc, tot);
        wbase = __shfl(wbase, 0, 64);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (key[u] == -1) continue;
          const int i = b0 + u * BLOCK + ti;
          __hip_atomic_store(&ov_key[4 * i], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ov_val[2 * i + 1], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          fold_lds(key[u], v[u], fold_cap);
          const int k = wbase + pre[u];
          if (k < cap34) {
            __hip_atomic_store(&touched[k], key[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ov_list[k], v[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            atomicOr(A.error_flag, 2);  // as dump_lds / ov_add at the same limit
          }
        }
      }
      __syncthreads();
      nov = min(s_novc, cap34);
    } else if (!LDS_ROW && !heavy && nov > 0) {
      // four entries per thread and round, their slot reads issued together
      // (the stretch compacts ~31k entries per source: the loop was a chain of
      // dependent random reads per entry)
      constexpr int U = 4;
      for (int k0 = tid; k0 < nov; k0 += U * BLOCK) {
        int32_t slot[U], key[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = k0 + u * BLOCK;
          slot[u] = k < nov ? __hip_atomic_load(&touched[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          key[u] = -1;
          v[u] = 0.0;
          if (slot[u] >= 0) {
            key[u] = __hip_atomic_load(&ov_key[4 * slot[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[u] = __hip_atomic_load(&ov_val[2 * slot[u] + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (slot[u] < 0) continue;
          __hip_atomic_store(&ov_key[4 * slot[u]], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ov_val[2 * slot[u] + 1], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          fold_lds(key[u], v[u], fold_cap);
          const int k = k0 + u * BLOCK;
          __hip_atomic_store(&touched[k], key[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ov_list[k], v[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      __syncthreads();
    }
    // hash mode: every thread takes its HASH_SLOTS / BLOCK slots into
    // registers and clears them.  Top-k rows only (no dense / sparse rows,
    // `regsel`): the selection passes below read those registers — no
    // compaction, no LDS re-reads, no re-zeroing pass (round 5).  Otherwise the
    // occupied slots are moved to the front once, so the passes scan only them.
    int NL = 0;
    constexpr int SPT = LDS_ROW ? 1 : HASH_SLOTS / BLOCK;
    static_assert(LDS_ROW || HASH_SLOTS % BLOCK == 0, "hash slots per thread");
    double vv[SPT];  // the values of this thread's slots (an empty slot holds 0.0)
    const bool regsel = !LDS_ROW && A.out_ids && !A.out_rows && !A.sp.cursor && !(kGwDiag && (A.diag & 4096));
    if (!LDS_ROW) {
#pragma unroll
      for (int i = 0; i < SPT; ++i) vv[i] = s_hval[tid + i * BLOCK];
    }
    if (!LDS_ROW && !regsel) {
      int32_t kk[SPT];
      int mine = 0;
#pragma unroll
      for (int i = 0; i < SPT; ++i) {
        kk[i] = s_hkey[tid + i * BLOCK];
        mine += kk[i] != -1;
      }
      // offsets: an inclusive scan inside the wave and one LDS atomic per
      // wave (the compacted order is free: selection and the sparse-row
      // writer do not depend on it); the barrier orders every read before the writes
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      int incl = mine;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      int wbase = 0;
      if (lane == 63) wbase = atomicAdd(&s_ncomp, incl);
      int o = __shfl(wbase, 63, 64) + incl - mine;
#pragma unroll
      for (int i = 0; i < SPT; ++i)
        if (kk[i] != -1) {
          s_hkey[tid + i * BLOCK] = -1;
          s_hval[tid + i * BLOCK] = 0.0;
        }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < SPT; ++i)
        if (kk[i] != -1) {
          s_hkey[o] = kk[i];
          s_hval[o] = vv[i];
          ++o;
        }
      __syncthreads();
      NL = s_ncomp;
    }
    const int NC = LDS_ROW ? n : NL + nov;  // LDS-side candidates (regsel: the overflow entries only)
    // the register-held candidates of this thread (regsel; the keys stay in
    // LDS until the re-zeroing, values in registers: every key's value > 0)
    auto each_reg = [&](auto&& f) {
      if (!LDS_ROW && regsel) {
#pragma unroll
        for (int i = 0; i < SPT; ++i)
          if (vv[i] > 0.0) f(i, vv[i]);
      }
    };
    auto cand = [&](int idx, int32_t* id, double* val) -> bool {
      if (LDS_ROW) {
        *id = idx;
        *val = s_row[idx];
      } else if (idx < NL) {
        *id = s_hkey[idx];
        *val = s_hval[idx];
      } else {  // the compact overflow list (relaxed atomic loads: plain ones here trip a gfx950 codegen bug)
        *id = __hip_atomic_load(&touched[idx - NL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *val = __hip_atomic_load(&ov_list[idx - NL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return *val > 0.0;
    };
    // f(id, value) for this thread's candidates idx = tid, tid + BLOCK, ... < NC
    // with a value > 0; the loads of kCandBatch of them are issued together
    // (the overflow list sits in L2 / HBM: a pass over ~36k stretch candidates
    // was ~70 dependent round trips per thread, one per entry)
    // (the append-and-reduce kernels only, whose heavy sources keep ~36k
    // candidates in the list: the unpipelined arxiv kernel measured +2.7% with
    // the batch, the others +-0; profiles/r06/tsab_r06e.jsonl)
    constexpr int kCandBatch = APPEND ? 8 : 1;
    auto for_cands = [&](auto&& f) {
      for (int b0 = tid; b0 < NC; b0 += kCandBatch * BLOCK) {
        int32_t id[kCandBatch];
        double v[kCandBatch];
#pragma unroll
        for (int u = 0; u < kCandBatch; ++u) {
          id[u] = 0;
          v[u] = 0.0;
          if (b0 + u * BLOCK < NC) cand(b0 + u * BLOCK, &id[u], &v[u]);
        }
#pragma unroll
        for (int u = 0; u < kCandBatch; ++u)
          if (v[u] > 0.0) f(id[u], v[u]);
      }
    };
    if (A.out_rows) {
      double* orow = A.out_rows + r * (int64_t)n;
      // (an opaque copy of tid: its row addresses are not hoisted out of the
      // source loop into a register held through the walker phase)
      int t0 = tid;
      asm volatile("" : "+v"(t0));
      if (LDS_ROW) {
        for (int t = t0; t < n; t += BLOCK) orow[t] = s_row[t];
      } else {
        for (int t = t0; t < n; t += BLOCK) orow[t] = 0.0;
        __syncthreads();
        for_cands([&](int32_t id, double v) { orow[id] = v; });
      }
    }
    if (A.sp.cursor) {
      // sparse row: every nonzero entry (accumulator order), packed at a
      // claimed offset; a row that does not fit is skipped (len -1) but still
      // counted, so the cursor ends at the room all rows need
      int mine = 0;
      for_cands([&](int32_t, double) { ++mine; });
      int tot;
      const int ex = block_excl_scan<NW>(mine, s_wave, &tot);
      if (tid == 0) s_spbase = atomicAdd(A.sp.cursor, (unsigned long long)tot);
      __syncthreads();
      const int64_t base = (int64_t)s_spbase;
      const bool fits = base + tot <= A.sp.cap;
      if (fits) {
        int64_t o = base + ex;
        for_cands([&](int32_t id, double v) {
          A.sp.ids[o] = id;
          A.sp.scores[o] = v;
          ++o;
        });
      }
      if (tid == 0) {
        A.sp.begin[r] = fits ? base : -1;
        A.sp.len[r] = fits ? tot : -1;
        if (!fits) atomicOr(A.error_flag, 4);
      }
    }
    if (A.out_ids) {
      const int K = A.topk;
      // the K-th key's bin may be taken whole once everything at or above it
      // fits the selection arrays: the ordering pass below then ranks the
      // extra entries out (bounded so that it keeps 4 threads per entry)
      const int kcoll = max(K, BLOCK / 4);
      mark(5);
      unsigned long long T = 0;  // threshold key (K-th largest)
      int32_t idT = 0x7fffffff;  // largest id taken at key == T
      bool take_all = false;     // at most K candidates (counted by the first radix pass)
      bool bin_exact = false;    // the K-th key's bin is taken whole: select by masked prefix
      unsigned long long Tmask = ~0ull;
      {
        for (int b = tid; b < 256; b += BLOCK) s_hist[b] = 0;
        if (tid == 0) {
          s_prefix = 0;
          s_mask = 0;
          s_need = K;
          s_exact = 0;
          s_total = 0;
          s_all = 0;
        }
        __syncthreads();
        // two barriers a pass: the histogram (the next pass's one is cleared
        // meanwhile), then wave 0 picks the bin and narrows the prefix
        int pass = 0;
        for (int shift = 56; shift >= 0; shift -= 8, ++pass) {
          unsigned* const H = (pass & 1) ? s_hist2 : s_hist;
          unsigned* const Hn = (pass & 1) ? s_hist : s_hist2;
          const unsigned long long pre = s_prefix, msk = s_mask;
          for (int b = tid; b < 256; b += BLOCK) Hn[b] = 0;
          each_reg([&](int, double v) {
            const unsigned long long k = dkey(v);
            if ((k & msk) == pre) atomicAdd(&H[(k >> shift) & 255], 1u);
          });
          for_cands([&](int32_t, double v) {
            const unsigned long long k = dkey(v);
            if ((k & msk) == pre) atomicAdd(&H[(k >> shift) & 255], 1u);
          });
          __syncthreads();
          if (tid < 64) {
            select_bin(H, s_need, true, &s_bin, &s_cum, shift == 56 ? &s_total : nullptr);
            if (tid == 0) {  // s_bin / s_cum / s_total were written by this thread
              if (shift == 56 && s_total <= K) {
                s_all = 1;
              } else {
                const int rest = s_need - s_cum;
                // everything above the chosen bin (K - rest keys) plus the bin fits
                if (K - rest + (int)H[s_bin] <= kcoll) s_exact = 1;
                s_need = rest;
                s_prefix = pre | ((unsigned long long)s_bin << shift);
                s_mask = msk | (255ull << shift);
              }
            }
          }
          __syncthreads();
          if (s_all) {
            take_all = true;
            break;
          }
          if (s_exact) break;
        }
        bin_exact = s_exact != 0;
        Tmask = s_mask;
        T = s_prefix;
      }
      mark(6);
      if (!take_all && !bin_exact) {
        // ties at the threshold: smallest ids first
        long long eq_local = 0;
        each_reg([&](int, double v) { eq_local += dkey(v) == T; });
        for_cands([&](int32_t, double v) { eq_local += dkey(v) == T; });
        const int EQ = (int)block_sum<long long, NW>(eq_local, s_red);
        if (EQ > s_need) {
          if (tid == 0) {
            s_prefix = 0;
            s_mask = 0;
          }
          __syncthreads();
          for (int shift = 24; shift >= 0; shift -= 8) {
            for (int b = tid; b < 256; b += BLOCK) s_hist[b] = 0;
            __syncthreads();
            const unsigned long long pre = s_prefix, msk = s_mask;
            each_reg([&](int i, double v) {
              if (dkey(v) != T) return;
              const unsigned long long k = (unsigned)s_hkey[tid + i * BLOCK];
              if ((k & msk) == pre) atomicAdd(&s_hist[(k >> shift) & 255], 1u);
            });
            for_cands([&](int32_t id, double v) {
              if (dkey(v) != T) return;
              const unsigned long long k = (unsigned)id;
              if ((k & msk) == pre) atomicAdd(&s_hist[(k >> shift) & 255], 1u);
            });
            __syncthreads();
            if (tid < 64) select_bin(s_hist, s_need, false, &s_bin, &s_cum);
            __syncthreads();
            if (tid == 0) {
              s_need = s_need - s_cum;
              s_prefix = pre | ((unsigned long long)s_bin << shift);
              s_mask = msk | (255ull << shift);
            }
            __syncthreads();
          }
          idT = (int32_t)s_prefix;
        }
      }
      mark(7);
      if (tid == 0) s_cnt = 0;
      __syncthreads();
      // one LDS atomic per wave and round (ballot + v_mbcnt ranks), not one
      // per selected entry on the same counter
      auto selected = [&](int32_t id, double v) {
        const unsigned long long k = dkey(v);
        return take_all || (bin_exact ? (k & Tmask) >= T : (k > T || (k == T && id <= idT)));
      };
      auto append = [&](bool sel, int32_t id, double v) {
        const unsigned long long sm = __ballot(sel);
        if (sm) {
          int wb = 0;
          if ((tid & 63) == __ffsll(sm) - 1) wb = atomicAdd(&s_cnt, __popcll(sm));
          wb = __shfl(wb, __ffsll(sm) - 1, 64);
          const int slot = wb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
          if (sel && slot < TOPK_MAX) {
            s_sel_id[slot] = id;
            s_sel_val[slot] = v;
          }
        }
      };
      if (!LDS_ROW && regsel) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
          const int32_t id = vv[i] > 0.0 ? s_hkey[tid + i * BLOCK] : 0;
          append(vv[i] > 0.0 && selected(id, vv[i]), id, vv[i]);
        }
      }
      for (int base = 0; base < NC; base += kCandBatch * BLOCK) {  // (wave-uniform: append's ballots)
        int32_t id[kCandBatch];
        double v[kCandBatch];
#pragma unroll
        for (int u = 0; u < kCandBatch; ++u) {
          id[u] = 0;
          v[u] = 0.0;
          const int idx = base + u * BLOCK + tid;
          if (idx < NC) cand(idx, &id[u], &v[u]);
        }
#pragma unroll
        for (int u = 0; u < kCandBatch; ++u) append(v[u] > 0.0 && selected(id[u], v[u]), id[u], v[u]);
      }
      __syncthreads();
      const int cnt = min(s_cnt, TOPK_MAX);
      mark(8);
      if (defer) {
        // deferred ordering: the selected entries go to the workgroup's HBM
        // scratch; the last wave ranks them during the next walker phase
        for (int k = tid; k < cnt; k += BLOCK) {
          // k made opaque here: otherwise the per-lane 64-bit store address is
          // hoisted out of the source loop and spilled (12 B scratch at STEP 5)
          asm volatile("" : "+v"(k));
          A.dsel_id[blk * TOPK_MAX + k] = s_sel_id[k];
          A.dsel_val[blk * TOPK_MAX + k] = s_sel_val[k];
        }
        pend_r = r;
        pend_n = cnt;
      } else {
        // order by (value desc, id asc): every selected entry counts the entries
        // that precede it (<= 256 entries, one pass, broadcast LDS reads)
        int32_t* oid = A.out_ids + r * (int64_t)K;
        double* osc = A.out_scores + r * (int64_t)K;
        {
          // G threads per entry (4 while cnt <= BLOCK / 4, then 2, then 1; more
          // entries than threads take several passes), partial counts summed with lane shuffles
          const int G = cnt <= BLOCK / 4 ? 4 : cnt <= BLOCK / 2 ? 2 : 1;
          for (int i0 = 0; i0 < cnt; i0 += BLOCK / G) {
            const int i = i0 + tid / G, sub = tid % G;
            int rank = 0;
            double vi = 0.0;
            int32_t ii = 0;
            if (i < cnt) {
              vi = s_sel_val[i];
              ii = s_sel_id[i];
  #pragma unroll 4
              for (int j = sub; j < cnt; j += G) {
                const double vj = s_sel_val[j];
                rank += (vj > vi) || (vj == vi && s_sel_id[j] < ii);
              }
            }
            for (int o = 1; o < G; o <<= 1) rank += __shfl_xor(rank, o, 64);
            if (i < cnt && sub == 0 && rank < K) {
              oid[rank] = ii;
              osc[rank] = vi;
            }
          }
        }
        for (int k = min(cnt, K) + tid; k < K; k += BLOCK) {
          oid[k] = -1;
          osc[k] = 0.0;
        }
      }
    }
    __syncthreads();
    mark(9);
    // re-zero the accumulator for the next source
    if (LDS_ROW) {
      for (int t = tid; t < n; t += BLOCK) s_row[t] = 0.0;
    } else {
      for (int j = tid; j < NL; j += BLOCK) {  // occupied slots were compacted to [0, NL)
        s_hval[j] = 0.0;
        s_hkey[j] = -1;
      }
      if (regsel) {  // this thread's own occupied slots
#pragma unroll
        for (int i = 0; i < SPT; ++i)
          if (vv[i] > 0.0) {
            s_hval[tid + i * BLOCK] = 0.0;
            s_hkey[tid + i * BLOCK] = -1;
          }
      }
    }
    __syncthreads();
    if (tid == 0) {
      s_ntouch = 0;
      s_hcount = 0;
      s_hdone = 0;
    }
    if (APPEND && tid < 64) s_pcur[tid] = 0;
    __syncthreads();
    mark(4);
    if (PIPE) cur ^= 1;
  }
  if (defer && pend_r >= 0 && tid >= BLOCK - 64) deferred_topk();  // the workgroup's last source

  if (kGwDiag && A.phase && tid == 0)
    for (int k = 0; k < 15; ++k) atomicAdd(&A.phase[k], s_ph[k]);
  if (kGwDiag && A.phase && tid == 64) {
    atomicAdd(&A.phase[15], w1_walk);
    atomicAdd(&A.phase[16], w1_wait);
  }
  // statistics
  long long e = block_sum<long long, NW>(my_ext, s_red);
  long long u = block_sum<long long, NW>(my_upd, s_red);
  long long w = block_sum<long long, NW>(my_walk, s_red);
  if (tid == 0 && A.stats) {
    atomicAdd((unsigned long long*)&A.stats[0], (unsigned long long)e);
    atomicAdd((unsigned long long*)&A.stats[1], (unsigned long long)u);
    atomicMax(&A.stats[2], my_maxf);
    atomicAdd((unsigned long long*)&A.stats[3], (unsigned long long)w);
  }
}

template <int STEP, int MODE>
__global__ void __launch_bounds__(TS_BLOCK) k_topsim(TsArgs A) {
  topsim_body<STEP, MODE>(A);
}
// two workgroups per CU (<= 72 KB dynamic LDS, <= 128 VGPRs): small dense rows and the 6144-slot hash
template <int STEP, int MODE>
__global__ void __launch_bounds__(TS_BLOCK) __attribute__((amdgpu_waves_per_eu(4, 4))) k_topsim_2wg(TsArgs A) {
  topsim_body<STEP, MODE>(A);
}

// pipelined TopSim_singleSample (hash accumulator, two workgroups per CU)
template <int STEP>
__global__ void __launch_bounds__(TS_BLOCK) __attribute__((amdgpu_waves_per_eu(4, 4))) k_topsim_pipe(TsArgs A) {
  topsim_body<STEP, 2, TS_BLOCK, true>(A);
}

// pipelined, dense LDS row over 72 KB (one workgroup per CU)
template <int STEP>
__global__ void __launch_bounds__(TS_BLOCK) k_topsim_pipe_row(TsArgs A) {
  topsim_body<STEP, 0, TS_BLOCK, true>(A);
}

template <typename T>
int ws_alloc(gw_graph* g, T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) count = 1;
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (size_t)count);
  if (e != hipSuccess) {
    g->err = std::string("hipMalloc(workspace ") + std::to_string(sizeof(T) * (size_t)count) + " B): " + hipGetErrorString(e);
    *p = nullptr;
    return GW_ERR_NOMEM;
  }
  return GW_OK;
}

__global__ void k_ts_ent(gw_dev_graph G, gw_ts_ent* __restrict__ ent) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= G.nnz) return;
  const int32_t x = G.nbrs[e];
  gw_ts_ent v;
  v.x = x;
  v.d = G.deg[x];
  v.off = G.offsets[x];
  ent[e] = v;
}

template <typename T>
void ws_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

constexpr size_t TS_2WG_LDS = 72 * 1024;  // dynamic LDS that still lets two workgroups share a CU

template <int STEP, int MODE, bool TWO>
hipError_t launch_step(const TsArgs& A, int blocks, size_t lds, hipStream_t s) {
  const void* fn = TWO ? (const void*)k_topsim_2wg<STEP, MODE> : (const void*)k_topsim<STEP, MODE>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (TWO)
    k_topsim_2wg<STEP, MODE><<<blocks, TS_BLOCK, lds, s>>>(A);
  else
    k_topsim<STEP, MODE><<<blocks, TS_BLOCK, lds, s>>>(A);
  return hipGetLastError();
}

template <int STEP>
hipError_t launch_mode(int mode, bool pipe, const TsArgs& A, int blocks, size_t lds, hipStream_t s) {
  if (mode == 2 && pipe) {
    hipError_t e = hipFuncSetAttribute((const void*)k_topsim_pipe<STEP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    k_topsim_pipe<STEP><<<blocks, TS_BLOCK, lds, s>>>(A);
    return hipGetLastError();
  }
  if (mode == 0 && pipe) {
    hipError_t e = hipFuncSetAttribute((const void*)k_topsim_pipe_row<STEP>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    k_topsim_pipe_row<STEP><<<blocks, TS_BLOCK, lds, s>>>(A);
    return hipGetLastError();
  }
  if (mode == 2) return launch_step<STEP, 2, true>(A, blocks, lds, s);
  if (mode == 1) return launch_step<STEP, 1, false>(A, blocks, lds, s);
  return lds <= TS_2WG_LDS ? launch_step<STEP, 0, true>(A, blocks, lds, s) : launch_step<STEP, 0, false>(A, blocks, lds, s);
}

// the kernel launch_mode() dispatches (gw_topsim_kernel_attrs)
template <int STEP>
const void* kernel_fn(int mode, bool pipe, size_t lds) {
  if (mode == 2 && pipe) return (const void*)k_topsim_pipe<STEP>;
  if (mode == 0 && pipe) return (const void*)k_topsim_pipe_row<STEP>;
  if (mode == 2) return (const void*)k_topsim_2wg<STEP, 2>;
  if (mode == 1) return (const void*)k_topsim<STEP, 1>;
  return lds <= TS_2WG_LDS ? (const void*)k_topsim_2wg<STEP, 0> : (const void*)k_topsim<STEP, 0>;
}

const void* kernel_fn(int step, int mode, bool pipe, size_t lds) {
  switch (step) {
    case 1: return kernel_fn<1>(mode, pipe, lds);
    case 2: return kernel_fn<2>(mode, pipe, lds);
    case 3: return kernel_fn<3>(mode, pipe, lds);
    case 4: return kernel_fn<4>(mode, pipe, lds);
    case 5: return kernel_fn<5>(mode, pipe, lds);
    case 6: return kernel_fn<6>(mode, pipe, lds);
    case 7: return kernel_fn<7>(mode, pipe, lds);
    case 8: return kernel_fn<8>(mode, pipe, lds);
    default: return nullptr;
  }
}

hipError_t launch(int step, int mode, bool pipe, const TsArgs& A, int blocks, size_t lds, hipStream_t s) {
  switch (step) {
    case 1: return launch_mode<1>(mode, pipe, A, blocks, lds, s);
    case 2: return launch_mode<2>(mode, pipe, A, blocks, lds, s);
    case 3: return launch_mode<3>(mode, pipe, A, blocks, lds, s);
    case 4: return launch_mode<4>(mode, pipe, A, blocks, lds, s);
    case 5: return launch_mode<5>(mode, pipe, A, blocks, lds, s);
    case 6: return launch_mode<6>(mode, pipe, A, blocks, lds, s);
    case 7: return launch_mode<7>(mode, pipe, A, blocks, lds, s);
    case 8: return launch_mode<8>(mode, pipe, A, blocks, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// Does the pipelined hash-mode kernel pay above kPipeMaxSample?  Its wave 0
// alone builds the next source's enumerated levels while seven waves walk the
// current one, so it pays while the enumerated part is small next to the
// walkers.  That part is deterministic (TopSim_singleSample.java:99-116: a
// path whose mass reaches its degree enumerates every neighbour with
// mass/degree), so the host replays it for 64 strided non-isolated sources:
// E = enumerated path extensions, W = walker steps (ceil(mass) walkers of a
// node with mass < degree at level l take 2*STEP - l steps).  W/E: P10M 35
// (SAMPLE 1000, STEP 3; the pipeline -7.1%) and 53 (SAMPLE 10000, STEP 5),
// lshrank arxiv 5.5-8 (levels of thousands of nodes per source at SAMPLE >=
// 2500), blog 41-85.
static bool pipe_pays_large_sample(const gw_graph* g, int sample, int step) {
  const int64_t n = g->n;
  if (n <= 0 || (int64_t)g->offsets.size() != n + 1) return false;
  const int L = 2 * step;
  std::vector<int32_t> src;
  for (int64_t v = 0; v < n; ++v)
    if (g->offsets[v + 1] > g->offsets[v]) src.push_back((int32_t)v);
  if (src.empty()) return false;
  double E = 0.0, W = 0.0;
  const int ns = (int)std::min<size_t>(64, src.size());
  std::vector<std::pair<int32_t, double>> lvl, nxt;
  for (int k = 0; k < ns; ++k) {
    lvl.assign(1, {src[(size_t)k * (src.size() - 1) / std::max(ns - 1, 1)], (double)sample});
    for (int l = 0; l < L && !lvl.empty(); ++l) {
      nxt.clear();
      for (const auto& vm : lvl) {
        const int64_t b = g->offsets[vm.first], e = g->offsets[vm.first + 1];
        const int64_t d = e - b;
        if (d == 0) continue;
        if (vm.second >= (double)d) {
          for (int64_t j = b; j < e; ++j) nxt.push_back({g->nbrs[j], vm.second / (double)d});
        } else {
          W += std::ceil(vm.second) * (double)(L - l);
        }
        if (nxt.size() > ((size_t)1 << 22)) return false;  // huge enumerated levels: keep the workgroup build
      }
      E += (double)nxt.size();
      lvl.swap(nxt);
    }
  }
  return W >= 16.0 * std::max(E, 1.0);
}

// -DGW_DIAG builds only: GW_DIAG_TS_PIPE_MAX=N runs the pipelined hash-mode
// kernel up to SAMPLE N instead of kPipeMaxSample (A/B knob; -1: no override)
static int diag_pipe_max() {
  const char* v = GW_DIAG_ENV("GW_DIAG_TS_PIPE_MAX");
  return v ? std::atoi(v) : -1;
}

int gw_dev_topsim_prepare(gw_graph* g, int variant, int sample, int step, int topk) {
  if (g->device < 0) {
    g->err = "graph is not on a device (call gw_graph_to_device)";
    return GW_ERR_STATE;
  }
  if (step < 1 || step > 8) {
    g->err = "step must be in [1, 8]";
    return GW_ERR_UNSUPPORTED;
  }
  if (sample < 1) {
    g->err = "sample must be >= 1";
    return GW_ERR_INVALID;
  }
  if (topk < 0 || topk > TOPK_MAX) {
    g->err = "topk must be in [0, 256]";
    return GW_ERR_UNSUPPORTED;
  }
  GW_HIP_TRY(hipSetDevice(g->device));
  gw_topsim_ws& t = g->ts;
  ws_free(t.lvl_vertex);
  ws_free(t.lvl_parent);
  ws_free(t.lvl_deg);
  ws_free(t.lvl_off);
  ws_free(t.lvl_mass);
  ws_free(t.child_off);
  ws_free(t.spawn_node);
  ws_free(t.spawn_level);
  ws_free(t.spawn_first);
  ws_free(t.spawn_mass);
  ws_free(t.acc_row);
  ws_free(t.ov_list);
  ws_free(t.touched);
  ws_free(t.app);
  ws_free(t.claim);
  ws_free(t.redo);
  ws_free(t.enum_tgt);
  ws_free(t.enum_val);
  ws_free(t.dsel_id);
  ws_free(t.dsel_val);
  ws_free(t.src_counter);
  ws_free(t.error_flag);
  const int64_t n = g->n;
  const int L = 2 * step;
  int64_t level_cap, spawn_cap;
  if (variant == GW_TOPSIM_SINGLE_SAMPLE) {
    level_cap = (int64_t)sample + 1;  // enumerated nodes carry mass >= 1
    spawn_cap = (int64_t)sample + 1;
  } else if (variant == GW_TOPSIM_ENUMERATE) {
    level_cap = std::max<int64_t>((int64_t)sample + 1, 1 << 20);
    spawn_cap = 1;
  } else if (variant == GW_TOPSIM_SINGLE_RW) {
    level_cap = 1;
    spawn_cap = 1;
  } else {
    g->err = "unknown TopSim variant";
    return GW_ERR_INVALID;
  }
  bool lds_row = n * 8 <= LDS_ROW_MAX_BYTES;
  int mode = lds_row ? 0 : 2;
  if (const char* hm = GW_DIAG_ENV("GW_DIAG_TS_HASH")) {  // A/B knob: force the 8192- (1) or 6144-slot (2) hash
    if (hm[0] == '1' || hm[0] == '2') {
      mode = hm[0] - '0';
      lds_row = false;
    }
  }
  // hash mode: HBM overflow table per workgroup (power of two) beyond the
  // 6144 keys the LDS table holds; distinct targets per source are bounded by
  // min(n, pair updates <= ~3*STEP*SAMPLE)
  int64_t touch_cap = 1;
  if (!lds_row) {
    const int64_t want = std::max<int64_t>(1 << 14, std::min<int64_t>(2 * n, 4LL * step * sample));
    touch_cap = 1;
    while (touch_cap < want) touch_cap <<= 1;
  }
  // TopSim_singleSample with the hash accumulator runs pipelined (k_topsim_pipe):
  // two level / spawner buffers per workgroup plus the enumerated nodes'
  // recorded pair updates (<= STEP even levels of level_cap nodes)
  // (wave 0 alone expands the enumerated levels: worth it while they are
  // small next to the walkers — P10M, SAMPLE 1000: ~130 enumerated nodes and
  // ~1,060 walkers per source — not for SAMPLE in the thousands on low-degree
  // graphs, whose levels reach thousands of nodes; above kPipeMaxSample the
  // host replay of the enumerated part decides, pipe_pays_large_sample)
  // The dense LDS row over 72 KB (one workgroup per CU, e.g. blog) runs
  // pipelined at any SAMPLE: its single workgroup otherwise leaves the CU idle
  // of walker reads during every level / output phase (blog, SAMPLE 10000:
  // 10.32 vs 10.52 ms, profiles/r04/ts_knob_ab_defer_order_pipe_row.jsonl).
  const int64_t pipe_max = diag_pipe_max() >= 0 ? diag_pipe_max() : kPipeMaxSample;
  bool pipe = variant == GW_TOPSIM_SINGLE_SAMPLE &&
              ((mode == 2 && (sample <= pipe_max ||
                              (diag_pipe_max() < 0 && pipe_pays_large_sample(g, sample, step)))) ||
               (mode == 0 && (size_t)n * 8 > TS_2WG_LDS));
  if (const char* np = GW_DIAG_ENV("GW_DIAG_TS_NOPIPE"))  // A/B knob: the unpipelined kernel
    if (np[0] == '1') pipe = false;
  t.diag_pipe = diag_pipe_max();
  const int64_t nb = pipe ? 2 : 1;
  const int64_t enum_cap = pipe ? (int64_t)step * level_cap : 1;
  // append-and-reduce buffers (pipelined hash mode): two of app_cap 16 B
  // entries per workgroup; a source whose pair-update bound is <= app_cap uses them
  const int64_t app_cap = (pipe && !lds_row) ? touch_cap / 2 : 0;
  const int64_t per_block = nb * ((int64_t)(L + 1) * level_cap * 20 + spawn_cap * 20 + 4) + 2 * level_cap * 8 +
                            (level_cap + 1) * 4 + (pipe ? 2 * enum_cap * 12 : 0) +
                            (lds_row ? 0 : touch_cap * 28) + (pipe ? TOPK_MAX * 12 : 0) + app_cap * 32 +
                            (app_cap > 0 ? touch_cap * 4 : 0);
  int dev_cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, g->device) == hipSuccess) dev_cus = prop.multiProcessorCount;
  const int64_t budget = (int64_t)16 << 30;  // 16 GB of the 288 GB HBM
  int64_t blocks = std::min<int64_t>(4 * dev_cus, budget / std::max<int64_t>(per_block, 1));  // persistent
  if (variant == GW_TOPSIM_ENUMERATE) blocks = std::min<int64_t>(blocks, dev_cus);
  if (blocks < 1) {
    g->err = "TopSim workspace exceeds the 16 GB budget";
    return GW_ERR_CAPACITY;
  }
  int rc;
  if ((rc = ws_alloc(g, &t.lvl_vertex, blocks * nb * (L + 1) * level_cap)) ||
      (rc = ws_alloc(g, &t.lvl_parent, blocks * nb * (L + 1) * level_cap)) ||
      (rc = ws_alloc(g, &t.lvl_deg, blocks * nb * (L + 1) * level_cap)) ||
      (rc = ws_alloc(g, &t.lvl_off, blocks * nb * (L + 1) * level_cap)) ||
      (rc = ws_alloc(g, &t.lvl_mass, blocks * 2 * level_cap)) ||
      (rc = ws_alloc(g, &t.child_off, blocks * (level_cap + 1))) ||
      (rc = ws_alloc(g, &t.spawn_node, blocks * nb * spawn_cap)) ||
      (rc = ws_alloc(g, &t.spawn_level, blocks * nb * spawn_cap)) ||
      (rc = ws_alloc(g, &t.spawn_first, blocks * nb * (spawn_cap + 1))) ||
      (rc = ws_alloc(g, &t.spawn_mass, blocks * nb * spawn_cap)) ||
      (rc = ws_alloc(g, &t.enum_tgt, blocks * 2 * enum_cap)) ||
      (rc = ws_alloc(g, &t.enum_val, blocks * 2 * enum_cap)) ||
      (rc = ws_alloc(g, &t.touched, blocks * touch_cap)) ||
      (rc = ws_alloc(g, &t.dsel_id, pipe ? blocks * TOPK_MAX : 1)) ||
      (rc = ws_alloc(g, &t.dsel_val, pipe ? blocks * TOPK_MAX : 1)) ||
      (rc = ws_alloc(g, &t.src_counter, 1)) || (rc = ws_alloc(g, &t.error_flag, 1)))
    return rc;
  if (!t.ent && g->nnz > 0) {  // slot entries {x, deg(x), offsets[x]}: one random line per path extension
    if ((rc = ws_alloc(g, &t.ent, g->nnz))) return rc;
    k_ts_ent<<<(unsigned)((g->nnz + 255) / 256), 256>>>(g->d, t.ent);
    GW_HIP_TRY(hipGetLastError());
  }
  if (!lds_row) {
    // overflow hash: 16 B slots {int32 key (-1 = empty), pad, f64 value}
    if ((rc = ws_alloc(g, &t.acc_row, 2 * blocks * touch_cap)) || (rc = ws_alloc(g, &t.ov_list, blocks * touch_cap)))
      return rc;
    GW_HIP_TRY(hipMemset(t.acc_row, 0, sizeof(double) * 2 * blocks * touch_cap));
    GW_HIP_TRY(hipMemset2D(t.acc_row, 16, 0xFF, 4, (size_t)(blocks * touch_cap)));
  }
  if (app_cap > 0 && ((rc = ws_alloc(g, &t.app, 4 * blocks * app_cap)) || (rc = ws_alloc(g, &t.claim, blocks * touch_cap)) ||
                      (rc = ws_alloc(g, &t.redo, 5))))
    return rc;
  t.variant = variant;
  t.sample = sample;
  t.step = step;
  t.topk = topk;
  t.blocks = (int)blocks;
  t.level_cap = level_cap;
  t.spawn_cap = spawn_cap;
  t.touch_cap = touch_cap;
  t.lds_row = mode;
  t.pipe = pipe ? 1 : 0;
  t.enum_cap = enum_cap;
  t.app_cap = app_cap;
  t.lds_bytes = lds_row ? (size_t)n * 8 : (size_t)(mode == 2 ? TsHash<2>::SLOTS : TsHash<1>::SLOTS) * 12;
  // the kernel launch() dispatches for this workspace (gw_topsim_kernel)
  if (mode == 2 && pipe)
    std::snprintf(t.kernel, sizeof t.kernel, "k_topsim_pipe<%d>", step);
  else if (mode == 0 && pipe)
    std::snprintf(t.kernel, sizeof t.kernel, "k_topsim_pipe_row<%d>", step);
  else if (mode == 2 || (mode == 0 && t.lds_bytes <= TS_2WG_LDS))
    std::snprintf(t.kernel, sizeof t.kernel, "k_topsim_2wg<%d, %d>", step, mode);
  else
    std::snprintf(t.kernel, sizeof t.kernel, "k_topsim<%d, %d>", step, mode);
  GW_HIP_TRY(hipDeviceSynchronize());
  return GW_OK;
}

int gw_dev_topsim(gw_graph* g, int variant, int sample, int step, double C, uint64_t seed,
                  const int32_t* sources_dev, int64_t nsrc, int topk, int32_t* out_ids_dev,
                  double* out_scores_dev, double* out_rows_dev, int64_t* stats_dev, void* stream,
                  const gw_ts_sparse* sparse) {
  gw_topsim_ws& t = g->ts;
  if (t.blocks == 0 || t.variant != variant || t.sample != sample || t.step != step ||
      (out_ids_dev && topk > t.topk) || (kGwDiag && t.diag_pipe != diag_pipe_max())) {
    int rc = gw_dev_topsim_prepare(g, variant, sample, step, std::max(topk, t.topk > 0 ? t.topk : topk));
    if (rc != GW_OK) return rc;
  }
  if (nsrc <= 0) return GW_OK;
  GW_HIP_TRY(hipSetDevice(g->device));
  hipStream_t s = (hipStream_t)stream;
  TsArgs A;
  A.G = g->d;
  A.variant = variant;
  {
    const char* dg = GW_DIAG_ENV("GW_DIAG_TS");
    A.diag = dg ? std::atoi(dg) : 0;
  }
  A.sample = sample;
  A.sampled = (double)sample;
  for (int i = 0; i < 16; ++i) A.cache[i] = 0.0;
  for (int i = 1; i <= step; ++i) A.cache[i] = std::pow(C, (double)i);  // Math.pow(C, i) (:43)
  A.k0 = (uint32_t)seed;
  A.k1 = (uint32_t)(seed >> 32) ^ GW_TAG_TOPSIM;
  A.sources = sources_dev;
  A.nsrc = nsrc;
  A.topk = topk;
  A.out_ids = out_ids_dev;
  A.out_scores = out_scores_dev;
  A.out_rows = out_rows_dev;
  A.sp = sparse ? *sparse : gw_ts_sparse{};
  A.stats = (long long*)stats_dev;
  A.level_cap = t.level_cap;
  A.spawn_cap = t.spawn_cap;
  A.touch_cap = t.touch_cap;
  A.lvl_vertex = t.lvl_vertex;
  A.lvl_parent = t.lvl_parent;
  A.lvl_deg = t.lvl_deg;
  A.lvl_off = t.lvl_off;
  A.ent = t.ent;
  A.lvl_mass = t.lvl_mass;
  A.child_off = t.child_off;
  A.spawn_node = t.spawn_node;
  A.spawn_level = t.spawn_level;
  A.spawn_first = t.spawn_first;
  A.spawn_mass = t.spawn_mass;
  A.ov_vals = t.acc_row;
  A.ov_list = t.ov_list;
  A.enum_tgt = t.enum_tgt;
  A.enum_val = t.enum_val;
  A.enum_cap = t.enum_cap;
  A.dsel_id = t.dsel_id;
  A.dsel_val = t.dsel_val;
  A.touched = t.touched;
  A.app = t.app;
  A.app_cap = t.app ? t.app_cap : 0;
  A.claim = t.claim;
  A.part_entries = 3584;  // ~ the distinct keys one 6144-slot LDS fill takes comfortably
  if (const char* pe = GW_DIAG_ENV("GW_DIAG_TS_PART"))  // A/B knob: partition size bound
    A.part_entries = std::max(256, std::atoi(pe));
  A.pcap_shrink = g->opt.topsim_part_shrink;  // (tests: partitions overflow -> re-run, flag 8)
  if (const char* pc = GW_DIAG_ENV("GW_DIAG_TS_PCAP_SHRINK"))
    A.pcap_shrink = std::min(8, std::max(0, std::atoi(pc)));
  A.heavy_min = 2 * (int64_t)(t.lds_row == 1 ? TsHash<1>::LIMIT : TsHash<2>::LIMIT);
  A.src_counter = t.src_counter;
  A.error_flag = t.error_flag;
  GW_HIP_TRY(hipMemsetAsync(t.src_counter, 0, sizeof(unsigned), s));
  GW_HIP_TRY(hipMemsetAsync(t.error_flag, 0, sizeof(int), s));
  const int blocks = (int)std::min<int64_t>(t.blocks, nsrc);
  // GW_DIAG_TS_PHASES=1: cycles per kernel phase summed over blocks, to stderr (diagnostics only)
  const char* dph = GW_DIAG_ENV("GW_DIAG_TS_PHASES");
  A.phase = nullptr;
  if (dph && dph[0] == '1') {
    GW_HIP_TRY(hipMalloc((void**)&A.phase, 17 * sizeof(unsigned long long)));
    GW_HIP_TRY(hipMemsetAsync(A.phase, 0, 17 * sizeof(unsigned long long), s));
  }
  // a heavy source's key-hash partition can overflow only when one key that
  // missed the LDS table takes thousands of its pair updates (flag 8): the
  // launch is then re-run without the append path, from the caller's
  // counters as they were (stats, sparse-row cursor: saved here)
  const bool may_redo = A.app_cap > 0 && (A.stats || A.sp.cursor);
  if (may_redo) {
    if (A.stats) GW_HIP_TRY(hipMemcpyAsync(t.redo, A.stats, 4 * sizeof(long long), hipMemcpyDeviceToDevice, s));
    if (A.sp.cursor) GW_HIP_TRY(hipMemcpyAsync(t.redo + 4, A.sp.cursor, sizeof(long long), hipMemcpyDeviceToDevice, s));
  }
  int flag = 0;
  for (int pass = 0; pass < 2; ++pass) {
    hipError_t e = launch(step, t.lds_row, t.pipe != 0, A, blocks, t.lds_bytes, s);
    if (e != hipSuccess) {
      g->err = std::string("k_topsim launch: ") + hipGetErrorString(e);
      return GW_ERR_DEVICE;
    }
    GW_HIP_TRY(hipMemcpyAsync(&flag, t.error_flag, sizeof(int), hipMemcpyDeviceToHost, s));
    GW_HIP_TRY(hipStreamSynchronize(s));
    if (!(flag & 8) || A.app_cap == 0) break;
    A.app_cap = 0;  // no heavy sources: every overflow key through the HBM hash
    if (A.stats) GW_HIP_TRY(hipMemcpyAsync(A.stats, t.redo, 4 * sizeof(long long), hipMemcpyDeviceToDevice, s));
    if (A.sp.cursor) GW_HIP_TRY(hipMemcpyAsync(A.sp.cursor, t.redo + 4, sizeof(long long), hipMemcpyDeviceToDevice, s));
    GW_HIP_TRY(hipMemsetAsync(t.src_counter, 0, sizeof(unsigned), s));
    GW_HIP_TRY(hipMemsetAsync(t.error_flag, 0, sizeof(int), s));
  }
  if (A.phase) {
    unsigned long long ph[17];
    GW_HIP_TRY(hipMemcpy(ph, A.phase, sizeof ph, hipMemcpyDeviceToHost));
    (void)hipFree(A.phase);
    const unsigned long long app = ph[10] + ph[11] + ph[12] + ph[13];
    std::fprintf(stderr, "[k_topsim phases, cycles summed over %d blocks] levels %llu walkers %llu output %llu "
                 "(count %llu radix %llu ties %llu collect %llu order %llu) clear %llu (spawn-prefix %llu) "
                 "[count: append-reduce %llu = fold %llu scatter+dump %llu partitions %llu pre %llu] "
                 "[wave 1: walking %llu, waiting at the walker barrier %llu]\n",
                 blocks, ph[0] + 0ull, ph[2], ph[3] + ph[5] + ph[6] + ph[7] + ph[8] + ph[9] + app, ph[5] + app, ph[6],
                 ph[7], ph[8], ph[9], ph[4], ph[1], app, ph[10], ph[11], ph[12], ph[13], ph[15], ph[16]);
  }
  if (flag & 3) {
    g->err = "TopSim frontier exceeded the workspace (level/spawn/touch capacity)";
    return GW_ERR_CAPACITY;
  }
  if (flag & 4) {
    g->err = "sparse rows exceed the output capacity (rows with len -1 did not fit; *used = room needed)";
    return GW_ERR_CAPACITY;
  }
  return GW_OK;
}

extern "C" const char* gw_topsim_kernel(const gw_graph* g) {
  return g ? g->ts.kernel : "";
}

extern "C" int gw_topsim_kernel_attrs(gw_graph* g, int32_t* vgprs, int32_t* scratch_bytes, int32_t* lds_bytes) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  const gw_topsim_ws& t = g->ts;
  if (t.blocks == 0) return gw_fail(g, GW_ERR_STATE, "no TopSim workspace (call gw_topsim_prepare)");
  GW_GUARD_DEVICE(g, g->device);
  const void* fn = kernel_fn(t.step, t.lds_row, t.pipe != 0, t.lds_bytes);
  if (!fn) return gw_fail(g, GW_ERR_STATE, "no TopSim kernel for step %d", t.step);
  hipFuncAttributes fa;
  const hipError_t e = hipFuncGetAttributes(&fa, fn);
  if (e != hipSuccess) return gw_fail(g, GW_ERR_DEVICE, "hipFuncGetAttributes: %s", hipGetErrorString(e));
  if (vgprs) *vgprs = (int32_t)fa.numRegs;
  if (scratch_bytes) *scratch_bytes = (int32_t)fa.localSizeBytes;
  if (lds_bytes) *lds_bytes = (int32_t)(fa.sharedSizeBytes + t.lds_bytes);
  return GW_OK;
}

// ---------------------------------------------------------------------------
// host-buffer conveniences (JNI shim / C++ host / CLI): stage through HBM
// ---------------------------------------------------------------------------
extern "C" int gw_topsim_host(gw_graph* g, int variant, int sample, int step, double C, uint64_t seed,
                              const int32_t* sources, int64_t nsrc, int topk, int32_t* out_ids,
                              double* out_scores, double* out_rows, int64_t* stats) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);  // restores the caller's current device on return
  if (g->device < 0) return gw_fail(g, GW_ERR_STATE, "graph is not on a device");
  if (nsrc < 0 || (nsrc > 0 && !sources) || (!out_rows && (!out_ids || !out_scores)) || topk < 0)
    return gw_fail(g, GW_ERR_INVALID, "bad arguments");
  for (int64_t i = 0; i < nsrc; ++i)
    if (sources[i] < 0 || sources[i] >= g->n) return gw_fail(g, GW_ERR_RANGE, "source %d out of [0,V)", sources[i]);
  GW_HIP_TRY(hipSetDevice(g->device));
  const int64_t n = g->n;
  // chunk so the staging buffers stay under ~1 GB
  const int64_t row_bytes = out_rows ? n * 8 : (int64_t)topk * 12;
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(nsrc, ((int64_t)1 << 30) / std::max<int64_t>(row_bytes, 1)));
  int32_t* d_src = nullptr;
  int32_t* d_ids = nullptr;
  double* d_sc = nullptr;
  double* d_rows = nullptr;
  int64_t* d_st = nullptr;
  int rc = GW_OK;
  if ((rc = ws_alloc(g, &d_src, chunk)) || (rc = ws_alloc(g, &d_st, 4)) ||
      (out_rows ? (rc = ws_alloc(g, &d_rows, chunk * n)) : ((rc = ws_alloc(g, &d_ids, chunk * (int64_t)std::max(topk, 1))) ||
                                                            (rc = ws_alloc(g, &d_sc, chunk * (int64_t)std::max(topk, 1)))))) {
    ws_free(d_src); ws_free(d_st); ws_free(d_rows); ws_free(d_ids); ws_free(d_sc);
    return rc;
  }
  hipError_t e = hipMemset(d_st, 0, 4 * sizeof(int64_t));
  for (int64_t c0 = 0; c0 < nsrc && rc == GW_OK && e == hipSuccess; c0 += chunk) {
    const int64_t cn = std::min(chunk, nsrc - c0);
    e = hipMemcpy(d_src, sources + c0, cn * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) break;
    rc = gw_dev_topsim(g, variant, sample, step, C, seed, d_src, cn, out_rows ? 0 : topk, out_rows ? nullptr : d_ids,
                       out_rows ? nullptr : d_sc, d_rows, d_st, nullptr);
    if (rc != GW_OK) break;
    if (out_rows) {
      e = hipMemcpy(out_rows + c0 * n, d_rows, cn * n * sizeof(double), hipMemcpyDeviceToHost);
    } else {
      e = hipMemcpy(out_ids + c0 * topk, d_ids, cn * topk * sizeof(int32_t), hipMemcpyDeviceToHost);
      if (e == hipSuccess) e = hipMemcpy(out_scores + c0 * topk, d_sc, cn * topk * sizeof(double), hipMemcpyDeviceToHost);
    }
  }
  if (rc == GW_OK && e == hipSuccess && stats) e = hipMemcpy(stats, d_st, 4 * sizeof(int64_t), hipMemcpyDeviceToHost);
  ws_free(d_src); ws_free(d_st); ws_free(d_rows); ws_free(d_ids); ws_free(d_sc);
  if (rc != GW_OK) return rc;
  if (e != hipSuccess) return gw_fail(g, GW_ERR_DEVICE, "%s", hipGetErrorString(e));
  return GW_OK;
}

// TopSim compute() + Print.printByOrder in one call, Java-exact at any V
// (TopSim_singleSample.java:47-54, Print.java:25-53): sources in batches
// through HBM as sparse rows (gw_topsim_sparse), each batch replayed through
// FixedMaxPQ on the host and appended to path / path.sim.txt in source order.
extern "C" int gw_topsim_write_text(gw_graph* g, int variant, int sample, int step, double C, uint64_t seed,
                                    const int32_t* sources, int64_t nsrc, int topk, const char* path, const char* sep,
                                    int decimals, int64_t* stats) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);
  if (g->device < 0) return gw_fail(g, GW_ERR_STATE, "graph is not on a device");
  if (nsrc < 0 || (nsrc > 0 && !sources) || topk < 0 || !path || decimals < 0 || decimals > 30)
    return gw_fail(g, GW_ERR_INVALID, "bad arguments");
  for (int64_t i = 0; i < nsrc; ++i)
    if (sources[i] < 0 || sources[i] >= g->n) return gw_fail(g, GW_ERR_RANGE, "source %d out of [0,V)", sources[i]);
  const std::string sp_sep = sep ? sep : ",";
  std::string err;
  int rc = gw_write_sim_sparse_impl(path, nullptr, nullptr, nullptr, nullptr, nullptr, 0, g->n, topk, sp_sep,
                                    decimals, false, &err);  // create / truncate both files
  if (rc != GW_OK) return gw_fail(g, rc, "%s", err.c_str());
  GW_HIP_TRY(hipSetDevice(g->device));
  const int64_t n = g->n;
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(nsrc, 65536));
  int64_t cap = std::max<int64_t>(1, std::min<int64_t>(chunk * n, (int64_t)1 << 26));
  int32_t *d_src = nullptr, *d_len = nullptr, *d_ids = nullptr;
  int64_t *d_begin = nullptr, *d_used = nullptr, *d_st = nullptr;
  double* d_sc = nullptr;
  auto release = [&]() {
    ws_free(d_src); ws_free(d_len); ws_free(d_ids); ws_free(d_begin); ws_free(d_used); ws_free(d_st); ws_free(d_sc);
  };
  if ((rc = ws_alloc(g, &d_src, chunk)) || (rc = ws_alloc(g, &d_len, chunk)) || (rc = ws_alloc(g, &d_begin, chunk)) ||
      (rc = ws_alloc(g, &d_used, 1)) || (rc = ws_alloc(g, &d_st, 4)) || (rc = ws_alloc(g, &d_ids, cap)) ||
      (rc = ws_alloc(g, &d_sc, cap))) {
    release();
    return rc;
  }
  int64_t tot_st[4] = {0, 0, 0, 0};
  std::vector<int64_t> h_begin;
  std::vector<int32_t> h_len, h_ids;
  std::vector<double> h_sc;
  hipError_t e = hipSuccess;
  for (int64_t c0 = 0; c0 < nsrc && rc == GW_OK;) {
    const int64_t cn = std::min(chunk, nsrc - c0);
    if ((e = hipMemcpy(d_src, sources + c0, cn * sizeof(int32_t), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemset(d_st, 0, 4 * sizeof(int64_t))) != hipSuccess || (e = hipMemset(d_used, 0, sizeof(int64_t))) != hipSuccess)
      break;
    gw_ts_sparse sp;
    sp.cap = cap;
    sp.begin = d_begin;
    sp.len = d_len;
    sp.ids = d_ids;
    sp.scores = d_sc;
    sp.cursor = reinterpret_cast<unsigned long long*>(d_used);
    rc = gw_dev_topsim(g, variant, sample, step, C, seed, d_src, cn, 0, nullptr, nullptr, nullptr, d_st, nullptr, &sp);
    int64_t used = 0;
    if ((e = hipMemcpy(&used, d_used, sizeof(int64_t), hipMemcpyDeviceToHost)) != hipSuccess) break;
    if (rc == GW_ERR_CAPACITY && used > cap) {  // the rows need more room: grow and redo this batch
      cap = used + used / 8;
      ws_free(d_ids);
      ws_free(d_sc);
      if ((rc = ws_alloc(g, &d_ids, cap)) || (rc = ws_alloc(g, &d_sc, cap))) break;
      continue;
    }
    if (rc != GW_OK) break;
    int64_t st[4];
    h_begin.resize(cn);
    h_len.resize(cn);
    h_ids.resize(std::max<int64_t>(used, 1));
    h_sc.resize(std::max<int64_t>(used, 1));
    if ((e = hipMemcpy(st, d_st, sizeof st, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(h_begin.data(), d_begin, cn * sizeof(int64_t), hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(h_len.data(), d_len, cn * sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess ||
        (used > 0 && (e = hipMemcpy(h_ids.data(), d_ids, used * sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess) ||
        (used > 0 && (e = hipMemcpy(h_sc.data(), d_sc, used * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess))
      break;
    tot_st[0] += st[0];
    tot_st[1] += st[1];
    tot_st[2] = std::max(tot_st[2], st[2]);
    tot_st[3] += st[3];
    rc = gw_write_sim_sparse_impl(path, h_begin.data(), h_len.data(), h_ids.data(), h_sc.data(), sources + c0, cn, n,
                                  topk, sp_sep, decimals, true, &err);
    if (rc != GW_OK) {
      gw_fail(g, rc, "%s", err.c_str());
      break;
    }
    c0 += cn;
  }
  release();
  if (rc != GW_OK) return rc;
  if (e != hipSuccess) return gw_fail(g, GW_ERR_DEVICE, "%s", hipGetErrorString(e));
  if (stats)
    for (int k = 0; k < 4; ++k) stats[k] = tot_st[k];
  return GW_OK;
}
