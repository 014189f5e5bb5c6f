// Naive (all-pairs) SimRank on gfx950 — the TopSim ground-truth generator.
//
// Reference: DeepSim/TopSimAll/src/simrank/SimRank.java
//   ctor        :21-31  sim = tempSim = I (n x n doubles)
//   compute     :36-57  STEP rounds of tempSim[i][j] = sim(i,j) for i<j,
//                       mirrored, then copied back to sim
//   postProcess :62-65  sim[i][i] = 0
//   sim(v,w)    :67-77  1 if v==w; 0 if deg(v)==0 or deg(w)==0; else
//                       C * (sum over neighbour pairs of sim) / (deg(v)*deg(w))
// The neighbour lists are the Java multigraph's (Graph.java: duplicates kept),
// so the double loop is the count-matrix product (A S A^T)[v][w].
//
// Design: the graph is undirected (A = A^T) and S is symmetric, so one round
// is two sparse row-gather passes with a dense fp64 matrix in HBM:
//   pass 1 (k_sr_gather<.., false>): U[j][i] = sum_{b in N(j)} S[i][b]   (U = A S)
//   pass 2 (k_sr_gather<.., true >): S'[i][j] = C * sum_{b in N(j)} U[i][b] / (d_i d_j)
//                                     for j > i, written to [i][j] and [j][i]
// Both passes run on the compact graph of non-isolated vertices (m <= n);
// each workgroup owns one row i: the row is staged in LDS (when m*8 fits),
// the adjacency is streamed as a row-padded entry list (4 B/entry, every row
// starts on a 16-entry chunk, padding reads a zero slot; 16 entries = 64 B
// per lane, prefetched one chunk ahead), so a lane's 16 entries belong to
// ONE row: the per-row sums are a plain 16-term lane sum + a DPP segmented
// scan over the wave's 64 chunk partials, with the row's carry kept in
// registers.  Work per pass = n * nnz gathered doubles (pass 2 about half of
// it) plus the padding (blog: +12.6%).  The reduction order differs
// from the Java double loop (fp64 reassociation only, ~1e-16 relative);
// each S'[i][j] is computed once and mirrored, so S stays exactly symmetric.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "gw_device_common.h"

namespace {

constexpr int SR_BLOCK = 1024;
constexpr int SR_WAVES = SR_BLOCK / 64;
constexpr int SR_K = 16;                         // adjacency entries per lane per chunk
constexpr int SR_CHUNK = 64 * SR_K;              // entries per wave per chunk
constexpr int64_t SR_LDS_BYTES = 152 * 1024;     // dynamic LDS per workgroup (input row + window)
constexpr int64_t SR_MIN_WIN = 2048;             // smallest output window (rows)

// The passes run over the compact graph of the m non-isolated vertices
// (isolated rows/columns of SimRank are 0): compact ids are consecutive, so
// the k-th head flag of the stream IS row k and a row's degree is its
// segment length — no per-row lookups inside the loop.
struct SrArgs {
  int64_t m;
  const int64_t* off;     // [m+1] compact CSR offsets (degrees)
  const int64_t* poff;    // [m+1] row starts in the padded stream (multiples of SR_K)
  const uint32_t* ent;    // [poff[m] + SR_CHUNK] byte offset (8 * compact neighbour) into a row; padding 8 * m
  const uint16_t* heads;  // [(poff[m] + SR_CHUNK) / 16] bit 0 of word g: chunk g (entries 16g..16g+15) starts a row
  double C;
};

__global__ void k_sr_identity(int64_t n, double* __restrict__ S) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v < n) S[v * n + v] = 1.0;  // SimRank.java:27-30
}

__global__ void k_sr_zero_diag(int64_t n, double* __restrict__ S) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (v < n) S[v * n + v] = 0.0;  // postProcess, SimRank.java:62-65
}

// out[rows[a]][rows[b]] = X[a][b] (out pre-zeroed: isolated rows/cols are 0)
__global__ void k_sr_expand(int64_t m, int64_t n, const int32_t* __restrict__ rows, const double* __restrict__ X,
                            double* __restrict__ out) {
  const int64_t a = blockIdx.y;
  const int64_t ra = rows[a];
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < m; b += (int64_t)gridDim.x * blockDim.x)
    out[ra * n + rows[b]] = X[a * m + b];
}

// first row r in [lo, hi] with off[r] >= e (off is non-decreasing)
__device__ __forceinline__ int64_t first_row_at(const int64_t* __restrict__ off, int64_t lo, int64_t hi, int64_t e) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (off[mid] < e)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// DPP lane moves (gfx9 wave64 controls): row_shr:d = 0x110+d, row_bcast:15 =
// 0x142, row_bcast:31 = 0x143, wave_shr:1 = 0x138.  Invalid sources read 0.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROW_MASK, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROW_MASK, 0xF, true);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xF, true);
}

// Segmented inclusive sum over the wave: lane l sums lanes [seg_start(l), l].
__device__ __forceinline__ double seg_scan(double S, int lane, int seg) {
  const int r = lane & 15;
  double t;
  t = dpp_f64<0x111>(S); if (r >= 1 && lane - 1 >= seg) S += t;
  t = dpp_f64<0x112>(S); if (r >= 2 && lane - 2 >= seg) S += t;
  t = dpp_f64<0x114>(S); if (r >= 4 && lane - 4 >= seg) S += t;
  t = dpp_f64<0x118>(S); if (r >= 8 && lane - 8 >= seg) S += t;
  t = dpp_f64<0x142, 0xA>(S); if ((lane & 16) && (lane & ~15) - 1 >= seg) S += t;
  t = dpp_f64<0x143, 0xC>(S); if (lane >= 32 && 31 >= seg) S += t;
  return S;
}

// One workgroup per row i of `src`.  The rows j are processed in windows of
// `win` rows whose totals land in an LDS window (no global stores inside
// the entry loop, so the one-chunk-ahead prefetch is never held up behind
// them); each wave owns a row-aligned slice of the window's entries and
// walks it 512 entries (8 per lane) at a time:
//   lane-local sequential sums -> wave segmented scan (DPP) of the lanes'
//   trailing segments -> each lane re-walks its entries from its carry-in
//   and writes a row total when the next row starts (or the slice ends).
// Flush: pass 1 writes U[j][i] (column i of U); pass 2 scales by
// C / (deg_i * deg_j) and writes S'[i][j] and S'[j][i].
template <bool LDS_ROW, bool PASS2>
__global__ void __launch_bounds__(SR_BLOCK) k_sr_gather(SrArgs A, const double* __restrict__ src,
                                                        double* __restrict__ dst, int last, int win) {
  extern __shared__ double lds[];
  const int64_t m = A.m;
  double* const in_row = lds;
  double* const out_win = LDS_ROW ? lds + m + 1 : lds;
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int32_t di = (int32_t)(A.off[i + 1] - A.off[i]);
  if (PASS2 && threadIdx.x == 0) dst[i * m + i] = last ? 0.0 : 1.0;  // tempSim[i][i] stays 1
  const double* row = src + i * m;
  if (LDS_ROW) {
    for (int64_t b = threadIdx.x; b < m; b += SR_BLOCK) in_row[b] = row[b];
    if (threadIdx.x == 0) in_row[m] = 0.0;  // the padding entries' slot
  }
  const uint32_t pad_off = (uint32_t)m * 8u;
  const uint64_t below_incl = (lane == 63) ? ~0ull : ((2ull << lane) - 1);

  for (int64_t j0 = PASS2 ? i + 1 : 0; j0 < m; j0 += win) {
    const int64_t j1 = min(m, j0 + (int64_t)win);
    __syncthreads();  // in_row staged / previous window flushed
    {
      const int64_t e_lo = A.poff[j0], tot = A.poff[j1] - e_lo;
      const int64_t t0 = e_lo + tot * wave / SR_WAVES, t1 = e_lo + tot * (wave + 1) / SR_WAVES;
      const int64_t ra = wave == 0 ? j0 : first_row_at(A.poff, j0, j1, t0);
      const int64_t rb = wave == SR_WAVES - 1 ? j1 : first_row_at(A.poff, j0, j1, t1);
      const int64_t eb = A.poff[ra], ee = A.poff[rb];
      if (eb < ee) {
        // eb, ee are row starts: multiples of SR_K, so every lane's chunk lies
        // inside one row and the slice is chunk-aligned
        const uint32_t* ep = A.ent + eb + SR_K * lane;
        const uint16_t* hp = A.heads + eb / SR_K + lane;
        const int pe = (int)(ee - eb);  // slice = chunk positions [0, pe)
        // the slice's first head flag is dropped: its row is cur_row from the start,
        // so every flag seen afterwards closes a row of this slice
        int cur_row = (int)(ra - j0);
        double chunk_carry = 0.0;
        uint4 n[4];
        uint32_t nh;
#pragma unroll
        for (int q = 0; q < 4; ++q) n[q] = *reinterpret_cast<const uint4*>(ep + 4 * q);
        nh = *hp;
        for (int pos = 0; pos < pe; pos += SR_CHUNK) {
          const uint32_t en[SR_K] = {n[0].x, n[0].y, n[0].z, n[0].w, n[1].x, n[1].y, n[1].z, n[1].w,
                                     n[2].x, n[2].y, n[2].z, n[2].w, n[3].x, n[3].y, n[3].z, n[3].w};
          uint32_t fl = nh & 1u;  // this lane's chunk starts a row
          if (pos + SR_CHUNK < pe) {
#pragma unroll
            for (int q = 0; q < 4; ++q) n[q] = *reinterpret_cast<const uint4*>(ep + pos + SR_CHUNK + 4 * q);
            nh = hp[(pos + SR_CHUNK) / SR_K];
          }
          const int p0 = pos + SR_K * lane;
          const bool live = p0 < pe;  // lanes past the slice end add zeros to its last row
          // one row's 16 entries (padding reads the zero slot), summed in entry order
          double p = 0.0;
#pragma unroll
          for (int k = 0; k < SR_K; ++k) {
            double x;
            if (LDS_ROW) {
              x = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(in_row) + en[k]);
            } else {  // the padding offset is one past the row: read a real element, use 0
              const uint32_t o = en[k] < pad_off ? en[k] : 0u;
              x = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(row) + o);
              if (en[k] >= pad_off) x = 0.0;
            }
            p += x;
          }
          if (!live) p = 0.0;
          if (!live || p0 == 0) fl = 0u;
          // heads at or below this lane: v_mbcnt over the head ballot (exclusive
          // count) + this lane's own flag, instead of a 6-step DPP scan
          const uint64_t headmask = __ballot(fl != 0);
          const int incl = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(headmask >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)headmask, 0u)) +
                           (int)fl;
          const int total = __popcll(headmask);
          // lane 0 without a head continues the row of the previous chunk
          if (lane == 0 && fl == 0) p = chunk_carry + p;
          const uint64_t hb = headmask & below_incl;
          const int seg_start = hb ? 63 - __builtin_clzll(hb) : 0;
          const double S = seg_scan(p, lane, seg_start);
          const double prevS = dpp_f64<0x138>(S);  // wave_shr:1
          const int r = cur_row + incl;            // this lane's row
          if (fl) out_win[r - 1] = lane == 0 ? chunk_carry : prevS;  // the previous row is complete
          // the lane holding the slice's last chunk writes that row
          if (live && p0 + SR_K >= pe) out_win[r] = S;
          const uint64_t Sb = __double_as_longlong(S);
          chunk_carry = __longlong_as_double(
              (long long)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(Sb >> 32), 63) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)Sb, 63)));
          cur_row += total;
        }
      }
    }
    __syncthreads();
    const int64_t nrow = j1 - j0;
    for (int64_t t = threadIdx.x; t < nrow; t += SR_BLOCK) {
      const int64_t j = j0 + t;
      const double val = out_win[t];
      if (!PASS2) {
        dst[j * m + i] = val;  // U = A S, stored transposed
      } else {
        // Java int product deg(v)*deg(w) (:76), wrap-around kept
        const int32_t dj = (int32_t)(A.off[j + 1] - A.off[j]);
        const int32_t dd = (int32_t)((uint32_t)di * (uint32_t)dj);
        const double sv = A.C * val / (double)dd;
        dst[i * m + j] = sv;
        dst[j * m + i] = sv;
      }
    }
  }
}

template <bool LDS_ROW, bool PASS2>
hipError_t launch_pass(const SrArgs& A, const double* src, double* dst, int last, int win, hipStream_t s) {
  const size_t lds = ((LDS_ROW ? (size_t)A.m + 1 : 0) + (size_t)win) * sizeof(double);
  hipError_t e = hipFuncSetAttribute((const void*)k_sr_gather<LDS_ROW, PASS2>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  k_sr_gather<LDS_ROW, PASS2><<<(unsigned)A.m, SR_BLOCK, lds, s>>>(A, src, dst, last, win);
  return hipGetLastError();
}

template <typename T>
void sr_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

}  // namespace

void gw_dev_simrank_release(gw_graph* g) {
  sr_free(g->sr_work);
  sr_free(g->sr_x);
  sr_free(g->sr_ent);
  sr_free(g->sr_heads);
  sr_free(g->sr_off);
  sr_free(g->sr_poff);
  sr_free(g->sr_rows);
  g->sr_n = 0;
  g->sr_m = 0;
}

// Compact layout (built once per graph on the host): non-isolated vertices
// in ascending id order, their CSR offsets, and the row-padded stream of
// neighbour ranks (each row starts on a 16-entry chunk; padding = 8 * m, the
// zero slot) with one head bit per chunk.
static int sr_build_layout(gw_graph* g) {
  const int64_t n = g->n;
  std::vector<int32_t> rank((size_t)n, -1), rows;
  std::vector<int64_t> off(1, 0), poff(1, 0);
  rows.reserve((size_t)n);
  for (int64_t v = 0; v < n; ++v) {
    const int64_t d = g->offsets[v + 1] - g->offsets[v];
    if (d > 0) {
      rank[v] = (int32_t)rows.size();
      rows.push_back((int32_t)v);
      off.push_back(g->offsets[v + 1]);
      poff.push_back(poff.back() + (d + SR_K - 1) / SR_K * SR_K);
    }
  }
  const int64_t m = (int64_t)rows.size();
  const int64_t padded = poff.back() + SR_CHUNK;  // + one chunk: the one-ahead prefetch stays in bounds
  std::vector<uint32_t> ent((size_t)padded, (uint32_t)m * (uint32_t)sizeof(double));
  std::vector<uint16_t> heads((size_t)(padded / SR_K), 0);
  for (int64_t r = 0; r < m; ++r) {
    const int64_t v = rows[(size_t)r], b = g->offsets[v], e = g->offsets[v + 1];
    heads[(size_t)(poff[(size_t)r] / SR_K)] = 1;
    for (int64_t k = b; k < e; ++k) ent[(size_t)(poff[(size_t)r] + (k - b))] = (uint32_t)rank[g->nbrs[k]] * (uint32_t)sizeof(double);
  }
  auto up = [&](auto*& dptr, const auto& vec) -> bool {
    const size_t bytes = std::max<size_t>(vec.size() * sizeof(vec[0]), 16);
    if (hipMalloc((void**)&dptr, bytes) != hipSuccess) {
      (void)hipGetLastError();
      dptr = nullptr;
      return false;
    }
    return vec.empty() || hipMemcpy(dptr, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(g->sr_ent, ent) || !up(g->sr_heads, heads) || !up(g->sr_off, off) || !up(g->sr_poff, poff) ||
      !up(g->sr_rows, rows)) {
    g->err = "naive SimRank adjacency layout does not fit in device memory";
    return GW_ERR_NOMEM;
  }
  g->sr_m = m;
  return GW_OK;
}

int gw_dev_simrank_naive(gw_graph* g, double C, int iters, double* sim_dev, void* stream) {
  GW_HIP_TRY(hipSetDevice(g->device));
  const int64_t n = g->n;
  hipStream_t s = (hipStream_t)stream;
  if (g->sr_n != n || !g->sr_ent) {
    gw_dev_simrank_release(g);
    int rc = sr_build_layout(g);
    if (rc != GW_OK) {
      gw_dev_simrank_release(g);
      return rc;
    }
    const int64_t m = g->sr_m;
    const size_t mb = std::max<size_t>((size_t)m * (size_t)m * sizeof(double), 8);
    if (hipMalloc((void**)&g->sr_work, mb) != hipSuccess || (m < n && hipMalloc((void**)&g->sr_x, mb) != hipSuccess)) {
      (void)hipGetLastError();
      gw_dev_simrank_release(g);
      g->err = "naive SimRank workspace (m*m doubles) does not fit in device memory";
      return GW_ERR_NOMEM;
    }
    g->sr_n = n;
  }
  if (n == 0) return GW_OK;
  const int64_t m = g->sr_m;
  double* X = m < n ? g->sr_x : sim_dev;  // compact S (the output itself when nothing is isolated)
  if (m < n) GW_HIP_TRY(hipMemsetAsync(sim_dev, 0, (size_t)n * n * sizeof(double), s));
  if (m > 0) {
    GW_HIP_TRY(hipMemsetAsync(X, 0, (size_t)m * m * sizeof(double), s));
    const unsigned mbk = (unsigned)((m + 255) / 256);
    k_sr_identity<<<mbk, 256, 0, s>>>(m, X);
    GW_HIP_TRY(hipGetLastError());
    SrArgs A{m, g->sr_off, g->sr_poff, g->sr_ent, g->sr_heads, C};
    // input row (+ the padding's zero slot) in LDS when it leaves room for a
    // window of SR_MIN_WIN rows; the handle's simrank_hbm_row option selects
    // the HBM-row variant (same bits; tests compare the two)
    const int64_t cap = SR_LDS_BYTES / (int64_t)sizeof(double);
    const bool lds_row = m + 1 + SR_MIN_WIN <= cap && !g->opt.simrank_hbm_row;
    const int win = (int)std::min<int64_t>(m, lds_row ? cap - m - 1 : cap);
    for (int r = 0; r < iters; ++r) {  // while (r++ < STEP), SimRank.java:38
      const int last = r == iters - 1;
      hipError_t e = lds_row ? launch_pass<true, false>(A, X, g->sr_work, 0, win, s)
                             : launch_pass<false, false>(A, X, g->sr_work, 0, win, s);
      if (e == hipSuccess)
        e = lds_row ? launch_pass<true, true>(A, g->sr_work, X, last, win, s)
                    : launch_pass<false, true>(A, g->sr_work, X, last, win, s);
      GW_HIP_TRY(e);
    }
    if (iters <= 0) {
      k_sr_zero_diag<<<mbk, 256, 0, s>>>(m, X);
      GW_HIP_TRY(hipGetLastError());
    }
    if (m < n) {
      dim3 grid((unsigned)std::min<int64_t>((m + 255) / 256, 64), (unsigned)m);
      k_sr_expand<<<grid, 256, 0, s>>>(m, n, g->sr_rows, X, sim_dev);
      GW_HIP_TRY(hipGetLastError());
    }
  }
  return GW_OK;
}

extern "C" int gw_simrank_naive_host(gw_graph* g, double C, int iters, double* sim) {
  if (!g) return gw_fail(nullptr, GW_ERR_INVALID, "NULL handle");
  GW_GUARD_DEVICE(g, g->device);  // restores the caller's current device on return
  if (g->device < 0) return gw_fail(g, GW_ERR_STATE, "graph is not on a device");
  if (g->directed) return gw_fail(g, GW_ERR_UNSUPPORTED, "naive SimRank needs an undirected graph");
  if (g->n > 0 && !sim) return gw_fail(g, GW_ERR_INVALID, "bad arguments");
  if (iters < 0) return gw_fail(g, GW_ERR_INVALID, "iters must be >= 0");
  GW_HIP_TRY(hipSetDevice(g->device));
  const int64_t n = g->n;
  if (n == 0) return GW_OK;
  double* d_sim = nullptr;
  if (hipMalloc((void**)&d_sim, (size_t)n * n * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    return gw_fail(g, GW_ERR_NOMEM, "n*n result does not fit in device memory");
  }
  int rc = gw_dev_simrank_naive(g, C, iters, d_sim, nullptr);
  hipError_t e = hipSuccess;
  if (rc == GW_OK) e = hipMemcpy(sim, d_sim, (size_t)n * n * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(d_sim);
  if (rc != GW_OK) return rc;
  if (e != hipSuccess) return gw_fail(g, GW_ERR_DEVICE, "%s", hipGetErrorString(e));
  return GW_OK;
}
