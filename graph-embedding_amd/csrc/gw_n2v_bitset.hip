// node2vec exact second-order sampling with per-edge common-neighbour
// bitsets (GW_N2V_BITSET) — the compressed form of the reference's per-edge
// alias tables.
//
// The reference precomputes, for every directed edge (src -> dst), an alias
// table over sorted N(dst) with weights  w/p (dst_nbr == src), w
// (has_edge(dst_nbr, src)), w/q (otherwise)   (node2vec.py:61-81).
// For unweighted undirected graphs that table is fully described by ONE BIT
// per entry ("dst_nbr is a common neighbour of src and dst") plus the position
// of src in N(dst): 1 bit instead of 12 bytes (q f64 + J), so sum(deg^2) bits
// (R-MAT-20: 8.8 GB) fit in HBM where the reference's tables (7.0e10 x 12 B)
// do not.  A step then samples the three-way mixture exactly:
//
//   Z = 1/p + c + (d - 1 - c)/q,  c = popcount(bitset)
//   r = U*Z < 1/p           -> return to prev
//   r - 1/p < c             -> the floor(r - 1/p)-th common neighbour (row order)
//   otherwise               -> uniform over the d-1-c others (rejection on the
//                              bitset: expected d/(d-1-c) ~ 1 trial)
//
// Per edge slot s = (u -> v):
//   bs_nbr[s] (64 B, one HBM sector): v, d = deg(v), offsets[v] (int64),
//            kp (position of u in N(v)), c, and either the bitset itself
//            (d <= 320, inline) or the word offset of its region
//   region   (d > 320 only) dir[ndir]  cumulative set bits before each
//                       512-bit block (d > 512 only), then
//            bits[ceil(d/32)]  bit k = (N(v)[k] != u) && has_edge(N(v)[k], u)
// The entry chosen by a step carries everything the next step needs, so a
// step into a vertex of degree <= 320 touches ONE random sector (the entry);
// larger degrees add the bitset word (~2 sectors, vs ~7 for rejection).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <string>

#include "gw_device_common.h"

namespace {

constexpr int kB = 256;
constexpr int kBlk = 16;         // words per 512-bit block: regions, directory and bits are block-aligned
constexpr int kDirBits = 512;    // bits per directory block
constexpr int kSmallD = 32;      // thread-per-slot fill up to this degree
constexpr int kStage = 16;

__host__ __device__ __forceinline__ int64_t bs_ndir(int64_t d) { return d > kDirBits ? (d + kDirBits - 1) / kDirBits : 0; }
__host__ __device__ __forceinline__ int64_t bs_round(int64_t w) { return (w + kBlk - 1) / kBlk * kBlk; }
// word offset of the bits inside a region (the directory is padded to a block)
__host__ __device__ __forceinline__ int64_t bs_boff(int64_t d) { return d <= GW_BS_INLINE_BITS ? 0 : bs_round(bs_ndir(d)); }
__host__ __device__ __forceinline__ int64_t bs_words(int64_t d) {
  return d <= GW_BS_INLINE_BITS ? 0 : bs_boff(d) + bs_round((d + 31) / 32);
}

__device__ __forceinline__ int32_t row_of_slot(const int64_t* __restrict__ off, int64_t n, int64_t e) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (off[mid + 1] <= e)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (int32_t)lo;
}

__device__ __forceinline__ bool bs_has_edge(const gw_dev_graph& G, int64_t rb, int64_t re, int32_t key) {
  if (G.bitmap) {
    const uint32_t h = (uint32_t)key * 0x9E3779B1u;
    const uint64_t bit = 16ull * (uint64_t)rb + (((uint64_t)h * (uint64_t)(16 * (re - rb))) >> 32);
    if (!((G.bitmap[bit >> 5] >> (bit & 31)) & 1u)) return false;
  }
  return gw_row_find(G.nbrs, rb, re, key) >= 0;
}

// position of the j-th (0-based) set bit of x (j < popc(x))
__device__ __forceinline__ int word_select(uint32_t x, uint32_t j) {
  int pos = 0;
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    const uint32_t lowc = (uint32_t)__popc(x & ((1u << w) - 1u));
    if (j >= lowc) {
      j -= lowc;
      x >>= w;
      pos += w;
    }
  }
  return pos;
}

__global__ void k_bs_sizes(int64_t nnz, const int32_t* __restrict__ nbrs, const int32_t* __restrict__ deg,
                           uint64_t* __restrict__ sz) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  sz[e] = (uint64_t)bs_words(deg[nbrs[e]]);
}

// thread per slot for small deg(v); larger slots are queued for the wave kernel
__global__ void k_bs_fill_small(gw_dev_graph G, const uint64_t* __restrict__ roff, uint32_t* __restrict__ reg,
                                gw_bs_nbr* __restrict__ bsn, int64_t* __restrict__ big,
                                unsigned long long* __restrict__ nbig) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= G.nnz) return;
  const int32_t v = G.nbrs[e];
  const uint64_t R = roff[e];
  const int64_t vb = G.offsets[v], d = G.offsets[v + 1] - vb;
  gw_bs_nbr en;
  en.x = (uint32_t)v;
  en.kp = 0xFFFFFFFFu;
  en.c = 0;
  en.d = (uint32_t)d;
  en.off_lo = (uint32_t)(uint64_t)vb;
  en.off_hi = (uint32_t)((uint64_t)vb >> 32);
#pragma unroll
  for (int t = 0; t < 10; ++t) en.w[t] = 0;
  if (d > GW_BS_INLINE_BITS) {
    en.w[0] = (uint32_t)R;
    en.w[1] = (uint32_t)(R >> 32);
  }
  if (d > kSmallD) {
    bsn[e] = en;  // c, kp filled by k_bs_fill_wave
    big[atomicAdd(nbig, 1ull)] = e;
    return;
  }
  const int32_t u = row_of_slot(G.offsets, G.n, e);
  const int64_t ub = G.offsets[u], ue = G.offsets[u + 1];
  uint32_t word = 0, c = 0;
  for (int64_t k = 0; k < d; ++k) {
    const int32_t x = G.nbrs[vb + k];
    if (x == u) {
      en.kp = (uint32_t)k;
    } else if (bs_has_edge(G, ub, ue, x)) {
      word |= 1u << (k & 31);
      ++c;
    }
  }
  en.c = c;
  if (gw_bs_is_list(c, (uint32_t)d)) {  // sorted positions, 0xFFFF padded
    uint16_t* lp = reinterpret_cast<uint16_t*>(en.w);
    for (int t = 0; t < 2 * 10; ++t) lp[t] = 0xFFFFu;
    int t = 0;
    for (uint32_t x = word; x; x &= x - 1) lp[t++] = (uint16_t)(__ffs(x) - 1);
  } else {
    en.w[0] = word;  // inline bitset (d <= 32)
  }
  bsn[e] = en;
}

// one wave per large slot: 64 neighbours per ballot
__global__ void k_bs_fill_wave(gw_dev_graph G, const uint64_t* __restrict__ roff, uint32_t* __restrict__ reg,
                               gw_bs_nbr* __restrict__ bsn, const int64_t* __restrict__ big,
                               const unsigned long long* __restrict__ nbig) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t total = (int64_t)*nbig;
  for (int64_t i = wave; i < total; i += nwaves) {
    const int64_t e = big[i];
    const int32_t v = G.nbrs[e];
    const int32_t u = row_of_slot(G.offsets, G.n, e);
    const int64_t vb = G.offsets[v], d = G.offsets[v + 1] - vb;
    const int64_t ub = G.offsets[u], ue = G.offsets[u + 1];
    const bool inl = d <= GW_BS_INLINE_BITS;
    uint32_t* h = inl ? bsn[e].w : reg + roff[e];
    const int64_t ndir = inl ? 0 : bs_ndir(d);
    uint32_t* dir = h;
    uint32_t* bits = h + bs_boff(d);
    uint32_t c = 0;
    int kp_local = -1;
    int my_pos = 0xFFFF;  // lane t < GW_BS_LIST: position of the t-th common neighbour
    for (int64_t base = 0; base < d; base += 64) {
      const int64_t k = base + lane;
      bool bit = false;
      if (k < d) {
        const int32_t x = G.nbrs[vb + k];
        if (x == u)
          kp_local = (int)k;
        else
          bit = bs_has_edge(G, ub, ue, x);
      }
      const unsigned long long m = __ballot(bit);
      {
        // lane t collects the t-th set bit overall when it falls in this ballot
        const int pc = __popcll(m);
        const int r = lane - (int)c;
        int src = 0;
        if (r >= 0 && r < pc) {
          const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
          const int plo = __popc(lo);
          src = r < plo ? word_select(lo, (uint32_t)r) : 32 + word_select(hi, (uint32_t)(r - plo));
        }
        const int got = __shfl((int)k, src, 64);
        if (r >= 0 && r < pc && lane < GW_BS_LIST) my_pos = got;
      }
      if (ndir && (base % kDirBits) == 0 && lane == 0) dir[base / kDirBits] = c;
      if (lane == 0) {
        bits[base / 32] = (uint32_t)m;
        if (base + 32 < d) bits[base / 32 + 1] = (uint32_t)(m >> 32);
      }
      c += (uint32_t)__popcll(m);
    }
    // kp: the lane that saw u
    const unsigned long long km = __ballot(kp_local >= 0);
    int kp = -1;
    if (km) {
      const int src = __ffsll(km) - 1;
      kp = __shfl(kp_local, src, 64);
    }
    if (gw_bs_is_list(c, (uint32_t)d)) {
      __threadfence();  // inline bit words written above by lane 0 land first
      if (lane < GW_BS_LIST) reinterpret_cast<uint16_t*>(bsn[e].w)[lane] = (uint16_t)my_pos;
    } else if (gw_bs_is_ef(c, (uint32_t)d) && lane == 0) {
      // Elias-Fano from the region bits lane 0 wrote above (same thread: visible)
      const int l = gw_bs_ef_l(c, (uint32_t)d);
      const uint32_t U = c + (uint32_t)((d - 1) >> l) + 1;
      uint32_t ef[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      uint32_t idx = 0;
      for (int64_t w = 0; w < (d + 31) / 32; ++w)
        for (uint32_t x = bits[w]; x; x &= x - 1) {
          const uint32_t p = (uint32_t)(32 * w + __ffs(x) - 1);
          const uint32_t up = (p >> l) + idx;  // high part, unary
          ef[up >> 5] |= 1u << (up & 31);
          for (int b = 0; b < l; ++b)
            if ((p >> b) & 1u) ef[(U + idx * l + b) >> 5] |= 1u << ((U + idx * l + b) & 31);
          ++idx;
        }
      for (int t = 0; t < 10; ++t) bsn[e].w[t] = ef[t];
    }
    if (lane == 0) {
      bsn[e].c = c;
      bsn[e].kp = (uint32_t)kp;
    }
  }
}

// j-th set bit among `nw` words held in registers (constant indices only)
template <int NW>
__device__ __forceinline__ int regs_select(const uint32_t (&wd)[NW], uint32_t j) {
  uint32_t x = 0;
  int base = 0;
  bool found = false;
#pragma unroll
  for (int t = 0; t < NW; ++t) {
    const uint32_t pc = (uint32_t)__popc(wd[t]);
    if (!found) {
      if (j < pc) {
        x = wd[t];
        base = 32 * t;
        found = true;
      } else {
        j -= pc;
      }
    }
  }
  return base + word_select(x, j);
}

// j-th set bit of an inline bitset (entry words, 8 B aligned; L2-resident)
__device__ __forceinline__ int64_t inl_select(const uint32_t* __restrict__ w, uint32_t j) {
  uint32_t wd[10];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const uint2 v = reinterpret_cast<const uint2*>(w)[t];
    wd[2 * t] = v.x;
    wd[2 * t + 1] = v.y;
  }
  return regs_select<10>(wd, j);
}

// j-th set bit of a region bitset (c set bits): the 512-bit block comes from
// the directory by interpolation (set bits are spread over the row), then
// the block is read as one 64 B sector and searched in registers
__device__ __forceinline__ int64_t bs_select(const uint32_t* __restrict__ h, int64_t d, uint32_t c, uint32_t j) {
  const int64_t ndir = bs_ndir(d);
  int64_t g = 0;
  if (ndir > 0) {
    g = (int64_t)((uint64_t)j * (uint64_t)ndir / c);
    if (g >= ndir) g = ndir - 1;
    uint32_t lo = h[g];
    uint32_t hi = g + 1 < ndir ? h[g + 1] : c;
    while (lo > j) {
      --g;
      hi = lo;
      lo = h[g];
    }
    while (hi <= j) {
      ++g;
      lo = hi;
      hi = g + 1 < ndir ? h[g + 1] : c;
    }
    j -= lo;
  }
  const uint4* blk = reinterpret_cast<const uint4*>(h + bs_boff(d) + g * kBlk);
  uint32_t wd[kBlk];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint4 v = blk[t];
    wd[4 * t] = v.x;
    wd[4 * t + 1] = v.y;
    wd[4 * t + 2] = v.z;
    wd[4 * t + 3] = v.w;
  }
  return g * kDirBits + regs_select<kBlk>(wd, j);
}

// pl[idx] for a per-lane idx without dynamic register indexing
__device__ __forceinline__ uint32_t pick10(const uint32_t (&pl)[10], uint32_t idx) {
  uint32_t r = 0;
#pragma unroll
  for (int t = 0; t < 10; ++t) r |= pl[t] & (0u - (uint32_t)(idx == (uint32_t)t));
  return r;
}

// ---- Elias-Fano payload ----------------------------------------------------
// The payload words live in registers; dynamic word picks are mask-selects.
// j-th one (ONE) / zero among the payload bits, from bit 0 (the high parts
// come first, so the first c ones and the first U - c zeros are theirs)
template <bool ONE>
__device__ __forceinline__ int ef_select_bit(const uint32_t (&pl)[10], uint32_t j) {
  uint32_t x = 0;
  int base = 0;
  bool found = false;
#pragma unroll
  for (int t = 0; t < 10; ++t) {
    const uint32_t m = ONE ? pl[t] : ~pl[t];
    const uint32_t pc = (uint32_t)__popc(m);
    if (!found) {
      if (j < pc) {
        x = m;
        base = 32 * t;
        found = true;
      } else {
        j -= pc;
      }
    }
  }
  return base + word_select(x, j);
}
__device__ __forceinline__ uint32_t ef_low(const uint32_t (&pl)[10], uint32_t U, uint32_t i, int l) {
  if (l == 0) return 0u;
  const uint32_t off = U + i * (uint32_t)l;
  const uint32_t w = off >> 5, sh = off & 31;
  const uint64_t v = ((uint64_t)pick10(pl, w + 1) << 32) | pick10(pl, w);
  return (uint32_t)(v >> sh) & ((1u << l) - 1u);
}
__device__ __forceinline__ int64_t ef_select(const uint32_t (&pl)[10], uint32_t U, int l, uint32_t j) {
  const int pos = ef_select_bit<true>(pl, j);
  return ((int64_t)(uint32_t)(pos - (int)j) << l) | ef_low(pl, U, j, l);
}
__device__ __forceinline__ bool ef_has(const uint32_t (&pl)[10], uint32_t c, uint32_t U, int l, uint32_t k) {
  const uint32_t h = k >> l, lowk = k & ((1u << l) - 1u);
  if (h > U - c) return false;  // beyond the largest high part
  // bucket h starts right after the (h-1)-th zero
  const uint32_t s = h > 0 ? (uint32_t)ef_select_bit<false>(pl, h - 1) + 1 : 0u;
  for (uint32_t q = s; q < U; ++q) {
    if (!((pick10(pl, q >> 5) >> (q & 31)) & 1u)) break;
    if (ef_low(pl, U, q - h, l) == lowk) return true;
  }
  return false;
}

// k in the inline common-neighbour list (registers, constant indices)
__device__ __forceinline__ bool list_has(const uint32_t (&pl)[10], uint32_t k) {
  bool hit = false;
#pragma unroll
  for (int t = 0; t < 10; ++t) hit |= (pl[t] & 0xFFFFu) == k || (pl[t] >> 16) == k;
  return hit;
}

struct BsParams {
  double a_p, a_q;
  uint32_t k0, k1, pk0, pk1;
  uint32_t diag;  // timing experiments only (GW_DIAG_BS): 1 = no select, 2 = no membership test
};

__global__ void __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_walk_bitset(gw_dev_graph G, BsParams P, int L, int64_t walk_begin, int64_t walk_count, int shuffle,
              int32_t* __restrict__ out, int32_t* __restrict__ lens, unsigned long long* __restrict__ counters) {
  __shared__ int32_t s_stage[kB / 64][kStage][64];
  const int lane = threadIdx.x & 63;
  int32_t* stage = &s_stage[threadIdx.x >> 6][0][lane];

  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long my_steps = 0, my_trials = 0;
  if (i < walk_count) {
    const int64_t w = walk_begin + i;
    const uint64_t it = (uint64_t)w / (uint64_t)G.n;
    const uint64_t pos = (uint64_t)w % (uint64_t)G.n;
    const uint64_t sp = shuffle ? gw_feistel_perm(pos, (uint64_t)G.n, P.pk0, P.pk1, (uint32_t)it) : pos;
    int32_t cur = G.order[sp];
    int32_t prev = -1;
    int32_t* row = out + i * (int64_t)L;
    const bool vec_ok = (L & 3) == 0;
    const uint32_t c0 = (uint32_t)w, c1 = (uint32_t)((uint64_t)w >> 32);
    stage[0] = cur;
    int len = 1;
    uint32_t trial = 0;
    // bitset of edge (prev -> cur): inside its entry (deg(cur) <= 320: the
    // entry's sector is already in L2, so reading a word is an L2 hit) or in
    // the region store
    const uint32_t* h = nullptr;
    int64_t b = G.offsets[cur], d = G.offsets[cur + 1] - b;  // row of cur
    uint32_t c = 0, kp = 0, boff = 0;
    bool inl = true, lst = false, efm = false;
    uint32_t efU = 0;
    int efl = 0;
    uint32_t pl[10];  // entry payload: the common-neighbour list in list mode
#pragma unroll
    for (int t = 0; t < 10; ++t) pl[t] = 0xFFFFFFFFu;
    while (len < L) {
      if (d == 0) break;
      int64_t k;
      bool acc = true;
      const gw_u4 u = gw_philox(c0, c1, (uint32_t)len, trial, P.k0, P.k1);
      ++trial;
      if (len == 1) {
        k = (int64_t)gw_bounded(u.x, (uint32_t)d);
      } else if (trial == 1) {
        const double Z = (P.a_p + (double)c) + (double)(d - 1 - (int64_t)c) * P.a_q;
        const double r = gw_u01(u.x) * Z;
        if (r < P.a_p) {
          k = kp;  // return to prev
        } else if (r - P.a_p < (double)c) {
          uint32_t j = (uint32_t)(r - P.a_p);
          if (j >= c) j = c - 1;
          k = (P.diag & 1) ? (int64_t)((uint64_t)j * (uint64_t)d / c)
              : lst        ? (int64_t)((pick10(pl, j >> 1) >> (16 * (j & 1))) & 0xFFFFu)
              : inl        ? (int64_t)regs_select<10>(pl, j)
              : efm        ? ef_select(pl, efU, efl, j)
                           : bs_select(h, d, c, j);
        } else {
          k = (int64_t)gw_bounded(u.y, (uint32_t)d);
          const bool common = (P.diag & 2) ? false
                              : lst ? list_has(pl, (uint32_t)k)
                              : inl ? ((pick10(pl, (uint32_t)(k >> 5)) >> (k & 31)) & 1u)
                              : efm ? ef_has(pl, c, efU, efl, (uint32_t)k)
                                    : ((h[boff + (k >> 5)] >> (k & 31)) & 1u);
          acc = (k != (int64_t)kp) && !common;
        }
      } else {  // retry of the "other" branch
        k = (int64_t)gw_bounded(u.y, (uint32_t)d);
        const bool common = lst ? list_has(pl, (uint32_t)k)
                            : inl ? ((pick10(pl, (uint32_t)(k >> 5)) >> (k & 31)) & 1u)
                            : efm ? ef_has(pl, c, efU, efl, (uint32_t)k)
                                  : ((h[boff + (k >> 5)] >> (k & 31)) & 1u);
        acc = ((k != (int64_t)kp) && !common) || trial >= (1u << 24);
      }
      if (acc) {
        my_trials += trial;
        trial = 0;
        const gw_bs_nbr* en = G.bs_nbr + (b + k);
        const uint4* ep = reinterpret_cast<const uint4*>(en);
        const uint4 e0 = ep[0], e1 = ep[1], e2 = ep[2], e3 = ep[3];  // one 64 B entry: next step's state
        prev = cur;
        cur = (int32_t)e0.x;
        d = (int64_t)e0.y;
        b = (int64_t)((uint64_t)e0.z | ((uint64_t)e0.w << 32));
        kp = e1.x;
        c = e1.y;
        lst = gw_bs_is_list(c, (uint32_t)d);
        inl = !lst && d <= GW_BS_INLINE_BITS;
        efm = gw_bs_is_ef(c, (uint32_t)d);
        if (efm) {
          efl = gw_bs_ef_l(c, (uint32_t)d);
          efU = c + (uint32_t)((d - 1) >> efl) + 1;
        }
        h = (lst || inl || efm) ? en->w : G.bs_region + ((uint64_t)e1.z | ((uint64_t)e1.w << 32));
        boff = (uint32_t)bs_boff(d);
        pl[0] = e1.z; pl[1] = e1.w; pl[2] = e2.x; pl[3] = e2.y; pl[4] = e2.z;
        pl[5] = e2.w; pl[6] = e3.x; pl[7] = e3.y; pl[8] = e3.z; pl[9] = e3.w;

        stage[64 * (len & (kStage - 1))] = cur;
        if ((len & (kStage - 1)) == kStage - 1) {
          int32_t* dst = row + (len - (kStage - 1));
          if (vec_ok) {
#pragma unroll
            for (int j = 0; j < kStage; j += 4)
              *reinterpret_cast<int4*>(dst + j) =
                  make_int4(stage[64 * j], stage[64 * (j + 1)], stage[64 * (j + 2)], stage[64 * (j + 3)]);
          } else {
#pragma unroll
            for (int j = 0; j < kStage; ++j) dst[j] = stage[64 * j];
          }
        }
        ++len;
      }
    }
    (void)prev;
    const int base = len & ~(kStage - 1);
    for (int t = base; t < len; ++t) row[t] = stage[64 * (t - base)];
    for (int t = len; t < L; ++t) row[t] = -1;
    if (lens) lens[i] = len;
    my_steps = (unsigned long long)(len - 1);
  }
  if (counters) {
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

template <typename T>
int bs_alloc(gw_graph* g, T** p, int64_t count) {
  *p = nullptr;
  if (count <= 0) count = 1;
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (size_t)count);
  if (e != hipSuccess) {
    g->err = std::string("hipMalloc(bitset ") + std::to_string(sizeof(T) * (size_t)count) + " B): " + hipGetErrorString(e);
    *p = nullptr;
    return GW_ERR_NOMEM;
  }
  return GW_OK;
}

template <typename T>
void bs_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

}  // namespace

void gw_dev_bitset_release(gw_graph* g) {
  bs_free(g->d.bs_region);
  bs_free(g->d.bs_nbr);
}

// Build the per-edge regions.  Requires the membership bitmap (has_edge).
int gw_dev_bitset_build(gw_graph* g, int64_t budget_bytes) {
  gw_dev_graph& d = g->d;
  gw_dev_bitset_release(g);
  const int64_t nnz = g->nnz;
  if (nnz == 0) return GW_OK;
  int rc;
  uint64_t* sz = nullptr;
  uint64_t* roff = nullptr;
  if ((rc = bs_alloc(g, &sz, nnz + 1)) || (rc = bs_alloc(g, &roff, nnz + 1))) {
    bs_free(sz);
    return rc;
  }
  k_bs_sizes<<<(unsigned)((nnz + kB - 1) / kB), kB>>>(nnz, d.nbrs, d.deg, sz);
  GW_HIP_TRY(hipMemset(sz + nnz, 0, sizeof(uint64_t)));
  size_t tmpb = 0;
  GW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, sz, roff, nnz + 1));
  void* tmp = nullptr;
  if ((rc = bs_alloc(g, (char**)&tmp, (int64_t)tmpb + 1))) {
    bs_free(sz);
    bs_free(roff);
    return rc;
  }
  GW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, sz, roff, nnz + 1));
  GW_HIP_TRY(hipDeviceSynchronize());
  bs_free(tmp);
  bs_free(sz);
  uint64_t words = 0;
  GW_HIP_TRY(hipMemcpy(&words, roff + nnz, sizeof(uint64_t), hipMemcpyDeviceToHost));
  const int64_t need = (int64_t)words * 4 + nnz * (int64_t)sizeof(gw_bs_nbr);
  if (words == 0) words = 1;  // every bitset is inline: keep a valid region pointer
  if (need > budget_bytes) {
    bs_free(roff);
    g->err = "per-edge bitsets need " + std::to_string(need) + " B (sum(deg^2) bits); over the " +
             std::to_string(budget_bytes) + " B budget: use GW_N2V_REJECTION";
    return GW_ERR_CAPACITY;
  }
  int64_t* big = nullptr;
  unsigned long long* nbig = nullptr;
  if ((rc = bs_alloc(g, &d.bs_region, (int64_t)words)) || (rc = bs_alloc(g, &d.bs_nbr, nnz)) ||
      (rc = bs_alloc(g, &big, nnz)) || (rc = bs_alloc(g, &nbig, 1))) {
    bs_free(roff);
    bs_free(big);
    bs_free(nbig);
    gw_dev_bitset_release(g);
    return rc;
  }
  GW_HIP_TRY(hipMemset(d.bs_region, 0, (size_t)words * 4));
  GW_HIP_TRY(hipMemset(nbig, 0, sizeof(unsigned long long)));
  k_bs_fill_small<<<(unsigned)((nnz + kB - 1) / kB), kB>>>(d, roff, d.bs_region, d.bs_nbr, big, nbig);
  GW_HIP_TRY(hipGetLastError());
  k_bs_fill_wave<<<2048, kB>>>(d, roff, d.bs_region, d.bs_nbr, big, nbig);
  GW_HIP_TRY(hipGetLastError());
  GW_HIP_TRY(hipDeviceSynchronize());
  bs_free(roff);
  bs_free(big);
  bs_free(nbig);
  g->bitset_words = (int64_t)words;
  return GW_OK;
}

int gw_dev_walk_bitset_launch(gw_graph* g, int L, uint64_t seed, int64_t walk_begin, int64_t walk_count,
                              int shuffle, int32_t* out_dev, int32_t* len_dev, uint64_t* counters_dev,
                              void* stream) {
  BsParams P;
  P.a_p = 1.0 / g->p;
  P.a_q = 1.0 / g->q;
  P.k0 = (uint32_t)seed;
  P.k1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_STEP;
  P.pk0 = (uint32_t)seed;
  P.pk1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_PERM;
  const char* dg = getenv("GW_DIAG_BS");  // diagnostic A/B knob only
  P.diag = dg ? (uint32_t)atoi(dg) : 0u;
  const unsigned grid = (unsigned)std::max<int64_t>(1, (walk_count + kB - 1) / kB);
  k_walk_bitset<<<grid, kB, 0, (hipStream_t)stream>>>(g->d, P, L, walk_begin, walk_count, shuffle, out_dev,
                                                       len_dev, (unsigned long long*)counters_dev);
  GW_HIP_TRY(hipGetLastError());
  return GW_OK;
}
