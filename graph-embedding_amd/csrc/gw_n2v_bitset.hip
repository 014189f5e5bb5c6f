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
//   bs_nbr[s] (64 B, one HBM sector): v, d = deg(v), offsets[v] (u32: this
//            mode needs < 2^32 slots), meta (payload mode, Elias-Fano l and U,
//            directory blocks), kp (position of u in N(v)) and c — one word
//            kp | c << 16 when d < 65536 — and a 44 B payload (40 B otherwise):
//            the common positions (u16 list or Elias-Fano), the bitset itself
//            (d <= 352), or for a region: w[0] = its 64 B block index, w[1..4]
//            = the directory (u16 counts, 512 < d <= 4096), then a draw filter
//            over u (w[5..10]: 192 buckets, or w[1..10]: 320 when the entry
//            holds no directory; bucket = u*F >> 32, bit set iff some u in the
//            bucket lands on a common position), so most "other"-branch
//            membership tests never read the region
//   region   (payload full) dir[ndir]  cumulative set bits before each 512-bit
//                       block (d > 4096 only), then
//            bits[ceil(d/32)]  bit k = (N(v)[k] != u) && has_edge(N(v)[k], u)
// The entry chosen by a step carries everything the next step needs, so a
// step into a vertex of degree <= 352 touches ONE random sector (the entry);
// region selects and unfiltered membership tests add one (1.34 per step on
// R-MAT-20, vs ~7 for rejection sampling with binary-search probes).
//
// Access shape (k_walk_bitset): entries and region blocks are fetched by a
// cooperative load (16 walkers' sectors per instruction) through a per-wave
// LDS exchange; region reads are pipelined so every loop iteration is one
// round trip for the wave; finished 16-position chunks of the walks are
// written by a cooperative flush.  See DESIGN.md §3.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "gw_device_common.h"

namespace {

constexpr int kB = 256;
constexpr int kBlk = 16;         // words per 512-bit block: regions, directory and bits are block-aligned
constexpr int kDirBits = 512;    // bits per directory block
constexpr int kStage = 16;

constexpr int kPDir = 8;         // region entries with <= this many directory blocks keep the directory in the entry

__host__ __device__ __forceinline__ int64_t bs_ndir(int64_t d) { return d > kDirBits ? (d + kDirBits - 1) / kDirBits : 0; }
__host__ __device__ __forceinline__ int64_t bs_round(int64_t w) { return (w + kBlk - 1) / kBlk * kBlk; }
// word offset of the bits inside a region (a directory kept in the region is padded to a block)
__host__ __device__ __forceinline__ int64_t bs_boff(int64_t d) {
  return (gw_bs_is_inline((uint32_t)d) || bs_ndir(d) <= kPDir) ? 0 : bs_round(bs_ndir(d));
}
__host__ __device__ __forceinline__ int64_t bs_words(int64_t d) {
  return gw_bs_is_inline((uint32_t)d) ? 0 : bs_boff(d) + bs_round((d + 31) / 32);
}

__device__ __forceinline__ bool bs_has_edge(const gw_dev_graph& G, int64_t rb, int64_t re, int32_t key) {
  if (G.eh) return gw_eh_has(G.eh, rb, re, key);
  if (G.bitmap) {
    const uint32_t h = (uint32_t)key * 0x9E3779B1u;
    const uint64_t bit = 16ull * (uint64_t)rb + (((uint64_t)h * (uint64_t)(16 * (re - rb))) >> 32);
    if (!((G.bitmap[bit >> 5] >> (bit & 31)) & 1u)) return false;
  }
  return gw_row_find(G.nbrs, rb, re, key) >= 0;
}

// region entries: the draw filter's bucket count (the payload words after
// w[0] and the in-entry directory) and first payload word
__host__ __device__ __forceinline__ uint32_t bs_filt_buckets(int64_t ndir, uint32_t d) {
  return 32u * (gw_bs_pw(d) - ((ndir > 0 && ndir <= kPDir) ? 5u : 1u));
}
__host__ __device__ __forceinline__ uint32_t bs_filt_word(int64_t ndir) { return (ndir > 0 && ndir <= kPDir) ? 5u : 1u; }

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

// ---- build ------------------------------------------------------------------
// Edge-centric common-neighbour enumeration (k_bs_tri).  Every undirected edge
// {u, v} is handled once, by its higher-degree end u (equal degrees: the
// smaller id).  A workgroup holds N(u) in an LDS hash (id -> position in N(u);
// hubs in chunks of kTriH ids, each chunk an id range), and one wave per edge
// streams N(v) through it — coalesced, 64 elements a round.  A hit x at index
// k of N(v) and position pu of N(u) is a common neighbour of BOTH directed
// slots of the edge:
//   (u -> v): position k in N(v), unless x == u;   (v -> u): position pu in N(u), unless x == v,
// and since both rows are sorted by id, the positions of both slots come out
// ascending.  The same stream finds kp(u -> v) (x == u at index k) and with it
// the reverse slot offsets[v] + k; kp(v -> u) is the edge's index j in N(u).
// Work: sum over edges of min(deg u, deg v) LDS probes plus one coalesced read
// of the shorter row (R-MAT-20: 6.9e9) — the per-slot build this replaces
// probed min(deg) for each DIRECTED slot with binary searches in HBM, twice.
// Pass 1 (COUNT) writes both entries' headers (x, deg, offsets, meta, kp, c);
// pass 2 (FILL), after the region layout, replays the stream and writes the
// payloads through BsEmit (common positions in ascending order with ranks).

enum { BS_LIST = 0, BS_INLINE = 1, BS_EF = 2, BS_REGION = 3 };
constexpr uint32_t kFiltL = 320;  // lists-only builds: a region-size common set leaves a 320-bucket draw filter

// The 32-bit draw words y whose index floor(y * d / 2^32) is k are
// [floor(k * 2^32 / d), ceil((k + 1) * 2^32 / d) - 1].  Both ends come from
// inv = 2^32 / d in double precision (k * inv is within 2^-20 of the quotient,
// k <= d < 2^31) and one integer correction, instead of two 64-bit divisions
// per common position.
__device__ __forceinline__ int64_t bs_div32(int64_t k, uint32_t d, double inv, bool* exact) {
  int64_t q = (int64_t)((double)k * inv);
  int64_t r = (k << 32) - q * (int64_t)d;
  if (r < 0) {
    --q;
    r += d;
  } else if (r >= (int64_t)d) {
    ++q;
    r -= d;
  }
  *exact = r == 0;
  return q;
}
__device__ __forceinline__ void bs_draw_range(int64_t k, uint32_t d, double inv, uint32_t* ylo, uint32_t* yhi) {
  bool ex;
  *ylo = (uint32_t)bs_div32(k, d, inv, &ex);
  const int64_t q1 = bs_div32(k + 1, d, inv, &ex);
  *yhi = (uint32_t)(q1 - (ex ? 1 : 0));
}
__device__ __forceinline__ double bs_inv32(uint32_t d) { return 4294967296.0 / (double)d; }

// lists-only builds (k_walk_listed): for common position k of a slot whose
// set needs a region, set the filter buckets of every draw (hi : lo) with
// index k, bucket = hi * kFiltL >> 32 (the listed draw's high word is u.x)
__device__ __forceinline__ void bs_filter_only(uint32_t* w, int64_t k, uint32_t d, double inv) {
  uint32_t ulo, uhi;
  bs_draw_range(k, d, inv, &ulo, &uhi);
  const uint32_t b0 = gw_bounded(ulo, kFiltL), b1 = gw_bounded(uhi, kFiltL);
  for (uint32_t b = b0; b <= b1; ++b) atomicOr(&w[b >> 5], 1u << (b & 31));
}
__device__ __forceinline__ int bs_mode(uint32_t c, uint32_t d) {
  return gw_bs_is_list(c, d) ? BS_LIST : gw_bs_is_inline(d) ? BS_INLINE : gw_bs_is_ef(c, d) ? BS_EF : BS_REGION;
}

// Return elision (k_walk_bitset).  When both directed slots of an edge have
// small common sets (c(u -> x) <= kDualC and c(x -> u) <= kDualC, both
// degrees < 65536), the builder writes E(u -> x) as a DUAL list entry: its
// own positions in N(x) in payload halfwords 0..5, the positions in N(u) of
// the reverse slot's common set (the payload of E(x -> u)) in halfwords 6..11,
// meta = kMetaDual | c(x -> u) << 2 (mode LIST).  Arriving through it, the
// walker keeps u's row and the index it drew at u in payload words 6..9
// (kMetaStash), so E(x -> u) is fully known: a return move (draw == kp) swaps
// rows, lists and counts in registers instead of fetching the reverse entry,
// and a return after that swaps back.  Membership in a dual entry's list
// looks at its first 3 words only.
constexpr uint32_t kDualC = 6;
constexpr uint32_t kMetaDual = 0x40000000u;
constexpr uint32_t kMetaStash = 0x80000000u;

// per-entry constants of the step kernel (no divisions per step):
// mode | Elias-Fano l << 2 | U << 7 | directory blocks before the bits << 16
__device__ __forceinline__ uint32_t bs_meta(uint32_t c, uint32_t d) {
  const uint32_t mode = (uint32_t)bs_mode(c, d);
  uint32_t l = 0, U = 0;
  if (mode == BS_EF) {
    l = (uint32_t)gw_bs_ef_l(c, d);
    U = c + ((d - 1) >> l) + 1;
  }
  const uint32_t bblk = (mode == BS_REGION) ? (uint32_t)(bs_boff(d) / kBlk) : 0u;
  return mode | (l << 2) | (U << 7) | (bblk << 16);
}
// meta of slot (u -> x): c common neighbours, d = deg x; dual entries (see
// above) carry the reverse slot's count c_rev (du = deg u)
__device__ __forceinline__ bool bs_dual(uint32_t c, uint32_t c_rev, uint32_t d, uint32_t du) {
  return c <= kDualC && c_rev <= kDualC && d < GW_BS_PACK_D && du < GW_BS_PACK_D;
}
__device__ __forceinline__ uint32_t bs_meta_slot(uint32_t c, uint32_t c_rev, uint32_t d, uint32_t du) {
  return bs_dual(c, c_rev, d, du) ? (kMetaDual | (c_rev << 2)) : bs_meta(c, d);
}

// payload writer for one common position (entry words zeroed beforehand)
struct BsEmit {
  int mode;
  bool nobits;     // region bits written by the caller (k_bs_tri's (u -> v) slot: whole words per round)
  uint32_t* w;     // entry payload (or a staging copy of it)
  uint32_t* dir;   // region directory (ndir > kPDir)
  uint16_t* pdir;  // directory in the entry (0 < ndir <= kPDir)
  uint32_t* bits;  // region bits
  int64_t ndir;
  uint32_t d;
  double inv;  // 2^32 / d (region filters)
  int l;
  uint32_t U;
  __device__ void operator()(int64_t k, uint32_t idx, int64_t kprev) const {
    const uint32_t bit = 1u << (k & 31);
    if (mode == BS_LIST) {
      reinterpret_cast<uint16_t*>(w)[idx] = (uint16_t)k;
    } else if (mode == BS_INLINE) {
      atomicOr(&w[k >> 5], bit);
    } else if (mode == BS_EF) {
      const uint32_t hp = (uint32_t)(k >> l) + idx;  // high part, unary
      atomicOr(&w[hp >> 5], 1u << (hp & 31));
      if (l > 0) {
        const uint32_t lowv = (uint32_t)k & ((1u << l) - 1u), off = U + idx * (uint32_t)l, sh = off & 31;
        atomicOr(&w[off >> 5], lowv << sh);
        if (sh + (uint32_t)l > 32u) atomicOr(&w[(off >> 5) + 1], lowv >> (32 - sh));
      }
    } else {
      if (!nobits) atomicOr(&bits[k >> 5], bit);
      set_dir((kprev < 0 ? -1 : kprev / kDirBits) + 1, k / kDirBits, idx);
      // filter over the draw's high word y (bucket floor(y*F / 2^32)): the 64-bit draws
      // (y:z) with index k have y in [floor(k*2^32/d), ceil((k+1)*2^32/d) - 1]
      uint32_t ulo, uhi;
      bs_draw_range(k, d, inv, &ulo, &uhi);
      const uint32_t F = bs_filt_buckets(ndir, d), w0 = bs_filt_word(ndir);
      const uint32_t b0 = gw_bounded(ulo, F), b1 = gw_bounded(uhi, F);
      for (uint32_t b = b0; b <= b1; ++b) atomicOr(&w[w0 + (b >> 5)], 1u << (b & 31));
    }
  }
  // directory blocks [g0, g1] start after `count` common positions
  __device__ void set_dir(int64_t g0, int64_t g1, uint32_t count) const {
    if (ndir == 0) return;
    for (int64_t g = g0; g <= g1 && g < ndir; ++g) {
      if (pdir)
        pdir[g] = (uint16_t)count;
      else
        dir[g] = count;
    }
  }
};

// payload words and common count of an entry (d < 65536: r[0] = kp | c << 16)
__device__ __forceinline__ uint32_t* bs_payload(gw_bs_nbr* en, uint32_t d) { return en->r + (d < GW_BS_PACK_D ? 1 : 2); }
__device__ __forceinline__ uint32_t bs_c(const gw_bs_nbr* en, uint32_t d) { return d < GW_BS_PACK_D ? en->r[0] >> 16 : en->r[1]; }

__device__ __forceinline__ BsEmit bs_emit(gw_bs_nbr* en, uint32_t* reg, const uint64_t* roff, int64_t e, uint32_t c,
                                          uint32_t d) {
  BsEmit E;
  E.mode = bs_mode(c, d);
  E.nobits = false;
  E.w = bs_payload(en, d);
  E.ndir = 0;
  E.dir = E.bits = nullptr;
  E.pdir = nullptr;
  E.d = d;
  E.inv = bs_inv32(d);
  E.l = 0;
  E.U = 0;
  if (E.mode == BS_EF) {
    E.l = gw_bs_ef_l(c, d);
    E.U = c + ((d - 1) >> E.l) + 1;
  } else if (E.mode == BS_REGION) {
    E.ndir = bs_ndir(d);
    E.dir = reg + roff[e];
    E.bits = E.dir + bs_boff(d);
    if (E.ndir <= kPDir) {
      E.pdir = reinterpret_cast<uint16_t*>(E.w + 1);
      E.dir = nullptr;
    }
  }
  return E;
}

// region words per slot: only slots whose payload is neither list, inline nor Elias-Fano
__global__ void k_bs_sizes(gw_dev_graph G, const gw_bs_nbr* __restrict__ bsn, uint64_t* __restrict__ sz,
                           int lists_only) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= G.nnz) return;
  const uint32_t d = (uint32_t)G.deg[G.nbrs[e]];
  sz[e] = (!lists_only && !gw_bs_is_inline(d) && bs_mode(bs_c(bsn + e, d), d) == BS_REGION)
              ? (uint64_t)bs_words(d) : 0ull;
}

constexpr int kTB = 512;                     // build workgroup: 8 waves
constexpr int kTW = kTB / 64;
constexpr int kTriH = 4096;                  // ids of N(u) per hash chunk
constexpr int kTriS = 2 * kTriH;             // LDS hash slots (load factor <= 1/2)
constexpr int kTriEB = 512;                  // edges of u's row per work item
constexpr int kTriAhead = 4;                 // rounds of N(v) in flight per wave
constexpr int32_t kTriNotOwned = INT32_MIN;

// build-time model constants (gw_bitset_build_model_s), measured on MI355X
// (R-MAT-20: 0.175 s for sum(min deg) = 6.9e9; R-MAT-24 ef 6: 1.17 s for 4.4e10)
constexpr double kBuildProbeRate = 7.7e10;     // k_bs_tri stream probes per second (one pass)
constexpr double kBuildSlotSeconds = 5.0e-11;  // per adjacency slot: memset, headers, sizes scan, payload stores

struct TriItem {
  int32_t u, j0;  // vertex, first edge index in N(u) (items of a vertex: j0 = 0, kTriEB, ...)
};

__global__ void k_bs_iota(int64_t n, int32_t* __restrict__ a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = (int32_t)i;
}

// work items per vertex (in the degree-descending order): ceil(deg / kTriEB)
__global__ void k_bs_nitems(gw_dev_graph G, const int32_t* __restrict__ order, uint32_t* __restrict__ nit) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > G.n) return;
  nit[i] = i < G.n ? (uint32_t)((G.deg[order[i]] + kTriEB - 1) / kTriEB) : 0u;
}

__global__ void k_bs_items(gw_dev_graph G, const int32_t* __restrict__ order, const uint32_t* __restrict__ itoff,
                           TriItem* __restrict__ items) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G.n) return;
  const int32_t u = order[i];
  const uint32_t b = itoff[i], e = itoff[i + 1];
  for (uint32_t t = b; t < e; ++t) items[t] = TriItem{u, (int32_t)((t - b) * kTriEB)};
}

// BsEmit for one slot of the edge (pass 2), or the lists-only draw filter.
// Payload words are staged in the wave's LDS copy `w` (E.w points there) and
// written to the entry by tri_flush: the many ORs into the same few words
// (bitsets, Elias-Fano, draw filters) stay off the global atomic path.
struct TriSlot {
  BsEmit E;
  uint32_t* gw;  // the entry's payload words in HBM
  bool filt;  // lists-only build, region-size set: draw filter only
  bool dual;  // dual list entry: the reverse slot's list goes to halfwords 6..11
  __device__ void operator()(int64_t k, uint32_t idx, int64_t kprev) const {
    if (filt)
      bs_filter_only(E.w, k, E.d, E.inv);
    else
      E(k, idx, kprev);
  }
};

__device__ __forceinline__ TriSlot tri_slot(gw_bs_nbr* en, uint32_t* reg, const uint64_t* roff, int64_t e, uint32_t c,
                                            uint32_t d, int lists_only, uint32_t* stage, int lane) {
  TriSlot T;
  T.filt = lists_only && bs_mode(c, d) == BS_REGION;
  T.dual = (en->meta & kMetaDual) != 0u;
  T.E = bs_emit(en, reg, roff, e, c, d);
  T.gw = T.E.w;
  T.E.w = stage;
  if (T.E.pdir) T.E.pdir = reinterpret_cast<uint16_t*>(stage + 1);
  if (lane < 12) stage[lane] = 0u;
  __builtin_amdgcn_wave_barrier();
  return T;
}

// prologue of a slot's payload (pass 2, first chunk): region block index
__device__ __forceinline__ void tri_prologue(const TriSlot& T, int64_t e, const uint64_t* roff, int lane) {
  if (!T.filt && T.E.mode == BS_REGION && lane == 0) T.E.w[0] = (uint32_t)(roff[e] / kBlk);
}

// epilogue (pass 2, last chunk): list padding, directory blocks after the last
// common position; c_rev = the reverse slot's count (dual entries)
__device__ __forceinline__ void tri_epilogue(const TriSlot& T, int64_t klast, uint32_t c, uint32_t c_rev, int lane) {
  if (T.filt) return;
  if (T.dual) {
    if (lane < 2 * (int)kDualC && (lane < (int)kDualC ? lane >= (int)c : lane - (int)kDualC >= (int)c_rev))
      reinterpret_cast<uint16_t*>(T.E.w)[lane] = 0xFFFFu;
    return;
  }
  if (T.E.mode == BS_LIST && lane >= (int)c && lane < 2 * (int)gw_bs_pw(T.E.d))
    reinterpret_cast<uint16_t*>(T.E.w)[lane] = 0xFFFFu;
  if (T.E.mode != BS_REGION) return;
  for (int64_t g = (klast < 0 ? -1 : klast / kDirBits) + 1 + lane; g < T.E.ndir; g += 64) T.E.set_dir(g, g, c);
}

// staged payload words -> the entry (once per chunk; the entry's payload is
// zero before the first flush, so later chunks OR into it)
__device__ __forceinline__ void tri_flush(const TriSlot& T, bool merge, int lane) {
  __builtin_amdgcn_wave_barrier();
  const int pw = (int)gw_bs_pw(T.E.d);
  if (lane < pw) {
    const uint32_t v = T.E.w[lane];
    if (!merge)
      T.gw[lane] = v;
    else if (v)
      atomicOr(&T.gw[lane], v);
  }
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void tri_header(gw_bs_nbr* en, uint32_t x, uint32_t d, uint32_t off, uint32_t meta,
                                           uint32_t kp, uint32_t c) {
  *reinterpret_cast<uint4*>(en) = make_uint4(x, d, off, meta);
  *reinterpret_cast<uint2*>(&en->r[0]) =
      d < GW_BS_PACK_D ? make_uint2((kp & 0xFFFFu) | (c << 16), 0u) : make_uint2(kp, c);
}

// wave-level emission of this round's common positions of one slot: lanes
// with `on` hold position pos; ranks continue from *cnt, kprev from *last;
// rev (dual entries): the other slot's staged halfwords, whose reverse list
// gets the same positions
// (positions < 2^31; the previous position is only needed by region slots'
// directories, and the round's last one and the count are wave-uniform)
template <class F>
__device__ __forceinline__ void tri_emit(const F& f, bool on, int64_t pos, uint32_t* cnt, int64_t* last, int lane,
                                         uint16_t* rev, bool need_prev) {
  const unsigned long long m = __ballot(on);
  if (!m) return;
  const unsigned long long lt = m & ((1ull << lane) - 1ull);
  const int32_t p32 = (int32_t)pos;
  int64_t prev = *last;
  if (need_prev) {
    const int32_t pin = __shfl(p32, lt ? 63 - __clzll(lt) : 0, 64);
    if (lt) prev = pin;
  }
  if (on) {
    const uint32_t idx = *cnt + (uint32_t)__popcll(lt);
    f(pos, idx, prev);
    if (rev) rev[kDualC + idx] = (uint16_t)pos;
  }
  *last = __builtin_amdgcn_readlane(p32, 63 - __clzll(m));
  *cnt += (uint32_t)__popcll(m);
}

// (a launch's work-items must stay below 2^32, so a workgroup takes items
// blockIdx.x, blockIdx.x + gridDim.x, ...; hubs come first in the item order)
template <bool FILL>
__global__ void __launch_bounds__(kTB) __attribute__((amdgpu_waves_per_eu(4))) k_bs_tri(gw_dev_graph G, const TriItem* __restrict__ items, uint32_t nitems,
                                                gw_bs_nbr* __restrict__ bsn,
                                                const uint64_t* __restrict__ roff, uint32_t* __restrict__ reg,
                                                int lists_only) {
  __shared__ int32_t s_key[kTriS];
  __shared__ uint16_t s_pos[kTriS];
  // per-edge state between chunks (hubs): common counts, last positions, kp(u -> v), cursor in N(v)
  __shared__ uint32_t s_cuv[kTriEB], s_cvu[kTriEB], s_cur[kTriEB];
  __shared__ int32_t s_luv[kTriEB], s_lvu[kTriEB], s_kp[kTriEB];
  __shared__ int32_t s_nx[kTriEB];  // hubs: N(v)'s next element (kTriNotOwned: edge owned by v)
  __shared__ uint32_t s_stage[kTW][2][12];  // pass 2: both slots' payload words, per wave
  // pass 2: the (v -> u) slot's region bits of this chunk (positions p0 ..
  // p0 + kTriH of N(u): one aligned window per chunk, written once)
  __shared__ uint32_t s_win[kTW][kTriH / 32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // diagnostics build only (GW_DIAG_BS_FILL, timing experiments, wrong tables):
  // 1 = no payload emission, 2 = no region-bit stores, 4 = no payload flush
  const int diag = kGwDiag ? (lists_only >> 8) : 0;
  lists_only &= 1;
  if (FILL) {
    for (int i = lane; i < kTriH / 32; i += 64) s_win[wave][i] = 0u;
  }
  for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
    if (item != blockIdx.x) __syncthreads();  // every wave is done with the previous item's hash and state
    const TriItem it = items[item];
    const int32_t u = it.u;
    const int64_t ub = G.offsets[u], du = G.offsets[u + 1] - ub;
    const int64_t j0 = it.j0, j1 = min(du, j0 + (int64_t)kTriEB);
    const int nch = (int)((du + kTriH - 1) / kTriH);
    const int64_t hk = min(du, (int64_t)kTriH);  // keys per chunk (at most)
    int lg = 6;
    while ((1 << lg) < 2 * hk) ++lg;
    const uint32_t S = 1u << lg, smask = S - 1u;
    const int sh = 32 - lg;
    for (int ch = 0; ch < nch; ++ch) {
      const int64_t p0 = (int64_t)ch * kTriH, p1 = min(du, p0 + kTriH);
      if (ch > 0) __syncthreads();  // every wave is done with the previous chunk
      for (uint32_t i = tid; i < S; i += kTB) s_key[i] = -1;
      __syncthreads();
      for (int64_t i = tid; i < p1 - p0; i += kTB) {
        const int32_t x = G.nbrs[ub + p0 + i];
        uint32_t h = ((uint32_t)x * 0x9E3779B1u) >> sh;
        while (atomicCAS(&s_key[h], -1, x) != -1) h = (h + 1) & smask;
        s_pos[h] = (uint16_t)i;
      }
      __syncthreads();
      // this chunk's id range is (previous chunk's last id, hi]: every element
      // of N(v) falls in exactly one chunk's stream
      const int32_t hi = ch == nch - 1 ? INT32_MAX : G.nbrs[ub + p1 - 1];
      // the wave's edges are software-pipelined: the row bounds of its next
      // edge and the neighbour id of the one after are requested at the top of
      // each edge, so an edge starts with (v, row) in registers instead of a
      // chain of two dependent reads
      int64_t jp = j0 + wave;
      int32_t pv_n = jp + kTW < j1 ? G.nbrs[ub + jp + kTW] : 0;
      int32_t pv = 0;
      int64_t pvb = 0, pve = 0;
      if (jp < j1) {
        pv = G.nbrs[ub + jp];
        pvb = G.offsets[pv];
        pve = G.offsets[pv + 1];
      }
      for (int64_t j = jp; j < j1; j += kTW) {
        const int32_t v = pv;
        const int64_t vb = pvb, dv = pve - pvb;
        if (j + kTW < j1) {
          pv = pv_n;
          pvb = G.offsets[pv];
          pve = G.offsets[pv + 1];
        }
        if (j + 2 * kTW < j1) pv_n = G.nbrs[ub + j + 2 * kTW];
        const int li = (int)(j - j0);
        if (ch > 0) {
          // hubs: an edge whose next element of N(v) lies past this chunk's
          // range has nothing here (the last chunk still closes every owned edge)
          const int32_t nx = s_nx[li];
          if (nx == kTriNotOwned || (ch + 1 < nch && nx > hi)) continue;
        }
        if (!(du > dv || (du == dv && u <= v))) {  // the other end owns this edge
          if (nch > 1 && lane == 0) s_nx[li] = kTriNotOwned;
          continue;
        }
        const int64_t e = ub + j;
        uint32_t cuv = 0, cvu = 0, cur = 0;
        int64_t luv = -1, lvu = -1, kp = -1;
        if (ch > 0) {
          cuv = s_cuv[li];
          cvu = s_cvu[li];
          cur = s_cur[li];
          luv = s_luv[li];
          lvu = s_lvu[li];
          kp = s_kp[li];
        }
        // the stream keeps kTriAhead rounds of N(v) in flight per wave (the
        // probes are latency-bound otherwise); the first ones are requested
        // before pass 2's header reads, so those latencies overlap too
        int64_t k = (int64_t)cur + lane;
        int32_t x = k < dv ? G.nbrs[vb + k] : INT32_MAX;
        int32_t xa[kTriAhead - 1];
#pragma unroll
        for (int r = 0; r < kTriAhead - 1; ++r) xa[r] = k + 64 * (r + 1) < dv ? G.nbrs[vb + k + 64 * (r + 1)] : INT32_MAX;
        // pass 2: both slots' payload writers (headers from pass 1)
        TriSlot Tuv, Tvu;
        int64_t er = -1;
        bool vu_win = false;
        if (FILL) {
          gw_bs_nbr* en = bsn + e;
          const uint32_t c = bs_c(en, (uint32_t)dv);
          Tuv = tri_slot(en, reg, roff, e, c, (uint32_t)dv, lists_only, s_stage[wave][0], lane);
          Tuv.E.nobits = true;  // (u -> v) positions are this round's lanes: whole bit words below
          if (ch == 0) tri_prologue(Tuv, e, roff, lane);
          if (u != v) {
            const uint32_t kpv = (uint32_t)dv < GW_BS_PACK_D ? (en->r[0] & 0xFFFFu) : en->r[0];
            er = vb + kpv;  // the reverse slot (v -> u)
            gw_bs_nbr* enr = bsn + er;
            const uint32_t cr = bs_c(enr, (uint32_t)du);
            Tvu = tri_slot(enr, reg, roff, er, cr, (uint32_t)du, lists_only, s_stage[wave][1], lane);
            if (ch == 0) tri_prologue(Tvu, er, roff, lane);
            vu_win = !Tvu.filt && Tvu.E.mode == BS_REGION;
            Tvu.E.nobits = vu_win;  // region bits go through the LDS window
          }
        }
        int32_t nx = INT32_MAX;  // first element of N(v) past this chunk (INT32_MAX: row done)
        for (;;) {
          // the round kTriAhead ahead is requested before this one is probed
          // (reads past the chunk's end cost a line each, past the row's end nothing)
          const int64_t kf = k + 64 * kTriAhead;
          const int32_t xf = kf < dv ? G.nbrs[vb + kf] : INT32_MAX;
          const bool inr = k < dv && x <= hi;
          bool hit = false;
          uint32_t pu = 0;
          if (inr) {
            uint32_t h = ((uint32_t)x * 0x9E3779B1u) >> sh;
            for (;;) {
              const int32_t kk = s_key[h];
              if (kk == x) {
                hit = true;
                pu = (uint32_t)p0 + s_pos[h];
                break;
              }
              if (kk == -1) break;
              h = (h + 1) & smask;
            }
          }
          const unsigned long long mu = __ballot(inr && x == u);
          if (mu) kp = (int64_t)cur + (__ffsll(mu) - 1);
          const bool cu = hit && x != u;              // (u -> v): position k in N(v)
          const bool cv = hit && x != v && u != v;    // (v -> u): position pu in N(u)
          if (FILL && !(diag & 1)) {
            if (!(diag & 2) && !Tuv.filt && Tuv.E.mode == BS_REGION) {
              // this round's positions are cur .. cur+63: its hits are whole
              // words of the region bitset (at most three)
              const unsigned long long m = __ballot(cu);
              if (m) {
                const uint32_t sh = cur & 31u;
                const unsigned long long lo = m << sh;
                const uint32_t hi3 = sh ? (uint32_t)(m >> (64 - sh)) : 0u;
                const uint32_t wv = lane == 0 ? (uint32_t)lo : lane == 1 ? (uint32_t)(lo >> 32) : hi3;
                if (lane < 3 && wv) atomicOr(&Tuv.E.bits[(cur >> 5) + lane], wv);
              }
            }
            const bool dual = u != v && Tuv.dual;  // (both slots or neither)
            tri_emit(Tuv, cu, k, &cuv, &luv, lane, dual ? reinterpret_cast<uint16_t*>(Tvu.E.w) : nullptr,
                     !Tuv.filt && Tuv.E.mode == BS_REGION);
            if (u != v) {
              tri_emit(Tvu, cv, (int64_t)pu, &cvu, &lvu, lane, dual ? reinterpret_cast<uint16_t*>(Tuv.E.w) : nullptr,
                       !Tvu.filt && Tvu.E.mode == BS_REGION);
              if (cv && vu_win && !(diag & 2)) atomicOr(&s_win[wave][(pu - (uint32_t)p0) >> 5], 1u << (pu & 31u));
            }
          } else if (!FILL) {
            const unsigned long long m1 = __ballot(cu), m2 = __ballot(cv);
            cuv += (uint32_t)__popcll(m1);
            cvu += (uint32_t)__popcll(m2);
          }
          const int nin = __popcll(__ballot(inr));  // a prefix of the lanes (rows are sorted)
          cur += (uint32_t)nin;
          if (nin < 64) {  // the chunk's id range or the row ended
            nx = __shfl(x, nin, 64);
            break;
          }
          k += 64;
          x = xa[0];
#pragma unroll
          for (int r = 0; r < kTriAhead - 2; ++r) xa[r] = xa[r + 1];
          xa[kTriAhead - 2] = xf;
        }
        if (FILL && ch + 1 == nch) {
          tri_epilogue(Tuv, luv, cuv, cvu, lane);
          if (u != v) tri_epilogue(Tvu, lvu, cvu, cuv, lane);
        }
        if (FILL && !(diag & 4)) {
          tri_flush(Tuv, nch > 1, lane);
          if (u != v) tri_flush(Tvu, nch > 1, lane);
          if (vu_win) {  // this chunk's window of (v -> u)'s region bits: plain stores, each word once
            __builtin_amdgcn_wave_barrier();
            for (int i = lane; i < kTriH / 32; i += 64) {
              const uint32_t wv = s_win[wave][i];
              if (wv) {
                Tvu.E.bits[(p0 >> 5) + i] = wv;
                s_win[wave][i] = 0u;
              }
            }
            __builtin_amdgcn_wave_barrier();
          }
        }
        if (ch + 1 < nch) {
          if (lane == 0) {
            s_cuv[li] = cuv;
            s_cvu[li] = cvu;
            s_cur[li] = cur;
            s_luv[li] = (int32_t)luv;
            s_lvu[li] = (int32_t)lvu;
            s_kp[li] = (int32_t)kp;
            s_nx[li] = nx;
          }
          continue;
        }
        if (!FILL) {
          const uint32_t k32 = kp >= 0 ? (uint32_t)kp : 0xFFFFFFFFu;
          if (lane == 0)
            tri_header(bsn + e, (uint32_t)v, (uint32_t)dv, (uint32_t)vb,
                       bs_meta_slot(cuv, u != v ? cvu : 0xFFFFu, (uint32_t)dv, (uint32_t)du), k32, cuv);
          if (lane == 1 && u != v && kp >= 0)
            tri_header(bsn + vb + kp, (uint32_t)u, (uint32_t)du, (uint32_t)ub,
                       bs_meta_slot(cvu, cuv, (uint32_t)du, (uint32_t)dv), (uint32_t)j, cvu);
        }
      }
    }
  }
}

// j-th set bit among `nw` words held in registers (constant indices only),
// branch-free: with running popcounts S_t, the target word is T = #{t : S_t
// <= j}; j - S_{T-1} is the rank inside it
template <int NW>
__device__ __forceinline__ int regs_select(const uint32_t* wd, uint32_t j) {
  uint32_t S = 0, T = 0, below = 0, x = wd[0];
#pragma unroll
  for (int t = 0; t < NW; ++t) {
    S += (uint32_t)__popc(wd[t]);
    const bool le = S <= j;
    T += le ? 1u : 0u;
    below = le ? S : below;
    if (t + 1 < NW) x = le ? wd[t + 1] : x;
  }
  return 32 * (int)T + word_select(x, j - below);
}

// pl[idx] for a per-lane idx < kPW without dynamic register indexing: a
// select tree on the index bits (10 v_cndmask + 4 bit tests; a mask-OR over
// all the words costs ~3 VALU per word).  idx >= kPW returns some payload word.
constexpr int kPW = 11;  // payload registers: 11 words for d < 65536 (packed kp | c), else 10 + a zero word
__device__ __forceinline__ uint32_t pickw(const uint32_t (&pl)[kPW], uint32_t idx) {
  const bool b0 = idx & 1u, b1 = idx & 2u, b2 = idx & 4u, b3 = idx & 8u;
  const uint32_t a0 = b0 ? pl[1] : pl[0], a1 = b0 ? pl[3] : pl[2], a2 = b0 ? pl[5] : pl[4];
  const uint32_t a3 = b0 ? pl[7] : pl[6], a4 = b0 ? pl[9] : pl[8];
  const uint32_t c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2, c2 = b1 ? pl[10] : a4;
  const uint32_t e0 = b2 ? c1 : c0;
  return b3 ? c2 : e0;
}

// 32 payload bits from bit position pos (pos < 320; bits past 320 are
// unspecified, callers use only bits inside the payload)
__device__ __forceinline__ uint32_t bits32(const uint32_t (&pl)[kPW], uint32_t pos) {
  const uint32_t w = pos >> 5;
  return __builtin_amdgcn_alignbit(pickw(pl, w + 1), pickw(pl, w), pos & 31u);
}

// ---- Elias-Fano payload ----------------------------------------------------
// High parts (unary, U bits: c ones, U - c zeros) come first, then c low
// parts of l bits.  Bucket h (elements with high part h) starts right after
// the (h-1)-th zero; its elements are the run of ones from there, indices
// e0 = s - h on.  k (high h, low k & (2^l - 1)) is a member iff one of the
// bucket's low parts equals k's (they ascend, so the scan stops early).
// lw = the 32 bits at U + e0 * l (already read by the caller).
__device__ __forceinline__ bool ef_bucket_has(const uint32_t (&pl)[kPW], uint32_t U, uint32_t l, uint32_t s,
                                              uint32_t e0, uint32_t k, uint32_t lw) {
  // the run of ones ends at a zero below U; a bucket spans 2^l positions, so
  // it can hold more than 32 elements (l >= 6): keep reading windows
  uint32_t hw = bits32(pl, s), run = 0;
  while (hw == 0xFFFFFFFFu && run < 320u) {
    run += 32u;
    hw = bits32(pl, s + run);
  }
  run += (uint32_t)__builtin_ctz(~hw);
  if (l == 0) return run > 0;
  const uint32_t mask = (1u << l) - 1u, lowk = k & mask;
  uint32_t o = 0;
  for (uint32_t i = 0; i < run; ++i) {
    if (o + l > 32u) {  // window exhausted (long bucket or wide low parts)
      lw = bits32(pl, U + (e0 + i) * l);
      o = 0;
    }
    const uint32_t f = (lw >> o) & mask;
    if (f >= lowk) return f == lowk;
    o += l;
  }
  return false;
}

// k in the inline common-neighbour list (registers, constant indices); a
// dual entry's own list is its first kDualC halfwords
__device__ __forceinline__ bool list_has(const uint32_t (&pl)[kPW], uint32_t k, bool dual = false) {
  bool hit = false;
#pragma unroll
  for (int t = 0; t < kPW; ++t)
    hit |= (t < (int)kDualC / 2 || !dual) && ((pl[t] & 0xFFFFu) == k || (pl[t] >> 16) == k);
  return hit;
}

struct BsParams {
  double a_p, a_q;
  uint32_t k0, k1, pk0, pk1;
  uint32_t diag;  // timing experiments only (GW_DIAG_BS): 1 = no select, 2 = no membership test,
                 // 4 = region blocks / 8 = region words read from a small hot area (wrong walks),
                 // 64 = lane-utilisation counters in counters[2..3] (the caller passes 4)
};

// an arrived entry's kp, c and payload (gw_bs_nbr: packed header when d < 65536)
__device__ __forceinline__ void unpack_entry(const uint32_t (&E)[16], uint32_t* kp, uint32_t* c, uint32_t (&pl)[kPW]) {
  const bool packed = E[1] < GW_BS_PACK_D;
  *kp = packed ? (E[4] & 0xFFFFu) : E[4];
  *c = packed ? (E[4] >> 16) : E[5];
#pragma unroll
  for (int q = 0; q < kPW - 1; ++q) pl[q] = packed ? E[5 + q] : E[6 + q];
  pl[kPW - 1] = packed ? E[15] : 0u;
}

// round j of a cooperative entry load: lane l fetches 16 B piece (l & 3) of
// the entry of the walker in lane 16 j + (l >> 2) (none if that walker
// fetches nothing)
__device__ __forceinline__ uint4 coop_piece(uint64_t sec, int lane, int j) {
  const int src = 16 * j + (lane >> 2);
  const uint64_t sj = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(sec >> 32), src, 64) << 32) |
                      (uint32_t)__shfl((int)(uint32_t)sec, src, 64);
  uint4 r = make_uint4(0u, 0u, 0u, 0u);
  if (sj != 0ull) r = reinterpret_cast<const uint4*>(sj)[lane & 3];
  return r;
}

// Entry reads are cooperative: a lane's 64 B entry read as four per-lane
// dwordx4 loads touches 64 random pages per instruction, which past ~3 GB of
// tables runs at 2e10 sectors/s (address translation bound, measured with
// tools/calib/calib_sweep.hip) against 4.9e10 when each instruction covers
// 16 sectors x 64 B.  So in round j lanes 4m..4m+3 load the four 16 B pieces
// of walker 16j+m's entry, and the pieces reach their walker through a 1 KB
// per-wave LDS exchange.  The walk loop is therefore wave-uniform (lanes
// whose walk is done idle in it until every lane of the wave is done).
__global__ void __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(5, 5)))
k_walk_bitset(gw_dev_graph G, BsParams P, int L, int64_t walk_begin, int64_t walk_count, int shuffle,
              int32_t* __restrict__ out, int32_t* __restrict__ lens, unsigned long long* __restrict__ counters) {
  __shared__ int32_t s_stage[kB / 64][kStage][64];
  __shared__ uint4 s_ex[kB / 64][64];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  int32_t* stage = &s_stage[wv][0][lane];
  uint4* ex = s_ex[wv];
  const uint4* __restrict__ ents = reinterpret_cast<const uint4*>(G.bs_nbr);

  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < walk_count;
  unsigned long long my_steps = 0;
  uint32_t my_trials = 0;
  const int64_t w = walk_begin + (valid ? i : 0);
  int32_t cur = -1;
  int len = L;  // lanes past walk_count take no step
  if (valid) {
    const uint64_t it = (uint64_t)w / (uint64_t)G.n;
    const uint64_t pos = (uint64_t)w % (uint64_t)G.n;
    const uint64_t sp = shuffle ? gw_feistel_perm(pos, (uint64_t)G.n, P.pk0, P.pk1, (uint32_t)it) : pos;
    cur = G.order[sp];
    len = 1;
  }
  const bool vec_ok = (L & 3) == 0;
  const uint32_t c0 = (uint32_t)w, c1 = (uint32_t)((uint64_t)w >> 32);
  stage[0] = cur;
  uint32_t trial = 0;
  // bitset of edge (prev -> cur): inside its entry (deg(cur) <= 320) or in
  // the region store at block pl[0]
  uint32_t b = 0, d = 0;  // row of cur (slot indices < 2^32: gw_dev_bitset_build)
  if (valid) {
    b = (uint32_t)G.offsets[cur];
    d = (uint32_t)(G.offsets[cur + 1] - G.offsets[cur]);
  }
  uint32_t c = 0, kp = 0, meta = 0;
  uint32_t pl[kPW];  // entry payload
#pragma unroll
  for (int t = 0; t < kPW; ++t) pl[t] = 0xFFFFFFFFu;
  // Region reads are pipelined with the entry loads: every loop iteration is
  // ONE memory round trip for the wave.  A step that selects inside a region
  // spends extra iterations (directory words dw0/dw1: ph 1; the 64 B block:
  // ph 2, searched as soon as it arrives -> ph 3 with the chosen position kb)
  // while the other lanes keep stepping; a region membership test reads its
  // bitset word together with the entry of the candidate (speculatively;
  // dropped when the candidate is common).
  uint32_t ph = 0, t = 0;  // phase; select rank (ph 1: j; ph 2: rank inside block g)
  int64_t g = 0;           // region block within the row
  uint32_t dw0 = 0u, dw1 = 0u, kb = 0u;  // ph 1: directory entries g, g+1; ph 3: selected position
  uint32_t dg_iter = 0, dg_act = 0;  // diag bit 64: wave iterations / this lane's active ones
  for (;;) {
    const bool active = len < L && d != 0;
    if (__ballot(active) == 0ull) break;
    if (kGwDiag && (P.diag & 64)) {
      ++dg_iter;
      dg_act += active ? 1u : 0u;
    }
    uint32_t slot = 0xFFFFFFFFu;  // entry to fetch (accepted or speculative step)
    bool spec = false;            // slot is accepted unless bit sbit of sw is set
    uint32_t sw = 0u, sbit = 0u;
    uint64_t sec = 0ull;  // 64 B sector this lane fetches: its next entry or a region block
    bool isblk = false;
    bool virt = false;    // return whose entry is already known (no fetch)
    if (active) {
      const uint32_t mode = meta & 3u;
      const int efl = (int)((meta >> 2) & 31u);
      const uint32_t efU = (meta >> 7) & 511u;
      const uint32_t* hreg = G.bs_region + (uint64_t)pl[0] * kBlk;  // region mode only
      const int64_t ndir = bs_ndir(d);
      int64_t k = 0;
      bool acc = false;
      if (ph == 3) {  // the region block arrived last iteration and was searched there
        k = kb;
        acc = true;
        ph = 0;
      } else if (ph == 1) {  // directory entries g, g+1 have arrived
        const uint32_t lo = dw0, hi = g + 1 < ndir ? dw1 : c;
        if (t < lo || t >= hi) {
          g += t < lo ? -1 : 1;
          dw0 = hreg[g];
          dw1 = g + 1 < ndir ? hreg[g + 1] : 0u;
        } else {
          t -= lo;
          ph = 2;
        }
      } else {
        const gw_u4 u = gw_philox(c0, c1, (uint32_t)len, trial, P.k0, P.k1);
        ++trial;
        int op = 0;  // 1: the j-th common position; 2: is draw k common
        uint32_t j = 0;
        if (len == 1) {
          k = (int64_t)gw_index(u.x, u.z, d);
          acc = true;
        } else {
          bool other = trial > 1;  // a retry is always the "other" branch
          if (!other) {
            const double Z = (P.a_p + (double)c) + (double)((int64_t)d - 1 - (int64_t)c) * P.a_q;
            const double r = gw_u01(u.x) * Z;
            if (r < P.a_p) {
              k = kp;  // return to prev
              acc = true;
            } else if (r - P.a_p < (double)c) {
              j = (uint32_t)(r - P.a_p);
              if (j >= c) j = c - 1;
              op = 1;
            } else {
              other = true;
            }
          }
          if (other) {
            k = (int64_t)gw_index(u.y, u.z, d);
            op = 2;
          }
        }
        if (kGwDiag && P.diag) {  // timing experiments only (-DGW_DIAG builds)
          if (op == 1 && (P.diag & 1)) {
            k = (int64_t)((uint64_t)j * (uint64_t)d / c);
            acc = true;
            op = 0;
          }
          if (op == 2 && (P.diag & 2)) {
            acc = k != (int64_t)kp;
            op = 0;
          }
        }
        bool common = false;
        // payload selects: the j-th one (inline bitset, Elias-Fano high
        // parts) or the (eh-1)-th zero (start of Elias-Fano bucket eh)
        const uint32_t eh = (uint32_t)k >> efl;
        const bool ef_mem = op == 2 && mode == BS_EF && eh <= efU - c;
        int pos = 0;
        if ((op == 1 && (mode == BS_INLINE || mode == BS_EF)) || (ef_mem && eh > 0)) {
          const bool inv = op == 2;
          uint32_t wp[kPW];
#pragma unroll
          for (int q = 0; q < kPW; ++q) wp[q] = inv ? ~pl[q] : pl[q];
          pos = regs_select<kPW>(wp, inv ? eh - 1 : j);
        }
        const uint32_t es = (ef_mem && eh > 0) ? (uint32_t)pos + 1u : 0u;  // first bit of bucket eh
        // ONE 32-bit payload window per lane serves every mode: the j-th u16
        // of a list, bit k of an inline bitset, the Elias-Fano low part j /
        // the low parts of bucket eh, the region draw-filter bucket
        const uint32_t fb = gw_bounded(u.y, bs_filt_buckets(ndir, d));
        const uint32_t wpos = mode == BS_LIST     ? 16u * j
                              : mode == BS_INLINE ? (uint32_t)k
                              : mode == BS_EF     ? efU + (op == 1 ? j : es - eh) * (uint32_t)efl
                                                  : 32u * bs_filt_word(ndir) + fb;
        const uint32_t win = bits32(pl, wpos);
        if (op == 1) {
          if (mode == BS_INLINE) {
            k = (int64_t)pos;
            acc = true;
          } else if (mode == BS_EF) {
            k = ((int64_t)(uint32_t)(pos - (int)j) << efl) | (win & ((1u << efl) - 1u));
            acc = true;
          } else if (mode == BS_LIST) {
            k = (int64_t)(win & 0xFFFFu);
            acc = true;
          } else {  // BS_REGION
            if (ndir > kPDir) {  // directory in the region: guess the block, verify next iteration
              g = (int64_t)((float)j * (float)ndir * __builtin_amdgcn_rcpf((float)c));
              if (g >= ndir) g = ndir - 1;
              dw0 = hreg[g];
              dw1 = g + 1 < ndir ? hreg[g + 1] : 0u;
              t = j;
              ph = 1;
            } else {  // <= 8 directory counts (u16) in w[1..4]: count those <= j
              uint32_t lo = 0;
              g = 0;
#pragma unroll
              for (int q = 1; q < kPDir; ++q) {
                const uint32_t dq = (pl[1 + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu;
                const bool in = q < ndir && dq <= j;
                g += in ? 1 : 0;
                lo = in ? dq : lo;
              }
              t = j - lo;
              ph = 2;
            }
          }
        } else if (op == 2) {
          if (mode == BS_LIST) {
            common = c != 0u && list_has(pl, (uint32_t)k, (meta & kMetaDual) != 0u);
          } else if (mode == BS_INLINE) {
            common = win & 1u;
          } else if (mode == BS_EF) {
            common = ef_mem && ef_bucket_has(pl, efU, (uint32_t)efl, es, es - eh, (uint32_t)k, win);
          } else if (k != (int64_t)kp && trial < (1u << 24)) {  // BS_REGION
            if (win & 1u) {  // the draw filter says maybe common: read the word
              sw = (kGwDiag && (P.diag & 8)) ? G.bs_region[((uint32_t)k >> 5) & 0xFFFFu]  // timing experiment: no TLB misses
                                : hreg[(meta >> 16) * kBlk + (k >> 5)];
              sbit = (uint32_t)(k & 31);
              spec = true;
            }
          }
          acc = (k != (int64_t)kp && !common) || trial >= (1u << 24);
        }
      }
      if (ph == 2 && !acc) {  // fetch the region block (this iteration's round trip)
        sec = (kGwDiag && (P.diag & 4)) ? (uint64_t)(G.bs_region + kBlk * ((pl[0] + (uint32_t)g) & 0xFFFu))
                           : (uint64_t)(hreg + ((meta >> 16) + (uint32_t)g) * kBlk);
        isblk = true;
      }
      if (acc) {
        if ((meta & kMetaStash) && k == (int64_t)kp) {
          // return over a dual entry's edge: the entry of the reverse slot
          // (cur -> prev) is {prev, its degree and row, kp = the index drawn
          // at prev (stash, pl[6..9]), its list (pl[3..5]) and count}
          virt = true;
        } else {
          slot = b + (uint32_t)k;
          sec = (uint64_t)(ents + (uint64_t)slot * 4u);
        }
      }
    }
    // cooperative sector load (entries and region blocks alike): all four
    // rounds in flight, then the exchange
    const uint4 r0 = coop_piece(sec, lane, 0), r1 = coop_piece(sec, lane, 1);
    const uint4 r2 = coop_piece(sec, lane, 2), r3 = coop_piece(sec, lane, 3);
    if (spec && ((sw >> sbit) & 1u)) {  // the candidate was common: rejected
      slot = 0xFFFFFFFFu;
      sec = 0ull;
    }
    // piece-major exchange: quarter q moves piece q (16 B) of EVERY walker —
    // the lanes that loaded it write their four rounds, then every lane reads
    // its own piece — so each lane's 16 words arrive unconditionally (no
    // per-round conditional copies of the entry / block registers)
    uint32_t E[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_wave_barrier();
      if ((lane & 3) == q) {
        ex[lane >> 2] = r0;
        ex[16 + (lane >> 2)] = r1;
        ex[32 + (lane >> 2)] = r2;
        ex[48 + (lane >> 2)] = r3;
      }
      __builtin_amdgcn_wave_barrier();
      const uint4 v = ex[lane];
      E[4 * q] = v.x;
      E[4 * q + 1] = v.y;
      E[4 * q + 2] = v.z;
      E[4 * q + 3] = v.w;
    }
    __builtin_amdgcn_wave_barrier();
    if (isblk) {  // the region block: pick the t-th set bit now
      kb = (uint32_t)(g * kDirBits) + (uint32_t)regs_select<kBlk>(E, t);
      ph = 3;
    }
    if (slot != 0xFFFFFFFFu) {
      const uint32_t ou = (uint32_t)cur, od = d, ob = b, ok = slot - b;
      cur = (int32_t)E[0];
      d = E[1];
      b = E[2];
      meta = E[3];
      unpack_entry(E, &kp, &c, pl);
      if (meta & kMetaDual) {
        // dual list entry (both degrees < 65536): its payload words 6..9
        // keep the row we came from, so a return needs no fetch
        pl[6] = ou;
        pl[7] = od;
        pl[8] = ob;
        pl[9] = ok;
        meta |= kMetaStash;
      }
    }
    if (virt) {  // the walker is back at prev: swap rows, lists and counts
      const uint32_t tc = (uint32_t)cur, td = d, tb = b, tk = kp;
      cur = (int32_t)pl[6];
      d = pl[7];
      b = pl[8];
      kp = pl[9];
      pl[6] = tc;
      pl[7] = td;
      pl[8] = tb;
      pl[9] = tk;
#pragma unroll
      for (int q = 0; q < (int)kDualC / 2; ++q) {
        const uint32_t t = pl[q];
        pl[q] = pl[q + kDualC / 2];
        pl[q + kDualC / 2] = t;
      }
      const uint32_t c_rev = (meta >> 2) & 7u;
      meta = kMetaDual | kMetaStash | (c << 2);
      c = c_rev;
    }
    const bool moved = slot != 0xFFFFFFFFu || virt;
    if (moved) {
      my_trials += trial;
      trial = 0;
    }
    bool ready = false;  // this lane completed 16 staged positions (flen-15 .. flen)
    int flen = 0;
    if (moved) {
      stage[64 * (len & (kStage - 1))] = cur;
      ready = (len & (kStage - 1)) == kStage - 1;
      flen = len;
      ++len;
    }
    // flush of the ready walkers' 64 B chunks, cooperative like the loads:
    // an instruction writes 16 whole sectors instead of a 16 B piece of 64.
    // The ready walkers are compacted first (each publishes its lane at its
    // rank among them), so a flush takes ceil(ready / 16) rounds, not 4:
    // walkers drift apart by their retries and region phases, so most
    // flushes serve a few walkers
    const unsigned long long rm = __ballot(ready);
    if (rm && !(kGwDiag && (P.diag & 32))) {
      if (vec_ok) {
        const int nready = __popcll(rm);
        int32_t* ids = reinterpret_cast<int32_t*>(ex);  // the exchange buffer is free here
        __builtin_amdgcn_wave_barrier();
        if (ready)
          ids[__builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u))] = lane;
        __builtin_amdgcn_wave_barrier();
        const int32_t* sw = &s_stage[wv][0][0];
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
    int32_t* row = out + i * (int64_t)L;
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
    if (kGwDiag && (P.diag & 64)) {  // lane utilisation: counters[2] += 64 x wave iterations, [3] += active lanes
      unsigned long long a = dg_act;
      for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off, 64);
      if ((threadIdx.x & 63) == 0) {
        atomicAdd(&counters[2], 64ull * dg_iter);
        atomicAdd(&counters[3], a);
      }
    }
  }
}

// ---- listed rejection sampler (GW_N2V_REJECTION, unweighted undirected) ----
// k_walk_scale's exact sampler — the same Philox draws, envelope, outlier
// return edge and acceptance tests, hence the same walks (oracle.walks_scale)
// — with one change: the lazy has_edge(x, prev) probe is answered from the
// payload of the entry that brought the walker to cur (the common neighbours
// of prev and cur as positions in N(cur), gw_dev_bitset_build(lists_only))
// whenever that payload is a list, an inline bitset or Elias-Fano; entries
// whose common set would need a region carry none, and those steps probe
// prev's neighbour hash as k_walk_scale does.  The candidate's 64 B entry is
// fetched cooperatively (k_walk_bitset's loads, exchange and flush).
struct LsParams {
  double a_q, M, lo, extra, h_prev;
  uint32_t k0, k1, pk0, pk1;
};

// k in the entry payload's common set (mode list / inline / Elias-Fano)
__device__ __forceinline__ bool payload_has(const uint32_t (&pl)[kPW], uint32_t meta, uint32_t c, uint32_t k) {
  const uint32_t mode = meta & 3u;
  const uint32_t efl = (meta >> 2) & 31u, efU = (meta >> 7) & 511u;
  if (mode == BS_LIST) return list_has(pl, k, (meta & 0x8000u) != 0u);  // bit 15: dual entry
  const uint32_t eh = k >> efl;
  uint32_t es = 0;
  if (mode == BS_EF && eh > 0) {  // bucket eh starts after the (eh-1)-th zero of the high parts
    uint32_t wp[kPW];
#pragma unroll
    for (int q = 0; q < kPW; ++q) wp[q] = ~pl[q];
    es = (uint32_t)regs_select<kPW>(wp, eh - 1) + 1u;
  }
  const uint32_t win = bits32(pl, mode == BS_INLINE ? k : efU + (es - eh) * efl);
  if (mode == BS_INLINE) return win & 1u;
  return eh <= efU - c && ef_bucket_has(pl, efU, efl, es, es - eh, k, win);
}

__global__ void __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(5, 5)))
k_walk_listed(gw_dev_graph G, LsParams P, int L, int64_t walk_begin, int64_t walk_count, int shuffle,
              int32_t* __restrict__ out, int32_t* __restrict__ lens, unsigned long long* __restrict__ counters) {
  __shared__ int32_t s_stage[kB / 64][kStage][64];
  __shared__ uint4 s_ex[kB / 64][64];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  int32_t* stage = &s_stage[wv][0][lane];
  uint4* ex = s_ex[wv];
  const uint4* __restrict__ ents = reinterpret_cast<const uint4*>(G.bs_nbr);

  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < walk_count;
  unsigned long long my_steps = 0, my_trials = 0;
  const int64_t w = walk_begin + (valid ? i : 0);
  int32_t cur = -1, prev = -1;
  int len = L;
  if (valid) {
    const uint64_t it = (uint64_t)w / (uint64_t)G.n;
    const uint64_t pos = (uint64_t)w % (uint64_t)G.n;
    const uint64_t sp = shuffle ? gw_feistel_perm(pos, (uint64_t)G.n, P.pk0, P.pk1, (uint32_t)it) : pos;
    cur = G.order[sp];
    len = 1;
  }
  const bool vec_ok = (L & 3) == 0;
  const uint32_t c0 = (uint32_t)w, c1 = (uint32_t)((uint64_t)w >> 32);
  stage[0] = cur;
  uint32_t trial = 0;
  uint32_t b = 0, d = 0, pb = 0, pd = 0;  // rows of cur and prev (slot indices < 2^32)
  if (valid) {
    b = (uint32_t)G.offsets[cur];
    d = (uint32_t)(G.offsets[cur + 1] - G.offsets[cur]);
  }
  // payload of the entry (prev -> cur): meta (mode, Elias-Fano l / U) with
  // min(c, 0xFFFF) in bits 16..31; mode BS_REGION = none, has_edge probes
  uint32_t meta = BS_REGION;
  uint32_t pl[kPW];
#pragma unroll
  for (int t = 0; t < kPW; ++t) pl[t] = 0u;
  // A probe is pipelined: the candidate's entry is parked (header below, its
  // payload in pl, which is unused while meta says BS_REGION) and the hash
  // slot of prev's row is read in the NEXT iteration beside the other lanes'
  // entry loads; the decision uses the draw kept in t.
  bool pend = false;
  int32_t px = 0;
  uint32_t pdx = 0, poff = 0, pmeta = 0;
  double t = 0.0;
  // a BS_REGION entry's pl is its draw filter (kFiltL buckets over the draw's
  // high word u.x; a clear bucket proves the candidate is not common) until a
  // parked candidate overwrites it
  bool filt = false;
  uint32_t fb = 0;
  for (;;) {
    const bool active = len < L && d != 0;
    if (__ballot(active) == 0ull) break;
    uint64_t sec = 0ull;  // the candidate's entry
    uint32_t k = 0;
    bool ret = false;  // outlier return to prev (no entry read)
    // pending probe: first slot of px's run in prev's neighbour hash
    uint32_t hs = 0;
    int4 h0 = make_int4(-1, -1, -1, -1);
    if (pend) {
      hs = gw_eh_slot(px, pd);
      h0 = gw_eh_row(G.eh, pb)[hs];
    }
    if (active && !pend) {
      if (len == 1) {  // first order (node2vec.py:28-29)
        const gw_u4 u = gw_philox(c0, c1, 1u, 0u, P.k0, P.k1);
        trial = 1;
        k = gw_index(u.x, u.z, d);
      } else {
        const gw_u4 u = gw_philox(c0, c1, (uint32_t)len, trial, P.k0, P.k1);
        ++trial;
        const double A = P.M * (double)d + P.extra;
        if (P.extra > 0.0 && gw_u01(u.z) * A < P.extra) {
          ret = true;
        } else {
          k = gw_index(u.x, u.y, d);
          t = gw_u01(u.w) * P.M;
          fb = (uint32_t)(((uint64_t)u.x * kFiltL) >> 32);
        }
      }
      if (!ret) sec = (uint64_t)(ents + (uint64_t)(b + k) * 4u);
    }
    const uint4 r0 = coop_piece(sec, lane, 0), r1 = coop_piece(sec, lane, 1);
    const uint4 r2 = coop_piece(sec, lane, 2), r3 = coop_piece(sec, lane, 3);
    uint32_t E[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_wave_barrier();
      if ((lane & 3) == q) {
        ex[lane >> 2] = r0;
        ex[16 + (lane >> 2)] = r1;
        ex[32 + (lane >> 2)] = r2;
        ex[48 + (lane >> 2)] = r3;
      }
      __builtin_amdgcn_wave_barrier();
      const uint4 v = ex[lane];
      E[4 * q] = v.x;
      E[4 * q + 1] = v.y;
      E[4 * q + 2] = v.z;
      E[4 * q + 3] = v.w;
    }
    __builtin_amdgcn_wave_barrier();
    bool acc = ret, take = false;  // take: adopt the entry in E (else the parked one)
    if (pend) {  // the probe's bucket arrived: a full bucket (rare) continues the query
      const int r0 = gw_eh_scan(h0, px);
      const bool adj = r0 > 0 || (r0 < 0 && gw_eh_has_from(G.eh, pb, pd, hs, px));
      acc = t < (adj ? 1.0 : P.a_q) || trial >= (1u << 24);
      pend = false;
    } else if (sec != 0ull) {
      const int32_t next = (int32_t)E[0];
      if (len == 1) {
        acc = true;
      } else if (next == prev) {
        acc = t < P.h_prev;
      } else if (t < P.lo) {
        acc = true;
      } else if ((meta & 3u) != BS_REGION) {
        acc = t < (payload_has(pl, meta, meta >> 16, k) ? 1.0 : P.a_q);
      } else if (filt && !((pickw(pl, fb >> 5) >> (fb & 31)) & 1u)) {
        acc = t < P.a_q;  // the filter proves "not common"
      } else if (G.eh) {  // park the candidate, probe next iteration
        pend = true;
        filt = false;  // pl will hold the parked payload
        px = next;
      } else {
        acc = t < (bs_has_edge(G, pb, (int64_t)pb + pd, next) ? 1.0 : P.a_q);
      }
      if (trial >= (1u << 24) && !pend) acc = true;
      take = true;
    }
    if (take && (pend || acc)) {  // the arrived entry becomes the parked or the current one
      uint32_t ekp, ec;
      unpack_entry(E, &ekp, &ec, pl);
      pdx = E[1];
      poff = E[2];
      pmeta = (E[3] & 0x7FFFu) | ((E[3] & kMetaDual) ? 0x8000u : 0u) | (min(ec, 0xFFFFu) << 16);
    }
    bool ready = false;
    int flen = 0;
    if (acc) {
      my_trials += trial;
      trial = 0;
      const int32_t next = ret ? prev : take ? (int32_t)E[0] : px;  // (E[0] == px when parked)
      const uint32_t ob = pb, od = pd;
      prev = cur;
      pb = b;
      pd = d;
      cur = next;
      if (ret) {  // back over the same edge: the old prev's row, no payload for (cur -> prev)
        b = ob;
        d = od;
        meta = BS_REGION;
      } else {  // the arrived or the parked entry: header in pdx / poff / pmeta, payload in pl
        d = pdx;
        b = poff;
        meta = pmeta;
      }
      filt = !ret && (meta & 3u) == BS_REGION;
      stage[64 * (len & (kStage - 1))] = cur;
      ready = (len & (kStage - 1)) == kStage - 1;
      flen = len;
      ++len;
    }
    const unsigned long long rm = __ballot(ready);
    if (rm) {
      if (vec_ok) {
        const int nready = __popcll(rm);
        int32_t* ids = reinterpret_cast<int32_t*>(ex);
        __builtin_amdgcn_wave_barrier();
        if (ready)
          ids[__builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u))] = lane;
        __builtin_amdgcn_wave_barrier();
        const int32_t* sw = &s_stage[wv][0][0];
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
    int32_t* row = out + i * (int64_t)L;
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

// row holding adjacency slot e (upper bound over offsets)
__device__ __forceinline__ int64_t bs_row_of(const gw_dev_graph& G, int64_t e) {
  int64_t lo = 0, hi = G.n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (G.offsets[mid + 1] <= e)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// sum over undirected edges of min(deg u, deg v) = k_bs_tri's probes (each
// edge counted at its owner u, where min = deg v).  Edge-centric: a thread
// takes kWorkChunk consecutive slots (one row search per row it enters), so a
// hub's row is spread over many threads instead of one serial loop.
constexpr int kWorkChunk = 16;
__global__ void k_bs_work(gw_dev_graph G, unsigned long long* __restrict__ acc) {
  const int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kWorkChunk;
  unsigned long long w = 0;
  if (e0 < G.nnz) {
    const int64_t e1 = e0 + kWorkChunk < G.nnz ? e0 + kWorkChunk : G.nnz;
    int64_t u = bs_row_of(G, e0);
    int64_t ue = G.offsets[u + 1];
    int64_t du = ue - G.offsets[u];
    for (int64_t e = e0; e < e1; ++e) {
      if (e >= ue) {
        u = bs_row_of(G, e);
        ue = G.offsets[u + 1];
        du = ue - G.offsets[u];
      }
      const int32_t v = G.nbrs[e];
      const int64_t dv = G.deg[v];
      if (du > dv || (du == dv && u <= v)) w += (unsigned long long)dv;
    }
  }
  for (int o = 32; o > 0; o >>= 1) w += __shfl_down(w, o, 64);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(acc, w);
}

// Build the per-edge entries and regions (k_bs_tri, see the build section):
// pass 1 writes every slot's header, regions are sized from the exact
// (c, d) (slots whose payload fits the entry take no region space) and
// placed by a scan, pass 2 writes the payloads.  Work items are scheduled
// hubs first (vertices in degree-descending order).  lists_only: no regions
// at all — entries whose payload would need one keep mode BS_REGION and a
// draw filter (the rejection sampler's listed entries, k_walk_listed, probes
// for those).
int gw_dev_bitset_build(gw_graph* g, int64_t budget_bytes, bool lists_only) {
  gw_dev_graph& d = g->d;
  gw_dev_bitset_release(g);
  const int64_t nnz = g->nnz, n = g->n;
  if (nnz == 0) return GW_OK;
  if (nnz >= (int64_t)0xFFFFFFFF) {  // the walk kernel passes slot indices as u32
    g->err = "bitset mode supports < 2^32 - 1 adjacency entries: use GW_N2V_REJECTION";
    return GW_ERR_CAPACITY;
  }
  if (nnz * (int64_t)sizeof(gw_bs_nbr) > budget_bytes) {
    g->err = "bitset entries need " + std::to_string(nnz * (int64_t)sizeof(gw_bs_nbr)) + " B; over the " +
             std::to_string(budget_bytes) + " B budget: use GW_N2V_REJECTION";
    return GW_ERR_CAPACITY;
  }
  // a REGION entry packs its directory block count in meta bits 16.. (about
  // deg / 8192); past 2^27 it would reach kMetaDual / kMetaStash (bits 30, 31)
  if (g->max_degree >= ((int64_t)1 << 27)) {
    g->err = "bitset mode supports vertex degrees < 2^27: use GW_N2V_REJECTION";
    return GW_ERR_UNSUPPORTED;
  }
  int rc;
  uint64_t* sz = nullptr;
  uint64_t* roff = nullptr;
  int32_t *ids = nullptr, *order = nullptr;
  int32_t* dkey = nullptr;  // sorted degrees (discarded)
  uint32_t* nit = nullptr;
  uint32_t* itoff = nullptr;
  TriItem* items = nullptr;
  void* tmp = nullptr;
  auto cleanup = [&]() {
    bs_free(sz);
    bs_free(roff);
    bs_free(ids);
    bs_free(order);
    bs_free(nit);
    bs_free(itoff);
    bs_free(items);
    bs_free(tmp);
    bs_free(dkey);
  };
  auto fail = [&](int code) {
    cleanup();
    gw_dev_bitset_release(g);
    return code;
  };
#define BS_TRY(expr)                                                 \
  do {                                                               \
    hipError_t _e = (expr);                                          \
    if (_e != hipSuccess) {                                          \
      g->err = std::string(#expr) + ": " + hipGetErrorString(_e);    \
      return fail(GW_ERR_DEVICE);                                    \
    }                                                                \
  } while (0)
  if ((rc = bs_alloc(g, &d.bs_nbr, nnz)) || (rc = bs_alloc(g, &ids, n)) ||
      (rc = bs_alloc(g, &order, n)) || (rc = bs_alloc(g, &nit, n + 1)) || (rc = bs_alloc(g, &itoff, n + 1)))
    return fail(rc);
  const unsigned gn = (unsigned)((n + kB - 1) / kB), gn1 = (unsigned)((n + 1 + kB - 1) / kB);
  BS_TRY(hipMemset(d.bs_nbr, 0, (size_t)nnz * sizeof(gw_bs_nbr)));
  k_bs_iota<<<gn, kB>>>(n, ids);
  BS_TRY(hipGetLastError());
  // work items: vertices by degree, descending (hubs first), kTriEB edges each
  size_t tb = 0, tb2 = 0;
  BS_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, (const int32_t*)nullptr, (int32_t*)nullptr,
                                                      (const int32_t*)nullptr, (int32_t*)nullptr, (int)n));
  BS_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, nit, itoff, (int)(n + 1)));
  if ((rc = bs_alloc(g, (char**)&tmp, (int64_t)std::max(tb, tb2) + 1))) return fail(rc);
  if ((rc = bs_alloc(g, &dkey, n))) return fail(rc);
  BS_TRY(hipcub::DeviceRadixSort::SortPairsDescending(tmp, tb, d.deg, dkey, ids, order, (int)n));
  // diagnostics build (GW_DIAG_BS_FILL & 8): both passes launched as two
  // dispatches, vertices of degree > 64 and the rest, to time them apart
  int bs_diag = 0;
  if (const char* dg = GW_DIAG_ENV("GW_DIAG_BS_FILL")) bs_diag = std::atoi(dg);
  int64_t nbig = 0;
  if (bs_diag & 8) {
    std::vector<int32_t> hk((size_t)n);
    BS_TRY(hipMemcpy(hk.data(), dkey, (size_t)n * 4, hipMemcpyDeviceToHost));
    while (nbig < n && hk[(size_t)nbig] > 64) ++nbig;
  }
  bs_free(dkey);
  k_bs_nitems<<<gn1, kB>>>(d, order, nit);
  BS_TRY(hipGetLastError());
  BS_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, nit, itoff, (int)(n + 1)));
  uint32_t nitems = 0, isplit = 0;
  BS_TRY(hipMemcpy(&nitems, itoff + n, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (bs_diag & 8) BS_TRY(hipMemcpy(&isplit, itoff + nbig, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if ((rc = bs_alloc(g, &items, std::max<int64_t>(nitems, 1)))) return fail(rc);
  k_bs_items<<<gn, kB>>>(d, order, itoff, items);
  BS_TRY(hipGetLastError());
  bs_free(tmp);
  bs_free(ids);
  bs_free(order);
  bs_free(nit);
  bs_free(itoff);
  // pass 1: headers
  auto tri = [&](bool fill, const TriItem* it, uint32_t cnt) {
    if (!cnt) return;
    const unsigned tgrid = std::min<uint32_t>(cnt, 1u << 20);  // <= 2^29 work-items per launch
    if (fill)
      k_bs_tri<true><<<tgrid, kTB>>>(d, it, cnt, d.bs_nbr, roff, d.bs_region, (lists_only ? 1 : 0) | (bs_diag << 8));
    else
      k_bs_tri<false><<<tgrid, kTB>>>(d, it, cnt, d.bs_nbr, nullptr, nullptr, lists_only ? 1 : 0);
  };
  auto tri_all = [&](bool fill) {
    if (bs_diag & 8) {
      tri(fill, items, isplit);
      tri(fill, items + isplit, nitems - isplit);
    } else {
      tri(fill, items, nitems);
    }
  };
  tri_all(false);
  BS_TRY(hipGetLastError());
  // region layout
  if ((rc = bs_alloc(g, &sz, nnz + 1)) || (rc = bs_alloc(g, &roff, nnz + 1))) return fail(rc);
  const unsigned grid = (unsigned)((nnz + kB - 1) / kB);
  k_bs_sizes<<<grid, kB>>>(d, d.bs_nbr, sz, lists_only ? 1 : 0);
  BS_TRY(hipGetLastError());
  BS_TRY(hipMemset(sz + nnz, 0, sizeof(uint64_t)));
  size_t tmpb = 0;
  BS_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, sz, roff, nnz + 1));
  if ((rc = bs_alloc(g, (char**)&tmp, (int64_t)tmpb + 1))) return fail(rc);
  BS_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, sz, roff, nnz + 1));
  BS_TRY(hipDeviceSynchronize());
  bs_free(tmp);
  bs_free(sz);
  uint64_t words = 0;
  BS_TRY(hipMemcpy(&words, roff + nnz, sizeof(uint64_t), hipMemcpyDeviceToHost));
  const int64_t need = (int64_t)words * 4 + nnz * (int64_t)sizeof(gw_bs_nbr);
  if (need > budget_bytes) {
    g->err = "per-edge bitsets need " + std::to_string(need) + " B; over the " + std::to_string(budget_bytes) +
             " B budget: use GW_N2V_REJECTION";
    return fail(GW_ERR_CAPACITY);
  }
  if (words == 0) words = 1;  // no region at all: keep a valid pointer
  if ((rc = bs_alloc(g, &d.bs_region, (int64_t)words))) return fail(rc);
  BS_TRY(hipMemset(d.bs_region, 0, (size_t)words * 4));
  // pass 2: payloads
  tri_all(true);
  BS_TRY(hipGetLastError());
  BS_TRY(hipDeviceSynchronize());
#undef BS_TRY
  cleanup();
  g->bitset_words = (int64_t)words;
  return GW_OK;
}

// Modelled wall time of gw_dev_bitset_build on this graph: two k_bs_tri
// passes over sum(min(deg u, deg v)) probes plus per-slot header / payload
// traffic, at rates measured on MI355X; < 0 on a device error.
double gw_bitset_build_model_s(gw_graph* g) {
  // GW_N2V_AUTO asks up to three times per prepare (pilot choice, listed_pays
  // twice): the O(nnz) model kernel runs once per resident graph
  if (g->bs_model_s >= 0.0) return g->bs_model_s;
  unsigned long long* acc = nullptr;
  if (hipMalloc((void**)&acc, sizeof(unsigned long long)) != hipSuccess) return -1.0;
  unsigned long long w = 0;
  bool ok = hipMemset(acc, 0, sizeof w) == hipSuccess;
  if (ok && g->nnz > 0) {
    const int64_t threads = (g->nnz + kWorkChunk - 1) / kWorkChunk;
    k_bs_work<<<(unsigned)((threads + kB - 1) / kB), kB>>>(g->d, acc);
    ok = hipGetLastError() == hipSuccess;
  }
  ok = ok && hipMemcpy(&w, acc, sizeof w, hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(acc);
  if (!ok) return -1.0;
  g->bs_model_s = 2.0 * (double)w / kBuildProbeRate + (double)g->nnz * kBuildSlotSeconds;
  return g->bs_model_s;
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
  const char* dg = GW_DIAG_ENV("GW_DIAG_BS");  // diagnostic A/B knob only
  P.diag = dg ? (uint32_t)atoi(dg) : 0u;
  if (const char* ns = GW_DIAG_ENV("GW_DIAG_NO_STORE")) P.diag |= ns[0] == '1' ? 32u : 0u;
  const unsigned grid = (unsigned)std::max<int64_t>(1, (walk_count + kB - 1) / kB);
  k_walk_bitset<<<grid, kB, 0, (hipStream_t)stream>>>(g->d, P, L, walk_begin, walk_count, shuffle, out_dev,
                                                       len_dev, (unsigned long long*)counters_dev);
  GW_HIP_TRY(hipGetLastError());
  return GW_OK;
}

int gw_dev_walk_listed_launch(gw_graph* g, int L, uint64_t seed, int64_t walk_begin, int64_t walk_count,
                              int shuffle, int32_t* out_dev, int32_t* len_dev, uint64_t* counters_dev,
                              void* stream) {
  LsParams P;
  const double a_p = 1.0 / g->p;
  P.a_q = 1.0 / g->q;
  P.M = std::max(1.0, P.a_q);
  P.lo = std::min(1.0, P.a_q);
  P.extra = a_p > P.M ? a_p - P.M : 0.0;
  P.h_prev = std::min(a_p, P.M);
  P.k0 = (uint32_t)seed;
  P.k1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_STEP;
  P.pk0 = (uint32_t)seed;
  P.pk1 = (uint32_t)(seed >> 32) ^ GW_TAG_N2V_PERM;
  const unsigned grid = (unsigned)std::max<int64_t>(1, (walk_count + kB - 1) / kB);
  k_walk_listed<<<grid, kB, 0, (hipStream_t)stream>>>(g->d, P, L, walk_begin, walk_count, shuffle, out_dev,
                                                       len_dev, (unsigned long long*)counters_dev);
  GW_HIP_TRY(hipGetLastError());
  return GW_OK;
}
