// Counter-based RNG shared by the HIP kernels and the host code.
//
// Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
// SC'11).  Every random decision on the scale-mode paths is a pure function
// of (seed, purpose, unit id, step, trial), so results are identical for any
// grid shape, any GPU count and any shard split.
//
// The reference draws from global, sequential streams instead
// (node2vec.py:156-157 `np.random.rand()`, Graph.java:17,72
// `java.util.Random.nextInt`); the exact-replay path for node2vec consumes a
// caller-supplied MT19937 uniform buffer instead of this generator.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GW_HD __host__ __device__ __forceinline__
#else
#define GW_HD static inline
#endif

// Purpose tags folded into key[1] so independent decisions never share a
// counter block.
#define GW_TAG_N2V_STEP 0x6E327632u   // "n2v2": walk transitions
#define GW_TAG_N2V_PERM 0x7065726Du   // "perm": per-iteration start shuffle
#define GW_TAG_TOPSIM 0x746F7053u     // "topS": TopSim random children
#define GW_TAG_RMAT 0x726D6174u       // "rmat": synthetic graph generator

struct gw_u4 {
  uint32_t x, y, z, w;
};

GW_HD void gw_mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

GW_HD struct gw_u4 gw_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                             uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    gw_mulhilo32(M0, c0, &hi0, &lo0);
    gw_mulhilo32(M1, c2, &hi1, &lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += W0;
    k1 += W1;
  }
  struct gw_u4 r;
  r.x = c0;
  r.y = c1;
  r.z = c2;
  r.w = c3;
  return r;
}

// u32 -> [0,1) double with 32 random bits (exact: x * 2^-32).
GW_HD double gw_u01(uint32_t x) { return (double)x * 2.3283064365386963e-10; }

// Bucket in [0, d) of a 32-bit draw: multiply-high (relative bias <= d / 2^32).
// Used for the small fixed bucket counts of the walk kernels' draw filters.
GW_HD uint32_t gw_bounded(uint32_t x, uint32_t d) {
  return (uint32_t)(((uint64_t)x * (uint64_t)d) >> 32);
}

// Uniform index in [0, d) of a 64-bit draw v = hi * 2^32 + lo: floor(v * d / 2^64),
// exactly (hi*d + floor(lo*d / 2^32) < 2^64 and its floor / 2^32 equals the full
// product's).  Relative bias <= d / 2^64, below the reference's floor(U*K) with
// a 53-bit U (node2vec.py:157, K / 2^53) for every d < 2^32.  Every neighbour
// index draw uses it; identical on host and device so parity is bitwise.
GW_HD uint32_t gw_index(uint32_t hi, uint32_t lo, uint32_t d) {
  return (uint32_t)(((uint64_t)hi * (uint64_t)d + (((uint64_t)lo * (uint64_t)d) >> 32)) >> 32);
}

// Keyed bijection on [0, n) (n < 2^62): a 4-round Feistel network over the
// smallest even-bit-width power-of-two domain >= n with cycle walking.  Used
// for the per-iteration start-node shuffle (reference: node2vec.py:49-51
// `random.shuffle(nodes)` once per walk iteration).
GW_HD uint64_t gw_feistel_perm(uint64_t i, uint64_t n, uint32_t k0, uint32_t k1,
                               uint32_t iter) {
  if (n <= 1) return 0;
  int bits = 2;
  while ((1ull << bits) < n) bits += 2;
  const int half = bits / 2;
  const uint64_t mask = (1ull << half) - 1ull;
  uint64_t x = i;
  do {
    uint64_t L = x >> half, R = x & mask;
    for (uint32_t r = 0; r < 4; ++r) {
      struct gw_u4 f = gw_philox((uint32_t)R, (uint32_t)(R >> 32), iter, r, k0, k1);
      uint64_t F = (((uint64_t)f.y << 32) | f.x) & mask;
      uint64_t nL = R;
      R = L ^ F;
      L = nL;
    }
    x = (L << half) | R;
  } while (x >= n);
  return x;
}
