// Device-side helpers shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "gw_internal.h"
#include "gw_philox.h"

#define GW_HIP_TRY(expr)                                                     \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) {                                                  \
      g->err = std::string(#expr) + ": " + hipGetErrorString(_e);            \
      return GW_ERR_DEVICE;                                                  \
    }                                                                        \
  } while (0)

// Binary search for `key` in the sorted row nbrs[b, e); returns the slot or
// -1.  Rows of NX_SIMPLE graphs are sorted by dense id (== label order), see
// gw_graph_host.cpp.
__device__ __forceinline__ int64_t gw_row_find(const int32_t* __restrict__ nbrs,
                                               int64_t b, int64_t e,
                                               int32_t key) {
  int64_t lo = b, hi = e;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (nbrs[mid] < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < e && nbrs[lo] == key) ? lo : -1;
}

// Exact neighbour sets for has_edge (GW_N2V_REJECTION): row r owns deg(r)
// buckets of 4 int32 slots (one 16 B-aligned dwordx4) at 4*offsets[r] (load
// factor 1/4).  A key hashes (multiply-shift) to a bucket and takes its first
// free slot, else the next bucket's (k_build_ehash, gw_n2v.hip), so a
// bucket's keys are a prefix of it and a bucket with a free slot ends every
// query that reaches it: one 16 B read answers a query unless the bucket is
// full (~1% of queries), never crossing a cache line.  (Round 1-4: 2*deg
// int32 slots with linear probing — 2.5 dependent slot reads per miss.)
__device__ __forceinline__ uint32_t gw_eh_slot(int32_t key, uint32_t buckets) {
  return (uint32_t)(((uint64_t)((uint32_t)key * 0x9E3779B1u) * (uint64_t)buckets) >> 32);
}
__device__ __forceinline__ const int4* gw_eh_row(const int32_t* __restrict__ eh, int64_t rb) {
  return reinterpret_cast<const int4*>(eh + 4 * rb);
}
// one bucket: 1 = key present, 0 = absent, -1 = full without it (continue)
__device__ __forceinline__ int gw_eh_scan(const int4 v, int32_t key) {
  if (v.x == key || v.y == key || v.z == key || v.w == key) return 1;
  return v.w == -1 ? 0 : -1;
}
// the rest of a query whose bucket hs was full without the key
__device__ __forceinline__ bool gw_eh_has_from(const int32_t* __restrict__ eh, int64_t rb, uint32_t buckets,
                                               uint32_t hs, int32_t key) {
  const int4* t = gw_eh_row(eh, rb);
  for (uint32_t i = 1; i < buckets; ++i) {
    hs = hs + 1 == buckets ? 0u : hs + 1;
    const int r = gw_eh_scan(t[hs], key);
    if (r >= 0) return r > 0;
  }
  return false;
}
__device__ __forceinline__ bool gw_eh_has(const int32_t* __restrict__ eh, int64_t rb, int64_t re, int32_t key) {
  const uint32_t nb = (uint32_t)(re - rb);
  if (nb == 0) return false;
  const uint32_t hs = gw_eh_slot(key, nb);
  const int r = gw_eh_scan(gw_eh_row(eh, rb)[hs], key);
  if (r >= 0) return r > 0;
  return gw_eh_has_from(eh, rb, nb, hs, key);
}

// Sequential Vose/Walker alias construction exactly as node2vec.py:116-147:
// q[k] = K*p_k; `smaller`/`larger` are LIFO lists filled in index order;
// J[small] = large; q[large] = (q[large] + q[small]) - 1.0.
// On entry q[] holds the probabilities; stack[] is K int32 scratch.  J is
// zero-filled here (np.zeros).  Both stacks share one array: `smaller`
// grows up from 0, `larger` grows down from K (an index is in at most one
// stack at a time, so they never collide).
template <typename JT>
__device__ __forceinline__ void gw_alias_build(double* q, JT* J, int32_t* stack,
                                               int64_t K) {
  const double Kd = (double)K;
  int64_t s_top = 0, l_top = K;
  for (int64_t k = 0; k < K; ++k) {
    J[k] = 0;
    double v = Kd * q[k];
    q[k] = v;
    if (v < 1.0)
      stack[s_top++] = (int32_t)k;
    else
      stack[--l_top] = (int32_t)k;
  }
  while (s_top > 0 && l_top < K) {
    int32_t small = stack[--s_top];
    int32_t large = stack[l_top++];
    J[small] = (JT)large;
    double nv = (q[large] + q[small]) - 1.0;
    q[large] = nv;
    if (nv < 1.0)
      stack[s_top++] = large;
    else
      stack[--l_top] = large;
  }
}

// One slot entry as ONE 16 B load (a struct copy is split into a dword and a
// dwordx3, i.e. two fabric requests for the same sector).
__device__ __forceinline__ gw_ts_ent gw_ts_load(const gw_ts_ent* p) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  gw_ts_ent e;
  e.x = (int32_t)v.x;
  e.d = (int32_t)v.y;
  e.off = (int64_t)((uint64_t)v.z | ((uint64_t)v.w << 32));
  return e;
}
