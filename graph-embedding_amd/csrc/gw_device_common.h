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

// Exact neighbour sets for has_edge (GW_N2V_REJECTION): row r owns 2*deg(r)
// int32 slots at 2*offsets[r] (load factor 1/2, linear probing from a
// multiply-shift hash); a query reads one slot run, almost always inside one
// 64 B sector (built by k_build_ehash, gw_n2v.hip).
__device__ __forceinline__ uint32_t gw_eh_slot(int32_t key, uint32_t cap) {
  return (uint32_t)(((uint64_t)((uint32_t)key * 0x9E3779B1u) * (uint64_t)cap) >> 32);
}
__device__ __forceinline__ bool gw_eh_has(const int32_t* __restrict__ eh, int64_t rb, int64_t re, int32_t key) {
  const uint32_t cap = (uint32_t)(2 * (re - rb));
  if (cap == 0) return false;
  const int32_t* __restrict__ t = eh + 2 * rb;
  uint32_t s = gw_eh_slot(key, cap);
  for (uint32_t i = 0; i < cap; ++i) {
    const int32_t k = t[s];
    if (k == key) return true;
    if (k == -1) return false;
    s = s + 1 == cap ? 0u : s + 1;
  }
  return false;
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
