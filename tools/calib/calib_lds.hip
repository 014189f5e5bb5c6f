// Random 8-byte LDS gather rate: the calibrated ceiling for naive SimRank's
// k_sr_gather (csrc/gw_simrank.hip), whose inner loop is "stream byte offsets
// from HBM/L2, gather one fp64 each from an LDS-resident row, add".
//
// One 1024-thread workgroup per CU holds a row of m doubles in LDS (m = 10313,
// lshrank blog: 82.5 KB, so one workgroup per CU as in k_sr_gather).  Every
// wave streams chunks of 1024 offsets (16 per lane, 64 B, prefetched one chunk
// ahead) and gathers the 16 doubles into four accumulators.  Patterns:
//   random  uniform offsets in [0, m)
//   rows    segments of random length (mean ~65, blog's mean degree) sorted
//           ascending, like a CSR adjacency stream
// No head flags, scans or output windows: this is the gather loop alone.
//
//   calib_lds [--m 10313] [--nent 667966] [--reps 40]
// Output: one JSON object per pattern:
//   {"pattern":"random","m":..,"gathers":..,"ms":..,"gathers_per_s":..,"per_cu_per_clk_at_2.4GHz":..}
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                               \
    }                                                                                        \
  } while (0)

constexpr int kBlock = 1024;
constexpr int kWaves = kBlock / 64;
constexpr int kK = 16;                 // offsets per lane per chunk
constexpr int kChunk = 64 * kK;        // offsets per wave per chunk

__global__ void __launch_bounds__(kBlock) k_lds_gather(const uint32_t* __restrict__ ent, long long nchunk, int m,
                                                      int reps, double* __restrict__ out) {
  extern __shared__ double row[];
  for (int b = threadIdx.x; b < m; b += kBlock) row[b] = (double)((b * 2654435761u) & 0xFFFFu) * 1e-5;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  const char* rb = reinterpret_cast<const char*>(row);
  for (int r = 0; r < reps; ++r) {
    long long c = (wave + (long long)blockIdx.x * 7 + r * 3) % kWaves;  // waves spread over the stream
    if (c >= nchunk) continue;
    const uint4* p = reinterpret_cast<const uint4*>(ent + c * kChunk + kK * lane);
    uint4 n0 = p[0], n1 = p[1], n2 = p[2], n3 = p[3];
    for (; c < nchunk; c += kWaves) {
      const uint32_t e[kK] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w,
                              n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
      if (c + kWaves < nchunk) {  // next chunk of this wave in flight during the gathers
        const uint4* q = reinterpret_cast<const uint4*>(ent + (c + kWaves) * kChunk + kK * lane);
        n0 = q[0];
        n1 = q[1];
        n2 = q[2];
        n3 = q[3];
      }
#pragma unroll
      for (int k = 0; k < kK; k += 4) {
        a0 += *reinterpret_cast<const double*>(rb + e[k]);
        a1 += *reinterpret_cast<const double*>(rb + e[k + 1]);
        a2 += *reinterpret_cast<const double*>(rb + e[k + 2]);
        a3 += *reinterpret_cast<const double*>(rb + e[k + 3]);
      }
    }
  }
  out[(long long)blockIdx.x * kBlock + threadIdx.x] = (a0 + a1) + (a2 + a3);
}

int main(int argc, char** argv) {
  int m = 10313, reps = 40;
  long long nent = 667966;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--m")) m = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--nent")) nent = atoll(argv[i + 1]);
    else if (!strcmp(argv[i], "--reps")) reps = atoi(argv[i + 1]);
  }
  const long long nchunk = (nent + kChunk - 1) / kChunk;
  const long long padded = nchunk * kChunk;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t lds = (size_t)m * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_lds_gather, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  uint32_t* d_ent;
  double* d_out;
  CK(hipMalloc(&d_ent, padded * sizeof(uint32_t)));
  const int grid = cus * 4;  // resident one at a time per CU (LDS), so 4 waves of workgroups
  CK(hipMalloc(&d_out, (size_t)grid * kBlock * sizeof(double)));
  std::mt19937_64 rng(42);
  for (int pat = 0; pat < 2; ++pat) {
    std::vector<uint32_t> h(padded);
    std::uniform_int_distribution<int> U(0, m - 1);
    if (pat == 0) {
      for (auto& v : h) v = (uint32_t)U(rng) * 8u;
    } else {
      std::geometric_distribution<int> G(1.0 / 65.0);
      long long i = 0;
      while (i < padded) {
        const long long len = std::min<long long>(padded - i, 1 + G(rng));
        std::vector<uint32_t> seg(len);
        for (auto& v : seg) v = (uint32_t)U(rng);
        std::sort(seg.begin(), seg.end());
        for (long long k = 0; k < len; ++k) h[i + k] = seg[k] * 8u;
        i += len;
      }
    }
    CK(hipMemcpy(d_ent, h.data(), padded * sizeof(uint32_t), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_lds_gather, dim3(grid), dim3(kBlock), lds, 0, d_ent, nchunk, m, 2, d_out);  // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_lds_gather, dim3(grid), dim3(kBlock), lds, 0, d_ent, nchunk, m, reps, d_out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    const double gathers = (double)grid * reps * (double)padded;
    const double rate = gathers / (ms * 1e-3);
    printf("{\"pattern\":\"%s\",\"m\":%d,\"grid\":%d,\"reps\":%d,\"gathers\":%.0f,\"ms\":%.3f,\"gathers_per_s\":%.4e,"
           "\"per_cu_per_clk_at_2.4GHz\":%.3f}\n",
           pat == 0 ? "random" : "rows", m, grid, reps, gathers, ms, rate, rate / cus / 2.4e9);
    fflush(stdout);
  }
  CK(hipFree(d_ent));
  CK(hipFree(d_out));
  return 0;
}
