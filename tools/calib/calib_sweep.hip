// Random-sector read rate vs table size (HBM vs Infinity Cache residency).
// Each lane follows `steps` reads; "dep" mode makes every address depend on
// the previous read (a walk's dependent chain), "ind" mode issues them
// independently.  Reads are 64 B (4 x dwordx4 of one sector) or 4 B.
// Prints sectors/s per (size, mode, width).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

template <bool DEP, bool WIDE>
__global__ void __launch_bounds__(256) chase(const uint4* __restrict__ buf, unsigned long long nsec, int steps,
                                             unsigned* __restrict__ out) {
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long h = 0x9E3779B97F4A7C15ull * (t + 1);
  unsigned acc = 0;
  unsigned long long s = h % nsec;
  for (int i = 0; i < steps; ++i) {
    const uint4* p = buf + s * 4;
    unsigned v;
    if (WIDE) {
      const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
      v = a.x ^ b.y ^ c.z ^ d.w;
    } else {
      v = p[0].x;
    }
    acc += v;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    s = DEP ? ((h ^ (unsigned long long)v) % nsec) : (h % nsec);
  }
  out[t] = acc;
}

// 4 lanes per sector: lane l of instruction j loads 16 B piece (l & 3) of the
// sector of walker 16 j + (l >> 2); 64 walkers' sectors in 4 instructions
__global__ void __launch_bounds__(256) coop(const uint4* __restrict__ buf, unsigned long long nsec, int steps,
                                            unsigned* __restrict__ out) {
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  unsigned long long h = 0x9E3779B97F4A7C15ull * (t + 1);
  unsigned acc = 0;
  for (int i = 0; i < steps; ++i) {
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    const unsigned long long s = h % nsec;  // this lane's walker sector
    const unsigned slo = (unsigned)s, shi = (unsigned)(s >> 32);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int src = 16 * j + (lane >> 2);
      const unsigned long long sj = ((unsigned long long)(unsigned)__shfl(shi, src) << 32) | (unsigned)__shfl(slo, src);
      const uint4 a = buf[sj * 4 + (lane & 3)];
      acc += a.x ^ a.w;
    }
  }
  out[t] = acc;
}

float run_coop(const uint4* buf, unsigned long long nsec, int blocks, int steps, unsigned* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  coop<<<blocks, 256>>>(buf, nsec, steps, out);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(a);
    coop<<<blocks, 256>>>(buf, nsec, steps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

template <bool DEP, bool WIDE>
float run(const uint4* buf, unsigned long long nsec, int blocks, int steps, unsigned* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  chase<DEP, WIDE><<<blocks, 256>>>(buf, nsec, steps, out);  // warm
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(a);
    chase<DEP, WIDE><<<blocks, 256>>>(buf, nsec, steps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return best;
}

int main() {
  const long long maxb = 32ll << 30;
  uint4* buf;
  unsigned* out;
  if (hipMalloc(&buf, maxb) != hipSuccess) return 1;
  hipMemset(buf, 0x5a, maxb);
  const int blocks = 8192, steps = 64;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  const long long sizes[] = {64ll << 20, 256ll << 20, 1ll << 30, 2ll << 30, 3ll << 30, 4ll << 30,
                             6ll << 30, 8ll << 30, 16ll << 30, 32ll << 30};
  for (long long sz : sizes) {
    const unsigned long long nsec = (unsigned long long)sz / 64;
    const double n = (double)blocks * 256 * steps;
    const float t0 = run<false, true>(buf, nsec, blocks, steps, out);
    const float t1 = run<true, true>(buf, nsec, blocks, steps, out);
    const float t2 = run<false, false>(buf, nsec, blocks, steps, out);
    const float t3 = run<true, false>(buf, nsec, blocks, steps, out);
    const float t4 = run_coop(buf, nsec, blocks, steps, out);
    printf("size %7.0f MB  ind64 %.3g  dep64 %.3g  ind4 %.3g  dep4 %.3g  coop64 %.3g sectors/s\n", sz / 1048576.0,
           n / (t0 * 1e-3), n / (t1 * 1e-3), n / (t2 * 1e-3), n / (t3 * 1e-3), n / (t4 * 1e-3));
  }
  return 0;
}
