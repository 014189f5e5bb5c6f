// Does the second half of a 128 B line come free after a 64 B read of its
// first half?  (Design question for the bitset walk's slot entries: a 64 B
// entry with its overflow payload in the other half of the same line.)
//
// Every lane is a walker that reads one random 64 B block per iteration from
// the first half of a random 128 B line of an S-byte table, cooperatively as
// k_walk_bitset does (4 lanes per walker, 16 walkers per instruction), with
// the next address depending on the data read.  MODE adds one per-lane dword
// read per iteration, issued beside the block loads:
//   0  none
//   1  a dword from the SECOND half of the line this walker read in the
//      previous iteration (the candidate layout)
//   2  a dword from an unrelated random line (control: one more request)
//   3  as 1, but from the second half of the line read two iterations earlier
//   4  the first 48 B of the line's second half fetched in the same
//      iteration by LDS-DMA (global_load_lds_dwordx4: lanes 4m..4m+2 of a
//      round, walker 16j+m's 64 B LDS record), one word of it folded into
//      the next address (the candidate bitset-entry layout: 64 B header +
//      payload in registers, 48 B extension in LDS)
// The dword's value enters the next address, so it is a dependent read.
//
//   calib_halfline [--sizes MB,..] [--modes 0,1,2,3] [--waves 5] [--iters N]
// Prints one JSON object per line; round 2 ran it with tools/gpu_halfline.sh (now `tools/gpu_run.sh py` / `counters`), which added rocprofv3
// TCC_EA0_RDREQ / TCC_HIT / TCC_MISS passes (requests per walker-iteration).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(2);                                                                                   \
    }                                                                                            \
  } while (0)

__device__ __forceinline__ unsigned long long mix64(unsigned long long h) {
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 29;
  return h;
}

template <int MODE>
__global__ void __launch_bounds__(256) k_half(const uint4* __restrict__ buf, unsigned long long nline, int iters,
                                              unsigned* __restrict__ out) {
  extern __shared__ unsigned s_pad[];
  __shared__ uint4 s_rec[4][64][4];  // MODE 4: per-wave 64 B records
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const unsigned* bw = reinterpret_cast<const unsigned*>(buf);
  unsigned long long h = mix64(0x9E3779B97F4A7C15ull * (t + 1));
  unsigned long long prev1 = h % nline, prev2 = prev1;
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    const unsigned long long s = h % nline;  // this walker's line
    const unsigned slo = (unsigned)s, shi = (unsigned)(s >> 32);
    unsigned extra = 0;
    if (MODE == 1) extra = bw[prev1 * 32 + 16 + (h >> 40) % 16];
    if (MODE == 2) extra = bw[(mix64(h + 7) % nline) * 32 + 16 + (h >> 40) % 16];
    if (MODE == 3) extra = bw[prev2 * 32 + 16 + (h >> 40) % 16];
    unsigned mine = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int src = 16 * j + lane / 4;
      const unsigned long long sj =
          ((unsigned long long)(unsigned)__shfl((int)shi, src, 64) << 32) | (unsigned)__shfl((int)slo, src, 64);
      const uint4 a = buf[sj * 8 + (lane % 4)];  // first 64 B of the 128 B line
      if (MODE == 4 && (lane & 3) != 3)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(buf + sj * 8 + 4 + (lane & 3)),
                                         &s_rec[threadIdx.x >> 6][16 * j][0], 16, 0, 0);
      acc += a.x ^ a.w;
      const unsigned v = (unsigned)__shfl((int)a.x, (lane % 16) * 4, 64);
      if (lane / 16 == j) mine = v;
    }
    if (MODE == 4) {
      __builtin_amdgcn_s_waitcnt(0);  // the LDS-DMA writes have landed (vmcnt 0)
      __builtin_amdgcn_wave_barrier();
      extra = reinterpret_cast<const unsigned*>(&s_rec[threadIdx.x >> 6][lane][0])[(h >> 40) % 12];
    }
    prev2 = prev1;
    prev1 = s;
    h = mix64(h ^ (unsigned long long)mine ^ ((unsigned long long)extra << 17));
  }
  out[t] = acc;
  if (acc == 0x12345678u) s_pad[threadIdx.x] = acc;
}

static std::vector<long long> parse_list(const char* s) {
  std::vector<long long> v;
  std::string a(s);
  size_t p = 0;
  while (p < a.size()) {
    size_t q = a.find(',', p);
    if (q == std::string::npos) q = a.size();
    v.push_back(atoll(a.substr(p, q - p).c_str()));
    p = q + 1;
  }
  return v;
}

typedef void (*KFn)(const uint4*, unsigned long long, int, unsigned*);

int main(int argc, char** argv) {
  std::vector<long long> sizes_mb = {8192};
  std::vector<long long> modes = {0, 1, 2, 3, 4};
  std::vector<long long> waves = {5};
  int reps = 3, iters = 256;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--sizes") && i + 1 < argc) sizes_mb = parse_list(argv[++i]);
    else if (!strcmp(argv[i], "--modes") && i + 1 < argc) modes = parse_list(argv[++i]);
    else if (!strcmp(argv[i], "--waves") && i + 1 < argc) waves = parse_list(argv[++i]);
    else if (!strcmp(argv[i], "--iters") && i + 1 < argc) iters = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--reps") && i + 1 < argc) reps = atoi(argv[++i]);
  }
  long long maxmb = 0;
  for (long long s : sizes_mb) maxmb = s > maxmb ? s : maxmb;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t maxb = (size_t)maxmb << 20;
  uint4* buf;
  CK(hipMalloc(&buf, maxb));
  CK(hipMemset(buf, 0x5a, maxb));
  unsigned* out;
  CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  KFn fs[5] = {k_half<0>, k_half<1>, k_half<2>, k_half<3>, k_half<4>};
  for (long long smb : sizes_mb)
    for (long long w : waves)
      for (long long m : modes) {
        if (m < 0 || m > 4 || w < 1 || w > 8) continue;
        KFn f = fs[m];
        const size_t lds = ((size_t)(160 * 1024 / w) & ~(size_t)1023) - 16384;  // + 16 KB static records
        if (lds > 64 * 1024) CK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        const unsigned long long nline = ((unsigned long long)smb << 20) / 128ull;
        const int blocks = cus * (int)w;
        hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, buf, nline, iters, out);
        CK(hipGetLastError());
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
          CK(hipEventRecord(a));
          hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, buf, nline, iters, out);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          best = ms < best ? ms : best;
        }
        const double walker_iters = (double)blocks * 256.0 * iters;
        printf("{\"mode\":%lld,\"waves\":%lld,\"table_mb\":%lld,\"walker_iters_per_s\":%.4g,\"ms\":%.4f,"
               "\"walker_iters\":%.0f,\"grid\":%d}\n",
               m, w, smb, walker_iters / (best * 1e-3), best, walker_iters, blocks * 256);
        fflush(stdout);
      }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
