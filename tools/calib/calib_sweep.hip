// Random-block read-rate calibration for the walk kernels (the denominator of
// bench.py's random_line_roofline).
//
// Every lane is a "walker" that reads one random RB-byte block (RB-aligned)
// per iteration from a table of S bytes, cooperatively as the walk kernels
// do: LP = RB/16 lanes load the 16 B pieces of one walker's block, so one
// wave-instruction covers 64/LP walkers and LP instructions serve the wave.
// DEP = 1 makes the next address depend on the data just read (a walk's
// dependent chain; the pieces are folded back to the walker through
// shuffles), DEP = 0 issues independent addresses.
//
// Occupancy is forced per run: 256-thread workgroups (one wave per SIMD)
// with 160 KiB / W of dynamic LDS each, so exactly W waves per SIMD are
// resident; the grid is 256 CUs x W workgroups (all resident, no tail).
//
//   calib_sweep [--quick] [--sizes MB,MB,..] [--rb 64,128] [--waves 5] [--dep 0,1] [--reps N]
//               [--alloc default|contiguous]   (hipMalloc or hipExtMallocWithFlags(hipDeviceMallocContiguous))
//
// Output: one JSON object per line:
//   {"rb":64,"dep":0,"waves":5,"table_mb":2048,"blocks_per_s":..,"bytes_per_s":..,"ms":..,"reads":..}
// tools/gpu_run.sh calib (rounds 1-4: tools/gpu_calib.sh) runs the sweep plus rocprofv3 TCC_EA0_RDREQ passes and
// writes profiles/calib_<tag>.json (bench.py reads the rate from there).
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

template <int RB, int DEP>
__global__ void __launch_bounds__(256) k_coop(const uint4* __restrict__ buf, unsigned long long nblk, int iters,
                                              unsigned* __restrict__ out) {
  extern __shared__ unsigned s_pad[];  // occupancy control only
  constexpr int LP = RB / 16;          // lanes per walker block
  constexpr int WPI = 64 / LP;         // walkers per wave-instruction
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  unsigned long long h = mix64(0x9E3779B97F4A7C15ull * (t + 1));
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    const unsigned long long s = h % nblk;  // this lane's walker block
    const unsigned slo = (unsigned)s, shi = (unsigned)(s >> 32);
    unsigned mine = 0;  // (DEP) the first dword of this walker's block
#pragma unroll
    for (int j = 0; j < LP; ++j) {
      const int src = WPI * j + lane / LP;
      const unsigned long long sj =
          ((unsigned long long)(unsigned)__shfl((int)shi, src, 64) << 32) | (unsigned)__shfl((int)slo, src, 64);
      const uint4 a = buf[sj * LP + (lane % LP)];
      acc += a.x ^ a.w;
      if (DEP) {
        // walker lane m reads piece 0 of its block from round m / WPI, lane (m % WPI) * LP
        const unsigned v = (unsigned)__shfl((int)a.x, (lane % WPI) * LP, 64);
        if (lane / WPI == j) mine = v;
      }
    }
    h = mix64(h ^ (DEP ? (unsigned long long)mine : 0ull));
  }
  out[t] = acc;
  if (acc == 0x12345678u) s_pad[threadIdx.x] = acc;  // keep the LDS allocation
}

struct Cfg {
  int rb, dep;
};

typedef void (*KFn)(const uint4*, unsigned long long, int, unsigned*);

static KFn pick(int rb, int dep) {
#define P(R)                                 \
  if (rb == R) return dep ? k_coop<R, 1> : k_coop<R, 0>;
  P(16) P(32) P(64) P(128) P(256)
#undef P
  return nullptr;
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

int main(int argc, char** argv) {
  std::vector<long long> sizes_mb = {64, 256, 1024, 2048, 8192, 32768};
  std::vector<long long> rbs = {32, 64, 128, 256};
  std::vector<long long> waves = {4, 5, 6, 8};
  std::vector<long long> deps = {0, 1};
  int reps = 3, iters = 256;
  int contiguous = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--quick")) {
      sizes_mb = {2048, 8192};
      waves = {5};
      deps = {1};
    } else if (!strcmp(argv[i], "--sizes") && i + 1 < argc) {
      sizes_mb = parse_list(argv[++i]);
    } else if (!strcmp(argv[i], "--rb") && i + 1 < argc) {
      rbs = parse_list(argv[++i]);
    } else if (!strcmp(argv[i], "--waves") && i + 1 < argc) {
      waves = parse_list(argv[++i]);
    } else if (!strcmp(argv[i], "--dep") && i + 1 < argc) {
      deps = parse_list(argv[++i]);
    } else if (!strcmp(argv[i], "--reps") && i + 1 < argc) {
      reps = atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--alloc") && i + 1 < argc) {
      contiguous = !strcmp(argv[++i], "contiguous");
    } else if (!strcmp(argv[i], "--iters") && i + 1 < argc) {
      iters = atoi(argv[++i]);
    }
  }
  long long maxmb = 0;
  for (long long s : sizes_mb) maxmb = s > maxmb ? s : maxmb;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t maxb = (size_t)maxmb << 20;
  uint4* buf;
  if (contiguous)
    CK(hipExtMallocWithFlags((void**)&buf, maxb, hipDeviceMallocContiguous));
  else
    CK(hipMalloc(&buf, maxb));
  CK(hipMemset(buf, 0x5a, maxb));
  unsigned* out;
  CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  fprintf(stderr, "device %s, %d CUs\n", prop.name, cus);
  for (long long smb : sizes_mb)
    for (long long w : waves)
      for (long long rb : rbs)
        for (long long dep : deps) {
          KFn f = pick((int)rb, (int)dep);
          if (!f || w < 1 || w > 8) continue;
          const size_t lds = (size_t)(160 * 1024 / w) & ~(size_t)1023;
          if (lds > 64 * 1024) CK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
          const unsigned long long nblk = ((unsigned long long)smb << 20) / (unsigned long long)rb;
          const int blocks = cus * (int)w;
          hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, buf, nblk, iters, out);  // warm
          CK(hipGetLastError());
          float best = 1e30f;
          for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, buf, nblk, iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
          }
          const double reads = (double)blocks * 256.0 * iters;
          printf("{\"rb\":%lld,\"dep\":%lld,\"waves\":%lld,\"table_mb\":%lld,\"blocks_per_s\":%.4g,"
                 "\"bytes_per_s\":%.4g,\"ms\":%.4f,\"reads\":%.0f,\"alloc\":\"%s\"}\n",
                 rb, dep, w, smb, reads / (best * 1e-3), reads * rb / (best * 1e-3), best, reads,
                 contiguous ? "contiguous" : "default");
          fflush(stdout);
        }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
