// FETCH_SIZE calibration for random 4-byte gathers (MI355X_MICROARCH.md §HBM:
// "Other access widths are uncalibrated: calibrate on a known byte count").
// Each lane reads `per_lane` int32 at hashed positions of a buffer far larger
// than the Infinity Cache; every read touches a distinct 128 B line with
// overwhelming probability.  Compare FETCH_SIZE*1024 with reads*64.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void gather(const int* __restrict__ buf, long long nwords, int per_lane, int* __restrict__ out) {
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long h = 0x9E3779B97F4A7C15ull * (unsigned long long)(t + 1);
  int acc = 0;
  for (int i = 0; i < per_lane; ++i) {
    h ^= h >> 31; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 29;
    long long idx = (long long)(h % (unsigned long long)(nwords / 32)) * 32;  // one word per 128 B line
    acc += buf[idx];
  }
  out[t] = acc;
}

int main(int argc, char** argv) {
  long long bytes = 8ll << 30;  // 8 GiB >> 256 MiB MALL
  long long nwords = bytes / 4;
  int blocks = 8192, threads = 256, per_lane = 64;
  int *buf, *out;
  hipMalloc(&buf, bytes);
  hipMemset(buf, 1, bytes);
  hipMalloc(&out, (size_t)blocks * threads * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    gather<<<blocks, threads>>>(buf, nwords, per_lane, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double reads = (double)blocks * threads * per_lane;
    printf("reads=%.0f  time=%.3f ms  reads/s=%.3g  64B-equiv GB/s=%.1f 128B-equiv GB/s=%.1f\n", reads, ms,
           reads / (ms * 1e-3), reads * 64 / (ms * 1e-3) / 1e9, reads * 128 / (ms * 1e-3) / 1e9);
  }
  return 0;
}
