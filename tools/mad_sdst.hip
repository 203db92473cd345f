// Microbenchmark: does the carry-out SGPR of v_mad_u64_u32 serialise a wave?
// Every v_mad_u64_u32 on gfx9-family targets writes a carry-out SGPR pair
// (there is no null destination).  The compiler gives independent multiplies
// the same dead pair, which makes consecutive mads write-after-write
// dependent.  Variants (8 independent accumulators, one wave per SIMD and 2):
//   same : all mads write s[40:41]
//   rot  : mad j writes its own pair s[40+2j : 41+2j]
//   vcc  : all mads write vcc
// Build: hipcc -O3 --offload-arch=gfx950 tools/mad_sdst.hip -o tools/mad_sdst
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                        \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

#define MAD(j, SD) asm volatile("v_mad_u64_u32 %0, " SD ", %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b) : CLOB)

template <int MODE>
__global__ void k_mad(uint64_t* out, int iters, uint32_t s) {
  uint32_t a = threadIdx.x * 77 + s, b = blockIdx.x * 31 + s;
  uint64_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = j;
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) {
#define CLOB "s40", "s41"
      MAD(0, "s[40:41]"); MAD(1, "s[40:41]"); MAD(2, "s[40:41]"); MAD(3, "s[40:41]");
      MAD(4, "s[40:41]"); MAD(5, "s[40:41]"); MAD(6, "s[40:41]"); MAD(7, "s[40:41]");
#undef CLOB
    } else if (MODE == 1) {
#define CLOB "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55"
      MAD(0, "s[40:41]"); MAD(1, "s[42:43]"); MAD(2, "s[44:45]"); MAD(3, "s[46:47]");
      MAD(4, "s[48:49]"); MAD(5, "s[50:51]"); MAD(6, "s[52:53]"); MAD(7, "s[54:55]");
#undef CLOB
    } else {
#define CLOB "vcc"
      MAD(0, "vcc"); MAD(1, "vcc"); MAD(2, "vcc"); MAD(3, "vcc");
      MAD(4, "vcc"); MAD(5, "vcc"); MAD(6, "vcc"); MAD(7, "vcc");
#undef CLOB
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int N>
__global__ void k_madn(uint64_t* out, int iters, uint32_t s) {
  uint32_t a = threadIdx.x * 77 + s, b = blockIdx.x * 31 + s;
  uint64_t acc[N];
#pragma unroll
  for (int j = 0; j < N; j++) acc[j] = j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < N; j++) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[j]) : "v"(a + j), "v"(b) : "vcc");
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < N; j++) r ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 4096;
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 8));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const char* names[3] = {"same sdst", "rotating sdst", "vcc sdst"};
  for (int waves = 1; waves <= 8; waves *= 2) {
    for (int mode = 0; mode < 3; mode++) {
      const int blocks = cus * waves;   // 256-thread blocks = 4 waves = 1 per SIMD
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        CHK(hipEventRecord(e0));
        if (mode == 0) hipLaunchKernelGGL(k_mad<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
        if (mode == 1) hipLaunchKernelGGL(k_mad<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
        if (mode == 2) hipLaunchKernelGGL(k_mad<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
      }
      const double mads = (double)blocks * 256 * iters * 8;
      const double cyc_per_mad = ms * 1e-3 * prop.clockRate * 1e3 / ((double)iters * 8) / waves;
      printf("waves/SIMD=%d %-14s %8.3f T mad/s  %6.2f cycles per wave-mad per SIMD\n", waves, names[mode],
             mads / (ms * 1e-3) / 1e12, cyc_per_mad);
    }
  }
  for (int w = 1; w <= 2; w *= 2) {
    const int blocks = cus * w;
    for (int N : {1, 2, 4, 16, 32}) {
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        CHK(hipEventRecord(e0));
        if (N == 1) hipLaunchKernelGGL(k_madn<1>, dim3(blocks), dim3(256), 0, 0, out, iters * 8, 1u);
        if (N == 2) hipLaunchKernelGGL(k_madn<2>, dim3(blocks), dim3(256), 0, 0, out, iters * 4, 1u);
        if (N == 4) hipLaunchKernelGGL(k_madn<4>, dim3(blocks), dim3(256), 0, 0, out, iters * 2, 1u);
        if (N == 16) hipLaunchKernelGGL(k_madn<16>, dim3(blocks), dim3(256), 0, 0, out, iters / 2, 1u);
        if (N == 32) hipLaunchKernelGGL(k_madn<32>, dim3(blocks), dim3(256), 0, 0, out, iters / 4, 1u);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
      }
      const double cyc = ms * 1e-3 * prop.clockRate * 1e3 / ((double)iters * 8) / w;
      printf("waves/SIMD=%d chains=%2d  %6.2f cycles per wave-mad per SIMD\n", w, N, cyc);
    }
  }
  return 0;
}
