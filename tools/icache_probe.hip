// Microbenchmark (round 5): does a long straight-line loop body cost issue
// rate through instruction-cache misses?  The same mad+and stream (8
// independent mad chains + 8 and chains, as tools/issue_probe.hip) runs as a
// loop body of 64, 4 K, 32 K and 64 K instructions (k_miller's per-step body
// is ~65 K instructions, ~0.5 MB of code), with the same total instruction
// count; in-kernel s_memtime cycles per instruction per wave at 1 and 2
// waves per SIMD.  Body: tools/gen_icache_probe.py > tools/icache_probe_body.inc
// Build: hipcc -O3 --offload-arch=gfx950 tools/icache_probe.hip -o tools/icache_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "icache_probe_body.inc"

#define CHK(x)                                                         \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(2);                                                         \
    }                                                                  \
  } while (0)

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int L>
__global__ __launch_bounds__(256) void k_body(uint64_t* out, int iters, uint32_t s) {
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = s;
  uint32_t a = threadIdx.x * 77 + s, b = blockIdx.x * 31 + s;
  uint64_t y[8];
  uint32_t x[8];
#pragma unroll
  for (int j = 0; j < 8; j++) y[j] = ((uint64_t)b << 32) + j, x[j] = a ^ j;
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t0 = stamp();
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < iters; it++) {
    if (L == 0) { BODY_L64 }
    if (L == 1) { BODY_L4K }
    if (L == 2) { BODY_L32K }
    if (L == 3) { BODY_L64K }
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t1 = stamp();
  __builtin_amdgcn_sched_barrier(0);
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= x[j] ^ y[j];
  const int w = blockIdx.x * 4 + threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) out[2 * w] = t1 - t0, out[2 * w + 1] = r;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int total = 1 << 22;   // instructions per wave in every variant
  const int lens[4] = {64, 4096, 32768, 65536};
  void (*fns[4])(uint64_t*, int, uint32_t) = {k_body<0>, k_body<1>, k_body<2>, k_body<3>};
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 4 * 2 * 8));
  std::vector<uint64_t> h((size_t)cus * 8 * 4 * 2);
  for (auto f : fns) CHK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  printf("# cycles per wave-instruction (in-kernel s_memtime, median over waves): loop body length vs waves/SIMD\n");
  printf("%-10s %10s %10s\n", "body", "W=1", "W=2");
  for (int v = 0; v < 4; v++) {
    printf("%-10d", lens[v]);
    for (int w : {1, 2}) {
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      const int blocks = cus * w, iters = total / lens[v];
      hipLaunchKernelGGL(fns[v], dim3(blocks), dim3(256), lds, 0, out, 2, 1u);
      hipLaunchKernelGGL(fns[v], dim3(blocks), dim3(256), lds, 0, out, iters, 1u);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), out, (size_t)blocks * 4 * 2 * 8, hipMemcpyDeviceToHost));
      std::vector<double> cyc;
      for (int i = 0; i < blocks * 4; i++) cyc.push_back((double)h[2 * i] / ((double)iters * lens[v]));
      std::sort(cyc.begin(), cyc.end());
      printf(" %10.3f", cyc[cyc.size() / 2]);
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
