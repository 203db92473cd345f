// Microbenchmark (round 5): VGPR bank conflicts and v_mad_u64_u32 issue.
// The operands are fixed physical VGPRs in the asm text
// (tools/gen_bank_probe.py): no conflict, a in the accumulator's high bank,
// a/b/accumulator-low in one bank, and a 3-way conflict.  In-kernel
// s_memtime cycles per mad per wave at 1 and 2 waves per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 -I tools tools/bank_probe.hip -o tools/bank_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "bank_probe_body.inc"

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

template <int C>
__global__ __launch_bounds__(256) void k_bank(uint64_t* out, int iters, uint32_t s) {
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = s;
  const uint32_t aa = threadIdx.x * 77 + s, bb = blockIdx.x * 31 + s;
  if (C == 0) { BANK_INIT_nocf }
  if (C == 1) { BANK_INIT_a_acchi }
  if (C == 2) { BANK_INIT_ab_same }
  if (C == 3) { BANK_INIT_all_b0 }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t0 = stamp();
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < iters; it++) {
    if (C == 0) { BANK_nocf }
    if (C == 1) { BANK_a_acchi }
    if (C == 2) { BANK_ab_same }
    if (C == 3) { BANK_all_b0 }
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t1 = stamp();
  const int w = blockIdx.x * 4 + threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) out[w] = t1 - t0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 8192;
  const char* names[4] = {"no conflict", "a = acc.hi bank", "a,b,acc.lo bank", "a,b bank0 3-way"};
  void (*fns[4])(uint64_t*, int, uint32_t) = {k_bank<0>, k_bank<1>, k_bank<2>, k_bank<3>};
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 4 * 8));
  std::vector<uint64_t> h((size_t)cus * 8 * 4);
  for (auto f : fns) CHK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  printf("# cycles per v_mad_u64_u32 per wave (in-kernel s_memtime, median), operand banks fixed\n");
  printf("%-18s %8s %8s\n", "case", "W=1", "W=2");
  for (int v = 0; v < 4; v++) {
    printf("%-18s", names[v]);
    for (int w : {1, 2}) {
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      const int blocks = cus * w;
      hipLaunchKernelGGL(fns[v], dim3(blocks), dim3(256), lds, 0, out, 4, 1u);
      hipLaunchKernelGGL(fns[v], dim3(blocks), dim3(256), lds, 0, out, iters, 1u);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), out, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost));
      std::vector<double> cyc;
      for (int i = 0; i < blocks * 4; i++) cyc.push_back((double)h[i] / (64.0 * iters));
      std::sort(cyc.begin(), cyc.end());
      printf(" %8.3f", cyc[cyc.size() / 2]);
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
