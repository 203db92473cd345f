// Microbenchmark (round 5): in-kernel cycle counts of the VALU issue stream the
// field arithmetic is made of, at 1 and 2 waves per SIMD.  Unlike
// tools/valu_rates.hip (HIP-event time x an assumed 2.4 GHz) every figure is
// measured with s_memtime around the loop on each wave (shader-clock cycles),
// and the clock itself is reported as d(s_memtime) / d(s_memrealtime) x 100 MHz.
//
// Each probe runs CH independent chains of one instruction, round-robin (ch=1:
// the dependent-issue latency; large ch: the issue throughput of one wave):
// v_mad_u64_u32 chained through its 64-bit addend (the product-scanning
// column), v_and_b32, v_lshrrev_b64, and mad+and pairs (the mix of a column).
// Build: hipcc -O3 --offload-arch=gfx950 tools/issue_probe.hip -o tools/issue_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);           \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ uint64_t rstamp() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// OP: 0 mad, 1 and, 2 lshrrev_b64, 3 mad+and pair (x[] chains are separate)
template <int OP, int CH>
__global__ __launch_bounds__(256) void k_probe(uint64_t* out, int iters, uint32_t s) {
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = s;
  uint32_t a = threadIdx.x * 77 + s, b = blockIdx.x * 31 + s;
  uint64_t y[CH];
  uint32_t x[2 * CH];
#pragma unroll
  for (int j = 0; j < CH; j++) y[j] = ((uint64_t)b << 32) + j, x[j] = a + j, x[CH + j] = a ^ j;
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t0 = stamp(), r0 = rstamp();
  __builtin_amdgcn_sched_barrier(0);
  for (int it = 0; it < iters; it++) {
    // 32 instructions per iteration (16 mad+and pairs), chains round-robin,
    // one asm statement per group (tools/gen_issue_probe.py)
#include "issue_probe_body.inc"
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t1 = stamp(), r1 = rstamp();
  __builtin_amdgcn_sched_barrier(0);
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < CH; j++) r ^= x[j] ^ x[CH + j] ^ y[j];
  const int w = blockIdx.x * 4 + threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    out[3 * w] = t1 - t0;
    out[3 * w + 1] = r1 - r0;
    out[3 * w + 2] = r;
  }
}

typedef void (*kfn)(uint64_t*, int, uint32_t);
struct P {
  kfn f;
  const char* name;
  int per_iter;
};
#define E(OP, CH, NM, PI) {k_probe<OP, CH>, NM " ch=" #CH, PI}
static const P kP[] = {
    E(0, 1, "mad", 32),  E(0, 2, "mad", 32),  E(0, 4, "mad", 32),  E(0, 8, "mad", 32),  E(0, 16, "mad", 32),
    E(1, 1, "and", 32),  E(1, 2, "and", 32),  E(1, 4, "and", 32),  E(1, 8, "and", 32),  E(1, 16, "and", 32),
    E(2, 1, "lshr64", 32), E(2, 2, "lshr64", 32), E(2, 4, "lshr64", 32), E(2, 8, "lshr64", 32),
    E(3, 1, "mad+and", 32), E(3, 2, "mad+and", 32), E(3, 4, "mad+and", 32), E(3, 8, "mad+and", 32),
};

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 4096;
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 4 * 3 * 8));
  std::vector<uint64_t> h((size_t)cus * 8 * 4 * 3);
  for (const auto& p : kP) CHK(hipFuncSetAttribute((const void*)p.f, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  printf("# cycles per wave-instruction (per wave, in-kernel s_memtime; median over waves) and clock\n");
  printf("%-16s %10s %8s %10s %8s\n", "probe", "W=1 cyc", "GHz", "W=2 cyc", "GHz");
  for (const auto& p : kP) {
    printf("%-16s", p.name);
    for (int w : {1, 2}) {
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      const int blocks = cus * w;
      hipLaunchKernelGGL(p.f, dim3(blocks), dim3(256), lds, 0, out, 64, 1u);
      hipLaunchKernelGGL(p.f, dim3(blocks), dim3(256), lds, 0, out, iters, 1u);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), out, (size_t)blocks * 4 * 3 * 8, hipMemcpyDeviceToHost));
      std::vector<double> cyc, ghz;
      for (int i = 0; i < blocks * 4; i++) {
        cyc.push_back((double)h[3 * i] / ((double)iters * p.per_iter));
        ghz.push_back((double)h[3 * i] / (double)h[3 * i + 1] * 0.1);
      }
      std::sort(cyc.begin(), cyc.end());
      std::sort(ghz.begin(), ghz.end());
      printf(" %10.2f %8.3f", cyc[cyc.size() / 2], ghz[ghz.size() / 2]);
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
