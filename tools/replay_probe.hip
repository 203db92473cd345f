// Replay probe (round 5): times windows of compiled instruction streams
// (tools/gen_replay_probe.py -> tools/replay_body.inc) at 1 and 2 waves per
// SIMD, in-kernel s_memtime; no memory instruction is replayed, so this is
// the issue rate of the instruction mix itself.  Values are garbage.
// Build: hipcc -O3 --offload-arch=gfx950 -I tools tools/replay_probe.hip -o tools/replay_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

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
__device__ __forceinline__ uint64_t rstamp() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int OP>
__global__ __launch_bounds__(256) void k_rp(uint64_t* out, int iters) {
  // wave index kept in an SGPR across the loop (the replayed code clobbers
  // every VGPR and AGPR)
  const uint32_t wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + threadIdx.x / 64);
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t0 = stamp(), r0 = rstamp();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
#include "replay_body.inc"
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t1 = stamp(), r1 = rstamp();
  __builtin_amdgcn_sched_barrier(0);
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == 0) {
    out[2 * wv] = t1 - t0;
    out[2 * wv + 1] = r1 - r0;
  }
}

#define RP_NAMES
#include "replay_body.inc"

typedef void (*kfn)(uint64_t*, int);

int main() {
  static const kfn all[] = {k_rp<0>, k_rp<1>, k_rp<2>, k_rp<3>, k_rp<4>, k_rp<5>, k_rp<6>, k_rp<7>};
  static_assert(RP_NPAT <= 8, "at most 8 windows");
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 64;
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 2 * 8));
  std::vector<uint64_t> h((size_t)cus * 8 * 2);
  for (int p = 0; p < RP_NPAT; p++)
    CHK(hipFuncSetAttribute((const void*)all[p], hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  printf("# replayed instruction windows: cycles per wave-instruction per wave (in-kernel s_memtime, median over waves)\n");
  printf("%-24s %6s %10s %8s %10s %8s\n", "window", "instrs", "W=1 cyc", "GHz", "W=2 cyc", "GHz");
  for (int p = 0; p < RP_NPAT; p++) {
    printf("%-24s %6d", kNames[p], kPer[p]);
    for (int w : {1, 2}) {
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      const int blocks = cus * w;
      hipLaunchKernelGGL(all[p], dim3(blocks), dim3(256), lds, 0, out, 4);
      hipLaunchKernelGGL(all[p], dim3(blocks), dim3(256), lds, 0, out, iters);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), out, (size_t)blocks * 4 * 2 * 8, hipMemcpyDeviceToHost));
      std::vector<double> cyc, ghz;
      for (int i = 0; i < blocks * 4; i++) {
        cyc.push_back((double)h[2 * i] / ((double)iters * kPer[p]));
        ghz.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 0.1);
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
