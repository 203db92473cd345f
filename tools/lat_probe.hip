// Latency / issue probe (round 5): cycles per wave-instruction of dependent
// and independent chains of the Montgomery column-boundary instructions
// (v_mad_u64_u32, v_mul_lo_u32, v_lshrrev_b64, v_lshl_add_u64, v_and_b32),
// 1,024 instructions per loop iteration (four 256-instruction asm statements
// on fixed registers, tools/gen_lat_probe.py), so the loop's own overhead is
// < 1 % -- unlike tools/issue_probe.hip, whose 32-instruction iterations add
// ~28 cycles of branch per iteration (its 4.88 cycles/instruction floor).
// In-kernel s_memtime / s_memrealtime; median over waves; W = waves per SIMD.
// Build: python3 tools/gen_lat_probe.py > tools/lat_probe_body.inc &&
//        hipcc -O3 --offload-arch=gfx950 tools/lat_probe.hip -o tools/lat_probe
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
__global__ __launch_bounds__(256) void k_lat(uint64_t* out, int iters, uint32_t s) {
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = s;
  // operands: small nonzero values in the probe registers
  asm volatile(
      "v_mov_b32 v40, 3\n\tv_mov_b32 v41, 0\n\tv_mov_b32 v42, 5\n\tv_mov_b32 v43, 7\n\t"
      "v_mov_b32 v44, 11\n\tv_mov_b32 v45, 0\n\tv_mov_b32 v46, 13\n\tv_mov_b32 v47, 17\n\t"
      "v_mov_b32 v48, 19\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 23\n\tv_mov_b32 v51, 0\n\t"
      "v_mov_b32 v52, 29\n\tv_mov_b32 v53, 0\n\tv_mov_b32 v54, 31\n\tv_mov_b32 v56, 37" ::
          : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53",
            "v54", "v56");
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t0 = stamp(), r0 = rstamp();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
#include "lat_probe_body.inc"
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t1 = stamp(), r1 = rstamp();
  __builtin_amdgcn_sched_barrier(0);
  const int w = blockIdx.x * 4 + threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = r1 - r0;
  }
}

#define LAT_NAMES
#include "lat_probe_body.inc"

typedef void (*kfn)(uint64_t*, int, uint32_t);

int main() {
  static_assert(LAT_NPAT == 21, "regenerate the table below");
  static const kfn fns[] = {k_lat<0>,  k_lat<1>,  k_lat<2>,  k_lat<3>,  k_lat<4>,  k_lat<5>,  k_lat<6>,
                            k_lat<7>,  k_lat<8>,  k_lat<9>,  k_lat<10>, k_lat<11>, k_lat<12>, k_lat<13>,
                            k_lat<14>, k_lat<15>, k_lat<16>, k_lat<17>, k_lat<18>, k_lat<19>, k_lat<20>};
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 256;
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 4 * 2 * 8));
  std::vector<uint64_t> h((size_t)cus * 8 * 4 * 2);
  for (auto f : fns) CHK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  printf("# cycles per wave-instruction per wave (in-kernel s_memtime; median over waves), 1,024 instructions per iteration\n");
  printf("%-20s %10s %8s %10s %8s\n", "probe", "W=1 cyc", "GHz", "W=2 cyc", "GHz");
  for (int p = 0; p < LAT_NPAT; p++) {
    printf("%-20s", kNames[p]);
    for (int w : {1, 2}) {
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      const int blocks = cus * w;
      hipLaunchKernelGGL(fns[p], dim3(blocks), dim3(256), lds, 0, out, 16, 1u);
      hipLaunchKernelGGL(fns[p], dim3(blocks), dim3(256), lds, 0, out, iters, 1u);
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
