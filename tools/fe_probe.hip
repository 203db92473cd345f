// Microbenchmark of the staged Fp12 operations (bls/staged.hpp) in isolation,
// one lane per "signature", the same LDS accumulator layout as k_miller/k_final.
// Prints per-op cycles per wave so the costs of the Miller-loop and
// final-exponentiation building blocks can be compared with the plain Fp
// multiply chain (the VALU floor).  Build on the CPU:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I cess_amd/csrc tools/fe_probe.hip -o tools/fe_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "soa.hpp"

using namespace bls;
using namespace cess;

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                 \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

enum Op { OP_FPMUL, OP_CYCSQ, OP_MUL12, OP_SQR12, OP_LINE, OP_N };
static const char* kNames[OP_N] = {"fp_mul chain", "cycsq12 (LDS)", "mul12 (LDS x HBM)", "sqr12 (LDS)",
                                   "mul014 line (LDS)"};
static const int kFpMuls[OP_N] = {1, 18, 54, 36, 39};

__global__ __launch_bounds__(256, 1) void k_probe(int op, int iters, uint4* __restrict__ slot, uint64_t stride,
                                                  uint32_t* __restrict__ sink) {
  __shared__ uint4 F[36][256];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  LdsF12 f{F, threadIdx.x};
  GlobF12 g{slot, stride, i};
  copy12(f, g);
  if (op == OP_FPMUL) {
    fp2 a = f.ld(0), b = f.ld(1);
    fp x = a.c0, y = b.c0;
#pragma unroll 1
    for (int it = 0; it < iters; it++) {
      x = mul(x, y);
      y = mul(y, x);
    }
    f.st(0, {x, y});
  } else if (op == OP_CYCSQ) {
#pragma unroll 1
    for (int it = 0; it < iters; it++) cycsq12(f);
  } else if (op == OP_MUL12) {
#pragma unroll 1
    for (int it = 0; it < iters; it++) mul12(f, g);
  } else if (op == OP_SQR12) {
#pragma unroll 1
    for (int it = 0; it < iters; it++) sqr12(f);
  } else {
    fp2 c0 = g.ld(3), c1 = g.ld(4), c4 = g.ld(5);
#pragma unroll 1
    for (int it = 0; it < iters; it++) mul014(f, c0, c1, c4);
  }
  fp2 r = f.ld(0);
  uint32_t h = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) h ^= r.c0.v[k] ^ r.c1.v[k];
  sink[i] = h;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 262144;
  const int iters = argc > 2 ? atoi(argv[2]) : 16;
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  uint4* slot;
  uint32_t* sink;
  CHK(hipMalloc(&slot, n * 36 * 16));
  CHK(hipMalloc(&sink, n * 4));
  // random limbs below 2^380 (valid Fp inputs)
  {
    uint32_t* h = (uint32_t*)malloc(n * 36 * 16);
    uint64_t s = 88172645463325252ull;
    for (uint64_t w = 0; w < n * 144; w++) {
      s ^= s << 13, s ^= s >> 7, s ^= s << 17;
      h[w] = (uint32_t)s;
    }
    // word (row*4 + q) of lane i: limb 11 of every Fp kept < 2^28
    for (uint64_t r = 0; r < 36; r++)
      for (uint64_t i = 0; i < n; i++)
        for (int q = 0; q < 4; q++)
          if ((r * 4 + q) % 12 == 11) h[(r * n + i) * 4 + q] &= 0x0fffffffu;
    CHK(hipMemcpy(slot, h, n * 36 * 16, hipMemcpyHostToDevice));
    free(h);
  }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double clk = prop.clockRate * 1e3;   // Hz
  const uint64_t waves = n / 64, simds = (uint64_t)prop.multiProcessorCount * 4;
  printf("device %s CUs %d clock %.0f MHz lanes %llu iters %d\n", prop.gcnArchName, prop.multiProcessorCount,
         clk / 1e6, (unsigned long long)n, iters);
  for (int op = 0; op < OP_N; op++) {
    for (int rep = 0; rep < 2; rep++) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_probe, dim3((unsigned)(n / 256)), dim3(256), 0, 0, op, iters, slot, n, sink);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 0) continue;
      const double ops = (double)iters * (op == OP_FPMUL ? 2 : 1);
      // cycles one wave spends per op (waves run one per SIMD, in rounds)
      const double rounds = (double)waves / simds;
      const double cyc = ms * 1e-3 * clk / rounds / ops;
      const double fpmul_rate = (double)n * ops * kFpMuls[op] / (ms * 1e-3);
      printf("%-22s %9.3f ms  %9.0f cycles/op/wave  %7.0f cycles per Fp mul  %6.1f G Fp-mul/s\n", kNames[op], ms, cyc,
             cyc / kFpMuls[op], fpmul_rate / 1e9);
    }
  }
  return 0;
}
