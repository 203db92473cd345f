// Microbenchmark of the staged Fp12 operations (bls/staged.hpp) in isolation,
// one lane per "signature", the same LDS accumulator layout as k_miller/k_final.
// Prints per-op cycles per wave so the costs of the Miller-loop and
// final-exponentiation building blocks can be compared with the plain Fp
// multiply chain (the VALU floor).  Build on the CPU:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I cess_amd/csrc tools/fe_probe.hip -o tools/fe_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "soa.hpp"
#include "pair2.hpp"   // tools/experimental (not a product header)

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

enum Op { OP_FPMUL, OP_CYCSQ, OP_MUL12, OP_SQR12, OP_LINE, OP_SQR12S, OP_N };
static const char* kNames[OP_N] = {"fp_mul chain", "cycsq12 (LDS)", "mul12 (LDS x HBM)", "sqr12 (LDS)",
                                   "mul014 line (LDS)", "sqr12 streamed (HBM, 2 waves)"};
static const int kFpMuls[OP_N] = {1, 18, 54, 36, 39, 36};

// --- streamed Fp6 operands (experiment): views compute operands from stores
template <class S> struct Half6 { const S& s; int h; __device__ fp2 get(int j) const { return s.ld(3 * h + j); } };
template <class A, class B> struct Sum6 { A a; B b; __device__ fp2 get(int j) const { return add(a.get(j), b.get(j)); } };
template <class A> struct MulV6 { A a; __device__ fp2 get(int j) const { return j == 0 ? mul_nr(a.get(2)) : a.get(j - 1); } };
template <class S> struct Sink6 { const S& s; int h; __device__ void put(int j, const fp2& x) const { s.st(3 * h + j, x); } };

template <class VA, class VB, class O>
__device__ __forceinline__ void mul6_stream(const VA& A, const VB& B, const O& out) {
  fp2 v0 = mul(A.get(0), B.get(0));
  CESS_MEMBAR();
  fp2 v1 = mul(A.get(1), B.get(1));
  CESS_MEMBAR();
  fp2 v2 = mul(A.get(2), B.get(2));
  CESS_MEMBAR();
  out.put(0, add(v0, mul_nr(sub(sub(mul(add(A.get(1), A.get(2)), add(B.get(1), B.get(2))), v1), v2))));
  CESS_MEMBAR();
  out.put(1, add(sub(sub(mul(add(A.get(0), A.get(1)), add(B.get(0), B.get(1))), v0), v1), mul_nr(v2)));
  CESS_MEMBAR();
  out.put(2, add(sub(sub(mul(add(A.get(0), A.get(2)), add(B.get(0), B.get(2))), v0), v2), v1));
  CESS_MEMBAR();
}
template <class S, class T>
__device__ __forceinline__ void sqr12_stream(const S& f, const T& t) {
  Half6<S> a0{f, 0}, a1{f, 1};
  mul6_stream(a0, a1, Sink6<T>{t, 0});                                   // ab
  mul6_stream(Sum6<Half6<S>, Half6<S>>{a0, a1}, Sum6<Half6<S>, MulV6<Half6<S>>>{a0, {a1}}, Sink6<T>{t, 1});  // X
#pragma unroll 1
  for (int j = 0; j < 3; j++) {
    fp2 ab = t.ld(j), vab = j == 0 ? mul_nr(t.ld(2)) : t.ld(j - 1);
    f.st(j, sub(sub(t.ld(3 + j), ab), vab));
    CESS_MEMBAR();
  }
#pragma unroll 1
  for (int j = 0; j < 3; j++) f.st(3 + j, dbl(t.ld(j)));
}

__global__ __launch_bounds__(256, 2) void k_probe2(int iters, uint4* __restrict__ slot, uint4* __restrict__ tslot,
                                                   uint4* __restrict__ fslot, uint64_t stride,
                                                   uint32_t* __restrict__ sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  GlobF12 f{fslot, stride, i}, t{tslot, stride, i}, g{slot, stride, i};
  copy12(f, g);
#pragma unroll 1
  for (int it = 0; it < iters; it++) sqr12_stream(f, t);
  fp2 r = f.ld(0);
  uint32_t h = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) h ^= r.c0.v[k] ^ r.c1.v[k];
  sink[i] = h;
}

__global__ __launch_bounds__(256, 1) void k_probe(int op, int iters, uint4* __restrict__ slot, uint64_t stride,
                                                  uint32_t* __restrict__ sink) {
  __shared__ uint4 F[36][256];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  LdsF12 f{F, wave_first_thread()};
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
  } else if (op == OP_LINE) {
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

// lane-pair versions: 512 threads = 256 signatures per block, two waves per SIMD.
// op: OP_CYCSQ, OP_SQR12, OP_LINE.  Output: the final Fp12 of each signature.
template <int op>
__global__ __launch_bounds__(512, 1) void k_probe_pair(int, int iters, uint4* __restrict__ slot, uint64_t stride,
                                                        uint4* __restrict__ out) {
  __shared__ uint4 F[36][256];
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  PairF12 f{F, threadIdx.x >> 1, (threadIdx.x & 1) != 0};
  GlobF12 g{slot, stride, i};
  if (!f.hi) copy12(f, g);
  __syncthreads();
  if (op == OP_CYCSQ) {
#pragma unroll 1
    for (int it = 0; it < iters; it++) cycsq12p(f);
  } else if (op == OP_SQR12) {
#pragma unroll 1
    for (int it = 0; it < iters; it++) sqr12p(f);
  } else if (op == OP_LINE) {
    fp2 c0 = g.ld(3), c1 = g.ld(4), c4 = g.ld(5);
#pragma unroll 1
    for (int it = 0; it < iters; it++) mul014p(f, c0, c1, c4);
  }
  __syncthreads();
  if (!f.hi) copy12(GlobF12{out, stride, i}, f);
}
// single-lane reference of the same ops, output for comparison
__global__ __launch_bounds__(256, 1) void k_probe_ref(int op, int iters, uint4* __restrict__ slot, uint64_t stride,
                                                       uint4* __restrict__ out) {
  __shared__ uint4 F[36][256];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  LdsF12 f{F, wave_first_thread()};
  GlobF12 g{slot, stride, i};
  copy12(f, g);
  if (op == OP_CYCSQ) {
#pragma unroll 1
    for (int it = 0; it < iters; it++) cycsq12(f);
  } else if (op == OP_SQR12) {
#pragma unroll 1
    for (int it = 0; it < iters; it++) sqr12(f);
  } else if (op == OP_LINE) {
    fp2 c0 = g.ld(3), c1 = g.ld(4), c4 = g.ld(5);
#pragma unroll 1
    for (int it = 0; it < iters; it++) mul014(f, c0, c1, c4);
  }
  copy12(GlobF12{out, stride, i}, f);
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 262144;
  const int iters = argc > 2 ? atoi(argv[2]) : 16;
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  uint4 *slot, *tslot, *fslot;
  uint32_t* sink;
  CHK(hipMalloc(&slot, n * 36 * 16));
  CHK(hipMalloc(&tslot, n * 36 * 16));
  CHK(hipMalloc(&fslot, n * 36 * 16));
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
      if (op == OP_SQR12S)
        hipLaunchKernelGGL(k_probe2, dim3((unsigned)(n / 256)), dim3(256), 0, 0, iters, slot, tslot, fslot, n, sink);
      else
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
  // lane-pair ops: correctness against the single-lane ops, then throughput
  {
    uint4 *o1, *o2;
    CHK(hipMalloc(&o1, n * 36 * 16));
    CHK(hipMalloc(&o2, n * 36 * 16));
    const int pops[3] = {OP_CYCSQ, OP_SQR12, OP_LINE};
    for (int q = 0; q < 3; q++) {
      const int op = pops[q];
      hipLaunchKernelGGL(k_probe_ref, dim3((unsigned)(n / 256)), dim3(256), 0, 0, op, 3, slot, n, o1);
      auto kp = op == OP_CYCSQ ? k_probe_pair<OP_CYCSQ> : op == OP_SQR12 ? k_probe_pair<OP_SQR12> : k_probe_pair<OP_LINE>;
      hipLaunchKernelGGL(kp, dim3((unsigned)(n / 256)), dim3(512), 0, 0, op, 3, slot, n, o2);
      CHK(hipDeviceSynchronize());
      std::vector<uint32_t> h1(n * 144), h2(n * 144);
      CHK(hipMemcpy(h1.data(), o1, n * 576, hipMemcpyDeviceToHost));
      CHK(hipMemcpy(h2.data(), o2, n * 576, hipMemcpyDeviceToHost));
      uint64_t bad = 0;
      for (uint64_t w = 0; w < n * 144; w++) bad += h1[w] != h2[w];
      float ms = 0;
      for (int rep = 0; rep < 2; rep++) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(kp, dim3((unsigned)(n / 256)), dim3(512), 0, 0, op, iters, slot, n, o2);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
      }
      const double fpmul_rate = (double)n * iters * kFpMuls[op] / (ms * 1e-3);
      printf("pair %-22s %9.3f ms  %6.1f G Fp-mul/s   mismatched words vs single-lane: %llu\n", kNames[op], ms,
             fpmul_rate / 1e9, (unsigned long long)bad);
    }
  }
  return 0;
}
