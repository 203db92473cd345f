// Microbenchmark (round 5): the shipped lazily reduced Fp2 product
// (bls/field.hpp mul(fp2, fp2)) and Fp2 additions on register operands, in a
// dependent loop, at 1 and 2 waves per SIMD: in-kernel s_memtime cycles per
// loop iteration per wave.  With the instruction count of the loop body
// (llvm-objdump of this binary) this is the product's own issue rate, without
// the Miller loop's LDS traffic.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=1000000 -I cess_amd/csrc tools/fp_probe.hip -o tools/fp_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "bls/field.hpp"

using namespace bls;

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


// (opaque(): bls/field.hpp)

// Lazy Fp2 product with the column work separated from the reduction chain:
// per column, the a*b products go to fresh partial sums (two per component,
// by digit parity), the m*p terms already known to another fresh sum, and
// only their merge, m_k and the shift are on the carried chain.
template <int SPLIT, bool QSEP = true, bool QBAL = false>
__device__ __forceinline__ fp2 mul_sep(const fp2& a, const fp2& b) {
  fp a0 = a.c0, a1 = a.c1, b0 = b.c0, b1 = b.c1;
  seq(a0); seq(a1); seq(b0); seq(b1);
  uint32_t x0[14], x1[14], y0[14], y1[14], y1n[14];
  unpack28(a0, x0); unpack28(a1, x1); unpack28(b0, y0); unpack28(b1, y1);
#pragma unroll
  for (int i = 0; i < 14; i++) y1n[i] = c::NEG_K28[i] - y1[i];
  uint32_t m0[14], m1[14], t0[14], t1[14];
  uint64_t acc0 = 0, acc1 = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    uint64_t s0[SPLIT], s1[SPLIT];
#pragma unroll
    for (int h = 0; h < SPLIT; h++) s0[h] = 0, s1[h] = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j < 0 || j >= 14) continue;
      const int h = i % SPLIT;
      mac(s0[h], x0[i], y0[j]);
      mac(s1[h], x0[i], y1[j]);
      mac(s0[h], x1[i], y1n[j]);
      mac(s1[h], x1[i], y0[j]);
    }
    uint64_t q0 = 0, q1 = 0;
    const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 14;
    if (QSEP) {
#pragma unroll
      for (int i = lo; i < hi; i++) {
        mac(q0, m0[i], c::P28[k - i]);
        mac(q1, m1[i], c::P28[k - i]);
      }
    } else if (QBAL) {   // the known m*p terms split over the chains by the parity of i
#pragma unroll
      for (int i = lo; i < hi; i++) {
        mac(s0[i % SPLIT], m0[i], c::P28[k - i]);
        mac(s1[i % SPLIT], m1[i], c::P28[k - i]);
      }
    } else {   // the known m*p terms continue the last a*b partial sum's chain
#pragma unroll
      for (int i = lo; i < hi; i++) {
        mac(s0[SPLIT - 1], m0[i], c::P28[k - i]);
        mac(s1[SPLIT - 1], m1[i], c::P28[k - i]);
      }
    }
#pragma unroll
    for (int h = 0; h < SPLIT; h++) {
      opaque(s0[h]);
      opaque(s1[h]);
      q0 += s0[h];
      q1 += s1[h];
    }
    opaque(q0);
    opaque(q1);
    acc0 += q0;
    acc1 += q1;
    if (k < 14) {
      m0[k] = ((uint32_t)acc0 * c::PINV28) & M28;
      m1[k] = ((uint32_t)acc1 * c::PINV28) & M28;
      mac(acc0, m0[k], c::P28[0]);
      mac(acc1, m1[k], c::P28[0]);
    } else {
      t0[k - 14] = (uint32_t)acc0 & M28;
      t1[k - 14] = (uint32_t)acc1 & M28;
    }
    acc0 >>= 28;
    acc1 >>= 28;
  }
  t0[13] = (uint32_t)acc0;
  t1[13] = (uint32_t)acc1;
  fp2 r;
  r.c0 = pack28(t0);
  r.c1 = pack28(t1);
  seq(r.c0); seq(r.c1);
  return r;
}

template <int OP>
__global__ __launch_bounds__(256) void k_fp(uint64_t* out, const uint32_t* in, int iters) {
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = in[0];
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  fp2 a, b;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    a.c0.v[i] = in[i * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
    a.c1.v[i] = in[(12 + i) * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
    b.c0.v[i] = in[(24 + i) * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
    b.c1.v[i] = in[(36 + i) * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t0 = stamp();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
    if (OP == 0) a = mul(a, b);                   // lazy Fp2 product
    if (OP == 1) a = sub(add(a, b), dbl(b));      // Fp2 add/sub chains
    if (OP == 2) a = dot2(a, b, b, a);            // one-reduction a b + c d
    if (OP == 3) mul2(a, b, b, a, a, b);          // two independent products, one column loop
    if (OP == 4) a = mul_sep<1>(a, b);            // column sums off the reduction chain
    if (OP == 5) a = mul_sep<2>(a, b);            // ... split by digit parity
    if (OP == 6) a = mul_sep<2, false>(a, b);     // ... m*p terms on the second a*b chain
    if (OP == 7) a = mul_sep<2, false, true>(a, b);
    if (OP == 8) a = mul_sep<3, false>(a, b);
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t1 = stamp();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r ^= a.c0.v[i] ^ a.c1.v[i] ^ b.c0.v[i];
  const int w = blockIdx.x * 4 + threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) out[2 * w] = t1 - t0;
  if (r == 0x12345678u) out[2 * w + 1] = r;
  if (OP >= 4 && iters == 1) {   // one step: compare with the shipped product
    fp2 a1, b1;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      a1.c0.v[i] = in[i * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
      a1.c1.v[i] = in[(12 + i) * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
      b1.c0.v[i] = in[(24 + i) * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
      b1.c1.v[i] = in[(36 + i) * 4096 + (t & 4095)] & (i == 11 ? 0x0fffffffu : ~0u);
    }
    const fp2 ref = mul(a1, b1);
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) d |= (ref.c0.v[i] ^ a.c0.v[i]) | (ref.c1.v[i] ^ a.c1.v[i]);
    if (d) out[2 * w + 1] = 0xBAD;
  }
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 2048;
  const char* names[9] = {"mul(fp2,fp2)", "sub(add,dbl) fp2", "dot2", "mul2 (2 products)", "mul_sep<1>", "mul_sep<2>",
                          "mul_sep<2,noq>", "mul_sep<2,bal>", "mul_sep<3,noq>"};
  void (*fns[9])(uint64_t*, const uint32_t*, int) = {k_fp<0>, k_fp<1>, k_fp<2>, k_fp<3>, k_fp<4>, k_fp<5>,
                                                      k_fp<6>, k_fp<7>, k_fp<8>};
  uint64_t* out;
  uint32_t* in;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 4 * 16));
  CHK(hipMalloc(&in, 48 * 4096 * 4));
  std::vector<uint32_t> hin(48 * 4096);
  uint64_t x = 88172645463325252ull;
  for (auto& v : hin) x ^= x << 13, x ^= x >> 7, x ^= x << 17, v = (uint32_t)x;
  CHK(hipMemcpy(in, hin.data(), hin.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint64_t> h((size_t)cus * 8 * 4 * 2);
  for (auto f : fns) CHK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  printf("# cycles per loop iteration per wave (in-kernel s_memtime, median over waves)\n");
  printf("%-18s %10s %10s\n", "op", "W=1", "W=2");
  for (int v = 0; v < 9; v++) {
    if (v >= 4) {   // correctness of the separated forms: one step against mul()
      hipLaunchKernelGGL(fns[v], dim3(cus), dim3(256), 0, 0, out, in, 1);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), out, (size_t)cus * 4 * 16, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int i = 0; i < cus * 4; i++) bad += h[2 * i + 1] == 0xBAD;
      printf("# %s: %s\n", names[v], bad ? "MISMATCH vs mul()" : "equal to mul() on every lane");
    }
    printf("%-18s", names[v]);
    for (int w : {1, 2}) {
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      const int blocks = cus * w;
      hipLaunchKernelGGL(fns[v], dim3(blocks), dim3(256), lds, 0, out, in, 16);
      hipLaunchKernelGGL(fns[v], dim3(blocks), dim3(256), lds, 0, out, in, iters);
      CHK(hipDeviceSynchronize());
      CHK(hipMemcpy(h.data(), out, (size_t)blocks * 4 * 16, hipMemcpyDeviceToHost));
      std::vector<double> cyc;
      for (int i = 0; i < blocks * 4; i++) cyc.push_back((double)h[2 * i] / iters);
      std::sort(cyc.begin(), cyc.end());
      printf(" %10.1f", cyc[cyc.size() / 2]);
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
