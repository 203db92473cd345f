// Microbenchmark: integer multiply-add rates on gfx950 (the roofline peak of
// the BLS verifier is the v_mad_u64_u32 rate, which the guides do not list).
// Variants:
//   mad      : independent v_mad_u64_u32 chains (64-bit addend, no carry use)
//   mac      : v_mad_u64_u32 (carry-out to SGPR) + v_addc_co_u32  (96-bit accumulate)
//   mul32    : the shipped Fp multiply (bls::mul: 12x32 storage, 14x28 carry-free compute)
//   mul28    : full 14x28-bit Montgomery multiply (carry-free 64-bit columns)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include "../cess_amd/csrc/bls/field.hpp"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// 96-bit accumulate with the carry-out in an SGPR pair (the 12 x 32 scheme)
__device__ __forceinline__ void mac(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& hi) {
  uint64_t c, d;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
  asm("v_addc_co_u32 %0, %1, %0, 0, %2" : "+v"(hi), "=s"(d) : "s"(c));
}

__global__ __launch_bounds__(256) void k_mad(uint64_t* out, int iters, uint32_t s) {
  uint32_t a = threadIdx.x * 77 + s, b = blockIdx.x * 31 + s;
  uint64_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b) : "vcc");
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mac(uint64_t* out, int iters, uint32_t s) {
  uint32_t a = threadIdx.x * 77 + s, b = blockIdx.x * 31 + s;
  uint64_t acc[8];
  uint32_t hi[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { acc[j] = j; hi[j] = 0; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) mac(a, b + j, acc[j], hi[j]);
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= acc[j] + hi[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mul32(uint32_t* io, int iters) {
  uint64_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bls::fp a, b;
#pragma unroll
  for (int k = 0; k < 12; k++) { a.v[k] = (uint32_t)(i * 2654435761u + k) & (k == 11 ? 0x0fffffffu : ~0u); b.v[k] = a.v[k] ^ 0x5555u; }
  for (int it = 0; it < iters; it++) { a = bls::mul(a, b); b = bls::mul(b, a); }
#pragma unroll
  for (int k = 0; k < 12; k++) io[k * 1048576 + (i & 1048575)] = a.v[k] ^ b.v[k];
}

// --- 14 x 28-bit variant, R = 2^392 ---
struct fq { uint32_t v[14]; };
static constexpr uint32_t M28 = (1u << 28) - 1;
// p in 28-bit limbs, pinv = -p^-1 mod 2^28 (filled from host-computed constants)
__constant__ uint32_t P28[14];
__constant__ uint32_t PINV28;
__device__ __forceinline__ fq mul28(const fq& a, const fq& b, const uint32_t (&p)[14], uint32_t pinv) {
  uint64_t acc = 0;
  uint32_t m[14];
  fq t;
#pragma unroll
  for (int k = 0; k < 14; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a.v[i] * b.v[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * p[k - i];
    m[k] = ((uint32_t)acc * pinv) & M28;
    acc += (uint64_t)m[k] * p[0];
    acc >>= 28;
  }
#pragma unroll
  for (int k = 14; k < 27; k++) {
#pragma unroll
    for (int i = k - 13; i < 14; i++) { acc += (uint64_t)a.v[i] * b.v[k - i]; acc += (uint64_t)m[i] * p[k - i]; }
    t.v[k - 14] = (uint32_t)acc & M28;
    acc >>= 28;
  }
  t.v[13] = (uint32_t)acc;
  // conditional subtract
  fq s;
  int32_t borrow = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    int32_t d = (int32_t)t.v[k] - (int32_t)p[k] + borrow;
    s.v[k] = (uint32_t)d & M28;
    borrow = d >> 28;
  }
#pragma unroll
  for (int k = 0; k < 14; k++) t.v[k] = borrow ? t.v[k] : s.v[k];
  return t;
}
__global__ __launch_bounds__(256) void k_mul28(uint32_t* io, int iters) {
  uint64_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t p[14];
#pragma unroll
  for (int k = 0; k < 14; k++) p[k] = P28[k];
  uint32_t pinv = PINV28;
  fq a, b;
#pragma unroll
  for (int k = 0; k < 14; k++) { a.v[k] = (uint32_t)(i * 2654435761u + k) & (k == 13 ? 0xffffu : M28); b.v[k] = a.v[k] ^ 0x5555u; }
  for (int it = 0; it < iters; it++) { a = mul28(a, b, p, pinv); b = mul28(b, a, p, pinv); }
#pragma unroll
  for (int k = 0; k < 14; k++) io[k * 1048576 + (i & 1048575)] = a.v[k] ^ b.v[k];
}

template <class F>
static double timeit(F f) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  f();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  f();
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e-3;
}

int main() {
  // p in 28-bit limbs
  const uint32_t* praw = bls::c::P_RAW;
  uint32_t p28[14] = {0};
  {
    // big-int shift: assemble bits
    for (int bit = 0; bit < 384; bit++) {
      uint32_t v = (praw[bit / 32] >> (bit % 32)) & 1;
      if (v) p28[bit / 28] |= 1u << (bit % 28);
    }
  }
  uint32_t inv = 1;  // p^-1 mod 2^28 by Newton
  for (int i = 0; i < 5; i++) inv *= 2 - p28[0] * inv;
  uint32_t pinv28 = (0u - inv) & M28;
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(P28), p28, sizeof(p28)));
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(PINV28), &pinv28, 4));

  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  uint64_t* out; CHK(hipMalloc(&out, 64ull << 20));
  uint32_t* io; CHK(hipMalloc(&io, 64ull << 20));
  for (int wpsimd = 1; wpsimd <= 8; wpsimd *= 2) {
    int blocks = cus * wpsimd;   // 256 threads = 4 waves = 1 wave per SIMD per block
    int iters = 4096;
    double t = timeit([&] { k_mad<<<blocks, 256>>>(out, iters, 1); });
    double mads = (double)blocks * 256 * iters * 8;
    printf("mad   waves/SIMD=%d : %.3f T mad/s  (%.2f lane-mads/CU/clk @2.4GHz)\n", wpsimd, mads / t * 1e-12, mads / t / cus / 2.4e9);
    t = timeit([&] { k_mac<<<blocks, 256>>>(out, iters, 1); });
    printf("mac   waves/SIMD=%d : %.3f T mac/s  (%.2f lane-macs/CU/clk)\n", wpsimd, mads / t * 1e-12, mads / t / cus / 2.4e9);
    int it2 = 256;
    t = timeit([&] { k_mul32<<<blocks, 256>>>(io, it2); });
    double muls = (double)blocks * 256 * it2 * 2;
    printf("mul32 waves/SIMD=%d : %.2f G fpmul/s (%.3f T mad-equiv/s at 288/mul)\n", wpsimd, muls / t * 1e-9, muls * 288 / t * 1e-12);
    t = timeit([&] { k_mul28<<<blocks, 256>>>(io, it2); });
    printf("mul28 waves/SIMD=%d : %.2f G fpmul/s\n", wpsimd, muls / t * 1e-9);
  }
  return 0;
}
