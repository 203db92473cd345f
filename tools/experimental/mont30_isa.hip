// ISA-count probe (round 4): one Montgomery product in
// 13 x 30-bit digits with split column accumulators, compiled for gfx950 and
// counted against field.hpp mul().  Not built
// into the library.  hipcc -O3 --offload-arch=gfx950 -I cess_amd/csrc
// --cuda-device-only -S tools/experimental/mont30_isa.hip -o /tmp/k30.s
// python tools/experimental/isa_count.py /tmp/k30.s k_fpmul30
#include <hip/hip_runtime.h>
#include "bls/field.hpp"
using namespace bls;
__device__ fp ldf(const uint32_t* p, int i) { fp r; for (int k = 0; k < 12; k++) r.v[k] = p[k * 256 + i]; return r; }
__device__ void stf(uint32_t* p, int i, const fp& a) { for (int k = 0; k < 12; k++) p[k * 256 + i] = a.v[k]; }
constexpr uint32_t P30D[13] = {0x3fffaaabu,0x27fbffffu,0x153ffffbu,0x2affffacu,0x30f6241eu,0x34a83dau,0x112bf673u,0x12e13ce1u,0x2cd76477u,0x1ed90d2eu,0x29a4b1bau,0x3a8e5ff9u,0x1a0111u};
constexpr uint32_t NPINV30 = 0x3ffcfffd, MM30 = 0x3fffffff;
__device__ __forceinline__ void unpack30(const fp& a, uint32_t (&l)[13]) {
#pragma unroll
  for (int k = 0; k < 13; k++) {
    const int off = 30 * k, i = off >> 5, sh = off & 31;
    uint32_t lo = a.v[i] >> sh;
    if (sh > 2 && i + 1 < 12) lo |= a.v[i + 1] << (32 - sh);
    l[k] = lo & MM30;
  }
}
__device__ __forceinline__ fp pack30(const uint32_t (&l)[13]) {
  fp r;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const int off = 32 * j, k = off / 30, sh = off - 30 * k;
    uint32_t w = l[k] >> sh;
    if (k + 1 < 13) w |= l[k + 1] << (30 - sh);
    if (sh > 28 && k + 2 < 13) w |= l[k + 2] << (60 - sh);
    r.v[j] = w;
  }
  return r;
}
__device__ __forceinline__ fp mul30(const fp& a0, const fp& b0) {
  fp a = a0, b = b0; seq(a); seq(b);
  uint32_t x[13], y[13], m[13], t[13];
  unpack30(a, x); unpack30(b, y);
  uint64_t A = 0, B = 0;
#pragma unroll
  for (int k = 0; k < 25; k++) {
#pragma unroll
    for (int i = 0; i < 13; i++) if (k - i >= 0 && k - i < 13) A += (uint64_t)x[i] * y[k - i];
#pragma unroll
    for (int i = 0; i < 13; i++) if (i < k && k - i < 13 && i < 13) B += (uint64_t)m[i] * P30D[k - i];
    B += (uint32_t)A & MM30; A >>= 30;
    if (k < 13) {
      m[k] = ((uint32_t)B * NPINV30) & MM30;
      B += (uint64_t)m[k] * P30D[0];
    } else {
      t[k - 13] = (uint32_t)B & MM30;
    }
    B >>= 30;
  }
  t[12] = (uint32_t)(B + A);
  fp r = pack30(t); seq(r); return r;
}
extern "C" __global__ void k_fpmul30(const uint32_t* in, uint32_t* out) {
  int i = threadIdx.x;
  fp r = mul30(ldf(in, i), ldf(in + 3072, i));
  stf(out, i, r);
}
