// SoA (limb-major) device-buffer helpers: element e of signature i lives at
// buf[e * stride + i], so consecutive lanes touch consecutive words.
#pragma once
#include "bls/h2c.hpp"
#include "bls/staged.hpp"
#include "kernels.hpp"

namespace cess {
using namespace bls;


// --- SoA helpers -----------------------------------------------------------
CESS_HD fp ld_fp(const uint32_t* __restrict__ base, uint64_t stride, uint32_t i) {
  fp r;
#pragma unroll
  for (int k = 0; k < 12; k++) r.v[k] = base[k * stride + i];
  return r;
}
CESS_HD void st_fp(uint32_t* __restrict__ base, uint64_t stride, uint32_t i, const fp& a) {
#pragma unroll
  for (int k = 0; k < 12; k++) base[k * stride + i] = a.v[k];
}
CESS_HD fp2 ld_fp2(const uint32_t* base, uint64_t stride, uint32_t i) {
  return {ld_fp(base, stride, i), ld_fp(base + 12 * stride, stride, i)};
}
CESS_HD void st_fp2(uint32_t* base, uint64_t stride, uint32_t i, const fp2& a) {
  st_fp(base, stride, i, a.c0);
  st_fp(base + 12 * stride, stride, i, a.c1);
}
CESS_HD uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// coefficient triple k of one signature: 6 Fp = 72 words, at word offset 72*k
CESS_HD coeff3 ld_coeff(const uint32_t* base, uint64_t stride, uint32_t i, int k) {
  const uint32_t* b = base + (uint64_t)(72 * k) * stride;
  return {ld_fp2(b, stride, i), ld_fp2(b + 24 * stride, stride, i), ld_fp2(b + 48 * stride, stride, i)};
}
CESS_HD void st_coeff(uint32_t* base, uint64_t stride, uint32_t i, int k, const coeff3& c) {
  uint32_t* b = base + (uint64_t)(72 * k) * stride;
  st_fp2(b, stride, i, c.c0);
  st_fp2(b + 24 * stride, stride, i, c.c1);
  st_fp2(b + 48 * stride, stride, i, c.c2);
}
// uint4-row layout (k_prepare output): row q of step k of sig i at base[(18k+q)*stride + i]
CESS_HD coeff3 ld_coeff4(const uint4* __restrict__ base, uint64_t stride, uint32_t i, int k) {
  coeff3 r;
  uint32_t* w = &r.c0.c0.v[0];
#pragma unroll
  for (int q = 0; q < 18; q++) {
    uint4 x = base[(uint64_t)(18 * k + q) * stride + i];
    w[4 * q] = x.x, w[4 * q + 1] = x.y, w[4 * q + 2] = x.z, w[4 * q + 3] = x.w;
  }
  return r;
}
CESS_HD void st_coeff4(uint4* __restrict__ base, uint64_t stride, uint32_t i, int k, const coeff3& c) {
  const uint32_t* w = &c.c0.c0.v[0];
#pragma unroll
  for (int q = 0; q < 18; q++)
    base[(uint64_t)(18 * k + q) * stride + i] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
// one coefficient (j = 0, 1, 2: c0, c1, c2) of line k, rows 18k + 6j .. +5
CESS_HD void st_coeff4_one(uint4* __restrict__ base, uint64_t stride, uint32_t i, int k, int j, const fp2& c) {
  const uint32_t* w = &c.c0.v[0];
#pragma unroll
  for (int q = 0; q < 6; q++)
    base[(uint64_t)(18 * k + 6 * j + q) * stride + i] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
// wave-uniform coefficient table (the -G2 constant): stride 1, same address in every lane
// c0 and c1 of a line of a table normalised to c2 = 1 (the -G2 table after
// k_norm_lines): 48 of the line's 72 dwords, so the 68 lines k_miller touches
// per signature (13 KB) stay resident in the scalar data cache instead of
// streaming 19.6 KB through it once per signature
CESS_HD coeff3 ld_coeff_uniform01(const uint32_t* tab, int k) {
  const uint32_t* b = tab + 72 * k;
  coeff3 r;
  fp* e = &r.c0.c0;
#pragma unroll
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int l = 0; l < 12; l++) e[j].v[l] = b[12 * j + l];
  r.c2 = fp2_one();
  return r;
}
CESS_HD coeff3 ld_coeff_uniform(const uint32_t* tab, int k) {
  const uint32_t* b = tab + 72 * k;
  coeff3 r;
  fp* e = &r.c0.c0;
#pragma unroll
  for (int j = 0; j < 6; j++)
#pragma unroll
    for (int l = 0; l < 12; l++) e[j].v[l] = b[12 * j + l];
  return r;
}


}  // namespace cess
