// CDNA4 (gfx950) generator-side kernels (PrivateKey, reference src/lib.rs:166-236, A15):
//   k_keygen : pk = compress([sk] G2)          PrivateKey::public_key   src/lib.rs:226-228
//   k_sign   : sig = compress([sk] H(msg))     PrivateKey::sign         src/lib.rs:233-236
//   k_hash_out: compress(H(msg))               hash_to_g1               src/lib.rs:25-31
// Secret keys are 32-byte big-endian scalars < r (PrivateKey::deserialize, :208-223).
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

namespace {
__device__ void load_sk(const uint8_t* sk, uint32_t (&k)[8]) {
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const uint8_t* q = sk + 28 - 4 * w;
    k[w] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
__device__ void store_bytes(uint8_t* dst, const uint8_t* src, int n) {
  for (int j = 0; j < n; j++) dst[j] = src[j];
}

// GLV split of a scalar for G1, where r = L^2 + L + 1 with L = x^2 - 1 (128
// bits) and [L]P = (beta^2 x, y) (beta: c::G1_BETA, phi = [-x^2] = [L^2]):
// k mod r = k1 + k2 L with 0 <= k1 < L and k2 < 2^128 -- plain long division
// by L (k is first reduced below r; a 32-byte key may exceed it).  Words
// little-endian.
constexpr uint32_t R_LE[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                              0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
constexpr uint32_t LAMBDA_LE[4] = {0xffffffffu, 0x00000000u, 0x0001a402u, 0xac45a401u};

__device__ __forceinline__ void sub_r_if_ge(uint32_t (&k)[8]) {
  uint32_t t[8], br = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) t[w] = subc32(k[w], R_LE[w], br, &br);
#pragma unroll
  for (int w = 0; w < 8; w++) k[w] = br ? k[w] : t[w];
}

__device__ __forceinline__ void glv_split(const uint32_t (&k0)[8], uint32_t (&k1)[4], uint32_t (&k2)[4]) {
  uint32_t k[8];
#pragma unroll
  for (int w = 0; w < 8; w++) k[w] = k0[w];
  sub_r_if_ge(k);
  sub_r_if_ge(k);   // 2^256 < 3 r
  uint32_t rem[5] = {0, 0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
#pragma unroll 1
  for (int bit = 255; bit >= 0; bit--) {
    // rem = 2 rem + bit (rem < L before, so < 2^129), q <<= 1
#pragma unroll
    for (int w = 4; w > 0; w--) rem[w] = (rem[w] << 1) | (rem[w - 1] >> 31);
    rem[0] = (rem[0] << 1) | ((k[bit >> 5] >> (bit & 31)) & 1u);
#pragma unroll
    for (int w = 3; w > 0; w--) q[w] = (q[w] << 1) | (q[w - 1] >> 31);
    q[0] <<= 1;
    uint32_t t[5], br = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) t[w] = subc32(rem[w], LAMBDA_LE[w], br, &br);
    t[4] = subc32(rem[4], 0u, br, &br);
    const bool ge = br == 0;
#pragma unroll
    for (int w = 0; w < 5; w++) rem[w] = ge ? t[w] : rem[w];
    q[0] |= ge ? 1u : 0u;
  }
#pragma unroll
  for (int w = 0; w < 4; w++) k1[w] = rem[w], k2[w] = q[w];
}

// [k]P for affine P in G1 (not the identity): [k1]P + [k2]([L]P) by 2-bit
// joint windows over the affine table {P, 2P, 3P} (one inversion) and its
// image (beta^2 x, y): 128 doublings + 128 complete mixed additions, against
// 256 doublings + 256 additions for the bitwise ladder (some lane of a wave
// always adds).  The additions are computed every window and kept by a select
// (digits differ per lane).
__device__ __forceinline__ g1p g1_mul_glv(const fp& px, const fp& py, const uint32_t (&k)[8]) {
  uint32_t k1[4], k2[4];
  glv_split(k, k1, k2);
  const g1p P2 = proj_dbl(g1p{px, py, fp_one()});
  const g1p P3 = proj_add_mixed(P2, px, py);
  const fp zi = inv(mul(P2.z, P3.z));
  const fp z2i = mul(zi, P3.z), z3i = mul(zi, P2.z);
  const fp x2 = mul(P2.x, z2i), y2 = mul(P2.y, z2i), x3 = mul(P3.x, z3i), y3 = mul(P3.y, z3i);
  const fp beta = fp_from(c::G1_BETA);
  const fp beta2 = mul(beta, beta);
  g1p acc = proj_identity<fp>();
#pragma unroll 1
  for (int w = 63; w >= 0; w--) {
    acc = proj_dbl(proj_dbl(acc));
    const int sh = 2 * (w & 15);
    const uint32_t d1 = (k1[w >> 4] >> sh) & 3u, d2 = (k2[w >> 4] >> sh) & 3u;
    {
      const fp tx = select(d1 == 1, px, select(d1 == 2, x2, x3)), ty = select(d1 == 1, py, select(d1 == 2, y2, y3));
      const g1p s = proj_add_mixed(acc, tx, ty);
      acc = {select(d1 != 0, s.x, acc.x), select(d1 != 0, s.y, acc.y), select(d1 != 0, s.z, acc.z)};
    }
    {
      const fp tx = mul(select(d2 == 1, px, select(d2 == 2, x2, x3)), beta2);
      const fp ty = select(d2 == 1, py, select(d2 == 2, y2, y3));
      const g1p s = proj_add_mixed(acc, tx, ty);
      acc = {select(d2 != 0, s.x, acc.x), select(d2 != 0, s.y, acc.y), select(d2 != 0, s.z, acc.z)};
    }
  }
  return acc;
}
}  // namespace

__global__ CESS_LB void k_keygen(uint64_t n, const uint8_t* __restrict__ sks, uint8_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_sk(sks + 32 * i, k);
  fp2 gx = {fp_from(c::G2_GEN_X0), fp_from(c::G2_GEN_X1)};
  fp2 gy = {fp_from(c::G2_GEN_Y0), fp_from(c::G2_GEN_Y1)};
  g2a p = proj_to_affine(proj_mul_scalar_mixed(gx, gy, k));
  uint8_t b[96];
  g2_compress(p, b);
  store_bytes(out + 96 * i, b, 96);
}

__global__ CESS_LB void k_sign(uint64_t n, const uint8_t* __restrict__ sks, const uint8_t* __restrict__ msgs,
                                               const uint64_t* __restrict__ offs, uint8_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_sk(sks + 32 * i, k);
  uint64_t o = offs[i];
  g1a h = hash_to_g1(msgs + o, (uint32_t)(offs[i + 1] - o));
  g1a s;
  if (h.inf) {
    s = h;
  } else {
    s = proj_to_affine(g1_mul_glv(h.x, h.y, k));
  }
  uint8_t b[48];
  g1_compress(s, b);
  store_bytes(out + 48 * i, b, 48);
}

__global__ CESS_LB void k_hash_out(uint64_t n, const uint8_t* __restrict__ msgs,
                                                   const uint64_t* __restrict__ offs, uint8_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t o = offs[i];
  g1a h = hash_to_g1(msgs + o, (uint32_t)(offs[i + 1] - o));
  uint8_t b[48];
  g1_compress(h, b);
  store_bytes(out + 48 * i, b, 48);
}
