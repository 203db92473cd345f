// CDNA4 (gfx950) kernels for batch BLS12-381 verification — one lane = one signature.
// Stage outputs live in HBM in limb-major SoA layout (soa.hpp).
// k_decode_sig: 48-B G1 encoding -> affine sig + code 1/2   (reference src/lib.rs:138-152, A3)
// k_decode_pk : 96-B G2 encoding -> affine pk  + code 3/4   (reference src/lib.rs:68-82, A5)
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

__global__ CESS_LB void k_decode_sig(uint64_t n, const uint8_t* __restrict__ sigs,
                                                     const uint8_t* __restrict__ pre, uint8_t* __restrict__ code,
                                                     uint8_t* __restrict__ inf, uint32_t* __restrict__ sig_aff,
                                                     uint64_t stride) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t pc = pre ? pre[i] : 0;
  uint8_t c = 0, f = 0;
  g1a p;
  p.inf = true;
  p.x = fp_zero();
  p.y = fp_one();
  if (pc & PRE_SIG_LEN_BAD) {
    c = CODE_SIG_LEN;
  } else {
    uint32_t w[12];
    const uint32_t* src = reinterpret_cast<const uint32_t*>(sigs + 48 * i);
#pragma unroll
    for (int k = 0; k < 12; k++) w[k] = bswap(src[k]);
    if (!g1_decompress(w, p)) c = CODE_SIG_POINT;
    else if (p.inf) f |= INF_SIG;
  }
  st_fp(sig_aff, stride, i, p.x);
  st_fp(sig_aff + 12 * stride, stride, i, p.y);
  code[i] = c;
  inf[i] = f;
}

__global__ CESS_LB void k_decode_pk(uint64_t n, const uint8_t* __restrict__ pks,
                                                    const uint8_t* __restrict__ pre, uint8_t* __restrict__ code,
                                                    uint8_t* __restrict__ inf, uint32_t* __restrict__ pk_aff,
                                                    uint64_t stride, uint32_t strict_identity) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t pc = pre ? pre[i] : 0;
  uint8_t c = code[i];
  uint8_t f = inf[i];
  g2a q;
  q.inf = true;
  q.x = {fp_from(c::G2_GEN_X0), fp_from(c::G2_GEN_X1)};
  q.y = {fp_from(c::G2_GEN_Y0), fp_from(c::G2_GEN_Y1)};
  if (c == 0) {
    if (pc & PRE_PK_LEN_BAD) {
      c = CODE_PK_LEN;
    } else {
      uint32_t w[24];
      const uint32_t* src = reinterpret_cast<const uint32_t*>(pks + 96 * i);
#pragma unroll
      for (int k = 0; k < 24; k++) w[k] = bswap(src[k]);
      g2a d;
      // on-curve decode only: the subgroup check runs in k_prepare, on the
      // [|x|]Q its G2Prepared iteration computes anyway
      if (!g2_decompress(w, d, RegPark2{}, false)) c = CODE_PK_POINT;
      else if (d.inf) {
        // the reference accepts the identity key (src/lib.rs:68-82); the
        // optional strict mode rejects it as KeyValidate does
        if (strict_identity) c = CODE_PK_POINT;
        else f |= INF_PK;
      } else {
        q = d;
      }
    }
  }
  // identity / rejected keys keep the generator so k_prepare stays well-defined
  st_fp2(pk_aff, stride, i, q.x);
  st_fp2(pk_aff + 24 * stride, stride, i, q.y);
  code[i] = c;
  inf[i] = f;
}

// keyed batch (cess_bls_verify_batch_keyed*): per-signature key verdicts taken
// from the distinct-key table in the reference's precedence -- a bad signature
// code stands, else the key's code, else the key's identity flag
// (src/lib.rs:244-245).  An index past the table (device-resident callers
// pass unchecked indices) names no key: the record is rejected as PK_POINT
// and k_miller, which skips records with a nonzero code, never reads its row.
__global__ CESS_LB void k_merge_pk(uint64_t n, const uint32_t* __restrict__ idx, uint32_t nkeys,
                                   const uint8_t* __restrict__ key_code, const uint8_t* __restrict__ key_inf,
                                   uint8_t* __restrict__ code, uint8_t* __restrict__ inf) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (code[i] != 0) return;
  const uint32_t j = idx[i];
  if (j >= nkeys) {
    code[i] = CODE_PK_POINT;
    return;
  }
  const uint8_t kc = key_code[j];
  if (kc != 0) code[i] = kc;
  else inf[i] |= key_inf[j] & INF_PK;
}
