// CDNA4 (gfx950) kernels for batch BLS12-381 verification — one lane = one signature.
// Stage outputs live in HBM in limb-major SoA layout (soa.hpp).
// k_hash: msg -> H(m) affine, RFC 9380 SSWU (reference src/lib.rs:25-31, A8/A9)
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

// CESS_HASH_PARK: the SSWU's waiting values parked in LDS (bls/h2c.hpp
// hash_to_g1_parked): 304 -> 24 B/lane scratch at equal time
// (profiles/round5_k_sweep.txt: 25.32 vs 25.27 ms per 1 M)
#ifndef CESS_HASH_PARK
#define CESS_HASH_PARK 1
#endif

__global__ CESS_LB void k_hash(uint64_t n, const uint8_t* __restrict__ msgs,
                                               const uint64_t* __restrict__ offs, const uint8_t* __restrict__ code,
                                               uint32_t* __restrict__ h_aff, uint64_t stride) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g1a h;
  h.x = fp_zero();
  h.y = fp_one();
  if (!code || code[i] == 0) {   // (no code array: the small-batch path hashes beside the decodes)
    uint64_t o = offs[i];
    uint32_t len = (uint32_t)(offs[i + 1] - o);
#if CESS_HASH_PARK
    __shared__ uint32_t park[48][256];   // 48 KiB per block
    h = hash_to_g1_parked(msgs + o, len, park, threadIdx.x);
#else
    h = hash_to_g1(msgs + o, len);
#endif
  }
  st_fp(h_aff, stride, i, h.x);
  st_fp(h_aff + 12 * stride, stride, i, h.y);
}
