// CDNA4 (gfx950) kernels for batch BLS12-381 verification — one lane = one signature.
// Stage outputs live in HBM in limb-major SoA layout (soa.hpp).
// k_final: final exponentiation -> code 0/5 + verdict bitmap (src/lib.rs:93-99, A13/A14)
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

__global__ CESS_LB void k_final(uint64_t n, uint8_t* __restrict__ code,
                                                const uint32_t* __restrict__ fin, uint64_t* __restrict__ bitmap,
                                                uint8_t* __restrict__ gt_out, uint64_t stride) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t c = CODE_SIG_LEN;
  if (i < n) {
    c = code[i];
    if (c == 0) {
      fp12 f;
      fp* e = &f.c0.c0.c0;
#pragma unroll
      for (int j = 0; j < 12; j++) e[j] = ld_fp(fin + 12 * j * stride, stride, i);
      fp12 g = final_exponentiation(f);
      if (!is_one(g)) c = CODE_PAIRING;
      if (gt_out) {   // optional Gt bytes for parity tests (576 B per signature)
        const fp* ge = &g.c0.c0.c0;
        for (int j = 0; j < 12; j++) {
          uint8_t b[48];
          raw_to_be48(from_mont(ge[j]), b);
          for (int t = 0; t < 48; t++) gt_out[576 * i + 48 * j + t] = b[t];
        }
      }
      code[i] = c;
    }
  }
  // one bitmap word per wave: bit (i mod 64) of word i/64 = (code == 0)
  uint64_t ball = __ballot(c == 0);
  if ((threadIdx.x & 63) == 0 && i < n) bitmap[i >> 6] = ball;
}
