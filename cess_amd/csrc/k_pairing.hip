// CDNA4 (gfx950) kernels for batch BLS12-381 verification — one lane = one signature.
// Stage outputs live in HBM in limb-major SoA layout (soa.hpp).
// (k_prepare lives in k_prepare.hip: it is compiled with the default scheduler)
// k_miller         : (sig,-G2),(H,pk) -> Miller-loop value (multi_miller_loop, src/lib.rs:90-93, A12)
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

// Miller accumulator placement (CESS_MILLER_MODE):
//   0: an LDS image (144 dwords x 256 lanes = 144 KiB, one wave per SIMD);
//   1: the lane's HBM output slot (L2/MALL-resident), two waves per SIMD;
//   2: split -- the c0 half (72 dwords) in LDS, the c1 half in the HBM output
//      slot: 72 KiB per block, two blocks (two waves per SIMD) per CU;
//   3: ping-pong -- the accumulator alternates between the HBM output slot and
//      a second HBM slot (`pp`), every Fp12 step streams its operands
//      (bls/staged.hpp mul014_stream / sqr12_stream) with one Fp6 temporary in
//      LDS (72 KiB per block): two waves per SIMD.
#ifndef CESS_MILLER_MODE
#define CESS_MILLER_MODE 0
#endif
#if CESS_MILLER_MODE
#define CESS_LB_F12 __launch_bounds__(256, 2)
#else
#define CESS_LB_F12 __launch_bounds__(256, 1)
#endif

// Fp12 store with the c0 half (store indices 0-2) in LDS and the c1 half (3-5)
// in HBM.  Indices are compile-time in the unrolled operations; the rolled
// copy loops branch wave-uniformly.
struct SplitF12 {
  LdsF12 lo;
  GlobF12 hi;
  CESS_HD fp2 ld(int k) const { return k < 3 ? lo.ld(k) : hi.ld(k); }
  CESS_HD void st(int k, const fp2& a) const {
    if (k < 3)
      lo.st(k, a);
    else
      hi.st(k, a);
  }
};

__global__ CESS_LB_F12 void k_miller(uint64_t n, const uint8_t* __restrict__ code,
                                     const uint8_t* __restrict__ inf, const uint32_t* __restrict__ sig_aff,
                                     const uint32_t* __restrict__ h_aff, const uint32_t* __restrict__ neg_g2,
                                     const uint4* __restrict__ coeffs, uint4* __restrict__ fout,
                                     uint4* __restrict__ pp, uint64_t stride,
                                     const uint32_t* __restrict__ cidx, uint64_t cstride) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (code[i] != 0) return;
  // coefficient row: the lane's own (per-signature prepare) or, for the keyed
  // batch, its key's row in the distinct-key table (cstride = table stride)
  const uint32_t cj = cidx ? cidx[i] : i;
  uint8_t fl = inf[i];
#if CESS_MILLER_MODE == 3
#elif CESS_MILLER_MODE == 1
  GlobF12 f{fout, stride, i};
#elif CESS_MILLER_MODE == 2
  __shared__ uint4 F[18][256];
  SplitF12 f{LdsF12{F, threadIdx.x}, GlobF12{fout, stride, i}};
#else
  __shared__ uint4 F[36][256];
  LdsF12 f{F, threadIdx.x};
#endif
  // the G1 points are re-read from HBM (L2) for every line instead of being
  // held in 48 registers across the loop
  auto pt = [&](int pair) {
    const uint32_t* b = pair ? h_aff : sig_aff;
    return g1a{ld_fp(b, stride, i), ld_fp(b + 12 * stride, stride, i), false};
  };
  auto src = [&](int pair, int k) { return pair ? ld_coeff4(coeffs, cstride, cj, k) : ld_coeff_uniform(neg_g2, k); };
#if CESS_MILLER_MODE == 3
  __shared__ uint4 T[18][256];
  const GlobF12 fa{fout, stride, i}, fb{pp, stride, i};
  if (miller_loop2_pp(fa, fb, LdsF12{T, threadIdx.x}, (fl & INF_SIG) == 0, (fl & INF_PK) == 0, pt, src))
    copy12(fa, fb);
#else
  miller_loop2_staged(f, (fl & INF_SIG) == 0, (fl & INF_PK) == 0, pt, src);
#if CESS_MILLER_MODE == 2
#pragma unroll 1
  for (int k = 0; k < 3; k++) f.hi.st(k, f.lo.ld(k));
#elif CESS_MILLER_MODE == 0
  copy12(GlobF12{fout, stride, i}, f);
#endif
#endif
}
