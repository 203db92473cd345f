// CDNA4 (gfx950) kernels for batch BLS12-381 verification — one lane = one signature.
// Stage outputs live in HBM in limb-major SoA layout (soa.hpp).
// (k_prepare lives in k_prepare.hip: it is compiled with the default scheduler)
// k_miller         : (sig,-G2),(H,pk) -> Miller-loop value (multi_miller_loop, src/lib.rs:90-93, A12)
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

// The Miller accumulator is an LDS image (144 dwords x 256 lanes = 144 KiB of
// the CU's 160 KiB), so one block (one wave per SIMD) per CU.  The
// alternative placements measured in round 1 (accumulator in HBM, split
// LDS/HBM, HBM ping-pong with streamed operands: 314 / 244 / 203 vs 191 ms
// per 1 M) were removed from the product source.
#define CESS_LB_F12 __launch_bounds__(256, 1)
#ifndef CESS_MILLER_UNIFORM01
#define CESS_MILLER_UNIFORM01 0
#endif

#if defined(CESS_DIAG)
CESS_DIAG_TABLE(k_miller)
#endif

__global__ CESS_LB_F12 void k_miller(uint64_t n, const uint8_t* __restrict__ code,
                                     const uint8_t* __restrict__ inf, const uint32_t* __restrict__ sig_aff,
                                     const uint32_t* __restrict__ h_aff, const uint32_t* __restrict__ neg_g2,
                                     const uint4* __restrict__ coeffs, uint4* __restrict__ fout,
                                     uint4* __restrict__ pp, uint64_t stride,
                                     const uint32_t* __restrict__ cidx, uint64_t cstride,
                                     const uint8_t* __restrict__ cnorm) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (code[i] != 0) return;
  // coefficient row: the lane's own (per-signature prepare) or, for the keyed
  // batch, its key's row in the distinct-key table (cstride = table stride)
  const uint32_t cj = cidx ? cidx[i] : i;
  uint8_t fl = inf[i];
  __shared__ uint4 F[36][256];
  LdsF12 f{F, wave_first_thread()};
  // the G1 points are re-read from L2 for every line: held in 48 registers
  // across the loop they cost 27 spilled VGPRs (112 B/lane of scratch) and
  // +0.4 ms (profiles/round3_z_sweep.txt; round 2: 163 -> 171 ms)
  auto pt = [&](int pair) {
    const uint32_t* b = pair ? h_aff : sig_aff;
    return g1a{ld_fp(b, stride, i), ld_fp(b + 12 * stride, stride, i), false};
  };
  // per-signature rows are read once: non-temporal loads, so the stream does
  // not evict the G1 points the lines re-read from L2 (keyed tables, shared by
  // many lanes, stay cached): k_miller 157.3 -> 152.9 ms per 1 M, counted
  // traffic 27.8 -> 21.2 KB/sig (profiles/round3_al_sweep.txt)
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  auto ld_nt = [&](int k) {
    coeff3 r;
    uint32_t* w = &r.c0.c0.v[0];
#pragma unroll
    for (int q = 0; q < 18; q++) {
      const u4v x = __builtin_nontemporal_load((const u4v*)(coeffs + (uint64_t)(18 * k + q) * cstride + cj));
      w[4 * q] = x.x, w[4 * q + 1] = x.y, w[4 * q + 2] = x.z, w[4 * q + 3] = x.w;
    }
    return r;
  };
  auto src = [&](int pair, int k) {
#if CESS_MILLER_UNIFORM01
    // pair 0 takes mul014_one, which reads c0 and c1 only
    return pair ? (cidx ? ld_coeff4(coeffs, cstride, cj, k) : ld_nt(k)) : ld_coeff_uniform01(neg_g2, k);
#else
    return pair ? (cidx ? ld_coeff4(coeffs, cstride, cj, k) : ld_nt(k)) : ld_coeff_uniform(neg_g2, k);
#endif
  };
  // cnorm (keyed batches): the key's lines were normalised to c2 = 1
  // (k_norm_keys), so pair 1 takes the 9-product sparse multiply as pair 0.
  // (Per-signature rows are not normalised: k_norm_keys over every record
  // costs 22 ms per 1 M against 18 ms saved here, profiles/round3_k_sweep.txt.)
  const bool norm1 = cnorm && cnorm[cj];
#if defined(CESS_DIAG)
  // regions: 0/1 pair-1 loads / sparse product, 2/3 pair 0, 4 squaring,
  // 5 prologue + epilogue
  Diag dg;
  dg.begin();
  miller_loop2_staged(f, (fl & INF_SIG) == 0, (fl & INF_PK) == 0, pt, src, norm1, &dg);
  copy12(GlobF12{fout, stride, i}, f);
  dg.mark<5>();
  dg.end(cess_diag_tab);
#else
  miller_loop2_staged(f, (fl & INF_SIG) == 0, (fl & INF_PK) == 0, pt, src, norm1);
  copy12(GlobF12{fout, stride, i}, f);
#endif
}
