// CDNA4 (gfx950) kernel of the distinct-key RLC mode (host_rlc.cpp rlcd_*):
// k_miller_rr : kRlcdPer (4) records per lane,
//               g_k = prod_j Miller(Q_i, pk_i) over the lane's records i = 4k + j,
//               Q_i = r_i H(m_i) (multi_miller_loop over the lane's pairs,
//               src/lib.rs:90-93, A12)
// One accumulator squaring per step serves all the lane's records: per record
// a quarter of a squaring and one general sparse product, against a squaring
// and a sparse product with one record per lane (k_miller with pair 0 off).
// Same LDS image and scheduling as k_miller (k_pairing.hip), own translation
// unit so k_miller's code is unchanged.
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

#define CESS_LB_F12 __launch_bounds__(256, 1)

// np lanes over the m records of a chunk: lane k takes records RPL k .. RPL k +
// RPL - 1 (those below m).  A record takes part when its code is 0 and neither
// Q_i nor its key is the identity (inf[i] & INF_PK clear, from k_rlcd_records).
// h_aff (affine Q_i), coeffs (the key's line rows) and inf have stride
// `stride`; g_k goes to fout with stride fstride (the batch-wide lane values).
// A lane with no record taking part stores one.
template <int RPL>
__device__ __forceinline__ void miller_rr(uint64_t np, uint64_t m, const uint8_t* __restrict__ code,
                                          const uint8_t* __restrict__ inf, const uint32_t* __restrict__ h_aff,
                                          const uint4* __restrict__ coeffs, uint4* __restrict__ fout, uint64_t stride,
                                          uint64_t fstride, uint4 (*F)[256]) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= np) return;
  uint32_t use = 0;
#pragma unroll
  for (int j = 0; j < RPL; j++) {
    const uint64_t r = (uint64_t)RPL * k + j;
    if (r < m && code[r] == 0 && (inf[r] & INF_PK) == 0) use |= 1u << j;
  }
  const GlobF12 out{fout, fstride, k};
  if (!use) {
    set_one12(out);
    return;
  }
  LdsF12 f{F, wave_first_thread()};
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const uint32_t r0 = RPL * k;
  // the G1 point is re-read per line (L2), as k_miller's; each record's
  // coefficient rows are read once: non-temporal loads (k_miller)
  auto pt = [&](int j) {
    return g1a{ld_fp(h_aff, stride, r0 + j), ld_fp(h_aff + 12 * stride, stride, r0 + j), false};
  };
  auto src = [&](int j, int s) {
    coeff3 c;
    uint32_t* w = &c.c0.c0.v[0];
#pragma unroll
    for (int q = 0; q < 18; q++) {
      const u4v x = __builtin_nontemporal_load((const u4v*)(coeffs + (uint64_t)(18 * s + q) * stride + r0 + j));
      w[4 * q] = x.x, w[4 * q + 1] = x.y, w[4 * q + 2] = x.z, w[4 * q + 3] = x.w;
    }
    return c;
  };
  miller_loopn_staged<RPL>(f, use, pt, src);
  copy12(out, f);
}

__global__ CESS_LB_F12 void k_miller_rr(uint64_t np, uint64_t m, const uint8_t* __restrict__ code,
                                        const uint8_t* __restrict__ inf, const uint32_t* __restrict__ h_aff,
                                        const uint4* __restrict__ coeffs, uint4* __restrict__ fout, uint64_t stride,
                                        uint64_t fstride) {
  __shared__ uint4 F[36][256];
  miller_rr<CESS_RLCD_PER>(np, m, code, inf, h_aff, coeffs, fout, stride, fstride, F);
}
