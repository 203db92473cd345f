// CDNA4 (gfx950) kernels for batch BLS12-381 verification — one lane = one signature.
// k_prepare : pk -> 68 line-coefficient triples (G2Prepared::from, src/lib.rs:88, A11)
//             (also builds the G2PREPARED_NEG_G table once per context, src/lib.rs:19-21, A10)
// Own translation unit so that k_miller's ILP scheduling (Makefile) does not
// apply here: k_prepare measured 40.6 ms per 1 M with it vs 38.3 without.
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

// The key's subgroup check (G2Affine::from_compressed's torsion check, A5) is
// done here: the G2Prepared iteration computes T = [|x|]Q anyway, and
// psi(Q) == -T is the check k_decode_pk used to run as a second scalar
// multiplication.  code/inf (null for the -G2 table): a key whose record still
// has code 0 and is not the identity is rejected as PK_POINT here, after the
// signature's code (precedence of src/lib.rs:244-245 unchanged: k_decode_pk and
// this kernel only touch records whose code is still 0).
__global__ CESS_LB void k_prepare(uint64_t n, const uint32_t* __restrict__ pk_aff,
                                  uint4* __restrict__ coeffs, uint64_t stride, uint8_t* __restrict__ code,
                                  const uint8_t* __restrict__ inf) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // the key (2 Fp2 = 12 uint4 per lane) parked in LDS for the whole
  // iteration: read at the five addition steps and the subgroup check only
  // (48 KiB per block, two blocks per CU)
  __shared__ uint4 QP[12][256];
  {
    const uint32_t t0 = threadIdx.x;
    const fp2 qx = ld_fp2(pk_aff, stride, i), qy = ld_fp2(pk_aff + 24 * stride, stride, i);
#pragma unroll
    for (int w = 0; w < 6; w++) {
      const fp& a = w < 3 ? qx.c0 : qx.c1;
      QP[w][t0] = make_uint4(a.v[4 * (w % 3)], a.v[4 * (w % 3) + 1], a.v[4 * (w % 3) + 2], a.v[4 * (w % 3) + 3]);
      const fp& b = w < 3 ? qy.c0 : qy.c1;
      QP[6 + w][t0] = make_uint4(b.v[4 * (w % 3)], b.v[4 * (w % 3) + 1], b.v[4 * (w % 3) + 2], b.v[4 * (w % 3) + 3]);
    }
  }
  const uint32_t w0 = wave_first_thread();
  auto q = [&](fp2& x, fp2& y) {
    const uint32_t t = w0 + lane_fresh();
#pragma unroll
    for (int w = 0; w < 6; w++) {
      const uint4 a = QP[w][t], b = QP[6 + w][t];
      fp& da = w < 3 ? x.c0 : x.c1;
      fp& db = w < 3 ? y.c0 : y.c1;
      const int o = 4 * (w % 3);
      da.v[o] = a.x, da.v[o + 1] = a.y, da.v[o + 2] = a.z, da.v[o + 3] = a.w;
      db.v[o] = b.x, db.v[o + 1] = b.y, db.v[o + 2] = b.z, db.v[o + 3] = b.w;
    }
  };
  const g2p t = g2_prepare_emit(q, [&](int k, int j, const fp2& c) { st_coeff4_one(coeffs, stride, i, k, j, c); });
  if (code && code[i] == 0 && !(inf[i] & INF_PK)) {
    CESS_MEMBAR();
    fp2 qx, qy;
    q(qx, qy);
    if (!g2_psi_is_neg_proj(qx, qy, t.x, t.y, t.z)) code[i] = CODE_PK_POINT;
  }
}

// The constant -G2 table (one lane per line, stride 1): scale every line to
// c2 = 1 (pairing.hpp normalize_line), once per context after k_prepare built it.
__global__ __launch_bounds__(128) void k_norm_lines(uint4* __restrict__ tab) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N_COEFFS) return;
  coeff3 c = ld_coeff4(tab, 1, 0, k);
  normalize_line(c);
  st_coeff4(tab, 1, 0, k, c);
}

// Normalise every line of each key of a distinct-key table to c2 = 1
// (pairing.hpp normalize_lines: one Fp2 inversion per key), once per
// cess_bls_keys_load, so the keyed Miller loop multiplies pair 1 by
// normalised lines as well (9 Fp2 products per line instead of 13).  tab:
// k_prepare's uint4-row table (n rows of stride K); pre: 68 Fp2 of scratch
// per key (word-SoA, stride K); norm[i] = 1 if key i was normalised, 0 if a
// zero c2 kept its lines as they were.
__global__ CESS_LB void k_norm_keys(uint64_t n, uint64_t K, uint4* __restrict__ tab, uint32_t* __restrict__ pre,
                                    uint8_t* __restrict__ norm) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool ok = normalize_lines([&](int k) { return ld_coeff4(tab, K, i, k); },
                                  [&](int k, const coeff3& c) { st_coeff4(tab, K, i, k, c); },
                                  [&](int k) { return ld_fp2(pre + (uint64_t)(24 * k) * K, K, i); },
                                  [&](int k, const fp2& v) { st_fp2(pre + (uint64_t)(24 * k) * K, K, i, v); });
  norm[i] = ok ? 1 : 0;
}
