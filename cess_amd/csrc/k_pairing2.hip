// k_miller2: the two-pair Miller loop (multi_miller_loop, src/lib.rs:90-93,
// SURVEY §8(a) A12) on a lane PAIR per signature (bls/pair.hpp): 256-thread
// blocks of 128 signatures with the accumulator image G[18][256] (72 KiB, the
// same bytes per signature as k_miller's F[36][256]), two blocks per CU, so
// two waves per SIMD.  (One 512-thread block per CU measured the same waves
// alive only ~80 % of the block's time: the older wave of a SIMD issues first
// and finishes first, and the younger then runs alone until the block ends;
// with two independent blocks a finished block is replaced at once.)
// Same arguments and output (fval rows) as k_miller (k_pairing.hip), so
// k_final and the keyed path consume it unchanged.
#include <hip/hip_runtime.h>
#include "soa.hpp"
#include "bls/pair.hpp"

using namespace bls;
using namespace cess;

__global__ __launch_bounds__(CESS_PAIR_THREADS, 2) void k_miller2(uint64_t n, const uint8_t* __restrict__ code,
                                                    const uint8_t* __restrict__ inf,
                                                    const uint32_t* __restrict__ sig_aff,
                                                    const uint32_t* __restrict__ h_aff,
                                                    const uint32_t* __restrict__ neg_g2,
                                                    const uint4* __restrict__ coeffs, uint4* __restrict__ fout,
                                                    uint4* __restrict__ pp, uint64_t stride,
                                                    const uint32_t* __restrict__ cidx, uint64_t cstride,
                                                    const uint8_t* __restrict__ cnorm) {
  // signature of the pair; both lanes of a pair take every branch together
  const uint32_t i = blockIdx.x * (blockDim.x >> 1) + (threadIdx.x >> 1);
  if (i >= n) return;
  if (code[i] != 0) return;
  const uint32_t h = threadIdx.x & 1u;
  const uint32_t cj = cidx ? cidx[i] : i;
  const uint8_t fl = inf[i];
  __shared__ uint4 G[18][CESS_PAIR_THREADS];
  LdsPair f{G, wave_first_thread()};
  // (the lambdas capture by value: with [&] captures the compiler kept the
  // captured pointers in a private frame and selected the pair's point through
  // it -- a dozen scratch accesses per line at 256 registers. The per-lane
  // offsets pass through an empty asm so each address is re-formed at its load
  // -- one 64-bit add -- instead of a dozen strength-reduced 64-bit pointers
  // held live, and spilled, across the step.)
  auto pt = [=](int pair) {
    const uint32_t* b = pair ? h_aff : sig_aff;
    uint32_t io = i;
    asm volatile("" : "+v"(io));
    return g1a{ld_fp(b, stride, io), ld_fp(b + 12 * stride, stride, io), false};
  };
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const uint64_t vo_c = 3 * h * cstride + cj, vo_t = 3 * h;
  // this lane's component of line coefficient j: rows 18k + 6j + 3h .. + 2
  // (vo = 3h st + column, this lane's offset)
  auto ld_row = [=](const uint4* base, uint64_t st, uint64_t vo, int k, int j, bool nt) {
    fph r;
    asm volatile("" : "+v"(vo));
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const uint4* a = base + (uint64_t)(18 * k + 6 * j + q) * st + vo;
      u4v x;
      if (nt)
        x = __builtin_nontemporal_load((const u4v*)a);
      else
        x = *(const u4v*)a;
      r.v.v[4 * q] = x.x, r.v.v[4 * q + 1] = x.y, r.v.v[4 * q + 2] = x.z, r.v.v[4 * q + 3] = x.w;
    }
    return r;
  };
  const uint4* g2tab = (const uint4*)neg_g2;   // 72 dwords = 18 uint4 per line, stride 1
  // (the -G2 table is normalised to c2 = 1: pair 0 reads c0 and c1 only)
  auto src = [=](int pair, int k, int j) {
    return pair ? ld_row(coeffs, cstride, vo_c, k, j, cidx == nullptr) : ld_row(g2tab, 1, vo_t, k, j, false);
  };
  const bool norm1 = cnorm && cnorm[cj];
  miller_loop2_pair(f, (fl & INF_SIG) == 0, (fl & INF_PK) == 0, pt, src, norm1);
  // this lane's rows of the GlobF12 output: 6k + 3h + q
#pragma unroll 1
  for (int k = 0; k < 6; k++) {
    const fph v = f.ld(k);
#pragma unroll
    for (int q = 0; q < 3; q++)
      fout[(uint64_t)(6 * k + 3 * h + q) * stride + i] =
          make_uint4(v.v.v[4 * q], v.v.v[4 * q + 1], v.v.v[4 * q + 2], v.v.v[4 * q + 3]);
  }
}

// k_miller_rr2: the distinct-key RLC's lane of CESS_RLCD_PER records
// (k_pairing_rr.hip k_miller_rr: g_k = prod_j Miller(Q_i, pk_i) over records
// i = 4k + j, src/lib.rs:90-93) on a lane pair per lane of records, as
// k_miller2: blocks of CESS_PAIR_THREADS / 2 record lanes, the accumulator in
// LDS, two waves per SIMD.  Same arguments and output rows as k_miller_rr.
__global__ __launch_bounds__(CESS_PAIR_THREADS, 2) void k_miller_rr2(uint64_t np, uint64_t m,
                                                                     const uint8_t* __restrict__ code,
                                                                     const uint8_t* __restrict__ inf,
                                                                     const uint32_t* __restrict__ h_aff,
                                                                     const uint4* __restrict__ coeffs,
                                                                     uint4* __restrict__ fout, uint64_t stride,
                                                                     uint64_t fstride) {
  constexpr int RPL = CESS_RLCD_PER;
  // the lane of records k of the pair; both lanes take every branch together
  const uint32_t k = blockIdx.x * (blockDim.x >> 1) + (threadIdx.x >> 1);
  if (k >= np) return;
  const uint32_t h = threadIdx.x & 1u;
  uint32_t use = 0;
#pragma unroll
  for (int j = 0; j < RPL; j++) {
    const uint64_t r = (uint64_t)RPL * k + j;
    if (r < m && code[r] == 0 && (inf[r] & INF_PK) == 0) use |= 1u << j;
  }
  auto out_row = [&](int kk, int q) { return fout + (uint64_t)(6 * kk + 3 * h + q) * fstride + k; };
  if (!use) {   // one
#pragma unroll 1
    for (int kk = 0; kk < 6; kk++) {
      const fph v = kk ? fph_zero() : fph_one();
#pragma unroll
      for (int q = 0; q < 3; q++)
        *out_row(kk, q) = make_uint4(v.v.v[4 * q], v.v.v[4 * q + 1], v.v.v[4 * q + 2], v.v.v[4 * q + 3]);
    }
    return;
  }
  __shared__ uint4 G[18][CESS_PAIR_THREADS];
  LdsPair f{G, wave_first_thread()};
  const uint32_t r0 = RPL * k;
  // (offsets through an empty asm, as in k_miller2: addresses re-formed at
  // each load rather than strength-reduced pointers spilled across the lane)
  auto pt = [=](int j) {
    uint32_t io = r0 + j;
    asm volatile("" : "+v"(io));
    return g1a{ld_fp(h_aff, stride, io), ld_fp(h_aff + 12 * stride, stride, io), false};
  };
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  auto src = [=](int j, int s, int cc) {
    fph c;
    uint64_t vo = 3 * h * stride + r0 + j;
    asm volatile("" : "+v"(vo));
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const u4v x = __builtin_nontemporal_load((const u4v*)(coeffs + (uint64_t)(18 * s + 6 * cc + q) * stride + vo));
      c.v.v[4 * q] = x.x, c.v.v[4 * q + 1] = x.y, c.v.v[4 * q + 2] = x.z, c.v.v[4 * q + 3] = x.w;
    }
    return c;
  };
  miller_loopn_pair<RPL>(f, use, pt, src);
#pragma unroll 1
  for (int kk = 0; kk < 6; kk++) {
    const fph v = f.ld(kk);
#pragma unroll
    for (int q = 0; q < 3; q++)
      *out_row(kk, q) = make_uint4(v.v.v[4 * q], v.v.v[4 * q + 1], v.v.v[4 * q + 2], v.v.v[4 * q + 3]);
  }
}
