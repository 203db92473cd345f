// Lane-pair Fp12 arithmetic: TWO lanes per signature.
//
// Why (measured on MI355X, tools/mad_sdst.hip): one wave alone on a SIMD issues
// at most one v_mad_u64_u32 per ~9.6 cycles however many independent chains it
// has; two waves per SIMD reach ~5 cycles.  The one-lane-per-signature Fp12
// kernels need the 144 KiB LDS image of 256 accumulators plus ~350 registers
// per lane, which pins them to one wave per SIMD.  Splitting every Fp12
// operation over an (even, odd) lane pair halves the per-lane register working
// set (~220) and lets a 512-lane block keep 256 accumulators in the same
// 144 KiB image: two waves per SIMD.
//
// Each operation gives both lanes the same instruction stream on lane-dependent
// operands (v_cndmask selects), e.g. squaring f = a0 + a1 w: the even lane
// computes (a0 + a1)(a0 + v a1), the odd lane a0 a1, in one Fp6 multiply; the
// products are exchanged with DPP quad-permutes (v_mov_b32_dpp, no LDS traffic)
// and each lane writes its half of the result in place.  Fp6 multiplies stream
// their Fp2 operands from LDS per product so only products stay in registers.
//
// The single-lane versions in staged.hpp are the executable specification;
// tools/fe_probe.hip and the GPU parity tests check these against them.
#pragma once
#include "bls/staged.hpp"

#if !defined(CESS_HOSTEMU)
namespace bls {

// --- lane-pair exchange ------------------------------------------------------
// value of the partner lane (lane ^ 1): DPP quad_perm [1,0,3,2]
CESS_HD uint32_t xchg32(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false); }
CESS_HD fp xchg(const fp& a) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = xchg32(a.v[i]);
  return r;
}
CESS_HD fp2 xchg(const fp2& a) { return {xchg(a.c0), xchg(a.c1)}; }
CESS_HD fp6 xchg(const fp6& a) { return {xchg(a.c0), xchg(a.c1), xchg(a.c2)}; }

CESS_HD fp2 sel(bool hi, const fp2& lo_v, const fp2& hi_v) { return select(hi, hi_v, lo_v); }
CESS_HD fp6 sel(bool hi, const fp6& lo_v, const fp6& hi_v) {
  return {sel(hi, lo_v.c0, hi_v.c0), sel(hi, lo_v.c1, hi_v.c1), sel(hi, lo_v.c2, hi_v.c2)};
}

// One signature's Fp12 in an LDS image F[36][256]: signature s = lane pair s
// of a 512-lane block; both lanes read the same rows (LDS broadcast).
struct PairF12 {
  uint4 (*F)[256];
  uint32_t s;   // signature slot in the block (threadIdx.x >> 1)
  bool hi;      // odd lane of the pair
  CESS_HD fp2 ld(int k) const {
    fp2 r;
#pragma unroll
    for (int q = 0; q < 6; q++) {
      uint4 x = F[6 * k + q][s];
      fp& d = q < 3 ? r.c0 : r.c1;
      const int o = 4 * (q % 3);
      d.v[o] = x.x, d.v[o + 1] = x.y, d.v[o + 2] = x.z, d.v[o + 3] = x.w;
    }
    return r;
  }
  CESS_HD void st(int k, const fp2& a) const {
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const fp& v = q < 3 ? a.c0 : a.c1;
      const int o = 4 * (q % 3);
      F[6 * k + q][s] = make_uint4(v.v[o], v.v[o + 1], v.v[o + 2], v.v[o + 3]);
    }
  }
};

// --- Fp6 multiply with operands produced on demand --------------------------
// A(j), B(j): the j-th Fp2 component of each operand (callables; re-evaluated
// per product so operands are not held across the multiply).  Karatsuba.
template <class FA, class FB>
CESS_HD fp6 mul6_on_demand(FA&& A, FB&& B) {
  fp2 v0 = mul(A(0), B(0));
  CESS_MEMBAR();
  fp2 v1 = mul(A(1), B(1));
  CESS_MEMBAR();
  fp2 v2 = mul(A(2), B(2));
  CESS_MEMBAR();
  fp2 c0 = add(v0, mul_nr(sub(sub(mul(add(A(1), A(2)), add(B(1), B(2))), v1), v2)));
  CESS_MEMBAR();
  fp2 c1 = add(sub(sub(mul(add(A(0), A(1)), add(B(0), B(1))), v0), v1), mul_nr(v2));
  CESS_MEMBAR();
  fp2 c2 = add(sub(sub(mul(add(A(0), A(2)), add(B(0), B(2))), v0), v2), v1);
  return {c0, c1, c2};
}
// (v a)_j for a in Fp6: v (c0, c1, c2) = (xi c2, c0, c1)
template <class FA>
CESS_HD fp2 mul_v_at(FA&& a, int j) {
  return j == 0 ? mul_nr(a(2)) : a(j - 1);
}

// --- f <- f^2 (complex squaring; even lane X = (a0+a1)(a0+v a1), odd ab) ----
template <class S>
CESS_HD void sqr12p(const S& f) {
  const bool hi = f.hi;
  auto a0 = [&](int j) { return f.ld(j); };
  auto a1 = [&](int j) { return f.ld(3 + j); };
  fp6 R = mul6_on_demand([&](int j) { return hi ? a0(j) : add(a0(j), a1(j)); },
                         [&](int j) { return hi ? a1(j) : add(a0(j), mul_v_at(a1, j)); });
  fp6 P = xchg(R);   // even lane receives ab
  // even: c0 = X - ab - v ab ; odd: c1 = 2 ab
  fp6 out = sel(hi, sub(sub(R, P), mul_v(P)), dbl(R));
  st6(f, hi ? 1 : 0, out);
}

// --- f <- f * (c0 + c1 v + c4 v w)  (sparse line; Fp12::mul_by_014) ---------
// even lane: aa = a0 (c0 + c1 v); odd lane: t = (a0 + a1)(c0 + (c1 + c4) v);
// bb = a1 (c4 v) = (xi a1.c2 c4, a1.c0 c4, a1.c1 c4) split 2 + 1 products.
template <class S>
CESS_HD void mul014p(const S& f, const fp2& c0, const fp2& c1, const fp2& c4) {
  const bool hi = f.hi;
  const fp2 b1 = hi ? add(c1, c4) : c1;
  // mul_by_01(A; c0, b1) with A = even ? a0 : a0 + a1, operands on demand
  auto A = [&](int j) { return hi ? add(f.ld(j), f.ld(3 + j)) : f.ld(j); };
  fp2 t0 = mul(A(0), c0);
  CESS_MEMBAR();
  fp2 t1 = mul(A(1), b1);
  CESS_MEMBAR();
  fp2 r0 = add(mul_nr(mul(A(2), b1)), t0);
  CESS_MEMBAR();
  fp2 r1 = sub(sub(mul(add(A(0), A(1)), add(c0, b1)), t0), t1);
  CESS_MEMBAR();
  fp2 r2 = add(mul(A(2), c0), t1);
  CESS_MEMBAR();
  // bb pieces: even computes a1.c2 c4 (-> bb0 = xi .) and a1.c0 c4 (bb1);
  // odd computes a1.c1 c4 (bb2) and repeats it (balanced issue)
  fp2 q1 = mul(f.ld(hi ? 4 : 5), c4);
  CESS_MEMBAR();
  fp2 q2 = mul(f.ld(hi ? 4 : 3), c4);
  // exchange: even gets t (unused) and bb2; odd gets aa, bb0, bb1
  fp6 Rx = xchg(fp6{r0, r1, r2});
  fp2 q1x = xchg(q1), q2x = xchg(q2);
  fp6 aa = sel(hi, fp6{r0, r1, r2}, Rx);
  fp6 bb = sel(hi, fp6{mul_nr(q1), q2, q1x}, fp6{mul_nr(q1x), q2x, q1});
  // even: a0' = aa + v bb ; odd: a1' = t - aa - bb
  fp6 out = sel(hi, add(aa, mul_v(bb)), sub(sub(fp6{r0, r1, r2}, aa), bb));
  st6(f, hi ? 1 : 0, out);
}

// --- f <- f^2 in the cyclotomic subgroup (Granger-Scott) --------------------
// z0 = k0, z4 = k1, z3 = k2, z2 = k3, z1 = k4, z5 = k5 (store index k).
// Nine Fp2 squarings, five per lane (z3^2 in both):
//   even: z0^2, z1^2, (z0+z1)^2, z2^2, z3^2   odd: (z2+z3)^2, z4^2, z5^2, (z4+z5)^2, z3^2
// even writes z0', z1', z4'; odd writes z5', z2', z3'.
template <class S>
CESS_HD void cycsq12p(const S& f) {
  const bool hi = f.hi;
  fp2 s0 = sqr(hi ? add(f.ld(3), f.ld(2)) : f.ld(0));
  CESS_MEMBAR();
  fp2 s1 = sqr(f.ld(hi ? 1 : 4));
  CESS_MEMBAR();
  fp2 s2 = sqr(hi ? f.ld(5) : add(f.ld(0), f.ld(4)));
  CESS_MEMBAR();
  fp2 s3 = sqr(hi ? add(f.ld(1), f.ld(5)) : f.ld(3));
  CESS_MEMBAR();
  const fp2 z3s = sqr(f.ld(2));
  const fp2 x0 = xchg(s0), x1 = xchg(s1), x2 = xchg(s2), x3 = xchg(s3);
  const fp2 z0s = sel(hi, s0, x0), z1s = sel(hi, s1, x1), z01s = sel(hi, s2, x2), z2s = sel(hi, s3, x3);
  const fp2 z23s = sel(hi, x0, s0), z4s = sel(hi, x1, s1), z5s = sel(hi, x2, s2), z45s = sel(hi, x3, s3);
  // fp4 squares: (t0, t1) of (z0, z1); (T0, T1) of (z2, z3); (U0, U1) of (z4, z5)
  // out = 2(x -/+ z) + x
  auto upd = [](const fp2& x, const fp2& z, bool plus) {
    fp2 d = plus ? add(x, z) : sub(x, z);
    return add(dbl(d), x);
  };
  if (!hi) {
    const fp2 t0 = add(mul_nr(z1s), z0s), t1 = sub(sub(z01s, z0s), z1s), T0 = add(mul_nr(z3s), z2s);
    f.st(0, upd(t0, f.ld(0), false));   // z0'
    f.st(4, upd(t1, f.ld(4), true));    // z1'
    f.st(1, upd(T0, f.ld(1), false));   // z4'
  } else {
    const fp2 T1 = sub(sub(z23s, z2s), z3s), U0 = add(mul_nr(z5s), z4s);
    const fp2 nU1 = mul_nr(sub(sub(z45s, z4s), z5s));
    f.st(5, upd(T1, f.ld(5), true));    // z5'
    f.st(3, upd(nU1, f.ld(3), true));   // z2'
    f.st(2, upd(U0, f.ld(2), false));   // z3'
  }
}

}  // namespace bls
#endif
