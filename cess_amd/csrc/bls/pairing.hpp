// Optimal-ate pairing pieces for the two-pair verification
//   e(sig, -G2) * e(H(m), pk) == 1
// Replaces (bls12_381 0.7.1, called from utils/verify-bls-signatures/src/lib.rs:85-100):
//   G2Prepared::from(pk)                  :88   -> g2_prepare (68 line-coefficient triples)
//   G2PREPARED_NEG_G lazy_static          :19-21 -> same routine, run once per context
//   multi_miller_loop(&[(sig,-G2),(H,pk)]) :90-93 -> miller_loop2
//   .final_exponentiation().is_identity() :93-95 -> final_exponentiation + is_one
// Line coefficients follow Costello-Lange-Naehrig (eprint 2010/354) Alg. 26/27 in
// Jacobian coordinates; the line is applied as f * (c2 + (c1*P.x) v + (c0*P.y) v w).
#pragma once
#include "curve.hpp"

namespace bls {

struct coeff3 {
  fp2 c0, c1, c2;
};

// R <- 2R (Jacobian), returns the line coefficients
CESS_HD coeff3 doubling_step(g2p& r) {
  fp2 tmp0 = sqr(r.x);
  fp2 tmp1 = sqr(r.y);
  fp2 tmp2 = sqr(tmp1);
  fp2 tmp3 = sub(sub(sqr(add(tmp1, r.x)), tmp0), tmp2);
  tmp3 = dbl(tmp3);
  fp2 tmp4 = mul3(tmp0);
  fp2 tmp6 = add(r.x, tmp4);
  fp2 tmp5 = sqr(tmp4);
  fp2 zsq = sqr(r.z);
  fp2 nx = sub(sub(tmp5, tmp3), tmp3);
  fp2 nz = sub(sub(sqr(add(r.z, r.y)), tmp1), zsq);
  fp2 ny = sub(mul(sub(tmp3, nx), tmp4), mul8(tmp2));
  fp2 t3 = neg(dbl(mul(tmp4, zsq)));
  fp2 t6 = sub(sub(sub(sqr(tmp6), tmp0), tmp5), mul4(tmp1));
  fp2 t0 = dbl(mul(nz, zsq));
  r = {nx, ny, nz};
  return {t0, t3, t6};
}

// R <- R + Q (Jacobian R, affine Q), returns the line coefficients
CESS_HD coeff3 addition_step(g2p& r, const fp2& qx, const fp2& qy) {
  fp2 zsq = sqr(r.z);
  fp2 ysq = sqr(qy);
  fp2 t0 = mul(zsq, qx);
  fp2 t1 = mul(sub(sub(sqr(add(qy, r.z)), ysq), zsq), zsq);
  fp2 t2 = sub(t0, r.x);
  fp2 t3 = sqr(t2);
  fp2 t4 = mul4(t3);
  fp2 t5 = mul(t4, t2);
  fp2 t6 = sub(sub(t1, r.y), r.y);
  fp2 t9 = mul(t6, qx);
  fp2 t7 = mul(t4, r.x);
  fp2 nx = sub(sub(sub(sqr(t6), t5), t7), t7);
  fp2 nz = sub(sub(sqr(add(r.z, t2)), zsq), t3);
  fp2 t10 = add(qy, nz);
  fp2 t8 = mul(sub(t7, nx), t6);
  fp2 ny = sub(t8, dbl(mul(r.y, t5)));
  t10 = sub(sub(sqr(t10), ysq), sqr(nz));
  t9 = sub(dbl(t9), t10);
  fp2 c0 = dbl(nz);
  fp2 c1 = dbl(neg(t6));
  r = {nx, ny, nz};
  return {c0, c1, t9};
}

// bits of |x| >> 1 below its leading one (bit 62), from bit 61 down to 0
CESS_HD bool loop_bit(int b) { return b == 61 || b == 59 || b == 56 || b == 47 || b == 15; }
constexpr int N_COEFFS = 68;

// G2Prepared: sink(index, coeff3) receives the 68 triples in Miller-loop order.
template <class Sink>
CESS_HD void g2_prepare(const fp2& qx, const fp2& qy, Sink&& sink) {
  g2p r = {qx, qy, fp2_one()};
  int idx = 0;
  for (int b = 61; b >= 0; b--) {
    sink(idx++, doubling_step(r));
    if (loop_bit(b)) sink(idx++, addition_step(r, qx, qy));
  }
  sink(idx++, doubling_step(r));
}

CESS_HD fp12 ell(const fp12& f, const coeff3& k, const fp& px, const fp& py) {
  return mul_by_014(f, k.c2, mul_fp(k.c1, px), mul_fp(k.c0, py));
}

// Two-pair Miller loop sharing one accumulator.  srcA(idx)/srcB(idx) return the
// coefficient triples; a pair whose G1 or G2 point is the identity is skipped.
template <class SrcA, class SrcB>
CESS_HD fp12 miller_loop2(const g1a& pa, bool skip_a, SrcA&& srcA, const g1a& pb, bool skip_b, SrcB&& srcB) {
  bool ua = !(skip_a || pa.inf), ub = !(skip_b || pb.inf);
  fp12 f = fp12_one();
  int idx = 0;
  for (int b = 61; b >= 0; b--) {
    if (ua) f = ell(f, srcA(idx), pa.x, pa.y);
    if (ub) f = ell(f, srcB(idx), pb.x, pb.y);
    idx++;
    if (loop_bit(b)) {
      if (ua) f = ell(f, srcA(idx), pa.x, pa.y);
      if (ub) f = ell(f, srcB(idx), pb.x, pb.y);
      idx++;
    }
    f = sqr(f);
  }
  if (ua) f = ell(f, srcA(idx), pa.x, pa.y);
  if (ub) f = ell(f, srcB(idx), pb.x, pb.y);
  return conj(f);   // x < 0
}

// MillerLoopResult::final_exponentiation: easy part (p^6 - 1)(p^2 + 1), then the
// hard part from five cyclotomic exponentiations by x.  Result = e^3 (canonical).
CESS_HD fp12 final_exponentiation(const fp12& f) {
  fp12 t0 = conj(f);   // f^(p^6)
  fp12 t1 = inv(f);
  fp12 t2 = mul(t0, t1);
  t1 = t2;
  t2 = frobenius<2>(t2);
  t2 = mul(t2, t1);
  t1 = conj(cyclotomic_square(t2));
  fp12 t3 = cyclotomic_exp(t2);
  fp12 t4 = cyclotomic_square(t3);
  fp12 t5 = mul(t1, t3);
  t1 = cyclotomic_exp(t5);
  t0 = cyclotomic_exp(t1);
  fp12 t6 = cyclotomic_exp(t0);
  t6 = mul(t6, t4);
  t4 = cyclotomic_exp(t6);
  t5 = conj(t5);
  t4 = mul(t4, mul(t5, t2));
  t5 = conj(t2);
  t1 = mul(t1, t2);
  t1 = frobenius<3>(t1);
  t6 = mul(t6, t5);
  t6 = frobenius<1>(t6);
  t3 = mul(t3, t0);
  t3 = frobenius<2>(t3);
  t3 = mul(t3, t1);
  t3 = mul(t3, t6);
  return mul(t3, t4);
}

}  // namespace bls
