// Optimal-ate pairing pieces for the two-pair verification
//   e(sig, -G2) * e(H(m), pk) == 1
// Replaces (bls12_381 0.7.1, called from utils/verify-bls-signatures/src/lib.rs:85-100):
//   G2Prepared::from(pk)                  :88   -> g2_prepare (68 line-coefficient triples)
//   G2PREPARED_NEG_G lazy_static          :19-21 -> same routine, run once per context
//   multi_miller_loop(&[(sig,-G2),(H,pk)]) :90-93 -> miller_loop2
//   .final_exponentiation().is_identity() :93-95 -> final_exponentiation + is_one
// Line coefficients: homogeneous projective doubling/addition (below); the line
// is applied as f * (c2 + (c1*P.x) v + (c0*P.y) v w).
#pragma once
#include "curve.hpp"

namespace bls {

struct coeff3 {
  fp2 c0, c1, c2;
};

// Line coefficients are (c0, c1, c2) = (y_P coefficient, x_P coefficient,
// constant) of the line through the step's points, applied as
// f * (c2 + (c1 x_P) v + (c0 y_P) v w).  Any Fp2 multiple of a line gives the
// same Gt (an Fp2 factor dies in the final exponentiation: (p^2 - 1) divides
// (p^12 - 1)/r), so the steps use homogeneous projective coordinates
// (x = X/Z, y = Y/Z) and the cheaper formulas of Costello-Lange-Naehrig /
// Aranha et al. (eprint 2010/526) for E': y^2 = x^3 + b', b' = 4(1 + u),
// instead of the crate's Jacobian ones; golden Gt bytes pin the result.

// R <- 2R: (X3, Y3, Z3) = 4 (A (B - F), G^2 - 3 E^2, B H) with A = XY/2,
// B = Y^2, C = Z^2, E = 3 b' C, F = 3E, G = (B + F)/2, H = 2YZ; tangent line
// Z^2 (2 y y_P - 3 x^2 x_P + 3 x^3 - 2 y^2) = H y_P - 3 X^2 x_P + (B - E)
// (X^3 / Z = Y^2 - b' Z^2 on the curve).  6 squarings + 3 products.
CESS_HD coeff3 doubling_step(g2p& r) {
  const fp2 B = sqr(r.y), C = sqr(r.z);
  const fp2 E = mul3(mul4(mul_nr(C)));              // 3 b' Z^2 = 12 (1 + u) Z^2
  const fp2 F = mul3(E);
  const fp2 H = sub(sub(sqr(add(r.y, r.z)), B), C);   // 2 Y Z
  const fp2 J = sqr(r.x);
  const fp2 A2 = mul(r.x, r.y);                       // 2A
  const fp2 nx = dbl(mul(A2, sub(B, F)));
  const fp2 ny = sub(sqr(add(B, F)), mul4(mul3(sqr(E))));
  const fp2 nz = mul4(mul(B, H));
  r = {nx, ny, nz};
  return {H, neg(mul3(J)), sub(B, E)};
}

// R <- R + Q (projective R, affine Q): theta = Y - y_Q Z, lambda = X - x_Q Z,
// X3 = lambda H, Y3 = theta (G - H) - Y lambda^3, Z3 = Z lambda^3 with
// G = X lambda^2, H = lambda^3 + Z theta^2 - 2G; chord line
// lambda y_P - theta x_P + (theta x_Q - lambda y_Q).
CESS_HD coeff3 addition_step(g2p& r, const fp2& qx, const fp2& qy) {
  const fp2 th = sub(r.y, mul(qy, r.z));
  const fp2 la = sub(r.x, mul(qx, r.z));
  const fp2 D = sqr(la);
  const fp2 E3 = mul(la, D);
  const fp2 G = mul(r.x, D);
  const fp2 H = sub(add(E3, mul(r.z, sqr(th))), dbl(G));
  const fp2 nx = mul(la, H);
  const fp2 ny = sub(mul(th, sub(G, H)), mul(r.y, E3));
  const fp2 nz = mul(r.z, E3);
  r = {nx, ny, nz};
  return {la, neg(th), sub(mul(th, qx), mul(la, qy))};
}

// bits of |x| >> 1 below its leading one (bit 62), from bit 61 down to 0
CESS_HD bool loop_bit(int b) { return b == 61 || b == 59 || b == 56 || b == 47 || b == 15; }
constexpr int N_COEFFS = 68;

// G2Prepared: sink(index, coeff3) receives the 68 triples in Miller-loop order.
// The iteration is the double-and-add of [|x|]Q (63 doublings, additions at
// |x|'s set bits 62, 60, 57, 48, 16), so on return `t` (optional) holds
// T = [|x|]Q in homogeneous projective coordinates.
template <class Sink>
CESS_HD void g2_prepare(const fp2& qx, const fp2& qy, Sink&& sink, g2p* t = nullptr) {
  g2p r = {qx, qy, fp2_one()};
  int idx = 0;
#pragma unroll 1
  for (int b = 61; b >= 0; b--) {
    sink(idx++, doubling_step(r));
    if (loop_bit(b)) sink(idx++, addition_step(r, qx, qy));
  }
  sink(idx++, doubling_step(r));
  if (t) *t = r;
}

// The same iteration with every coefficient handed to emit(k, j, c_j) as soon
// as it is computed and the key read through q(x, y) where it is needed (a
// store, e.g. LDS), so fewer Fp2 values are live at the doubling step's peak:
// k_prepare (two waves per SIMD, 256 VGPRs) spilled 195 VGPRs (940 B/lane of
// scratch) with the value-returning steps above and the key in registers.
// Every multiply is sequenced (field.hpp seq), so the program order below is
// the order the values are produced and die in.
#ifndef CESS_DBL_SQR_XY
#define CESS_DBL_SQR_XY 1
#endif
template <class Emit>
CESS_HD void doubling_step_emit(g2p& r, int k, Emit&& emit) {
#if CESS_DBL_SQR_XY
  // 2XY = 4A as (X + Y)^2 - X^2 - Y^2: a squaring for a product (2M + 7S);
  // X3 = 2 (2A)(B - F) = (4A)(B - F) below takes it without the doubling
  const fp2 J = sqr(r.x);
  emit(k, 1, neg(mul3(J)));                             // -3 X^2
  const fp2 B = sqr(r.y);
  const fp2 A4 = sub(sub(sqr(add(r.x, r.y)), J), B);    // 4A; X dead
  const fp2 C = sqr(r.z);
#else
  emit(k, 1, neg(mul3(sqr(r.x))));                      // -3 X^2
  const fp2 A2 = mul(r.x, r.y);                         // 2A; X dead
  const fp2 B = sqr(r.y), C = sqr(r.z);
#endif
  const fp2 H = sub(sub(sqr(add(r.y, r.z)), B), C);     // 2YZ; Y, Z dead
  emit(k, 0, H);
  const fp2 E = mul3(mul4(mul_nr(C)));                  // 3 b' Z^2; C dead
  emit(k, 2, sub(B, E));
  const fp2 F = mul3(E);
#if CESS_DBL_SQR_XY
  const fp2 nx = mul(A4, sub(B, F));
#else
  const fp2 nx = dbl(mul(A2, sub(B, F)));
#endif
  const fp2 ny = sub(sqr(add(B, F)), mul4(mul3(sqr(E))));
  r = {nx, ny, mul4(mul(B, H))};
}
template <class QL, class Emit>
CESS_HD void addition_step_emit(g2p& r, QL&& q, int k, Emit&& emit) {
  fp2 qx, qy;
  q(qx, qy);
  const fp2 th = sub(r.y, mul(qy, r.z));
  const fp2 la = sub(r.x, mul(qx, r.z));
  emit(k, 0, la);
  emit(k, 1, neg(th));
  emit(k, 2, sub(mul(th, qx), mul(la, qy)));
  const fp2 D = sqr(la);
  const fp2 E3 = mul(la, D);
  const fp2 G = mul(r.x, D);
  const fp2 H = sub(add(E3, mul(r.z, sqr(th))), dbl(G));
  r = {mul(la, H), sub(mul(th, sub(G, H)), mul(r.y, E3)), mul(r.z, E3)};
}
// g2_prepare with emit(k, j, c_j) per coefficient and the key behind q(x, y);
// returns T = [|x|]Q (by value: an out-pointer to a local puts it in scratch)
template <class QL, class Emit>
CESS_HD g2p g2_prepare_emit(QL&& q, Emit&& emit) {
  g2p r;
  q(r.x, r.y);
  r.z = fp2_one();
  int idx = 0;
#pragma unroll 1
  for (int b = 61; b >= 0; b--) {
    doubling_step_emit(r, idx++, emit);
    CESS_MEMBAR();
    if (loop_bit(b)) addition_step_emit(r, q, idx++, emit);
    CESS_MEMBAR();
  }
  doubling_step_emit(r, idx++, emit);
  return r;
}

// Scale a line by 1/c2: (c0, c1, c2) -> (c0/c2, c1/c2, 1).  Every Fp2 factor of
// the Miller-loop value dies in the final exponentiation ((p^2 - 1) divides
// (p^12 - 1)/r), so the Gt value is unchanged, and the sparse product with a
// line whose c2 is one costs 9 Fp2 products instead of 13 (staged.hpp
// mul014_one).  Used for the constant -G2 table (G2PREPARED_NEG_G, A10), built
// once per context.
CESS_HD void normalize_line(coeff3& k) {
  const fp2 ic2 = inv(k.c2);
  k.c0 = mul(k.c0, ic2);
  k.c1 = mul(k.c1, ic2);
  k.c2 = fp2_one();
}

// normalize_line for a whole G2Prepared table (the keys of a distinct-key
// table, built once and used by many signatures) with ONE Fp2 inversion:
// Montgomery's simultaneous inversion, prefix products of the c2 kept in a
// scratch Fp2 per line.  ld(k) / st(k, c) access line k, pre(k) / set_pre(k, v)
// its scratch.  A table with a zero c2 (never for a key of G2 in practice, but
// a crafted key could force one) is left unchanged and false returned; the
// Miller loop then uses the general sparse product for it.
template <class Ld, class St, class PreLd, class PreSt>
CESS_HD bool normalize_lines(Ld&& ld, St&& st, PreLd&& pre, PreSt&& set_pre) {
  fp2 prod = fp2_one();
#pragma unroll 1
  for (int k = 0; k < N_COEFFS; k++) {
    set_pre(k, prod);
    prod = mul(prod, ld(k).c2);
  }
  if (is_zero(prod)) return false;
  fp2 iv = inv(prod);
#pragma unroll 1
  for (int k = N_COEFFS - 1; k >= 0; k--) {
    coeff3 c = ld(k);
    const fp2 ic2 = mul(iv, pre(k));   // 1 / c2_k
    iv = mul(iv, c.c2);
    c.c0 = mul(c.c0, ic2);
    c.c1 = mul(c.c1, ic2);
    c.c2 = fp2_one();
    st(k, c);
  }
  return true;
}

CESS_HD fp12 ell(const fp12& f, const coeff3& k, const fp& px, const fp& py) {
  return mul_by_014(f, k.c2, mul_fp(k.c1, px), mul_fp(k.c0, py));
}

// Coefficient step s (0..67) is followed by f <- f^2 unless it is a doubling
// step whose addition step follows, or the last step.
CESS_HD bool square_after_step(int s) {
  // step order: for b = 61..0: D(b) [A(b) if loop_bit(b)]; final D
  int idx = 0;
#pragma unroll 1
  for (int b = 61; b >= 0; b--) {
    int last = idx + (loop_bit(b) ? 1 : 0);
    if (s >= idx && s <= last) return s == last;
    idx = last + 1;
  }
  return false;
}

// Two-pair Miller loop sharing one accumulator.  src(pair, idx) returns the
// coefficient triple of pair 0 (sig, -G2) or 1 (H(m), pk); a pair whose G1 or
// G2 point is the identity is skipped.  The body holds a single copy of the
// sparse line multiplication and of the Fp12 squaring (code size on CDNA4).
template <class Src>
CESS_HD fp12 miller_loop2(const g1a& pa, bool skip_a, const g1a& pb, bool skip_b, Src&& src) {
  bool use[2] = {!(skip_a || pa.inf), !(skip_b || pb.inf)};
  fp12 f = fp12_one();
#pragma unroll 1
  for (int s = 0; s < N_COEFFS; s++) {
#pragma unroll 1
    for (int pair = 0; pair < 2; pair++) {
      if (!use[pair]) continue;
      const fp& px = pair ? pb.x : pa.x;
      const fp& py = pair ? pb.y : pa.y;
      f = ell(f, src(pair, s), px, py);
    }
    if (square_after_step(s)) f = sqr(f);
  }
  return conj(f);   // x < 0
}

// ---------------------------------------------------------------------------
// Value-based final exponentiation: HOST EMULATION ONLY (tests/hostemu: the
// CPU baseline and an independent cross-check of the staged program the
// k_final kernel runs, bls/staged.hpp).  Not compiled for the device, so no
// out-of-line (__noinline__) device function exists in the product library.
// ---------------------------------------------------------------------------
#if defined(CESS_HOSTEMU)
CESS_NOINLINE void fe_mul(fp12* r, const fp12* a, const fp12* b) { *r = mul(*a, *b); }
CESS_NOINLINE void fe_cycsq(fp12* r, const fp12* a) { *r = cyclotomic_square(*a); }
CESS_NOINLINE void fe_frob(fp12* r, const fp12* a, int k) {
  fp12 x = *a;
  fp2* v[6] = {&x.c0.c0, &x.c1.c0, &x.c0.c1, &x.c1.c1, &x.c0.c2, &x.c1.c2};
#pragma unroll
  for (int i = 0; i < 6; i++) {
    fp2 y = (k & 1) ? conj(*v[i]) : *v[i];
    if (i) y = mul(y, frob_coeff(k, i));
    *v[i] = y;
  }
  *r = x;
}
// r = a^x (x = -|x|) in the cyclotomic subgroup
CESS_NOINLINE void fe_cycexp(fp12* r, const fp12* a) {
  fp12 t = *a;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    t = cyclotomic_square(t);
    if (b == 62 || b == 60 || b == 57 || b == 48 || b == 16) fe_mul(&t, &t, a);
  }
  *r = conj(t);
}
CESS_NOINLINE void fe_inv(fp12* r, const fp12* a) { *r = inv(*a); }

// MillerLoopResult::final_exponentiation: easy part (p^6 - 1)(p^2 + 1), then the
// hard part from five cyclotomic exponentiations by x.  Result = e^3 (canonical).
CESS_HD fp12 final_exponentiation(const fp12& f) {
  fp12 t0, t1, t2, t3, t4, t5, t6, fin = f;
  t0 = conj(fin);   // f^(p^6)
  fe_inv(&t1, &fin);
  fe_mul(&t2, &t0, &t1);
  t1 = t2;
  fe_frob(&t2, &t2, 2);
  fe_mul(&t2, &t2, &t1);
  fe_cycsq(&t1, &t2);
  t1 = conj(t1);
  fe_cycexp(&t3, &t2);
  fe_cycsq(&t4, &t3);
  fe_mul(&t5, &t1, &t3);
  fe_cycexp(&t1, &t5);
  fe_cycexp(&t0, &t1);
  fe_cycexp(&t6, &t0);
  fe_mul(&t6, &t6, &t4);
  fe_cycexp(&t4, &t6);
  t5 = conj(t5);
  fe_mul(&t5, &t5, &t2);
  fe_mul(&t4, &t4, &t5);
  t5 = conj(t2);
  fe_mul(&t1, &t1, &t2);
  fe_frob(&t1, &t1, 3);
  fe_mul(&t6, &t6, &t5);
  fe_frob(&t6, &t6, 1);
  fe_mul(&t3, &t3, &t0);
  fe_frob(&t3, &t3, 2);
  fe_mul(&t3, &t3, &t1);
  fe_mul(&t3, &t3, &t6);
  fe_mul(&t3, &t3, &t4);
  return t3;
}
#endif  // CESS_HOSTEMU

}  // namespace bls
