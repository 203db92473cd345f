// Final exponentiation on a lane pair per signature (MillerLoopResult::
// final_exponentiation + Gt::is_identity, utils/verify-bls-signatures/src/
// lib.rs:93-99): the program of staged.hpp
// (CESS_FE_PROGRAM) with every Fp2 split over the pair as in bls/pair.hpp.
//
// Why: the one-lane k_final keeps its accumulators in HBM (two waves per SIMD
// leave 288 B of LDS per lane, half an Fp12) and streams every operand of an
// Fp12 product from there -- ~324 KB of counted traffic per signature, which
// costs it its clock (2.13-2.20 against 2.36 GHz with the same instructions
// on L2-resident slots, profiles/round5_v_diag_l2.txt).  A lane pair holds an
// Fp12 in 288 B per lane, so the accumulator lives in LDS (G[18][256], 72 KiB
// per 128-signature block, two blocks per CU) and every opcode works on it in
// place: FE_MUL reads its slot operand once per Fp6 product (1.15 KB per
// signature against 6.9 KB), the compressed squarings keep z2..z5 in
// registers (48 per lane).
#pragma once
#include "pair.hpp"

#if !defined(CESS_HOSTEMU)
namespace bls {

// One signature's Fp12 in an HBM slot (the GlobF12 rows, stride `stride`):
// lane h reads / writes rows 6k + 3h + q of column (signature) base + lane/2.
// `base` points at the wave's first signature (uniform); the lane part is
// recomputed per access (staged.hpp GlobF12W).
struct GlobPair {
  uint4* base;
  uint64_t stride;
  CESS_HD uint64_t at(int k, int q) const {
    const uint32_t l = lane_fresh();
    return (uint64_t)(6 * k + q + 3 * (l & 1u)) * stride + (l >> 1);
  }
  CESS_HD fph ld(int k) const {
    fph r;
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const uint4 x = base[at(k, q)];
      r.v.v[4 * q] = x.x, r.v.v[4 * q + 1] = x.y, r.v.v[4 * q + 2] = x.z, r.v.v[4 * q + 3] = x.w;
    }
    return r;
  }
  CESS_HD void st(int k, const fph& a) const {
#pragma unroll
    for (int q = 0; q < 3; q++)
      base[at(k, q)] = make_uint4(a.v.v[4 * q], a.v.v[4 * q + 1], a.v.v[4 * q + 2], a.v.v[4 * q + 3]);
  }
  // both components of coefficient k (k may differ between the two lanes)
  CESS_HD fp2 ld_full(int k) const {
    const uint32_t l = lane_fresh() >> 1;
    fp2 r;
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const uint4 x = base[(uint64_t)(6 * k + q) * stride + l];
      fp& d = q < 3 ? r.c0 : r.c1;
      const int o = 4 * (q % 3);
      d.v[o] = x.x, d.v[o + 1] = x.y, d.v[o + 2] = x.z, d.v[o + 3] = x.w;
    }
    return r;
  }
  CESS_HD void st_full(int k, const fp2& a) const {
    const uint32_t l = lane_fresh() >> 1;
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const fp& s = q < 3 ? a.c0 : a.c1;
      const int o = 4 * (q % 3);
      base[(uint64_t)(6 * k + q) * stride + l] = make_uint4(s.v[o], s.v[o + 1], s.v[o + 2], s.v[o + 3]);
    }
  }
};

template <class D, class S>
CESS_HD void pcopy12(const D& d, const S& s) {
#pragma unroll 1
  for (int k = 0; k < 6; k++) d.st(k, s.ld(k));
}
template <class S>
CESS_HD void pconj12(const S& f) {
#pragma unroll 1
  for (int k = 3; k < 6; k++) f.st(k, neg(f.ld(k)));
}
// f == 1, the same answer in both lanes
template <class S>
CESS_HD bool pis_one12(const S& f) {
  bool r = eq(f.ld(0).v, fph_one().v);
#pragma unroll 1
  for (int k = 1; k < 6; k++) r = r && is_zero(f.ld(k).v);
  return pair_and(r);
}
// a == conj(b) (a b == 1 for b cyclotomic), the same answer in both lanes
template <class A, class B>
CESS_HD bool pis_conj12(const A& a, const B& b) {
  bool r = true;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r = r && eq(a.ld(k).v, k < 3 ? b.ld(k).v : neg(b.ld(k).v));
  return pair_and(r);
}

// Karatsuba Fp6 product with the first operand fetched per use (a(j): this
// lane's component of coefficient j, e.g. an LDS load or a sum of two) and
// the second held in registers
template <class LA>
CESS_HD fp6h pmul6_lr(LA&& a, const fp6h& b) {
#if CESS_PAIR_SB
  return pmul6_sb(a, b);
#endif
  const fph v0 = pmul(a(0), b.c0);
  CESS_MEMBAR();
  const fph v1 = pmul(a(1), b.c1);
  CESS_MEMBAR();
  const fph v2 = pmul(a(2), b.c2);
  CESS_MEMBAR();
  const fph c0 = add(mul_nr(sub(sub(pmul(add_nr(a(1), a(2)), add_nr(b.c1, b.c2)), v1), v2)), v0);
  CESS_MEMBAR();
  const fph c1 = add(sub(sub(pmul(add_nr(a(0), a(1)), add_nr(b.c0, b.c1)), v0), v1), mul_nr(v2));
  CESS_MEMBAR();
  const fph c2 = add(sub(sub(pmul(add_nr(a(0), a(2)), add_nr(b.c0, b.c2)), v0), v2), v1);
  return {c0, c1, c2};
}

// f <- f g in place (f: the LDS accumulator, g: a slot), Karatsuba over Fp6
// ordered so that at most one Fp6 product is held: t0 = f0 g0;
// x = (f0 + f1)(g0 + g1); f0 <- x - t0 (f0 is dead: t1 needs f1 only);
// t1 = f1 g1; f1 <- f0 - t1 = f0 g1 + f1 g0; f0 <- t0 + v t1.
// CESS_PAIR_FE_LOOP (default 1): the three Fp6 products as a three-iteration
// loop over ONE inlined pmul6_lr body (a third of the code, as pair.hpp
// CESS_PAIR_LOOP): k_final2 98.3 K -> 87.3 K instructions, 129.6-129.9 ->
// 129.1 ms same box (profiles/round6_ac_sweep_feloop.txt)
#ifndef CESS_PAIR_FE_LOOP
#define CESS_PAIR_FE_LOOP 1
#endif
template <class S, class G>
CESS_HD void pmul12(const S& f, const G& g) {
#if CESS_PAIR_FE_LOOP
  fp6h t0;
#pragma unroll 1
  for (int it = 0; it < 3; it++) {
    // it 0: t0 = f0 g0; it 1: x = (f0 + f1)(g0 + g1); it 2: t1 = f1 g1
    fp6h b;
    if (it == 1) {
      b = add_nr(pld6(g, 0), pld6(g, 1));
    } else {
      b = pld6(g, it >> 1);
    }
    const fp6h r = pmul6_lr(
        [&](int j) {
          const int lo = it == 2 ? 3 : 0;
          const fph a = f.ld(lo + j);
          return it == 1 ? add_nr(a, f.ld(3 + j)) : a;
        },
        b);
    CESS_MEMBAR();
    if (it == 0) {
      t0 = r;
    } else if (it == 1) {
      pst6(f, 0, sub(r, t0));
    } else {
      pst6(f, 1, sub(pld6(f, 0), r));
      pst6(f, 0, add(t0, mul_v(r)));
    }
  }
#else
  fp6h t0;
  {
    const fp6h g0 = pld6(g, 0);
    t0 = pmul6_lr([&](int j) { return f.ld(j); }, g0);
  }
  CESS_MEMBAR();
  {
    fp6h gs;
    {
      const fp6h g0 = pld6(g, 0), g1 = pld6(g, 1);
      gs = add_nr(g0, g1);
    }
    const fp6h x = pmul6_lr([&](int j) { return add_nr(f.ld(j), f.ld(3 + j)); }, gs);
    CESS_MEMBAR();
    pst6(f, 0, sub(x, t0));
  }
  CESS_MEMBAR();
  fp6h t1;
  {
    const fp6h g1 = pld6(g, 1);
    t1 = pmul6_lr([&](int j) { return f.ld(3 + j); }, g1);
  }
  CESS_MEMBAR();
  pst6(f, 1, sub(pld6(f, 0), t1));
  pst6(f, 0, add(t0, mul_v(t1)));
#endif
}

// Fp6 square of the store half h (a pmul6 of the half with itself)
template <class S>
CESS_HD fp6h psqr6(const S& f, int h) {
  const fp6h a = pld6(f, h);
  return pmul6_lr([&](int j) { return f.ld(3 * h + j); }, a);
}

// f <- f^-1 in place (staged.hpp inv12_stream): t = a0^2 - v a1^2,
// t^-1 = (c0, c1, c2) / (t0 c0 + xi (t2 c1 + t1 c2)), f = (a0 t^-1, -a1 t^-1)
template <class S>
CESS_HD void pinv12(const S& f) {
  fp6h ti;
  {
    fp6h t;
    {
      const fp6h s0 = psqr6(f, 0);
      CESS_MEMBAR();
      t = sub(s0, mul_v(psqr6(f, 1)));
    }
    CESS_MEMBAR();
    const fph c0 = sub(pmul(t.c0, t.c0), mul_nr(pmul(t.c1, t.c2)));
    CESS_MEMBAR();
    const fph c1 = sub(mul_nr(pmul(t.c2, t.c2)), pmul(t.c0, t.c1));
    CESS_MEMBAR();
    const fph c2 = sub(pmul(t.c1, t.c1), pmul(t.c0, t.c2));
    CESS_MEMBAR();
    const fph den = add(pmul(t.c0, c0), mul_nr(pdot2(t.c2, c1, t.c1, c2)));
    const fph di = pinv(den);
    CESS_MEMBAR();
    ti = {pmul(c0, di), pmul(c1, di), pmul(c2, di)};
  }
  CESS_MEMBAR();
  pst6(f, 0, pmul6_lr([&](int j) { return f.ld(j); }, ti));
  CESS_MEMBAR();
  const fp6h r1 = pmul6_lr([&](int j) { return f.ld(3 + j); }, ti);
  pst6(f, 1, {neg(r1.c0), neg(r1.c1), neg(r1.c2)});
}

// the lane's component of the Frobenius constant gamma_{k,i} (field.hpp frob_coeff)
CESS_HD fph pfrob_coeff(int k, int i) {
  const uint32_t hm = pair_hi_mask();
  fp r;
#pragma unroll
  for (int w = 0; w < 12; w++) r.v[w] = (c::FROB[k - 1][i][1][w] & hm) | (c::FROB[k - 1][i][0][w] & ~hm);
  return {r};
}
// f <- f^(p^k) in place (staged.hpp frob12)
template <class S>
CESS_HD void pfrob12(const S& f, int k) {
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int i = (s % 3) * 2 + s / 3;
    fph y = f.ld(s);
    if (k & 1) y = conj(y);
    if (i) y = pmul(y, pfrob_coeff(k, i));
    f.st(s, y);
  }
}

// (a + b s)^2 in Fp4 (field.hpp fp4_square)
// (a + b s)^2 = (a^2 + xi b^2) + 2 a b s in two products, as the Karabina
// squaring: t0 = a b, t = (a + b)(a + xi b) = a^2 + xi b^2 + (1 + xi) a b
// (against three: a^2, b^2, (a + b)^2)
CESS_HD void pfp4_square(fph& c0, fph& c1, const fph& a, const fph& b) {
  const fph t0 = pmul(a, b);
  CESS_MEMBAR();
  const fph t = pmul(add_nr(a, b), add_xi_nr(a, b));
  c0 = sub(sub(t, t0), mul_nr(t0));
  c1 = dbl(t0);
}
// n Granger-Scott cyclotomic squarings (staged.hpp cyc_square_run / cycsq12)
// of the six coefficients z (in registers, 72 per lane)
CESS_HD void pcyc_square_regs(fph (&z)[6], int n) {
#pragma unroll 1
  for (int r = 0; r < n; r++) {
    CESS_MEMBAR();
    fph t0, t1;
    pfp4_square(t0, t1, z[0], z[4]);
    z[0] = add(dbl(sub(t0, z[0])), t0);
    z[4] = add(dbl(add(t1, z[4])), t1);
    CESS_MEMBAR();
    fph t2, t3;
    pfp4_square(t0, t1, z[3], z[2]);
    CESS_MEMBAR();
    pfp4_square(t2, t3, z[1], z[5]);
    z[1] = add(dbl(sub(t0, z[1])), t0);
    z[5] = add(dbl(add(t1, z[5])), t1);
    const fph n3 = mul_nr(t3);
    z[3] = add(dbl(add(n3, z[3])), n3);
    z[2] = add(dbl(sub(t2, z[2])), t2);
  }
}
// n Granger-Scott squarings of the store f in place
template <class S>
CESS_HD void pcyc_square_run(const S& f, int n) {
  fph z[6];
#pragma unroll
  for (int k = 0; k < 6; k++) z[k] = f.ld(k);
  pcyc_square_regs(z, n);
#pragma unroll
  for (int k = 0; k < 6; k++) f.st(k, z[k]);
}

// n Karabina compressed squarings (staged.hpp kcyc_run) of (z2, z3, z4, z5),
// all in registers
CESS_HD void pkcyc_run(fph& z2, fph& z3, fph& z4, fph& z5, int n) {
#pragma unroll 1
  for (int r = 0; r < n; r++) {
    CESS_MEMBAR();
    fph u, v;
    {
      const fph b3 = pmul_scaled<3>(z4, z5);
      CESS_MEMBAR();
      const fph t3 = pmul_scaled<3>(add_nr(z4, z5), add_xi_nr(z4, z5));
      const fph nb3 = mul_nr(b3);
      u = sub(sub(t3, b3), nb3);   // 3 (z4^2 + xi z5^2)
      v = dbl(nb3);                // 6 xi z4 z5
    }
    CESS_MEMBAR();
    {
      const fph b3 = pmul_scaled<3>(z2, z3);
      CESS_MEMBAR();
      const fph t3 = pmul_scaled<3>(add_nr(z2, z3), add_xi_nr(z2, z3));
      z4 = sub(sub(sub(t3, b3), mul_nr(b3)), dbl(z4));
      z5 = dbl(add(z5, b3));
    }
    CESS_MEMBAR();
    z2 = add(dbl(z2), v);
    z3 = sub(u, dbl(z3));
  }
}

CESS_HD fp2 xchg2(const fp2& a) { return {xchg(a.c0), xchg(a.c1)}; }

// n Karabina compressed squarings split by PRODUCTS over the pair: the
// squaring's two halves are independent -- (z4, z5) gives 3 (z4^2 + xi z5^2)
// and 6 xi z4 z5, which update z3 and z2; (z2, z3) gives 3 (z2^2 + xi z3^2)
// and 6 z2 z3, which update z4 and z5 -- so each lane holds one half as FULL
// Fp2 values, runs its two lazily reduced products (mul_scaled<3>, no
// per-product exchange) and the lanes swap two Fp2 results per squaring.
// Lane 0 holds (u, w) = (z4, z5), lane 1 (u, w) = (z3, z2), so that both
// lanes apply the same update to what they receive:
//   b3 = 3 u w,  A = 3 (u^2 + xi w^2) on lane 0, 3 (w^2 + xi u^2) on lane 1
//   (the second product's operand is u + xi w or w + xi u);
//   lane 0 sends (A, xi b3), lane 1 sends (A, b3); with (P, Q) received
//   u' = P - 2u,  w' = 2 (w + Q)
// (lane 0: z4' = 3 (z2^2 + xi z3^2) - 2 z4, z5' = 2 (z5 + 3 z2 z3); lane 1:
// z3' = 3 (z4^2 + xi z5^2) - 2 z3, z2' = 2 (z2 + 3 xi z4 z5)).
// (u + w, u + xi w | w + xi u), unreduced (< 4p, < 6p), in one pass: the
// xi term is the lane's own select of (w, u)
CESS_HD void ps_operands(const fp2& u, const fp2& w, bool hi, fp2& s, fp2& y) {
  uint32_t bn = 0, k0 = 0, k1 = 0, k2 = 0, k3 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t z0 = hi ? u.c0.v[i] : w.c0.v[i], z1 = hi ? u.c1.v[i] : w.c1.v[i];
    const uint32_t nz1 = subc32(c::P2_RAW[i], z1, bn, &bn);
    s.c0.v[i] = addc32(u.c0.v[i], w.c0.v[i], k0, &k0);
    s.c1.v[i] = addc32(u.c1.v[i], w.c1.v[i], k1, &k1);
    y.c0.v[i] = addc32(s.c0.v[i], nz1, k2, &k2);   // x0 + z0 - z1, {x, z} = {u, w}
    y.c1.v[i] = addc32(s.c1.v[i], z0, k3, &k3);    // x1 + z1 + z0
  }
}
CESS_HD void pkcyc_run_ps(fp2& u, fp2& w, int n) {
  const bool hi = pair_hi_mask() != 0;
#pragma unroll 1
  for (int r = 0; r < n; r++) {
    CESS_MEMBAR();
    fp2 P, Q;
    {
      const fp2 b3 = mul_scaled<3>(u, w);
      CESS_MEMBAR();
      fp2 s, y;
      ps_operands(u, w, hi, s, y);
      const fp2 t3 = mul_scaled<3>(s, y);
      const fp2 nb3 = mul_nr(b3);
      P = sub(sub(t3, b3), nb3);
      Q = select(hi, b3, nb3);
    }
    CESS_MEMBAR();
    P = xchg2(P);
    Q = xchg2(Q);
    u = sub(P, dbl(u));
    w = dbl(add(w, Q));
  }
}

// staged.hpp cyc_z1_frac / cyc_z1_den / cyc_z0
CESS_HD void pcyc_z1_frac(const fph& z2, const fph& z3, const fph& z4, const fph& z5, fph& num, fph& den) {
  if (is_zero(z2)) {   // pair-uniform, practically never taken
    num = dbl(pmul(z4, z5));
    den = z3;
  } else {
    num = sub(add(mul_nr(psqr(z5)), mul3(psqr(z4))), dbl(z3));
    den = dbl(dbl(z2));
  }
}
CESS_HD fph pcyc_z1_den(const fph& z2, const fph& z3) { return is_zero(z2) ? z3 : dbl(dbl(z2)); }
CESS_HD fph pcyc_z0(const fph& z1, const fph& z2, const fph& z3, const fph& z4, const fph& z5) {
  return add(mul_nr(add(dbl(psqr(z1)), pdot2(z2, z5, neg(mul3(z3)), z4))), fph_one());
}

// FE_CHAIN (staged.hpp cyc_chain): the powers a^(2^k), k = 16, 48, 57, 60, 62,
// 63, of the cyclotomic element in `base` into the stores X(0..5).
// CESS_CHAIN_TAIL (staged.hpp, default 1): only a^(2^16), a^(2^48) and
// a^(2^57) come from the compressed run and its decompression; a^(2^60),
// a^(2^62) and a^(2^63) follow from a^(2^57) by 3 + 2 + 1 Granger-Scott
// squarings.  Per exponentiation by x that is 6 GS squarings (6 products each,
// against 4 for a Karabina squaring) for 3 decompressions (~8.5 products each).
template <class B, class XFn>
CESS_HD void pcyc_chain(const B& base, XFn&& X) {
  constexpr int ND = CESS_CHAIN_TAIL ? 3 : 6;   // decompressed powers
#ifndef CESS_PAIR_KCYC_PS
#define CESS_PAIR_KCYC_PS 1
#endif
#if CESS_PAIR_KCYC_PS
  {
    // store indices of (u, w): lane 0 (z4, z5) = (1, 5), lane 1 (z3, z2) = (2, 3)
    const bool hi = pair_hi_mask() != 0;
    const int ku = hi ? 2 : 1, kw = hi ? 3 : 5;
    fp2 u = base.ld_full(ku), w = base.ld_full(kw);
    int k = 0;
#pragma unroll 1
    for (int j = 0; j < ND; j++) {
      const int stop = j == 0 ? 16 : j == 1 ? 48 : j == 2 ? 57 : j == 3 ? 60 : j == 4 ? 62 : 63;
      pkcyc_run_ps(u, w, stop - k);
      k = stop;
      CESS_MEMBAR();
      const auto x = X(j);
      x.st_full(ku, u);
      x.st_full(kw, w);
    }
  }
#else
  {
    fph z4 = base.ld(1), z5 = base.ld(5), z2 = base.ld(3), z3 = base.ld(2);
    int k = 0;
#pragma unroll 1
    for (int j = 0; j < ND; j++) {
      const int stop = j == 0 ? 16 : j == 1 ? 48 : j == 2 ? 57 : j == 3 ? 60 : j == 4 ? 62 : 63;
      pkcyc_run(z2, z3, z4, z5, stop - k);
      k = stop;
      CESS_MEMBAR();
      const auto x = X(j);
      x.st(3, z2);
      x.st(2, z3);
      x.st(1, z4);
      x.st(5, z5);
    }
  }
#endif
  CESS_MEMBAR();
  bool degen = false;
  fph prod = fph_one();
#pragma unroll 1
  for (int j = 0; j < ND; j++) {
    const auto x = X(j);
    fph num, den;
    pcyc_z1_frac(x.ld(3), x.ld(2), x.ld(1), x.ld(5), num, den);
    const bool z = is_zero(den);
    degen = degen || z;
    x.st(4, num);
    x.st(0, prod);   // product of the denominators before j
    prod = pmul(prod, select(z, fph_one(), den));
    CESS_MEMBAR();
  }
  fph iv = pinv(prod);
#pragma unroll 1
  for (int j = ND - 1; j >= 0; j--) {
    const auto x = X(j);
    const fph den = pcyc_z1_den(x.ld(3), x.ld(2));
    const fph ivj = pmul(iv, x.ld(0));   // 1 / den_j
    iv = pmul(iv, select(is_zero(den), fph_one(), den));
    CESS_MEMBAR();
    const fph z1 = pmul(x.ld(4), ivj);
    x.st(4, z1);
    CESS_MEMBAR();
    x.st(0, pcyc_z0(z1, x.ld(3), x.ld(2), x.ld(1), x.ld(5)));
    CESS_MEMBAR();
  }
  if (degen) {   // pair-uniform; Granger-Scott squarings with X(5) as the running power
    const auto w = X(5);
    pcopy12(w, base);
#pragma unroll 1
    for (int j = 0; j < 5; j++) {
      const int run = j == 0 ? 16 : j == 1 ? 32 : j == 2 ? 9 : j == 3 ? 3 : 2;
      pcyc_square_run(w, run);
      pcopy12(X(j), w);
    }
    pcyc_square_run(w, 1);
  }
#if CESS_CHAIN_TAIL
  else {   // X3..X5 from X2 = a^(2^57): 3, 2, 1 squarings
    fph z[6];
    {
      const auto x2 = X(2);
#pragma unroll
      for (int k = 0; k < 6; k++) z[k] = x2.ld(k);
    }
#pragma unroll 1
    for (int j = 3; j < 6; j++) {
      pcyc_square_regs(z, j == 3 ? 3 : j == 4 ? 2 : 1);
      CESS_MEMBAR();
      const auto x = X(j);
#pragma unroll
      for (int k = 0; k < 6; k++) x.st(k, z[k]);
    }
  }
#endif
}

// The program (staged.hpp final_exp_staged) on ONE in-place accumulator
// (FE_MUL and FE_INV work in place here); slot(s) returns the store of slot s.
template <class A, class SlotFn>
CESS_HD void final_exp_pair(const A& acc, const uint8_t (*prog)[2], SlotFn&& slot) {
#pragma unroll 1
  for (int pc = 0;; pc++) {
    const uint8_t op = prog[pc][0], arg = prog[pc][1];
    if (op == FE_END) break;
    switch (op) {
      case FE_LOAD: pcopy12(acc, slot(arg)); break;
      case FE_STORE: pcopy12(slot(arg), acc); break;
      case FE_MUL: pmul12(acc, slot(arg)); break;
      case FE_SQN: pcyc_square_run(acc, arg); break;
      case FE_CONJ: pconj12(acc); break;
      case FE_FROB: pfrob12(acc, arg); break;
      case FE_INV: pinv12(acc); break;
      case FE_CHAIN: pcyc_chain(slot(arg), [&](int j) { return slot(SL_X0 + j); }); break;
      default: break;
    }
    CESS_MEMBAR();
  }
}

}  // namespace bls
#endif
