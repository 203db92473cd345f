// Lane-pair (component-split) Fp2 arithmetic: TWO lanes per signature, lane h
// of the pair (h = lane & 1) holds component h of every Fp2 value.
//
// Why (MI355X, k_miller): the one-lane Miller loop keeps its Fp12
// accumulator in a 144 KiB LDS image of 256 signatures and needs ~490
// registers, so it runs ONE wave per SIMD (VALU-active 0.77, 5.29 cycles per
// instruction; profiles/round5_ax_pmc_stall.txt).  Splitting every Fp2 value
// over a lane pair keeps the same 144 KiB image for the same 256 signatures
// but with 512 lanes (two waves per SIMD), and halves the registers every
// held Fp2 / Fp6 intermediate needs.
//
// The split follows the lazily reduced schoolbook Fp2 product (field.hpp
// mul_scaled): component 0 of a b is a0 b0 + a1 (K - b1), component 1 is
// a0 b1 + a1 b0 -- each ONE Montgomery reduction over two half-products, so
// the pair does exactly the one-lane product's mads, half per lane.  A lane
// unpacks only its own components into 28-bit digits and takes the partner's
// digits with DPP quad-permutes (v_mov_b32_dpp, no LDS): for lane h,
//   xa = own a digits, xb = partner's a digits (swap),
//   ya = b0 digits (broadcast from the even lane),
//   yb = b1 digits (broadcast from the odd lane), K - b1 on the even lane,
// and component h = sum xa[i] ya[j] + xb[i] yb[j] (lane 0: a0 b0 + a1 (K - b1),
// lane 1: a1 b0 + a0 b1).  Additions and subtractions are per component, so
// each lane does half of them; multiplication by xi = 1 + u needs the partner's
// component (own - partner on the even lane, own + partner on the odd one).
//
// Every condition that steers control flow must be the same in both lanes of a
// pair (per signature): DPP reads the partner's register at the instant of the
// instruction, so both lanes have to execute it.
//
// Reference: bls12_381 0.7.1's Fp2/Fp6/Fp12 arithmetic under
// MillerLoopResult / multi_miller_loop, called at
// utils/verify-bls-signatures/src/lib.rs:90-93.
#pragma once
#include "staged.hpp"
#include "../kernels.hpp"

#if !defined(CESS_HOSTEMU)
namespace bls {

// --- lane-pair exchange ------------------------------------------------------
// quad_perm controls: swap [1,0,3,2], even broadcast [0,0,2,2], odd [1,1,3,3]
// (bound_ctrl with full row/bank masks: no 'old' operand, so no v_mov
// initialising the destination before each v_mov_b32_dpp)
CESS_HD uint32_t dpp_swap(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true); }
CESS_HD uint32_t dpp_even(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xF, 0xF, true); }
CESS_HD uint32_t dpp_odd(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xF5, 0xF, 0xF, true); }

// all ones on the odd lane of a pair (component 1), zero on the even lane
CESS_HD uint32_t pair_hi_mask() { return 0u - (__lane_id() & 1u); }

// the lane's component of an Fp2 value
struct fph {
  fp v;
};
struct fp6h {
  fph c0, c1, c2;
};

CESS_HD fph fph_of(const fp& v) { return {v}; }
CESS_HD fph add(const fph& a, const fph& b) { return {add(a.v, b.v)}; }
CESS_HD fph sub(const fph& a, const fph& b) { return {sub(a.v, b.v)}; }
CESS_HD fph add_nr(const fph& a, const fph& b) { return {add_nr(a.v, b.v)}; }
CESS_HD fph dbl(const fph& a) { return {dbl(a.v)}; }
CESS_HD fph neg(const fph& a) { return {neg(a.v)}; }
CESS_HD fp xchg(const fp& a) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = dpp_swap(a.v[i]);
  return r;
}
// the partner's component, negated (2p - x, in [0, 2p]) on the even lane:
// lane 0 gets -a1, lane 1 gets +a0 -- the second term of xi a and of x + xi y
CESS_HD fp partner_signed(const fp& own) {
  const fp p = xchg(own);
  const uint32_t hm = pair_hi_mask();
  fp r;
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t n = subc32(c::P2_RAW[i], p.v[i], bw, &bw);
    r.v[i] = (p.v[i] & hm) | (n & ~hm);
  }
  return r;
}
// * xi = 1 + u: (a0 - a1) + (a0 + a1) u -- own - partner on the even lane,
// own + partner on the odd lane (a summand of 2p, for a1 = 0, is removed by
// add's conditional subtraction)
CESS_HD fph mul_nr(const fph& a) { return {add(a.v, partner_signed(a.v))}; }
// xi a unreduced (< 4p): for products only
CESS_HD fph mul_nr_nr(const fph& a) { return {add_nr(a.v, partner_signed(a.v))}; }
// a + xi b unreduced (< 6p), field.hpp add_xi_nr: for products only
CESS_HD fph add_xi_nr(const fph& a, const fph& b) { return {add_nr(add_nr(a.v, b.v), partner_signed(b.v))}; }
// both lanes of the pair agree on a predicate (AND of the two lanes' values)
CESS_HD bool pair_and(bool b) {
  const uint32_t x = b ? 1u : 0u;
  return (x & dpp_swap(x)) != 0;
}
CESS_HD bool is_zero(const fph& a) { return pair_and(is_zero(a.v)); }
CESS_HD bool eq(const fph& a, const fph& b) { return pair_and(eq(a.v, b.v)); }
CESS_HD fph select(bool c, const fph& a, const fph& b) { return {select(c, a.v, b.v)}; }
CESS_HD fph mul3(const fph& a) { return {mul3(a.v)}; }
// the pair's Fp2 value (1, 0) / (0, 0)
CESS_HD fph fph_one() {
  const uint32_t hm = pair_hi_mask();
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = c::ONE[i] & ~hm;
  return {r};
}
CESS_HD fph fph_zero() { return {fp_zero()}; }
// conjugate: the odd lane negates
CESS_HD fph conj(const fph& a) {
  const fp n = neg(a.v);
  const uint32_t hm = pair_hi_mask();
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = (n.v[i] & hm) | (a.v.v[i] & ~hm);
  return {r};
}

// digit vectors of one Fp2 operand pair (x = a, y = b) for this lane's
// component: xa own a, xb partner's a, ya = b0, yb = b1 (odd lane) or K - b1
// (even lane)
// (S: a's digits scaled by S <= 3 before the exchange, as mul_scaled<S>)
template <uint32_t S = 1>
CESS_HD void pair_digits(const fp& a, const fp& b, uint32_t (&xa)[14], uint32_t (&xb)[14], uint32_t (&ya)[14],
                         uint32_t (&yb)[14]) {
  uint32_t yo[14];
  unpack28(a, xa);
  unpack28(b, yo);
  const uint32_t hm = pair_hi_mask();
#pragma unroll
  for (int i = 0; i < 14; i++) {
    if (S != 1) xa[i] *= S;
    xb[i] = dpp_swap(xa[i]);
    ya[i] = dpp_even(yo[i]);
    const uint32_t t = dpp_odd(yo[i]);
    yb[i] = (t & hm) | ((c::NEG_K28[i] - t) & ~hm);
  }
}

// this lane's component of S a b (a, b: the pair's Fp2 values, inputs < 8p as
// mul_scaled<S>); result < 2p
template <uint32_t S>
CESS_HD fph pmul_scaled(const fph& a0, const fph& b0) {
  static_assert(S >= 1 && S <= 3, "digit bound");
  CESS_COUNT_MUL2();
  fp a = a0.v, b = b0.v;
  seq(a);
  seq(b);
  uint32_t xa[14], xb[14], ya[14], yb[14];
  pair_digits<S>(a, b, xa, xb, ya, yb);
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
      mac(acc, xa[i], ya[j]);
      mac(acc, xb[i], yb[j]);
    }
  });
  seq(r);
  return {r};
}
CESS_HD fph pmul(const fph& a, const fph& b) { return pmul_scaled<1>(a, b); }

// a^2: ONE Fp product per lane -- component 0 = (a0 + a1)(a0 - a1) on the
// even lane, component 1 = (2 a1) a0 on the odd lane (against two
// half-products and the operand exchange of pmul(a, a)); factors < 4p
CESS_HD fph psqr(const fph& a) {
  const fp p = xchg(a.v);
  const bool hi = pair_hi_mask() != 0;
  fp x, y;
  uint32_t cx = 0, bn = 0, cy = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    x.v[i] = addc32(a.v.v[i], hi ? a.v.v[i] : p.v[i], cx, &cx);   // a0 + a1 | 2 a1
    const uint32_t n = subc32(c::P2_RAW[i], p.v[i], bn, &bn);      // 2p - a1
    const uint32_t t = addc32(a.v.v[i], n, cy, &cy);                // a0 + 2p - a1
    y.v[i] = hi ? p.v[i] : t;                                       // a0 - a1 | a0
  }
  return {mul(x, y)};
}

// a^-1 in Fp2: a / (a0^2 + a1^2) conjugated (field.hpp inv(fp2)); the norm
// and its Fp inversion are computed by both lanes
CESS_HD fph pinv(const fph& a) {
  const fp n = sqr(a.v);
  const fp t = inv(add(n, xchg(n)));
  return conj(fph{mul(a.v, t)});
}

// this lane's component of a b + c d (one reduction; bounds as dot2)
CESS_HD fph pdot2(const fph& a0, const fph& b0, const fph& c0, const fph& d0) {
  CESS_COUNT_HALVES(8);
  fp a = a0.v, b = b0.v, c = c0.v, d = d0.v;
  seq(a);
  seq(b);
  seq(c);
  seq(d);
  uint32_t xa[14], xb[14], ya[14], yb[14], ua[14], ub[14], wa[14], wb[14];
  pair_digits(a, b, xa, xb, ya, yb);
  pair_digits(c, d, ua, ub, wa, wb);
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
      mac(acc, xa[i], ya[j]);
      mac(acc, xb[i], yb[j]);
      mac(acc, ua[i], wa[j]);
      mac(acc, ub[i], wb[j]);
    }
  });
  seq(r);
  return {r};
}

// Prepared operands: the digit vectors of pair_digits computed once for an
// operand that several products share (each preparation is an unpack plus
// 14-28 DPP moves and, for a y operand, the K - b1 selection).
struct pxd {   // x side: own digits, partner's digits
  uint32_t a[14], b[14];
};
struct pyd {   // y side: b0 digits, b1 (odd lane) or K - b1 (even lane) digits
  uint32_t a[14], b[14];
};
CESS_HD pxd prep_x(const fph& x0) {
  fp x = x0.v;
  seq(x);
  pxd r;
  unpack28(x, r.a);
#pragma unroll
  for (int i = 0; i < 14; i++) r.b[i] = dpp_swap(r.a[i]);
  return r;
}
CESS_HD pyd prep_y(const fph& y0) {
  fp y = y0.v;
  seq(y);
  uint32_t yo[14];
  unpack28(y, yo);
  const uint32_t hm = pair_hi_mask();
  pyd r;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    r.a[i] = dpp_even(yo[i]);
    const uint32_t t = dpp_odd(yo[i]);
    r.b[i] = (t & hm) | ((c::NEG_K28[i] - t) & ~hm);
  }
  return r;
}
// this lane's component of x y / x y + u w from prepared operands (bounds as
// pmul / pdot2)
CESS_HD fph pmul_p(const pxd& x, const pyd& y) {
  CESS_COUNT_MUL2();
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
      mac(acc, x.a[i], y.a[j]);
      mac(acc, x.b[i], y.b[j]);
    }
  });
  seq(r);
  return {r};
}
CESS_HD fph pdot2_p(const pxd& x, const pyd& y, const pxd& u, const pyd& w) {
  CESS_COUNT_HALVES(8);
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
      mac(acc, x.a[i], y.a[j]);
      mac(acc, x.b[i], y.b[j]);
      mac(acc, u.a[i], w.a[j]);
      mac(acc, u.b[i], w.b[j]);
    }
  });
  seq(r);
  return {r};
}

// this lane's component of x y + u w + s t from prepared operands: ONE
// reduction over six half-products.  Columns < 3 x 14 x (2^56 + 2^57) + 14 x
// 2^56 < 2^63.2 (x digits < 2^28, y digits < 2^29: K - b1), and the value
// < 3 x 8p x 2^385 < p R for inputs < 8p, so the reduction returns < 2p.
CESS_HD fph pdot3_p(const pxd& x, const pyd& y, const pxd& u, const pyd& w, const pxd& s, const pyd& t) {
  CESS_COUNT_HALVES(12);
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
      mac(acc, x.a[i], y.a[j]);
      mac(acc, x.b[i], y.b[j]);
      mac(acc, u.a[i], w.a[j]);
      mac(acc, u.b[i], w.b[j]);
      mac(acc, s.a[i], t.a[j]);
      mac(acc, s.b[i], t.b[j]);
    }
  });
  seq(r);
  return {r};
}

// a * s for s in Fp (both lanes hold s): one Fp product per lane
CESS_HD fph pmul_fp(const fph& a, const fp& s) { return {mul(a.v, s)}; }

// --- Fp6 over lane pairs ------------------------------------------------------
CESS_HD fp6h add(const fp6h& a, const fp6h& b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
CESS_HD fp6h sub(const fp6h& a, const fp6h& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1), sub(a.c2, b.c2)}; }
CESS_HD fp6h dbl(const fp6h& a) { return {dbl(a.c0), dbl(a.c1), dbl(a.c2)}; }
CESS_HD fp6h add_nr(const fp6h& a, const fp6h& b) {
  return {add_nr(a.c0, b.c0), add_nr(a.c1, b.c1), add_nr(a.c2, b.c2)};
}
CESS_HD fp6h mul_v(const fp6h& a) { return {mul_nr(a.c2), a.c0, a.c1}; }

// Schoolbook Fp6 product as three lazily reduced dot products (one reduction
// per output component; v^3 = xi):
//   c0 = a0 b0 + a1 (xi b2) + a2 (xi b1),  c1 = a0 b1 + a1 b0 + a2 (xi b2),
//   c2 = a0 b2 + a1 b1 + a2 b0.
// 17 % more mads than Karatsuba's six products, but the three x operands and
// five y operands are prepared once (unpack + DPP exchange) and there are no
// operand sums, no re-preparation of them and no recombination: fewer VALU
// instructions per Fp6 product (CESS_PAIR_SB).  a(j): this lane's component of
// a's coefficient j (a loader or register values), < 8p; b's coefficients < 4p.
// Measured, not adopted: static VALU -2.5 % (k_miller2) / -2.9 % (k_final2),
// but 15 / 62 spilled VGPRs, and equal time on the same box (k_miller2
// 126.8-126.9 vs 126.7-127.0, k_final2 140.8-141.9 vs 140.9-141.0 ms,
// profiles/round6_k_sweep_schoolbook.txt).
#ifndef CESS_PAIR_SB
#define CESS_PAIR_SB 0
#endif
template <class LA>
CESS_HD fp6h pmul6_sb(LA&& a, const fp6h& b) {
  const pxd x0 = prep_x(a(0)), x1 = prep_x(a(1)), x2 = prep_x(a(2));
  fp6h c;
  {
    const pyd y0 = prep_y(b.c0), y1 = prep_y(b.c1);
    c.c2 = pdot3_p(x0, prep_y(b.c2), x1, y1, x2, y0);
    CESS_MEMBAR();
    // xi b2, xi b1 from b reduced below 2p: callers pass unreduced sums (< 4p:
    // add_nr(a0, v a1) in the squaring, g0 + g1 in FE_MUL), and xi's 2p - b
    // on the even lane needs b < 2p
    const pyd xy2 = prep_y(mul_nr_nr(fph{fp_reduce2(b.c2.v)}));
    c.c1 = pdot3_p(x0, y1, x1, y0, x2, xy2);
    CESS_MEMBAR();
    c.c0 = pdot3_p(x0, y0, x1, xy2, x2, prep_y(mul_nr_nr(fph{fp_reduce2(b.c1.v)})));
  }
  return c;
}

// Karatsuba Fp6 product (as field.hpp mul(fp6, fp6))
CESS_HD fp6h pmul6(const fp6h& a, const fp6h& b) {
#if CESS_PAIR_SB
  return pmul6_sb([&](int j) { return j == 0 ? a.c0 : j == 1 ? a.c1 : a.c2; }, b);
#endif
  const fph t0 = pmul(a.c0, b.c0);
  const fph t1 = pmul(a.c1, b.c1);
  const fph t2 = pmul(a.c2, b.c2);
  const fph c0 = add(mul_nr(sub(sub(pmul(add_nr(a.c1, a.c2), add_nr(b.c1, b.c2)), t1), t2)), t0);
  const fph c1 = add(sub(sub(pmul(add_nr(a.c0, a.c1), add_nr(b.c0, b.c1)), t0), t1), mul_nr(t2));
  const fph c2 = add(sub(sub(pmul(add_nr(a.c0, a.c2), add_nr(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}
// a * (b1 v)
#ifndef CESS_PAIR_PREP
#define CESS_PAIR_PREP 1
#endif
CESS_HD fp6h pmul_by_1(const fp6h& a, const fph& b1) {
#if CESS_PAIR_PREP
  const pyd y = prep_y(b1);   // shared by the three products
  const fph p2 = pmul_p(prep_x(a.c2), y);
  CESS_MEMBAR();
  const fph p0 = pmul_p(prep_x(a.c0), y);
  CESS_MEMBAR();
  return {mul_nr(p2), p0, pmul_p(prep_x(a.c1), y)};
#else
  const fph p2 = pmul(a.c2, b1);
  CESS_MEMBAR();
  const fph p0 = pmul(a.c0, b1);
  CESS_MEMBAR();
  return {mul_nr(p2), p0, pmul(a.c1, b1)};
#endif
}

// One signature's Fp12 in the lane pair's LDS image G[18][CESS_PAIR_THREADS]: lane t owns
// column t (signature t / 2, component t & 1), row 3k + q holds words
// 4q..4q+3 of its component of coefficient k (store index as staged.hpp).
// Conflict-free ds_read_b128 as LdsF12; t = w0 + lane id, w0 uniform.
struct LdsPair {
  uint4 (*G)[CESS_PAIR_THREADS];
  uint32_t w0;
  CESS_HD fph ld(int k) const {
    const uint32_t t = w0 + lane_fresh();
    fph r;
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const uint4 x = G[3 * k + q][t];
      r.v.v[4 * q] = x.x, r.v.v[4 * q + 1] = x.y, r.v.v[4 * q + 2] = x.z, r.v.v[4 * q + 3] = x.w;
    }
    return r;
  }
  CESS_HD void st(int k, const fph& a) const {
    const uint32_t t = w0 + lane_fresh();
#pragma unroll
    for (int q = 0; q < 3; q++) G[3 * k + q][t] = make_uint4(a.v.v[4 * q], a.v.v[4 * q + 1], a.v.v[4 * q + 2], a.v.v[4 * q + 3]);
  }
};

template <class S>
CESS_HD fp6h pld6(const S& s, int h) {
  return {s.ld(3 * h), s.ld(3 * h + 1), s.ld(3 * h + 2)};
}
template <class S>
CESS_HD void pst6(const S& s, int h, const fp6h& a) {
  s.st(3 * h, a.c0);
  s.st(3 * h + 1, a.c1);
  s.st(3 * h + 2, a.c2);
}

// f <- f^2 (complex squaring: 2 Fp6 products), staged.hpp sqr12
// CESS_PAIR_LOOP (bit mask): the Miller step's repeated Fp6 products as
// two-iteration loops over ONE inlined product body each -- bit 1 psqr12's two
// pmul6, bit 2 pmul014's two mul_by_01 halves, bit 4 pmul014_one's -- a
// smaller step body for the instruction cache (staged.hpp CESS_MUL014_LOOP
// for k_miller_rr).  Default 5: k_miller2 31.6 K -> 23.7 K instructions,
// 120.0-120.4 -> 119.5 ms same box (profiles/round6_ab_sweep_loop.txt); bit
// 2 spills 27 VGPRs (the loop-carried u beside the dot products' operands).
#ifndef CESS_PAIR_LOOP
#define CESS_PAIR_LOOP 5
#endif
template <class S>
CESS_HD void psqr12(const S& f) {
#if CESS_PAIR_LOOP & 1
  fp6h ab;
#pragma unroll 1
  for (int it = 0; it < 2; it++) {
    const fp6h a0 = pld6(f, 0), a1 = pld6(f, 1);
    fp6h A = a0, B = a1;
    if (it) {
      A = add_nr(a0, a1);
      B = add_nr(a0, mul_v(a1));
    }
    const fp6h r = pmul6(A, B);
    CESS_MEMBAR();
    if (it == 0) {
      ab = r;
    } else {
      pst6(f, 0, sub(sub(r, ab), mul_v(ab)));
      pst6(f, 1, dbl(ab));
    }
  }
#else
  fp6h ab;
  {
    const fp6h a0 = pld6(f, 0), a1 = pld6(f, 1);
    ab = pmul6(a0, a1);
  }
  CESS_MEMBAR();
  fp6h x;
  {
    const fp6h a0 = pld6(f, 0), a1 = pld6(f, 1);
    x = pmul6(add_nr(a0, a1), add_nr(a0, mul_v(a1)));
  }
  pst6(f, 0, sub(sub(x, ab), mul_v(ab)));
  pst6(f, 1, dbl(ab));
#endif
}

// a * (b0 + b1 v) for the Fp6 in store half h, as staged.hpp mul_by_01_dot
template <class S>
CESS_HD fp6h pmul_by_01_dot(const S& f, int h, const fph& b0, const fph& b1, const fph& xb1) {
#if CESS_PAIR_PREP
  // b0 enters all three dot products, b1 two, each coefficient of f two
  const pyd y0 = prep_y(b0);
  fp6h r;
  {
    const pxd x0 = prep_x(f.ld(3 * h));
    r.c0 = pdot2_p(x0, y0, prep_x(f.ld(3 * h + 2)), prep_y(xb1));
    CESS_MEMBAR();
    r.c1 = pdot2_p(x0, prep_y(b1), prep_x(f.ld(3 * h + 1)), y0);
  }
  CESS_MEMBAR();
  r.c2 = pdot2_p(prep_x(f.ld(3 * h + 1)), prep_y(b1), prep_x(f.ld(3 * h + 2)), y0);
  return r;
#else
  fp6h r;
  r.c0 = pdot2(f.ld(3 * h), b0, f.ld(3 * h + 2), xb1);
  CESS_MEMBAR();
  r.c1 = pdot2(f.ld(3 * h), b1, f.ld(3 * h + 1), b0);
  CESS_MEMBAR();
  r.c2 = pdot2(f.ld(3 * h + 1), b1, f.ld(3 * h + 2), b0);
  return r;
#endif
}

// f <- f * (c0 + c1 v + c4 v w), staged.hpp mul014
template <class S>
CESS_HD void pmul014(const S& f, const fph& c0, const fph& c1, const fph& c4) {
  const fp6h bb = pmul_by_1(pld6(f, 1), c4);
  CESS_MEMBAR();
#if CESS_PAIR_LOOP & 2
  {
    fp6h u;
    const fph d = add(c1, c4);
#pragma unroll 1
    for (int it = 0; it < 2; it++) {
      const fph b1 = it ? d : c1;
      const fp6h r = pmul_by_01_dot(f, it, c0, b1, mul_nr_nr(b1));
      CESS_MEMBAR();
      if (it == 0) {
        pst6(f, 1, add(pld6(f, 0), pld6(f, 1)));   // f.c1 <- a0 + a1 (read by it = 1)
        pst6(f, 0, add(mul_v(bb), r));
        u = add(r, bb);
      } else {
        pst6(f, 1, sub(r, u));
      }
    }
    return;
  }
#endif
  const fp6h aa = pmul_by_01_dot(f, 0, c0, c1, mul_nr_nr(c1));
  CESS_MEMBAR();
  pst6(f, 1, add(pld6(f, 0), pld6(f, 1)));   // f.c1 <- a0 + a1 (consumed below)
  pst6(f, 0, add(mul_v(bb), aa));
  const fp6h u = add(aa, bb);
  CESS_MEMBAR();
  const fph d = add(c1, c4);
  const fp6h t = pmul_by_01_dot(f, 1, c0, d, mul_nr_nr(d));
  pst6(f, 1, sub(t, u));
}

// a * (1 + b1 v)
CESS_HD fp6h pmul_by_01_one(const fp6h& a, const fph& b1) {
#if CESS_PAIR_PREP
  const pyd y = prep_y(b1);   // shared by the three products
  const fph p2 = pmul_p(prep_x(a.c2), y);
  CESS_MEMBAR();
  const fph p0 = pmul_p(prep_x(a.c0), y);
  CESS_MEMBAR();
  return {add(a.c0, mul_nr(p2)), add(a.c1, p0), add(a.c2, pmul_p(prep_x(a.c1), y))};
#else
  const fph p2 = pmul(a.c2, b1);
  CESS_MEMBAR();
  const fph p0 = pmul(a.c0, b1);
  CESS_MEMBAR();
  return {add(a.c0, mul_nr(p2)), add(a.c1, p0), add(a.c2, pmul(a.c1, b1))};
#endif
}

// f <- f * (1 + c1 v + c4 v w), staged.hpp mul014_one
template <class S>
CESS_HD void pmul014_one(const S& f, const fph& c1, const fph& c4) {
  const fp6h bb = pmul_by_1(pld6(f, 1), c4);
  CESS_MEMBAR();
#if CESS_PAIR_LOOP & 4
  {
    fp6h u;
    const fph d = add(c1, c4);
#pragma unroll 1
    for (int it = 0; it < 2; it++) {
      const fp6h r = pmul_by_01_one(pld6(f, it), it ? d : c1);
      CESS_MEMBAR();
      if (it == 0) {
        pst6(f, 1, add(pld6(f, 0), pld6(f, 1)));
        pst6(f, 0, add(mul_v(bb), r));
        u = add(r, bb);
      } else {
        pst6(f, 1, sub(r, u));
      }
    }
    return;
  }
#endif
  const fp6h aa = pmul_by_01_one(pld6(f, 0), c1);
  CESS_MEMBAR();
  pst6(f, 1, add(pld6(f, 0), pld6(f, 1)));
  pst6(f, 0, add(mul_v(bb), aa));
  const fp6h u = add(aa, bb);
  CESS_MEMBAR();
  const fp6h t = pmul_by_01_one(pld6(f, 1), add(c1, c4));
  pst6(f, 1, sub(t, u));
}

// The two-pair Miller loop of staged.hpp miller_loop2_staged over a lane
// pair: pt(pair) the pair's affine G1 point (both lanes), src(pair, step, j):
// this lane's component of the line's coefficient c_j (returned by value:
// coefficients written through reference parameters from pair-dependent
// branches were lowered to a dynamically indexed private array -- ~40
// scratch accesses per Miller step).
template <class S, class Pt, class Src>
CESS_HD void miller_loop2_pair(const S& f, bool use0, bool use1, Pt&& pt, Src&& src, bool norm1) {
  f.st(0, fph_one());
#pragma unroll 1
  for (int k = 1; k < 6; k++) f.st(k, fph_zero());
#pragma unroll 1
  for (int s = 0; s < N_COEFFS; s++) {
#pragma unroll 1
    for (int pair = 0; pair < 2; pair++) {
      const int pr = 1 - pair;
      if (!(pr ? use1 : use0)) continue;
      const g1a p = pt(pr);
      const fph c1 = pmul_fp(src(pr, s, 1), p.x), c4 = pmul_fp(src(pr, s, 0), p.y);
      if (pr && !norm1)
        pmul014(f, src(pr, s, 2), c1, c4);
      else
        pmul014_one(f, c1, c4);
      CESS_MEMBAR();
    }
    if (square_after_step(s)) psqr12(f);
    CESS_MEMBAR();
  }
#pragma unroll 1
  for (int k = 3; k < 6; k++) f.st(k, neg(f.ld(k)));   // conj: x < 0
}

// Miller loop over up to NP pairs with general lines sharing one accumulator
// (staged.hpp miller_loopn_staged, the distinct-key RLC's lane of records) on
// a lane pair: bit j of `use` (the same in both lanes) -- pair j takes part;
// pt(j) its affine G1 point, src(j, step, c) this lane's component of its
// line coefficient c (by value, as in miller_loop2_pair).
template <int NP, class S, class Pt, class Src>
CESS_HD void miller_loopn_pair(const S& f, uint32_t use, Pt&& pt, Src&& src) {
  f.st(0, fph_one());
#pragma unroll 1
  for (int k = 1; k < 6; k++) f.st(k, fph_zero());
#pragma unroll 1
  for (int s = 0; s < N_COEFFS; s++) {
#pragma unroll 1
    for (int j = 0; j < NP; j++) {
      if (!((use >> j) & 1u)) continue;
      const g1a p = pt(j);
      const fph c1 = pmul_fp(src(j, s, 1), p.x), c4 = pmul_fp(src(j, s, 0), p.y);
      pmul014(f, src(j, s, 2), c1, c4);
      CESS_MEMBAR();
    }
    if (square_after_step(s)) psqr12(f);
    CESS_MEMBAR();
  }
#pragma unroll 1
  for (int k = 3; k < 6; k++) f.st(k, neg(f.ld(k)));   // conj: x < 0
}

}  // namespace bls
#endif
