// Two-waves-per-SIMD Miller loop: the Fp12 accumulator ping-pongs between two
// HBM stores (every step reads one and writes the other) and each operation's
// Fp6 temporary (3 Fp2) lives in a 72 KiB LDS park per 256-lane block, so two
// blocks fit a CU.  Same arithmetic as miller_loop2_staged (staged.hpp: the
// one-wave loop on a 144 KiB LDS image): 9 Fp2 products per normalised -G2
// line, 3 products + 6 dot2 per key line, two Fp6 products per squaring.
//
// EXPERIMENTAL, not in the product library: measured on MI355X as a k_miller
// variant (CESS_MILLER_2W, two waves per SIMD, 708-832 B/lane scratch) at
// 178.3 ms per 1 M with the default scheduler and 186.8 with max-ilp, against
// 170.6 for the one-wave LDS loop (profiles/r03a_sweep.txt); correct on all 40
// GPU tests.  Kept here, cross-checked in host emulation
// (tests/test_hostemu.py::test_miller_pingpong_matches_inplace).
#pragma once
#include "../../cess_amd/csrc/bls/staged.hpp"

namespace bls {

// d <- f * (1 + c1 v + c4 v w) (a line normalised to c2 = 1); d distinct from
// f; t: 3-Fp2 temporary.  bb = f.c1 (c4 v) goes to t, d.c0 = aa + v bb with
// aa = f.c0 (1 + c1 v), d.c1 = (f.c0 + f.c1)(1 + (c1 + c4) v) - aa - bb with
// aa recovered as d.c0 - v bb.
template <class D, class S, class T>
CESS_HD void mul014_one_st(const D& d, const S& f, const fp2& c1, const fp2& c4, const T& t) {
  t.st(0, mul(f.ld(5), c4));   // bb = (xi c4 f12, c4 f10, c4 f11); t0 holds c4 f12 (xi applied on use)
  CESS_MEMBAR();
  t.st(1, mul(f.ld(3), c4));
  CESS_MEMBAR();
  t.st(2, mul(f.ld(4), c4));
  CESS_MEMBAR();
  // d.c0 = (f00 + xi (c1 f02) + xi bb2, f01 + c1 f00 + bb0, f02 + c1 f01 + bb1)
  d.st(0, add(f.ld(0), mul_nr(add(mul(f.ld(2), c1), t.ld(2)))));
  CESS_MEMBAR();
  d.st(1, add(add(f.ld(1), mul(f.ld(0), c1)), mul_nr(t.ld(0))));
  CESS_MEMBAR();
  d.st(2, add(add(f.ld(2), mul(f.ld(1), c1)), t.ld(1)));
  CESS_MEMBAR();
  const fp2 e = add(c1, c4);
  // g = f.c0 + f.c1; d.c1_j = (g (1 + e v))_j - aa_j - bb_j
  {
    const fp2 x = add(add(f.ld(0), f.ld(3)), mul_nr(mul(add_nr(f.ld(2), f.ld(5)), e)));
    // aa0 + bb0 = (d0 - xi t2) + xi t0
    d.st(3, sub(sub(x, d.ld(0)), mul_nr(sub(t.ld(0), t.ld(2)))));
  }
  CESS_MEMBAR();
  {
    const fp2 x = add(add(f.ld(1), f.ld(4)), mul(add_nr(f.ld(0), f.ld(3)), e));
    // aa1 + bb1 = (d1 - xi t0) + t1
    d.st(4, sub(add(sub(x, d.ld(1)), mul_nr(t.ld(0))), t.ld(1)));
  }
  CESS_MEMBAR();
  {
    const fp2 x = add(add(f.ld(2), f.ld(5)), mul(add_nr(f.ld(1), f.ld(4)), e));
    // aa2 + bb2 = (d2 - t1) + t2
    d.st(5, sub(add(sub(x, d.ld(2)), t.ld(1)), t.ld(2)));
  }
}

// d <- f * (c2 + c1 v + c4 v w) (Fp12::mul_by_014 with the key's line); aa and
// the d.c1 products as dot2 (one reduction per component), bb in t.
template <class D, class S, class T>
CESS_HD void mul014_st(const D& d, const S& f, const fp2& c2, const fp2& c1, const fp2& c4, const T& t) {
  t.st(0, mul(f.ld(5), c4));
  CESS_MEMBAR();
  t.st(1, mul(f.ld(3), c4));
  CESS_MEMBAR();
  t.st(2, mul(f.ld(4), c4));
  CESS_MEMBAR();
  {
    const fp2 xc1 = mul_nr(c1);
    d.st(0, add(dot2(f.ld(0), c2, f.ld(2), xc1), mul_nr(t.ld(2))));
  }
  CESS_MEMBAR();
  d.st(1, add(dot2(f.ld(1), c2, f.ld(0), c1), mul_nr(t.ld(0))));
  CESS_MEMBAR();
  d.st(2, add(dot2(f.ld(2), c2, f.ld(1), c1), t.ld(1)));
  CESS_MEMBAR();
  const fp2 e = add(c1, c4);
  {
    const fp2 xe = mul_nr(e);
    const fp2 x = dot2(add_nr(f.ld(0), f.ld(3)), c2, add_nr(f.ld(2), f.ld(5)), xe);
    d.st(3, sub(sub(x, d.ld(0)), mul_nr(sub(t.ld(0), t.ld(2)))));
  }
  CESS_MEMBAR();
  {
    const fp2 x = dot2(add_nr(f.ld(1), f.ld(4)), c2, add_nr(f.ld(0), f.ld(3)), e);
    d.st(4, sub(add(sub(x, d.ld(1)), mul_nr(t.ld(0))), t.ld(1)));
  }
  CESS_MEMBAR();
  {
    const fp2 x = dot2(add_nr(f.ld(2), f.ld(5)), c2, add_nr(f.ld(1), f.ld(4)), e);
    d.st(5, sub(add(sub(x, d.ld(2)), t.ld(1)), t.ld(2)));
  }
}

// d <- f^2 (complex squaring) with streamed operands; d distinct from f.
// ab = f.c0 f.c1 goes to t; d.c0 = (f.c0 + f.c1)(f.c0 + v f.c1) - ab - v ab,
// d.c1 = 2 ab.
template <class D, class S, class T>
CESS_HD void sqr12_st(const D& d, const S& f, const T& t) {
  mul6_stream([&](int j) { return f.ld(j); }, [&](int j) { return f.ld(3 + j); },
              [&](int j, const fp2& v) { t.st(j, v); });
  mul6_stream([&](int j) { return add_nr(f.ld(j), f.ld(3 + j)); },
              [&](int j) { return j == 0 ? add_nr(f.ld(0), mul_nr(f.ld(5))) : add_nr(f.ld(j), f.ld(2 + j)); },
              [&](int j, const fp2& x) {
                const fp2 vab = j == 0 ? mul_nr(t.ld(2)) : t.ld(j - 1);
                d.st(j, sub(sub(x, t.ld(j)), vab));
              });
#pragma unroll 1
  for (int j = 0; j < 3; j++) d.st(3 + j, dbl(t.ld(j)));
}

// The two-pair Miller loop on stores fa (initial accumulator) and fb; returns
// the index (0: fa, 1: fb) of the store holding the result.  mk(w) builds the
// store of index w for this lane.
template <class MK, class T, class Pt, class Src>
CESS_HD int miller_loop2_pp(MK&& mk, const T& t, bool use0, bool use1, Pt&& pt, Src&& src) {
  set_one12(mk(0));
  int cur = 0;
#pragma unroll 1
  for (int s = 0; s < N_COEFFS; s++) {
    if (use0) {
      const coeff3 k = src(0, s);
      const g1a p = pt(0);
      mul014_one_st(mk(cur ^ 1), mk(cur), mul_fp(k.c1, p.x), mul_fp(k.c0, p.y), t);
      cur ^= 1;
    }
    CESS_MEMBAR();
    if (use1) {
      const coeff3 k = src(1, s);
      const g1a p = pt(1);
      mul014_st(mk(cur ^ 1), mk(cur), k.c2, mul_fp(k.c1, p.x), mul_fp(k.c0, p.y), t);
      cur ^= 1;
    }
    CESS_MEMBAR();
    if (square_after_step(s)) {
      sqr12_st(mk(cur ^ 1), mk(cur), t);
      cur ^= 1;
    }
    CESS_MEMBAR();
  }
  conj12(mk(cur));   // x < 0
  return cur;
}

}  // namespace bls
