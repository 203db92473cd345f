// Staged Fp12 arithmetic: the 576-byte Fp12 operands of the Miller loop and of
// the final exponentiation live OUTSIDE the register file -- in an LDS column
// (the hot accumulator) or in an HBM slot (cold temporaries of the final
// exponentiation) -- and every operation streams its Fp2 pieces in, computes in
// VGPRs, and writes the result back in place.
//
// Why (MI355X, one signature per lane): an Fp12 is 144 dwords; a value-based
// Fp12 multiply keeps ~4 of them live, which overflows the 256 arch VGPRs + 256
// AGPRs and spills to scratch (measured: 2.2 KB/lane in the Miller loop,
// 8.9 KB/lane in the final exponentiation, 30-34 % of wave cycles waiting on
// those spills).  With the accumulator in LDS (144 dwords x 256 lanes = 144 KiB
// of the CU's 160 KiB) the register working set is one Fp12 operation's
// temporaries only.
//
// Replaces bls12_381 0.7.1's Fp12 Miller loop / final exponentiation called at
// utils/verify-bls-signatures/src/lib.rs:90-95.
//
// Store concept: `fp2 ld(int k) const` / `void st(int k, const fp2&)`, with
// k = 3*i + j addressing coefficient c_i.c_j of (c0 + c1 w), c_i = (c_i.c0 +
// c_i.c1 v + c_i.c2 v^2).  Word w of the 144-word image = limb (w % 12) of Fp
// component ((w / 12) % 2) of fp2 (w / 24); rows of 4 words are uint4.
#pragma once
#include "pairing.hpp"
#include "diag.hpp"

namespace bls {

#if !defined(CESS_HOSTEMU)
// The lane's id within its wave, recomputed at every call (v_mbcnt_lo/hi in a
// volatile asm, so LLVM can neither merge two calls nor hoist one): the
// per-lane part of a store address then lives for one access only.  With the
// address kept in a register for the whole kernel, k_miller's allocator
// spilled it and reloaded it from scratch -- one serialised scratch round trip
// (s_waitcnt vmcnt(0)) in front of every LDS access, ~110 per Miller step --
// and k_final did the same with the 64-bit HBM slot addresses.
CESS_HD uint32_t lane_fresh() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// first thread (block-relative) of the calling lane's wave, wave-uniform (SGPR)
CESS_HD uint32_t wave_first_thread() { return __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u); }

// One lane's Fp12 in an LDS image F[36][256] (uint4 rows; lane t owns column t,
// so a wave reads 16 consecutive bytes per lane: conflict-free ds_read_b128).
// t = w0 + lane_fresh(): w0 is the wave's first thread (uniform).
struct LdsF12 {
  uint4 (*F)[256];
  uint32_t w0;
  CESS_HD fp2 ld(int k) const {
    const uint32_t t = w0 + lane_fresh();
    fp2 r;
#pragma unroll
    for (int q = 0; q < 6; q++) {
      uint4 x = F[6 * k + q][t];
      fp& d = q < 3 ? r.c0 : r.c1;
      const int o = 4 * (q % 3);
      d.v[o] = x.x, d.v[o + 1] = x.y, d.v[o + 2] = x.z, d.v[o + 3] = x.w;
    }
    return r;
  }
  CESS_HD void st(int k, const fp2& a) const {
    const uint32_t t = w0 + lane_fresh();
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const fp& s = q < 3 ? a.c0 : a.c1;
      const int o = 4 * (q % 3);
      F[6 * k + q][t] = make_uint4(s.v[o], s.v[o + 1], s.v[o + 2], s.v[o + 3]);
    }
  }
};

// One lane's Fp12 in an HBM slot, addressed like LdsF12: `base` already points
// at the wave's first lane (uniform), the lane id is recomputed per access
// (k_final: scratch 2,012 -> 800 B/lane, 158.0 -> 147.0 ms per 1 M,
// profiles/round3_n_sweep.txt).  (Uniform row bases + a 32-bit lane byte
// offset, global_load voffset s[base], measured no better: 147.8 ms.)
struct GlobF12W {
  uint4* base;
  uint64_t stride;
  CESS_HD fp2 ld(int k) const {
    const uint32_t l = lane_fresh();
    fp2 r;
#pragma unroll
    for (int q = 0; q < 6; q++) {
      uint4 x = base[(uint64_t)(6 * k + q) * stride + l];
      fp& d = q < 3 ? r.c0 : r.c1;
      const int o = 4 * (q % 3);
      d.v[o] = x.x, d.v[o + 1] = x.y, d.v[o + 2] = x.z, d.v[o + 3] = x.w;
    }
    return r;
  }
  CESS_HD void st(int k, const fp2& a) const {
    const uint32_t l = lane_fresh();
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const fp& s = q < 3 ? a.c0 : a.c1;
      const int o = 4 * (q % 3);
      const uint4 v = make_uint4(s.v[o], s.v[o + 1], s.v[o + 2], s.v[o + 3]);
      base[(uint64_t)(6 * k + q) * stride + l] = v;
    }
  }
};

// One lane's Fp12 in an HBM slot: 36 uint4 rows of `stride` lanes (SoA,
// coalesced 1 KiB per wave per row).
struct GlobF12 {
  uint4* base;
  uint64_t stride;
  uint32_t i;
  CESS_HD fp2 ld(int k) const {
    fp2 r;
#pragma unroll
    for (int q = 0; q < 6; q++) {
      uint4 x = base[(uint64_t)(6 * k + q) * stride + i];
      fp& d = q < 3 ? r.c0 : r.c1;
      const int o = 4 * (q % 3);
      d.v[o] = x.x, d.v[o + 1] = x.y, d.v[o + 2] = x.z, d.v[o + 3] = x.w;
    }
    return r;
  }
  CESS_HD void st(int k, const fp2& a) const {
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const fp& s = q < 3 ? a.c0 : a.c1;
      const int o = 4 * (q % 3);
      base[(uint64_t)(6 * k + q) * stride + i] = make_uint4(s.v[o], s.v[o + 1], s.v[o + 2], s.v[o + 3]);
    }
  }
};
#endif

// Plain-memory store (host emulation; also the Gt output path)
struct ArrF12 {
  fp12* p;
  CESS_HD fp2 ld(int k) const { return (&p->c0.c0)[k]; }
  CESS_HD void st(int k, const fp2& a) const { (&p->c0.c0)[k] = a; }
};

template <class S>
CESS_HD fp6 ld6(const S& s, int h) {
  return {s.ld(3 * h), s.ld(3 * h + 1), s.ld(3 * h + 2)};
}
template <class S>
CESS_HD void st6(const S& s, int h, const fp6& a) {
  s.st(3 * h, a.c0);
  s.st(3 * h + 1, a.c1);
  s.st(3 * h + 2, a.c2);
}
template <class D, class S>
CESS_HD void copy12(const D& d, const S& s) {
#pragma unroll 1
  for (int k = 0; k < 6; k++) d.st(k, s.ld(k));
}
template <class S>
CESS_HD void set_one12(const S& s) {
  s.st(0, fp2_one());
#pragma unroll 1
  for (int k = 1; k < 6; k++) s.st(k, fp2_zero());
}
template <class S>
CESS_HD void conj12(const S& s) {
#pragma unroll 1
  for (int k = 3; k < 6; k++) s.st(k, neg(s.ld(k)));
}
template <class S>
CESS_HD bool is_one12(const S& s) {
  bool r = eq(s.ld(0), fp2_one());
#pragma unroll 1
  for (int k = 1; k < 6; k++) r = r && is_zero(s.ld(k));
  return r;
}

// a == conj(b), i.e. a b == 1 for b in the cyclotomic subgroup
template <class A, class B>
CESS_HD bool is_conj12(const A& a, const B& b) {
  bool r = true;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r = r && eq(a.ld(k), k < 3 ? b.ld(k) : neg(b.ld(k)));
  return r;
}

#ifndef CESS_SQR12_LOOP
#define CESS_SQR12_LOOP 0
#endif
#ifndef CESS_MUL014_LOOP
#define CESS_MUL014_LOOP 0
#endif
// f <- f^2  (complex squaring: 2 Fp6 multiplies)
template <class S>
CESS_HD void sqr12(const S& f) {
#if CESS_SQR12_LOOP
  // the two Fp6 products share ONE copy of the code (a two-pass loop over
  // operands chosen per pass): half the instruction bytes of the squaring, so
  // more of k_miller's step body stays in the instruction cache
  fp6 ab;
#pragma unroll 1
  for (int it = 0; it < 2; it++) {
    fp6 x, y;
    {
      const fp6 a0 = ld6(f, 0), a1 = ld6(f, 1);
      if (it) {
        x = add_nr(a0, a1);
        y = add_nr(a0, mul_v(a1));
      } else {
        x = a0;
        y = a1;
      }
    }
    const fp6 r = mul(x, y);
    CESS_MEMBAR();
    if (it) {
      st6(f, 0, sub(sub(r, ab), mul_v(ab)));
      st6(f, 1, dbl(ab));
    } else {
      ab = r;
    }
  }
#else
  fp6 ab;
  {
    fp6 a0 = ld6(f, 0), a1 = ld6(f, 1);
    ab = mul(a0, a1);
  }
  CESS_MEMBAR();
  fp6 x;
  {
    fp6 a0 = ld6(f, 0), a1 = ld6(f, 1);
    x = mul(add_nr(a0, a1), add_nr(a0, mul_v(a1)));
  }
  st6(f, 0, sub(sub(x, ab), mul_v(ab)));
  st6(f, 1, dbl(ab));
#endif
}

// a * (b0 + b1 v) for an Fp6 `a` in store half h (coefficients fetched per
// use): each output coefficient is a sum of two Fp2 products, taken as one
// dot2 (one reduction per component): (a0 b0 + a2 (xi b1), a0 b1 + a1 b0,
// a1 b1 + a2 b0) -- 3 x 1,568 mads against mul_by_01's 5 x 980 plus the
// reductions and additions of its Karatsuba recombination (k_miller 179.6 vs
// 184.4 ms per 1 M, profiles/r02g_sweep.txt).  xb1 = xi * b1.
template <class S>
CESS_HD fp6 mul_by_01_dot(const S& f, int h, const fp2& b0, const fp2& b1, const fp2& xb1) {
  fp6 r;
  r.c0 = dot2(f.ld(3 * h), b0, f.ld(3 * h + 2), xb1);
  CESS_MEMBAR();
  r.c1 = dot2(f.ld(3 * h), b1, f.ld(3 * h + 1), b0);
  CESS_MEMBAR();
  r.c2 = dot2(f.ld(3 * h + 1), b1, f.ld(3 * h + 2), b0);
  return r;
}

// f <- f * (c0 + c1 v + c4 v w)   (bls12_381 Fp12::mul_by_014, in place)
template <class S>
CESS_HD void mul014(const S& f, const fp2& c0, const fp2& c1, const fp2& c4) {
#if CESS_MUL014_LOOP
  // aa = f0 (c0 + c1 v) and t = (f0 + f1)(c0 + (c1 + c4) v) share one copy
  // of mul_by_01_dot (a two-pass loop: half 0, then half 1 after f.c1 holds
  // f0 + f1)
  fp6 bb = mul_by_1(ld6(f, 1), c4);
  CESS_MEMBAR();
  fp6 aa;
  const fp2 d = add(c1, c4);
#pragma unroll 1
  for (int it = 0; it < 2; it++) {
    const fp2 b1 = it ? d : c1;
    const fp6 r = mul_by_01_dot(f, it, c0, b1, mul_nr(b1));
    CESS_MEMBAR();
    if (it) {
      st6(f, 1, sub(r, add(aa, bb)));
    } else {
      aa = r;
      {
        fp6 s = add(ld6(f, 0), ld6(f, 1));
        st6(f, 1, s);                    // f.c1 <- a0 + a1 (consumed by pass 1)
      }
      st6(f, 0, add(mul_v(bb), aa));
    }
  }
#else
  fp6 bb = mul_by_1(ld6(f, 1), c4);
  CESS_MEMBAR();
  fp6 aa = mul_by_01_dot(f, 0, c0, c1, mul_nr(c1));
  CESS_MEMBAR();
  {
    fp6 s = add(ld6(f, 0), ld6(f, 1));
    st6(f, 1, s);                    // f.c1 <- a0 + a1 (consumed below)
  }
  st6(f, 0, add(mul_v(bb), aa));
  fp6 u = add(aa, bb);
  CESS_MEMBAR();
  const fp2 d = add(c1, c4);
  fp6 t = mul_by_01_dot(f, 1, c0, d, mul_nr(d));
  st6(f, 1, sub(t, u));
#endif
}

// a * (1 + b1 v): mul_by_01 with b0 = 1 (a reduced)
CESS_HD fp6 mul_by_01_one(const fp6& a, const fp2& b1) {
#if CESS_MUL2
  fp2 p2, p0;
  mul2(a.c2, b1, a.c0, b1, p2, p0);
  return {add(a.c0, mul_nr(p2)), add(a.c1, p0), add(a.c2, mul(a.c1, b1))};
#else
  return {add(a.c0, mul_nr(mul(a.c2, b1))), add(a.c1, mul(a.c0, b1)), add(a.c2, mul(a.c1, b1))};
#endif
}

// f <- f * (1 + c1 v + c4 v w): mul014 for a line normalised to c0 = 1
// (pairing.hpp normalize_line), 9 Fp2 products instead of 13
template <class S>
CESS_HD void mul014_one(const S& f, const fp2& c1, const fp2& c4) {
#if CESS_MUL014_LOOP
  fp6 bb = mul_by_1(ld6(f, 1), c4);
  CESS_MEMBAR();
  fp6 aa;
  const fp2 d = add(c1, c4);
#pragma unroll 1
  for (int it = 0; it < 2; it++) {
    const fp6 r = mul_by_01_one(ld6(f, it), it ? d : c1);
    CESS_MEMBAR();
    if (it) {
      st6(f, 1, sub(r, add(aa, bb)));
    } else {
      aa = r;
      {
        fp6 s = add(ld6(f, 0), ld6(f, 1));
        st6(f, 1, s);                    // f.c1 <- a0 + a1 (consumed by pass 1)
      }
      st6(f, 0, add(mul_v(bb), aa));
    }
  }
#else
  fp6 bb = mul_by_1(ld6(f, 1), c4);
  CESS_MEMBAR();
  fp6 aa = mul_by_01_one(ld6(f, 0), c1);
  CESS_MEMBAR();
  {
    fp6 s = add(ld6(f, 0), ld6(f, 1));
    st6(f, 1, s);                    // f.c1 <- a0 + a1 (consumed below)
  }
  st6(f, 0, add(mul_v(bb), aa));
  fp6 u = add(aa, bb);
  CESS_MEMBAR();
  fp6 t = mul_by_01_one(ld6(f, 1), add(c1, c4));
  st6(f, 1, sub(t, u));
#endif
}

// f <- f * g  (Karatsuba over Fp6: 3 Fp6 multiplies)
template <class S, class G>
CESS_HD void mul12(const S& f, const G& g) {
  fp6 t0, t1;
  t0 = mul(ld6(f, 0), ld6(g, 0));
  CESS_MEMBAR();
  t1 = mul(ld6(f, 1), ld6(g, 1));
  CESS_MEMBAR();
  fp6 x = mul(add_nr(ld6(f, 0), ld6(f, 1)), add_nr(ld6(g, 0), ld6(g, 1)));
  st6(f, 1, sub(sub(x, t0), t1));
  st6(f, 0, add(t0, mul_v(t1)));
}

// Fp6 product a * b with the operands' Fp2 pieces fetched on demand (a(j),
// b(j): loaders, typically loads from a store) and each coefficient of the
// result handed to sink(j, c_j) as soon as it is complete.  Only the three
// diagonal products stay in registers (72 dwords); the value-based mul(fp6,
// fp6) keeps both 72-dword operands live as well, which spills at two waves
// per SIMD.  Loaders may return unreduced sums (< 4p); sums of two of them
// (< 8p) still satisfy mul()'s input bound.
// CESS_FE_PF (measurement variant): the next diagonal product's operands are
// loaded before the current product, so their HBM latency overlaps its mads
// (48 more live VGPRs).
#ifndef CESS_FE_PF
#define CESS_FE_PF 0
#endif
template <class LA, class LB, class SK>
CESS_HD void mul6_stream(LA&& a, LB&& b, SK&& sink) {
#if CESS_FE_PF
  fp2 pa = a(0), pb = b(0);
  fp2 qa = a(1), qb = b(1);
  const fp2 v0 = mul(pa, pb);
  CESS_MEMBAR();
  pa = a(2), pb = b(2);
  const fp2 v1 = mul(qa, qb);
  CESS_MEMBAR();
  const fp2 v2 = mul(pa, pb);
  CESS_MEMBAR();
#else
  const fp2 v0 = mul(a(0), b(0));
  CESS_MEMBAR();
  const fp2 v1 = mul(a(1), b(1));
  CESS_MEMBAR();
  const fp2 v2 = mul(a(2), b(2));
  CESS_MEMBAR();
#endif
  sink(0, add(mul_nr(sub(sub(mul(add_nr(a(1), a(2)), add_nr(b(1), b(2))), v1), v2)), v0));
  CESS_MEMBAR();
  sink(1, add(sub(sub(mul(add_nr(a(0), a(1)), add_nr(b(0), b(1))), v0), v1), mul_nr(v2)));
  CESS_MEMBAR();
  sink(2, add(sub(sub(mul(add_nr(a(0), a(2)), add_nr(b(0), b(2))), v0), v2), v1));
  CESS_MEMBAR();
}

// d <- f * g (Karatsuba over Fp6) with every operand streamed: d must be a
// store distinct from f and g; t is a one-Fp6 temporary store (3 Fp2, indices
// 0-2).  t0 = f0 g0 goes to t, t1 = f1 g1 to d.c1, then d.c0 = t0 + v t1 and
// d.c1 = (f0 + f1)(g0 + g1) - t0 - t1 in place.  (Parking the diagonal products
// in an HBM slot instead of registers measured slower: k_final 186 vs 173 ms
// per 1 M, profiles/r02q_sweep.txt.)
template <class D, class S, class G, class T>
CESS_HD void mul12_stream(const D& d, const S& f, const G& g, const T& t) {
  mul6_stream([&](int j) { return f.ld(j); }, [&](int j) { return g.ld(j); },
              [&](int j, const fp2& v) { t.st(j, v); });
  mul6_stream([&](int j) { return f.ld(3 + j); }, [&](int j) { return g.ld(3 + j); },
              [&](int j, const fp2& v) { d.st(3 + j, v); });
  d.st(0, add(t.ld(0), mul_nr(d.ld(5))));
  d.st(1, add(t.ld(1), d.ld(3)));
  d.st(2, add(t.ld(2), d.ld(4)));
  CESS_MEMBAR();
  mul6_stream([&](int j) { return add_nr(f.ld(j), f.ld(3 + j)); },
              [&](int j) { return add_nr(g.ld(j), g.ld(3 + j)); },
              [&](int j, const fp2& x) { d.st(3 + j, sub(sub(x, t.ld(j)), d.ld(3 + j))); });
}

// mul12_stream with the park `pk` (3 Fp2, LDS) caching each Fp6 product's
// FIRST operand (f0, f1, then f0 + f1) instead of holding the temporary t0
// (now the store `t`, an HBM slot): every a(j) of mul6_stream is an LDS read,
// so f is read from HBM 12 times (Fp2) per product instead of 36 -- 60 Fp2
// loads + 12 stores against 78 + 9 (k_final's HBM traffic is its clock:
// the same instruction stream with L2-resident slots runs 2.36 instead of
// 2.13 GHz, profiles/round5_v_diag_l2.txt).
#ifndef CESS_FE_APARK
#define CESS_FE_APARK 1
#endif
template <class D, class S, class G, class T, class P>
CESS_HD void mul12_stream_ap(const D& d, const S& f, const G& g, const T& t, const P& pk) {
#pragma unroll 1
  for (int j = 0; j < 3; j++) pk.st(j, f.ld(j));
  CESS_MEMBAR();
  mul6_stream([&](int j) { return pk.ld(j); }, [&](int j) { return g.ld(j); },
              [&](int j, const fp2& v) { t.st(j, v); });
  CESS_MEMBAR();
#pragma unroll 1
  for (int j = 0; j < 3; j++) pk.st(j, f.ld(3 + j));
  CESS_MEMBAR();
  mul6_stream([&](int j) { return pk.ld(j); }, [&](int j) { return g.ld(3 + j); },
              [&](int j, const fp2& v) { d.st(3 + j, v); });
  d.st(0, add(t.ld(0), mul_nr(d.ld(5))));
  d.st(1, add(t.ld(1), d.ld(3)));
  d.st(2, add(t.ld(2), d.ld(4)));
  CESS_MEMBAR();
  // unreduced sums (< 4p) in the park: mul6_stream's own sums of two of them
  // stay below 8p, mul()'s input bound (as in mul12_stream)
#pragma unroll 1
  for (int j = 0; j < 3; j++) pk.st(j, add_nr(f.ld(j), f.ld(3 + j)));
  CESS_MEMBAR();
  mul6_stream([&](int j) { return pk.ld(j); }, [&](int j) { return add_nr(g.ld(j), g.ld(3 + j)); },
              [&](int j, const fp2& x) { d.st(3 + j, sub(sub(x, t.ld(j)), d.ld(3 + j))); });
}

// f <- f^2 for f in the cyclotomic subgroup (Granger-Scott, eprint 2009/565)
template <class S>
CESS_HD void cycsq12(const S& f) {
  // (z0,z1) = (c0.c0, c1.c1)
  {
    fp2 z0 = f.ld(0), z1 = f.ld(4), t0, t1;
    fp4_square(t0, t1, z0, z1);
    f.st(0, add(dbl(sub(t0, z0)), t0));
    f.st(4, add(dbl(add(t1, z1)), t1));
  }
  CESS_MEMBAR();
  // (z2,z3) = (c1.c0, c0.c2), (z4,z5) = (c0.c1, c1.c2)
  fp2 t0, t1, t2, t3;
  fp4_square(t0, t1, f.ld(3), f.ld(2));
  fp4_square(t2, t3, f.ld(1), f.ld(5));
  f.st(1, add(dbl(sub(t0, f.ld(1))), t0));
  f.st(5, add(dbl(add(t1, f.ld(5))), t1));
  fp2 n3 = mul_nr(t3);
  f.st(3, add(dbl(add(n3, f.ld(3))), n3));
  f.st(2, add(dbl(sub(t2, f.ld(2))), t2));
}

// f <- f^(p^k), k = 1, 2, 3.  w-basis index i of store index k': c0.c0=0,
// c1.c0=1, c0.c1=2, c1.c1=3, c0.c2=4, c1.c2=5 (field.hpp frobenius).
template <class S>
CESS_HD void frob12(const S& f, int k) {
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int i = (s % 3) * 2 + s / 3;
    fp2 y = f.ld(s);
    if (k & 1) y = conj(y);
    if (i) y = mul(y, frob_coeff(k, i));
    f.st(s, y);
  }
}

// f <- f^-1
template <class S>
CESS_HD void inv12(const S& f) {
  fp6 t;
  {
    fp6 a0 = ld6(f, 0), a1 = ld6(f, 1);
    t = sub(sqr(a0), mul_v(sqr(a1)));
  }
  t = inv(t);
  CESS_MEMBAR();
  fp6 a0 = ld6(f, 0);
  st6(f, 0, mul(a0, t));
  fp6 a1 = ld6(f, 1);
  st6(f, 1, neg(mul(a1, t)));
}

// d <- f^-1 with every Fp6 operand streamed (FE_INV): d distinct from f, t a
// 3-Fp2 temporary store (the LDS park).  f = a0 + a1 w: t = a0^2 - v a1^2,
// t^-1 = (c0, c1, c2) / (t0 c0 + xi (t2 c1 + t1 c2)) with c0 = t0^2 - xi t1 t2,
// c1 = xi t2^2 - t0 t1, c2 = t1^2 - t0 t2, then d = (a0 t^-1, -a1 t^-1).  The
// value-based inv12 above keeps a0, a1 and the squares' temporaries live at
// once: k_final's largest spill region (575 of its 653 scratch accesses).
template <class D, class S, class T>
CESS_HD void inv12_stream(const D& d, const S& f, const T& t) {
  mul6_stream([&](int j) { return f.ld(j); }, [&](int j) { return f.ld(j); }, [&](int j, const fp2& v) { d.st(j, v); });
  mul6_stream([&](int j) { return f.ld(3 + j); }, [&](int j) { return f.ld(3 + j); },
              [&](int j, const fp2& v) { d.st(3 + j, v); });
  t.st(0, sub(d.ld(0), mul_nr(d.ld(5))));   // a0^2 - v a1^2, v (x0, x1, x2) = (xi x2, x0, x1)
  t.st(1, sub(d.ld(1), d.ld(3)));
  t.st(2, sub(d.ld(2), d.ld(4)));
  CESS_MEMBAR();
  d.st(0, sub(sqr(t.ld(0)), mul_nr(mul(t.ld(1), t.ld(2)))));
  CESS_MEMBAR();
  d.st(1, sub(mul_nr(sqr(t.ld(2))), mul(t.ld(0), t.ld(1))));
  CESS_MEMBAR();
  d.st(2, sub(sqr(t.ld(1)), mul(t.ld(0), t.ld(2))));
  CESS_MEMBAR();
  const fp2 den = inv(add(mul(t.ld(0), d.ld(0)), mul_nr(add(mul(t.ld(2), d.ld(1)), mul(t.ld(1), d.ld(2))))));
  CESS_MEMBAR();
#pragma unroll 1
  for (int j = 0; j < 3; j++) t.st(j, mul(d.ld(j), den));
  CESS_MEMBAR();
  mul6_stream([&](int j) { return f.ld(j); }, [&](int j) { return t.ld(j); }, [&](int j, const fp2& v) { d.st(j, v); });
  mul6_stream([&](int j) { return f.ld(3 + j); }, [&](int j) { return t.ld(j); },
              [&](int j, const fp2& v) { d.st(3 + j, neg(v)); });
}

// ---------------------------------------------------------------------------
// Final exponentiation as a program over one in-place accumulator A and HBM
// slots (MillerLoopResult::final_exponentiation, A13).  Each opcode body exists
// once in the code object; the hard part's five cyclotomic exponentiations by
// x are spelled out as square runs and multiplies by the base.
// ---------------------------------------------------------------------------
enum FeOp : uint8_t { FE_LOAD, FE_STORE, FE_MUL, FE_SQN, FE_CONJ, FE_FROB, FE_INV, FE_CHAIN, FE_END };
// SL_TM: FE_MUL's Fp6 temporary when the park caches its first operand
// (CESS_FE_APARK)
enum FeSlot : uint8_t { SL_F = 0, SL_M, SL_T0, SL_T1, SL_T3, SL_T4, SL_T5, SL_T6,
                        SL_X0, SL_X1, SL_X2, SL_X3, SL_X4, SL_X5, SL_TM, SL_N };

// a^x (x = -0xd201000000010000) for a in slot s: |x| has bits 63, 62, 60, 57,
// 48, 16, so a^|x| = a^(2^63) a^(2^62) a^(2^60) a^(2^57) a^(2^48) a^(2^16).
// FE_CHAIN s runs the 63 squarings in Karabina's compressed form and leaves
// the six powers, decompressed with one Fp2 inversion, in slots X5..X0; five
// multiplies and the conjugation (x < 0) follow.
#define CESS_FE_CYCEXP(s) \
  {FE_CHAIN, s}, {FE_LOAD, SL_X5}, {FE_MUL, SL_X4}, {FE_MUL, SL_X3}, {FE_MUL, SL_X2}, {FE_MUL, SL_X1}, \
      {FE_MUL, SL_X0}, {FE_CONJ, 0}

// easy part: m = f^((p^6 - 1)(p^2 + 1)); hard part as in pairing.hpp
// final_exponentiation (t2 = m).  SL_T0 doubles as scratch in the easy part.
#define CESS_FE_BODY                                                                                              \
  {FE_LOAD, SL_F}, {FE_CONJ, 0}, {FE_STORE, SL_T0}, {FE_LOAD, SL_F}, {FE_INV, 0}, {FE_MUL, SL_T0},                 \
      {FE_STORE, SL_T0}, {FE_FROB, 2}, {FE_MUL, SL_T0}, {FE_STORE, SL_M},                                          \
      /* t1 = conj(cycsq(m)) */ {FE_SQN, 1}, {FE_CONJ, 0}, {FE_STORE, SL_T1},                                     \
      /* t3 = m^x */ CESS_FE_CYCEXP(SL_M), {FE_STORE, SL_T3},                                                      \
      /* t4 = cycsq(t3) */ {FE_SQN, 1}, {FE_STORE, SL_T4},                                                          \
      /* t5 = t1 * t3 */ {FE_LOAD, SL_T1}, {FE_MUL, SL_T3}, {FE_STORE, SL_T5},                                     \
      /* t1 = t5^x */ CESS_FE_CYCEXP(SL_T5), {FE_STORE, SL_T1},                                                    \
      /* t0 = t1^x */ CESS_FE_CYCEXP(SL_T1), {FE_STORE, SL_T0},                                                    \
      /* t6 = t0^x * t4 */ CESS_FE_CYCEXP(SL_T0), {FE_MUL, SL_T4}, {FE_STORE, SL_T6},                             \
      /* t4 = t6^x */ CESS_FE_CYCEXP(SL_T6), {FE_STORE, SL_T4},                                                    \
      /* t4 = t4 * conj(t5) * m */ {FE_LOAD, SL_T5}, {FE_CONJ, 0}, {FE_MUL, SL_M}, {FE_MUL, SL_T4},              \
      {FE_STORE, SL_T4},                                                                                           \
      /* t1 = frob3(t1 * m) */ {FE_LOAD, SL_T1}, {FE_MUL, SL_M}, {FE_FROB, 3}, {FE_STORE, SL_T1},                 \
      /* t6 = frob1(t6 * conj(m)) */ {FE_LOAD, SL_M}, {FE_CONJ, 0}, {FE_MUL, SL_T6}, {FE_FROB, 1},              \
      {FE_STORE, SL_T6},                                                                                           \
      /* t3 = frob2(t3 * t0) * t1 * t6 * t4 */ {FE_LOAD, SL_T3}, {FE_MUL, SL_T0}, {FE_FROB, 2}, {FE_MUL, SL_T1},  \
      {FE_MUL, SL_T6}
#define CESS_FE_PROGRAM CESS_FE_BODY, {FE_MUL, SL_T4}, {FE_END, 0}
// Verdict-only form (no Gt output): the result t3 * t4 is 1 iff t3 equals
// t4^-1 = conj(t4) (t4 is in the cyclotomic subgroup), so the last multiply
// becomes a comparison (is_conj12 of the accumulator and slot SL_T4).
#define CESS_FE_PROGRAM_VERIFY CESS_FE_BODY, {FE_END, 0}

// n cyclotomic squarings of acc (Granger-Scott formulas, as cyclotomic_square
// in field.hpp): pair (z0, z1) updates itself; the square of (z2, z3) updates
// z4, z5 and the square of (z4, z5) updates z2, z3, so the latter is taken
// first and its t3 parked while the former runs.  z0, z1 and that temporary
// are parked in the 3-Fp2 store `pk` (LDS in k_final), z4, z5 stay in the
// accumulator store `acc` (HBM in k_final) for the whole run, and only z2, z3
// live in registers: the register peak is one Fp4 square's working set plus
// three Fp2, which the two-waves-per-SIMD budget (256 VGPRs) nearly holds
// (57 scratch accesses per squaring, against 101 with z2..z5 in registers;
// same time, profiles/r02j_sweep.txt), for 4 Fp2 loads + 2 Fp2 stores of
// `acc` per squaring.
// store index: z0 = 0, z4 = 1, z3 = 2, z2 = 3, z1 = 4, z5 = 5
template <class A, class P>
CESS_HD void cyc_square_run(const A& acc, const P& pk, int n) {
  pk.st(0, acc.ld(0));
  pk.st(1, acc.ld(4));
  fp2 z2 = acc.ld(3), z3 = acc.ld(2);
#pragma unroll 1
  for (int r = 0; r < n; r++) {
    CESS_MEMBAR();
    {
      const fp2 a = pk.ld(0), b = pk.ld(1);
      fp2 t0, t1;
      fp4_square(t0, t1, a, b);
      pk.st(0, add(dbl(sub(t0, a)), t0));
      pk.st(1, add(dbl(add(t1, b)), t1));
    }
    CESS_MEMBAR();
    fp2 u0;
    {
      fp2 u1;
      fp4_square(u0, u1, acc.ld(1), acc.ld(5));   // (z4, z5)
      pk.st(2, u1);
    }
    CESS_MEMBAR();
    {
      fp2 t0, t1;
      fp4_square(t0, t1, z2, z3);
      acc.st(1, add(dbl(sub(t0, acc.ld(1))), t0));   // z4
      acc.st(5, add(dbl(add(t1, acc.ld(5))), t1));   // z5
    }
    CESS_MEMBAR();
    const fp2 n3 = mul_nr(pk.ld(2));
    z2 = add(dbl(add(n3, z2)), n3);
    z3 = add(dbl(sub(u0, z3)), u0);
  }
  CESS_MEMBAR();
  acc.st(0, pk.ld(0));
  acc.st(4, pk.ld(1));
  acc.st(3, z2);
  acc.st(2, z3);
}

// Karabina compressed squaring (eprint 2010/542) on (z2, z3, z4, z5) (store
// indices 3, 2, 1, 5; naming as cyc_square_run), which the square's (z2..z5)
// depend on alone:
//   z2' = 2 (z2 + 3 xi z4 z5),   z3' = 3 (z4^2 + xi z5^2) - 2 z3,
//   z4' = 3 (z2^2 + xi z3^2) - 2 z4,   z5' = 2 (z5 + 3 z2 z3),
// with z4^2 + xi z5^2 = (z4 + z5)(z4 + xi z5) - (1 + xi) z4 z5 (likewise z2, z3):
// four lazily reduced Fp2 products per squaring against Granger-Scott's nine
// Fp2 squarings.  The factor 3 of both products of a half rides in the digits
// of one operand (mul_scaled<3>), so b3 = 3 z4 z5 and t3 = 3 (z4 + z5)(z4 + xi
// z5) give 3 (z4^2 + xi z5^2) = t3 - b3 - xi b3 and 6 xi z4 z5 = 2 xi b3 with
// four Fp2 additions instead of seven; z4 + xi z5 is formed unreduced
// (add_xi_nr, < 6p: 3 (4p)(6p) < p R).  z2, z3 stay in registers, z4, z5 in
// the parking store `pk` (LDS in k_final, indices 0, 1), and the (z4, z5)
// half's two results stay in registers while the (z2, z3) half runs: the run
// touches no HBM (k_final 171.3 -> 160.8 ms per 1 M against z4, z5 in the HBM
// accumulator with the results parked in LDS, profiles/r02w_sweep.txt).
#ifndef CESS_KCYC_LOOP
#define CESS_KCYC_LOOP 0
#endif
template <class P>
CESS_HD void kcyc_run(const P& pk, fp2& z2, fp2& z3, int n) {
#if CESS_KCYC_LOOP
  // the two halves share ONE copy of their products (b3 = 3 x y and
  // t3 = 3 (x + y)(x + xi y)): a two-pass inner loop, (x, y) = (z4, z5) from
  // the park, then (z2, z3); half the loop body's instruction bytes
#pragma unroll 1
  for (int r = 0; r < n; r++) {
    fp2 u, v;
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
      CESS_MEMBAR();
      fp2 x, y;
      if (h) {
        x = z2;
        y = z3;
      } else {
        x = pk.ld(0);
        y = pk.ld(1);
      }
      const fp2 b3 = mul_scaled<3>(x, y);
      CESS_MEMBAR();
      const fp2 t3 = mul_scaled<3>(add_nr(x, y), add_xi_nr(x, y));
      const fp2 nb3 = mul_nr(b3);
      const fp2 w = sub(sub(t3, b3), nb3);   // 3 (x^2 + xi y^2)
      if (h) {
        pk.st(0, sub(w, dbl(pk.ld(0))));
        pk.st(1, dbl(add(pk.ld(1), b3)));
      } else {
        u = w;
        v = dbl(nb3);   // 6 xi z4 z5
      }
    }
    CESS_MEMBAR();
    z2 = add(dbl(z2), v);
    z3 = sub(u, dbl(z3));
  }
#else
#pragma unroll 1
  for (int r = 0; r < n; r++) {
    CESS_MEMBAR();
    fp2 u, v;
    {
      const fp2 b3 = mul_scaled<3>(pk.ld(0), pk.ld(1));
      CESS_MEMBAR();
      const fp2 t3 = mul_scaled<3>(add_nr(pk.ld(0), pk.ld(1)), add_xi_nr(pk.ld(0), pk.ld(1)));
      const fp2 nb3 = mul_nr(b3);
      u = sub(sub(t3, b3), nb3);   // 3 (z4^2 + xi z5^2)
      v = dbl(nb3);                // 6 xi z4 z5
    }
    CESS_MEMBAR();
    {
      const fp2 b3 = mul_scaled<3>(z2, z3);
      CESS_MEMBAR();
      const fp2 t3 = mul_scaled<3>(add_nr(z2, z3), add_xi_nr(z2, z3));
      pk.st(0, sub(sub(sub(t3, b3), mul_nr(b3)), dbl(pk.ld(0))));
      pk.st(1, dbl(add(pk.ld(1), b3)));
    }
    CESS_MEMBAR();
    z2 = add(dbl(z2), v);
    z3 = sub(u, dbl(z3));
  }
#endif
}

// numerator / denominator of z1 of a compressed cyclotomic element:
//   z2 != 0: z1 = (xi z5^2 + 3 z4^2 - 2 z3) / (4 z2);  z2 == 0: z1 = 2 z4 z5 / z3
// (den = 0, i.e. z2 = z3 = 0, cannot be decompressed: the caller falls back)
CESS_HD void cyc_z1_frac(const fp2& z2, const fp2& z3, const fp2& z4, const fp2& z5, fp2& num, fp2& den) {
  num = sub(add(mul_nr(sqr(z5)), mul3(sqr(z4))), dbl(z3));
  den = dbl(dbl(z2));
  if (is_zero(z2)) {   // divergent, practically never taken
    num = dbl(mul(z4, z5));
    den = z3;
  }
}
// the denominator alone (backward pass of cyc_chain)
CESS_HD fp2 cyc_z1_den(const fp2& z2, const fp2& z3) { return is_zero(z2) ? z3 : dbl(dbl(z2)); }
// z0 = xi (2 z1^2 + z2 z5 - 3 z3 z4) + 1, with z2 z5 - 3 z3 z4 as one dot2
// (one reduction per component instead of two products and a subtraction)
CESS_HD fp2 cyc_z0(const fp2& z1, const fp2& z2, const fp2& z3, const fp2& z4, const fp2& z5) {
  return add(mul_nr(add(dbl(sqr(z1)), dot2(z2, z5, neg(mul3(z3)), z4))), fp2_one());
}

// FE_CHAIN: the powers a^(2^k), k = 16, 48, 57, 60, 62, 63, of the cyclotomic
// element a (store `base`) into the stores X(0..5): compressed squarings, then
// z1 of the compressed powers with ONE Fp2 inversion (Montgomery's
// simultaneous inversion: numerators parked in the z1 words, prefix products
// of the denominators in the z0 words; safegcd inversion), then z0.  A lane
// whose denominator vanishes (z2 = z3 = 0, e.g. a = 1 from an identity pair)
// redoes its chain with Granger-Scott squarings (divergent, rare).
// CESS_CHAIN_TAIL (default 1): the compressed run stops at a^(2^57); only
// a^(2^16), a^(2^48), a^(2^57) are decompressed, and a^(2^60), a^(2^62),
// a^(2^63) follow by 3 + 2 + 1 Granger-Scott squarings -- six uncompressed
// squarings for three decompressions (pair_fe.hpp pcyc_chain).
#ifndef CESS_CHAIN_TAIL
#define CESS_CHAIN_TAIL 1
#endif
template <class B, class XFn, class P, class DG = NoDiag>
CESS_HD void cyc_chain(const B& base, XFn&& X, const P& pk, DG* dg = nullptr) {
  constexpr int ND = CESS_CHAIN_TAIL ? 3 : 6;   // decompressed powers
  {
    pk.st(0, base.ld(1));   // z4, z5 of the running power
    pk.st(1, base.ld(5));
    fp2 z2 = base.ld(3), z3 = base.ld(2);
    int k = 0;
#pragma unroll 1
    for (int j = 0; j < ND; j++) {
      const int stop = j == 0 ? 16 : j == 1 ? 48 : j == 2 ? 57 : j == 3 ? 60 : j == 4 ? 62 : 63;
      if (dg) dg->template mark<0>();
      kcyc_run(pk, z2, z3, stop - k);
      if (dg) dg->template mark<3>();   // compressed squarings
      k = stop;
      CESS_MEMBAR();
      const auto x = X(j);
      x.st(3, z2);
      x.st(2, z3);
      x.st(1, pk.ld(0));
      x.st(5, pk.ld(1));
    }
  }
  CESS_MEMBAR();
  bool degen = false;
  fp2 prod = fp2_one();
#pragma unroll 1
  for (int j = 0; j < ND; j++) {
    const auto x = X(j);
    fp2 num, den;
    cyc_z1_frac(x.ld(3), x.ld(2), x.ld(1), x.ld(5), num, den);
    const bool z = is_zero(den);
    degen = degen || z;
    x.st(4, num);
    x.st(0, prod);   // product of the denominators before j
    prod = mul(prod, select(z, fp2_one(), den));
    CESS_MEMBAR();
  }
  fp2 iv = inv(prod);
#pragma unroll 1
  for (int j = ND - 1; j >= 0; j--) {
    const auto x = X(j);
    const fp2 den = cyc_z1_den(x.ld(3), x.ld(2));
    const fp2 ivj = mul(iv, x.ld(0));   // 1 / den_j
    iv = mul(iv, select(is_zero(den), fp2_one(), den));
    CESS_MEMBAR();
    const fp2 z1 = mul(x.ld(4), ivj);
    x.st(4, z1);
    CESS_MEMBAR();
    x.st(0, cyc_z0(z1, x.ld(3), x.ld(2), x.ld(1), x.ld(5)));
    CESS_MEMBAR();
  }
  if (degen) {   // Granger-Scott squarings with X(5) as the running power
    const auto w = X(5);
    copy12(w, base);
#pragma unroll 1
    for (int j = 0; j < 5; j++) {
      const int run = j == 0 ? 16 : j == 1 ? 32 : j == 2 ? 9 : j == 3 ? 3 : 2;
      cyc_square_run(w, pk, run);
      copy12(X(j), w);
    }
    cyc_square_run(w, pk, 1);
  }
#if CESS_CHAIN_TAIL
  else {   // X3..X5 from X2 = a^(2^57): 3, 2, 1 squarings
#pragma unroll 1
    for (int j = 3; j < 6; j++) {
      copy12(X(j), X(j - 1));
      cyc_square_run(X(j), pk, j == 3 ? 3 : j == 4 ? 2 : 1);
    }
  }
#endif
  if (dg) dg->template mark<4>();   // decompression (and the rare fallback)
}

// Run the program.  The accumulator alternates between the stores acc0 and
// acc1: FE_MUL writes the product of the current one and a slot into the other
// (mul12_stream, with the parking store `pk` as its Fp6 temporary); every other
// opcode works in place.  slot(s) returns the store of slot s (slot SL_F holds
// the Miller-loop output on entry); `pk` is also the parking store of
// cyc_square_run.  Returns the index (0/1) of the store holding the
// result.
template <class A, class SlotFn, class P, class DG = NoDiag>
CESS_HD int final_exp_staged(const A& acc0, const A& acc1, const uint8_t (*prog)[2], SlotFn&& slot, const P& pk,
                             DG* dg = nullptr) {
  int cur = 0;
#pragma unroll 1
  for (int pc = 0;; pc++) {
    const uint8_t op = prog[pc][0], arg = prog[pc][1];
    if (op == FE_END) break;
    const A& acc = cur ? acc1 : acc0;
    switch (op) {
      case FE_LOAD: copy12(acc, slot(arg)); break;
      case FE_STORE: copy12(slot(arg), acc); break;
      case FE_MUL:
#if CESS_FE_APARK
        mul12_stream_ap(cur ? acc0 : acc1, acc, slot(arg), slot(SL_TM), pk);
#else
        mul12_stream(cur ? acc0 : acc1, acc, slot(arg), pk);
#endif
        cur ^= 1;
        if (dg) dg->template mark<1>();
        break;
      case FE_SQN: cyc_square_run(acc, pk, arg); break;
      case FE_CONJ: conj12(acc); break;
      case FE_FROB: frob12(acc, arg); break;
      case FE_INV:   // into the other accumulator, like FE_MUL
        inv12_stream(cur ? acc0 : acc1, acc, pk);
        cur ^= 1;
        if (dg) dg->template mark<2>();
        break;
      case FE_CHAIN: cyc_chain(slot(arg), [&](int j) { return slot(SL_X0 + j); }, pk, dg); break;
      default: break;
    }
    if (dg) dg->template mark<0>();   // LOAD / STORE / SQN / CONJ / FROB (and the switch itself)
  }
  return cur;
}

// Miller loop for the two pairs of PublicKey::verify on an accumulator store:
// pair 0 = (sig, -G2) (uniform -G2 table, lines normalised to c2 = 1 by
// normalize_line), pair 1 = (H(m), pk).  use0/use1:
// the pair's points are both non-identity (identity terms contribute 1).
// pt(pair) yields the pair's affine G1 point; src(pair, step) its coefficients.
// norm1: pair 1's lines are normalised to c2 = 1 as well (a distinct-key table
// after normalize_lines); otherwise they take the general sparse product.
template <class S, class Pt, class Src, class DG = NoDiag>
CESS_HD void miller_loop2_staged(const S& f, bool use0, bool use1, Pt&& pt, Src&& src, bool norm1 = false,
                                 DG* dg = nullptr) {
  set_one12(f);
  if (dg) dg->template mark<5>();
#pragma unroll 1
  for (int s = 0; s < N_COEFFS; s++) {
    // pair 1 (H(m), key) first: with pair 0 (sig, -G2) second k_miller's
    // register allocation spills less (160.7 vs 163.2 ms per 1 M,
    // profiles/round3_h_sweep.txt)
#pragma unroll 1
    for (int pair = 0; pair < 2; pair++) {
      const int pr = 1 - pair;
      if (!(pr ? use1 : use0)) continue;
      coeff3 k = src(pr, s);
      g1a p = pt(pr);
      fp2 c1 = mul_fp(k.c1, p.x), c4 = mul_fp(k.c0, p.y);
      if (dg) {
        if (pr) dg->template mark<0>(); else dg->template mark<2>();
      }
      if (pr && !norm1)
        mul014(f, k.c2, c1, c4);
      else
        mul014_one(f, c1, c4);   // -G2 table (and normalised key tables): c2 = 1
      CESS_MEMBAR();
      if (dg) {
        if (pr) dg->template mark<1>(); else dg->template mark<3>();
      }
    }
    if (square_after_step(s)) sqr12(f);
    CESS_MEMBAR();
    if (dg) dg->template mark<4>();
  }
  conj12(f);   // x < 0
  if (dg) dg->template mark<5>();
}

// Miller loop over up to NP pairs with general lines sharing one accumulator
// (the distinct-key RLC's lane of records, k_miller_rr): the product of the
// pairs' Miller values, one squaring per step for all of them.  Bit j of `use`:
// pair j takes part; pt(j) yields its affine G1 point, src(j, step) its
// coefficients.
template <int NP, class S, class Pt, class Src>
CESS_HD void miller_loopn_staged(const S& f, uint32_t use, Pt&& pt, Src&& src) {
  set_one12(f);
#pragma unroll 1
  for (int s = 0; s < N_COEFFS; s++) {
#pragma unroll 1
    for (int j = 0; j < NP; j++) {
      if (!((use >> j) & 1u)) continue;
      const coeff3 k = src(j, s);
      const g1a p = pt(j);
      const fp2 c1 = mul_fp(k.c1, p.x), c4 = mul_fp(k.c0, p.y);
      mul014(f, k.c2, c1, c4);
      CESS_MEMBAR();
    }
    if (square_after_step(s)) sqr12(f);
    CESS_MEMBAR();
  }
  conj12(f);   // x < 0
}

}  // namespace bls
