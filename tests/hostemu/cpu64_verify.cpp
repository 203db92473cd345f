// CPU BASELINE ONLY (bench.py cpu_baseline leg, tests): verify_bls_signature
// (utils/verify-bls-signatures/src/lib.rs:243-247) restated for the host in
// the reference crate's own representation -- bls12_381 0.7.1's Fp is
// 6 x u64 Montgomery (R = 2^384) -- so the CPU number is not penalised by the
// GPU's 28-bit digit scheme.  Structure follows the
// crate's published algorithms as restated in oracle/bls_oracle.py:
//   * Fp: CIOS Montgomery product with unsigned __int128 and the "no final
//     carry" form (p's top limb < 2^63), Fp2 = Fp[u]/(u^2+1) with
//     Karatsuba, Fp6 = Fp2[v]/(v^3 - (u+1)), Fp12 = Fp6[w]/(w^2 - v);
//   * decode: ZCash flags, x < p, square roots by a^((p+1)/4) (Fp) and
//     eprint 2012/685 Alg. 9 (Fp2); G1 check phi(P) = -x^2 P, G2 check
//     psi(Q) = [x] Q (G1Affine / G2Affine::is_torsion_free);
//   * hash_to_g1: expand_message_xmd(SHA-256), RFC 9380 simplified SWU with
//     sqrt_ratio (App. F.2), 11-isogeny, h_eff = 1 - x (src/lib.rs:25-31);
//   * G2Prepared (Jacobian doubling / addition steps, oracle _doubling_step /
//     _addition_step), multi_miller_loop with mul_by_014, final
//     exponentiation with cyclotomic squarings (oracle final_exponentiation).
// Constants: cpu64_consts.h (generated from the oracle by gen_cpu64_consts.py).
// Never linked into the product library; test infrastructure like oracle/.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

namespace {

typedef unsigned __int128 u128;
struct Fp {
  uint64_t l[6];
};
struct Fp2 {
  Fp c0, c1;
};
#include "cpu64_consts.h"
struct Fp6 {
  Fp2 c0, c1, c2;
};
struct Fp12 {
  Fp6 c0, c1;
};

// ---------------------------------------------------------------- Fp -------
inline bool geq_p(const uint64_t* a) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > P_MOD.l[i]) return true;
    if (a[i] < P_MOD.l[i]) return false;
  }
  return true;
}
inline void sub_p(uint64_t* a) {
  uint64_t b = 0;
  for (int i = 0; i < 6; i++) {
    const u128 d = (u128)a[i] - P_MOD.l[i] - b;
    a[i] = (uint64_t)d;
    b = (uint64_t)(d >> 64) & 1;
  }
}
inline Fp fadd(const Fp& a, const Fp& b) {
  Fp r;
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    const u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (geq_p(r.l)) sub_p(r.l);
  return r;
}
inline Fp fsub(const Fp& a, const Fp& b) {
  Fp r;
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    const u128 d = (u128)a.l[i] - b.l[i] - br;
    r.l[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      const u128 s = (u128)r.l[i] + P_MOD.l[i] + c;
      r.l[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  return r;
}
inline bool fzero(const Fp& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3] | a.l[4] | a.l[5]) == 0; }
inline bool feq(const Fp& a, const Fp& b) { return memcmp(a.l, b.l, 48) == 0; }
inline Fp fneg(const Fp& a) { return fzero(a) ? a : fsub(Fp{{0, 0, 0, 0, 0, 0}}, a); }
inline Fp fdbl(const Fp& a) { return fadd(a, a); }

// CIOS Montgomery product, no final carry word (p's top limb < 2^63 - 1)
inline Fp fmul(const Fp& a, const Fp& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a.l[0] * b.l[i] + t[0];
    uint64_t A = (uint64_t)(s >> 64);
    t[0] = (uint64_t)s;
    const uint64_t m = t[0] * P_INV;
    u128 r = (u128)m * P_MOD.l[0] + t[0];
    uint64_t C = (uint64_t)(r >> 64);
    for (int j = 1; j < 6; j++) {
      s = (u128)a.l[j] * b.l[i] + t[j] + A;
      A = (uint64_t)(s >> 64);
      t[j] = (uint64_t)s;
      r = (u128)m * P_MOD.l[j] + t[j] + C;
      C = (uint64_t)(r >> 64);
      t[j - 1] = (uint64_t)r;
    }
    t[5] = C + A;
  }
  if (geq_p(t)) sub_p(t);
  Fp o;
  memcpy(o.l, t, 48);
  return o;
}
inline Fp fsqr(const Fp& a) { return fmul(a, a); }
Fp fpow(const Fp& a, const uint64_t* e, int nw) {
  Fp r = ONE_M;
  bool started = false;
  for (int w = nw - 1; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      if (started) r = fsqr(r);
      if ((e[w] >> b) & 1) {
        r = started ? fmul(r, a) : a;
        started = true;
      }
    }
  return r;
}
#define NW(a) (int)(sizeof(a) / sizeof((a)[0]))
inline Fp finv(const Fp& a) { return fpow(a, E_INV, NW(E_INV)); }
inline Fp to_mont(const Fp& raw) { return fmul(raw, R2_MOD); }
inline Fp from_mont(const Fp& a) { return fmul(a, Fp{{1, 0, 0, 0, 0, 0}}); }
// raw value > (p - 1) / 2
inline bool lex_largest(const Fp& a) {
  const Fp r = from_mont(a);
  // compare 2 r > p - 1, i.e. 2 r >= p (r < p)
  uint64_t d[6];
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    d[i] = (r.l[i] << 1) | c;
    c = r.l[i] >> 63;
  }
  return geq_p(d);
}
inline Fp from_be48(const uint8_t* b) {
  Fp r;
  for (int i = 0; i < 6; i++) {
    uint64_t w = 0;
    for (int k = 0; k < 8; k++) w = (w << 8) | b[8 * (5 - i) + k];
    r.l[i] = w;
  }
  return r;
}
inline void to_be48(const Fp& raw, uint8_t* b) {
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[8 * (5 - i) + k] = (uint8_t)(raw.l[i] >> (8 * (7 - k)));
}

// ---------------------------------------------------------------- Fp2 ------
inline Fp2 f2add(const Fp2& a, const Fp2& b) { return {fadd(a.c0, b.c0), fadd(a.c1, b.c1)}; }
inline Fp2 f2sub(const Fp2& a, const Fp2& b) { return {fsub(a.c0, b.c0), fsub(a.c1, b.c1)}; }
inline Fp2 f2neg(const Fp2& a) { return {fneg(a.c0), fneg(a.c1)}; }
inline Fp2 f2dbl(const Fp2& a) { return f2add(a, a); }
inline Fp2 f2conj(const Fp2& a) { return {a.c0, fneg(a.c1)}; }
inline bool f2zero(const Fp2& a) { return fzero(a.c0) && fzero(a.c1); }
inline bool f2eq(const Fp2& a, const Fp2& b) { return feq(a.c0, b.c0) && feq(a.c1, b.c1); }
inline Fp2 f2mul(const Fp2& a, const Fp2& b) {
  const Fp v0 = fmul(a.c0, b.c0), v1 = fmul(a.c1, b.c1);
  const Fp s = fmul(fadd(a.c0, a.c1), fadd(b.c0, b.c1));
  return {fsub(v0, v1), fsub(fsub(s, v0), v1)};
}
inline Fp2 f2sqr(const Fp2& a) {
  const Fp t = fmul(a.c0, a.c1);
  return {fmul(fadd(a.c0, a.c1), fsub(a.c0, a.c1)), fdbl(t)};
}
inline Fp2 f2mulfp(const Fp2& a, const Fp& s) { return {fmul(a.c0, s), fmul(a.c1, s)}; }
inline Fp2 f2nr(const Fp2& a) { return {fsub(a.c0, a.c1), fadd(a.c0, a.c1)}; }   // * (u + 1)
inline Fp2 f2inv(const Fp2& a) {
  const Fp t = finv(fadd(fsqr(a.c0), fsqr(a.c1)));
  return {fmul(a.c0, t), fneg(fmul(a.c1, t))};
}
Fp2 f2pow(const Fp2& a, const uint64_t* e, int nw) {
  Fp2 r{ONE_M, Fp{}};
  bool started = false;
  for (int w = nw - 1; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      if (started) r = f2sqr(r);
      if ((e[w] >> b) & 1) {
        r = started ? f2mul(r, a) : a;
        started = true;
      }
    }
  return r;
}
inline bool f2lex_largest(const Fp2& a) { return lex_largest(a.c1) || (fzero(a.c1) && lex_largest(a.c0)); }
// eprint 2012/685 Alg. 9 (p = 3 mod 4); false if a is not a square
bool f2sqrt(const Fp2& a, Fp2& out) {
  if (f2zero(a)) {
    out = a;
    return true;
  }
  const Fp2 a1 = f2pow(a, E_SQRT_RATIO, NW(E_SQRT_RATIO));   // a^((p-3)/4)
  const Fp2 alpha = f2mul(f2sqr(a1), a);
  const Fp2 x0 = f2mul(a1, a);
  const Fp2 minus_one{fneg(ONE_M), Fp{}};
  Fp2 x;
  if (f2eq(alpha, minus_one)) {
    x = {fneg(x0.c1), x0.c0};
  } else {
    const Fp2 b = f2pow(f2add(alpha, Fp2{ONE_M, Fp{}}), E_LEGENDRE, NW(E_LEGENDRE));
    x = f2mul(b, x0);
  }
  if (!f2eq(f2sqr(x), a)) return false;
  out = x;
  return true;
}

// ---------------------------------------------------------------- Fp6/12 ---
inline Fp6 f6add(const Fp6& a, const Fp6& b) { return {f2add(a.c0, b.c0), f2add(a.c1, b.c1), f2add(a.c2, b.c2)}; }
inline Fp6 f6sub(const Fp6& a, const Fp6& b) { return {f2sub(a.c0, b.c0), f2sub(a.c1, b.c1), f2sub(a.c2, b.c2)}; }
inline Fp6 f6neg(const Fp6& a) { return {f2neg(a.c0), f2neg(a.c1), f2neg(a.c2)}; }
inline Fp6 f6mulv(const Fp6& a) { return {f2nr(a.c2), a.c0, a.c1}; }
Fp6 f6mul(const Fp6& a, const Fp6& b) {
  const Fp2 t0 = f2mul(a.c0, b.c0), t1 = f2mul(a.c1, b.c1), t2 = f2mul(a.c2, b.c2);
  const Fp2 c0 = f2add(t0, f2nr(f2sub(f2sub(f2mul(f2add(a.c1, a.c2), f2add(b.c1, b.c2)), t1), t2)));
  const Fp2 c1 = f2add(f2sub(f2sub(f2mul(f2add(a.c0, a.c1), f2add(b.c0, b.c1)), t0), t1), f2nr(t2));
  const Fp2 c2 = f2add(f2sub(f2sub(f2mul(f2add(a.c0, a.c2), f2add(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}
// bls12_381 Fp6::mul_by_01 / mul_by_1
Fp6 f6mul01(const Fp6& a, const Fp2& c0, const Fp2& c1) {
  const Fp2 aa = f2mul(a.c0, c0), bb = f2mul(a.c1, c1);
  const Fp2 t1 = f2add(f2nr(f2mul(a.c2, c1)), aa);
  const Fp2 t2 = f2sub(f2sub(f2mul(f2add(c0, c1), f2add(a.c0, a.c1)), aa), bb);
  const Fp2 t3 = f2add(f2mul(a.c2, c0), bb);
  return {t1, t2, t3};
}
Fp6 f6mul1(const Fp6& a, const Fp2& c1) { return {f2nr(f2mul(a.c2, c1)), f2mul(a.c0, c1), f2mul(a.c1, c1)}; }
Fp6 f6inv(const Fp6& a) {
  const Fp2 c0 = f2sub(f2sqr(a.c0), f2nr(f2mul(a.c1, a.c2)));
  const Fp2 c1 = f2sub(f2nr(f2sqr(a.c2)), f2mul(a.c0, a.c1));
  const Fp2 c2 = f2sub(f2sqr(a.c1), f2mul(a.c0, a.c2));
  const Fp2 t = f2inv(f2add(f2mul(a.c0, c0), f2nr(f2add(f2mul(a.c2, c1), f2mul(a.c1, c2)))));
  return {f2mul(c0, t), f2mul(c1, t), f2mul(c2, t)};
}
Fp12 f12mul(const Fp12& a, const Fp12& b) {
  const Fp6 t0 = f6mul(a.c0, b.c0), t1 = f6mul(a.c1, b.c1);
  return {f6add(t0, f6mulv(t1)), f6sub(f6sub(f6mul(f6add(a.c0, a.c1), f6add(b.c0, b.c1)), t0), t1)};
}
Fp12 f12sqr(const Fp12& a) {
  const Fp6 ab = f6mul(a.c0, a.c1);
  const Fp6 c0 = f6sub(f6sub(f6mul(f6add(a.c0, a.c1), f6add(a.c0, f6mulv(a.c1))), ab), f6mulv(ab));
  return {c0, f6add(ab, ab)};
}
inline Fp12 f12conj(const Fp12& a) { return {a.c0, f6neg(a.c1)}; }
Fp12 f12inv(const Fp12& a) {
  const Fp6 t = f6inv(f6sub(f6mul(a.c0, a.c0), f6mulv(f6mul(a.c1, a.c1))));
  return {f6mul(a.c0, t), f6neg(f6mul(a.c1, t))};
}
// bls12_381 Fp12::mul_by_014
Fp12 f12mul014(const Fp12& f, const Fp2& c0, const Fp2& c1, const Fp2& c4) {
  const Fp6 aa = f6mul01(f.c0, c0, c1);
  const Fp6 bb = f6mul1(f.c1, c4);
  const Fp2 o = f2add(c1, c4);
  const Fp6 t = f6sub(f6sub(f6mul01(f6add(f.c1, f.c0), c0, o), aa), bb);
  return {f6add(f6mulv(bb), aa), t};
}
// Frobenius: w-basis coefficients (c00, c10, c01, c11, c02, c12) times gamma_i
Fp12 f12frob(const Fp12& a) {
  static const Fp2* G[6] = {&GAMMA0, &GAMMA1, &GAMMA2, &GAMMA3, &GAMMA4, &GAMMA5};
  return {{f2mul(f2conj(a.c0.c0), *G[0]), f2mul(f2conj(a.c0.c1), *G[2]), f2mul(f2conj(a.c0.c2), *G[4])},
          {f2mul(f2conj(a.c1.c0), *G[1]), f2mul(f2conj(a.c1.c1), *G[3]), f2mul(f2conj(a.c1.c2), *G[5])}};
}
inline void fp4_square(Fp2& c0, Fp2& c1, const Fp2& a, const Fp2& b) {
  const Fp2 t0 = f2sqr(a), t1 = f2sqr(b);
  c0 = f2add(f2nr(t1), t0);
  c1 = f2sub(f2sub(f2sqr(f2add(a, b)), t0), t1);
}
// Granger-Scott cyclotomic square (bls12_381 Fp12::cyclotomic_square)
Fp12 cyc_sqr(const Fp12& f) {
  Fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  Fp2 t0, t1, t2, t3;
  fp4_square(t0, t1, z0, z1);
  z0 = f2add(f2dbl(f2sub(t0, z0)), t0);
  z1 = f2add(f2dbl(f2add(t1, z1)), t1);
  fp4_square(t0, t1, z2, z3);
  fp4_square(t2, t3, z4, z5);
  z4 = f2add(f2dbl(f2sub(t0, z4)), t0);
  z5 = f2add(f2dbl(f2add(t1, z5)), t1);
  t0 = f2nr(t3);
  z2 = f2add(f2dbl(f2add(t0, z2)), t0);
  z3 = f2add(f2dbl(f2sub(t2, z3)), t2);
  return {{z0, z4, z3}, {z2, z1, z5}};
}
constexpr uint64_t BLS_X = 0xd201000000010000ull;   // |x|, x < 0
Fp12 cyc_exp(const Fp12& f) {   // f^x (conjugated f^|x|)
  Fp12 t = f;
  for (int b = 62; b >= 0; b--) {
    t = cyc_sqr(t);
    if ((BLS_X >> b) & 1) t = f12mul(t, f);
  }
  return f12conj(t);
}
Fp12 final_exp(const Fp12& f) {
  Fp12 t0 = f12conj(f);   // f^(p^6)
  Fp12 t1 = f12inv(f);
  Fp12 t2 = f12mul(t0, t1);
  t1 = t2;
  t2 = f12frob(f12frob(t2));
  t2 = f12mul(t2, t1);
  t1 = f12conj(cyc_sqr(t2));
  Fp12 t3 = cyc_exp(t2);
  Fp12 t4 = cyc_sqr(t3);
  Fp12 t5 = f12mul(t1, t3);
  t1 = cyc_exp(t5);
  t0 = cyc_exp(t1);
  Fp12 t6 = cyc_exp(t0);
  t6 = f12mul(t6, t4);
  t4 = cyc_exp(t6);
  t5 = f12conj(t5);
  t4 = f12mul(t4, f12mul(t5, t2));
  t5 = f12conj(t2);
  t1 = f12mul(t1, t2);
  t1 = f12frob(f12frob(f12frob(t1)));
  t6 = f12mul(t6, t5);
  t6 = f12frob(t6);
  t3 = f12mul(t3, t0);
  t3 = f12frob(f12frob(t3));
  t3 = f12mul(t3, t1);
  t3 = f12mul(t3, t6);
  return f12mul(t3, t4);
}

// ------------------------------------------------------------ curves -------
// Jacobian points over F (Fp or Fp2), a = 0; Z = 0 is the identity
template <class F>
struct Jac {
  F x, y, z;
};
struct FpOps {
  using T = Fp;
  static Fp add(const Fp& a, const Fp& b) { return fadd(a, b); }
  static Fp sub(const Fp& a, const Fp& b) { return fsub(a, b); }
  static Fp mul(const Fp& a, const Fp& b) { return fmul(a, b); }
  static Fp sqr(const Fp& a) { return fsqr(a); }
  static Fp neg(const Fp& a) { return fneg(a); }
  static bool zero(const Fp& a) { return fzero(a); }
  static bool eq(const Fp& a, const Fp& b) { return feq(a, b); }
  static Fp one() { return ONE_M; }
  static Fp inv(const Fp& a) { return finv(a); }
};
struct Fp2Ops {
  using T = Fp2;
  static Fp2 add(const Fp2& a, const Fp2& b) { return f2add(a, b); }
  static Fp2 sub(const Fp2& a, const Fp2& b) { return f2sub(a, b); }
  static Fp2 mul(const Fp2& a, const Fp2& b) { return f2mul(a, b); }
  static Fp2 sqr(const Fp2& a) { return f2sqr(a); }
  static Fp2 neg(const Fp2& a) { return f2neg(a); }
  static bool zero(const Fp2& a) { return f2zero(a); }
  static bool eq(const Fp2& a, const Fp2& b) { return f2eq(a, b); }
  static Fp2 one() { return {ONE_M, Fp{}}; }
  static Fp2 inv(const Fp2& a) { return f2inv(a); }
};
// dbl-2009-l
template <class O>
Jac<typename O::T> jdbl(const Jac<typename O::T>& p) {
  using T = typename O::T;
  if (O::zero(p.z)) return p;
  const T A = O::sqr(p.x), B = O::sqr(p.y), C = O::sqr(B);
  T D = O::sub(O::sub(O::sqr(O::add(p.x, B)), A), C);
  D = O::add(D, D);
  const T E = O::add(O::add(A, A), A);
  const T Fq = O::sqr(E);
  const T X3 = O::sub(Fq, O::add(D, D));
  T C8 = O::add(C, C);
  C8 = O::add(C8, C8);
  C8 = O::add(C8, C8);
  const T Y3 = O::sub(O::mul(E, O::sub(D, X3)), C8);
  const T yz = O::mul(p.y, p.z);
  return {X3, Y3, O::add(yz, yz)};
}
// mixed addition with an affine point (madd-2007-bl), complete for this use
template <class O>
Jac<typename O::T> jadd_aff(const Jac<typename O::T>& p, const typename O::T& qx, const typename O::T& qy) {
  using T = typename O::T;
  if (O::zero(p.z)) return {qx, qy, O::one()};
  const T Z1Z1 = O::sqr(p.z);
  const T U2 = O::mul(qx, Z1Z1);
  const T S2 = O::mul(O::mul(qy, p.z), Z1Z1);
  const T H = O::sub(U2, p.x);
  const T Rr = O::sub(S2, p.y);
  if (O::zero(H)) {
    if (O::zero(Rr)) return jdbl<O>(p);
    return {O::one(), O::one(), T{}};
  }
  const T HH = O::sqr(H), HHH = O::mul(H, HH), V = O::mul(p.x, HH);
  const T X3 = O::sub(O::sub(O::sub(O::sqr(Rr), HHH), V), V);
  const T Y3 = O::sub(O::mul(Rr, O::sub(V, X3)), O::mul(p.y, HHH));
  return {X3, Y3, O::mul(p.z, H)};
}
// [k] (x, y) for a 64-bit k (MSB first)
template <class O>
Jac<typename O::T> jmul64(const typename O::T& x, const typename O::T& y, uint64_t k) {
  using T = typename O::T;
  Jac<T> acc{O::one(), O::one(), T{}};
  for (int b = 63; b >= 0; b--) {
    acc = jdbl<O>(acc);
    if ((k >> b) & 1) acc = jadd_aff<O>(acc, x, y);
  }
  return acc;
}
// Jacobian (X : Y : Z) equals affine (x, y)
template <class O>
bool jeq_aff(const Jac<typename O::T>& p, const typename O::T& x, const typename O::T& y) {
  using T = typename O::T;
  if (O::zero(p.z)) return false;
  const T z2 = O::sqr(p.z);
  return O::eq(p.x, O::mul(x, z2)) && O::eq(p.y, O::mul(y, O::mul(z2, p.z)));
}

struct G1 {
  Fp x, y;
  bool inf;
};
struct G2 {
  Fp2 x, y;
  bool inf;
};

// G1Affine::from_compressed (src/lib.rs:144)
bool g1_decompress(const uint8_t* b, G1& out) {
  const int c = b[0] >> 7 & 1, i = b[0] >> 6 & 1, s = b[0] >> 5 & 1;
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  const Fp xr = from_be48(t);
  if (geq_p(xr.l)) return false;
  if (i && c && !s && fzero(xr)) {
    out.inf = true;
    return true;
  }
  const Fp x = to_mont(xr);
  const Fp rhs = fadd(fmul(fsqr(x), x), B1_M);
  Fp y = fpow(rhs, E_SQRT, NW(E_SQRT));
  if (!feq(fsqr(y), rhs)) return false;
  if (lex_largest(y) != (bool)s) y = fneg(y);
  if (i || !c) return false;
  // phi(P) = -x^2 P: [|x|]([|x|] P) (x^2 > 0), then negate
  Jac<Fp> t1 = jmul64<FpOps>(x, y, BLS_X);
  if (FpOps::zero(t1.z)) return false;
  const Fp zi = finv(t1.z), zi2 = fsqr(zi);
  const Fp ax = fmul(t1.x, zi2), ay = fmul(t1.y, fmul(zi2, zi));
  const Jac<Fp> t2 = jmul64<FpOps>(ax, ay, BLS_X);
  if (!jeq_aff<FpOps>(Jac<Fp>{t2.x, fneg(t2.y), t2.z}, fmul(x, BETA_M), y)) return false;
  out = {x, y, false};
  return true;
}
// G2Affine::from_compressed (src/lib.rs:74)
bool g2_decompress(const uint8_t* b, G2& out) {
  const int c = b[0] >> 7 & 1, i = b[0] >> 6 & 1, s = b[0] >> 5 & 1;
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  const Fp x1r = from_be48(t), x0r = from_be48(b + 48);
  if (geq_p(x1r.l) || geq_p(x0r.l)) return false;
  if (i && c && !s && fzero(x1r) && fzero(x0r)) {
    out.inf = true;
    return true;
  }
  const Fp2 x{to_mont(x0r), to_mont(x1r)};
  const Fp2 rhs = f2add(f2mul(f2sqr(x), x), B2_M);
  Fp2 y;
  if (!f2sqrt(rhs, y)) return false;
  if (f2lex_largest(y) != (bool)s) y = f2neg(y);
  if (i || !c) return false;
  // psi(Q) = [x] Q = -[|x|] Q
  const Jac<Fp2> q = jmul64<Fp2Ops>(x, y, BLS_X);
  const Fp2 px = f2mul(f2conj(x), PSI_CX), py = f2mul(f2conj(y), PSI_CY);
  if (!jeq_aff<Fp2Ops>(Jac<Fp2>{q.x, f2neg(q.y), q.z}, px, py)) return false;
  out = {x, y, false};
  return true;
}

// ----------------------------------------------------------- hashing -------
struct Sha256 {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len = 0;
  int fill = 0;
  Sha256() {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(h, iv, 32);
  }
  static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    len += n;
    while (n) {
      const size_t k = std::min<size_t>(n, 64 - fill);
      memcpy(buf + fill, p, k);
      fill += (int)k, p += k, n -= k;
      if (fill == 64) block(buf), fill = 0;
    }
  }
  void final(uint8_t* out) {
    const uint64_t bits = len * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (fill != 56) update(&zero, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(l, 8);
    for (int i = 0; i < 8; i++)
      for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
  }
};
const char DST[] = "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_";   // src/lib.rs:23
constexpr int DST_LEN = 43;

// expand_message_xmd(msg, DST, 128) (RFC 9380 §5.3.1)
void expand_xmd(const uint8_t* msg, size_t mlen, uint8_t out[128]) {
  uint8_t b0[32];
  {
    Sha256 s;
    const uint8_t z[64] = {0};
    s.update(z, 64);
    s.update(msg, mlen);
    const uint8_t lib[3] = {0, 128, 0};
    s.update(lib, 3);
    s.update((const uint8_t*)DST, DST_LEN);
    const uint8_t dl = DST_LEN;
    s.update(&dl, 1);
    s.final(b0);
  }
  uint8_t prev[32];
  for (int i = 1; i <= 4; i++) {
    Sha256 s;
    uint8_t x[32];
    for (int k = 0; k < 32; k++) x[k] = i == 1 ? b0[k] : (uint8_t)(b0[k] ^ prev[k]);
    s.update(x, 32);
    const uint8_t ib = (uint8_t)i;
    s.update(&ib, 1);
    s.update((const uint8_t*)DST, DST_LEN);
    const uint8_t dl = DST_LEN;
    s.update(&dl, 1);
    s.final(prev);
    memcpy(out + 32 * (i - 1), prev, 32);
  }
}
// OS2IP(64 bytes) mod p, Montgomery form: hi * 2^256 + lo
Fp field_elem(const uint8_t* b) {
  Fp hi{}, lo{};
  for (int i = 0; i < 4; i++) {
    uint64_t wh = 0, wl = 0;
    for (int k = 0; k < 8; k++) wh = (wh << 8) | b[8 * (3 - i) + k], wl = (wl << 8) | b[32 + 8 * (3 - i) + k];
    hi.l[i] = wh, lo.l[i] = wl;
  }
  static const Fp TWO256 = to_mont(Fp{{0, 0, 0, 0, 1, 0}});
  return fadd(fmul(to_mont(hi), TWO256), to_mont(lo));
}
inline bool sgn0(const Fp& a) { return from_mont(a).l[0] & 1; }
// RFC 9380 App. F.2 simplified SWU onto E' (x, y affine)
void sswu(const Fp& u, Fp& xo, Fp& yo) {
  Fp tv1 = fmul(SSWU_Z, fsqr(u));
  Fp tv2 = fadd(fsqr(tv1), tv1);
  Fp tv3 = fmul(SSWU_B, fadd(tv2, ONE_M));
  Fp tv4 = fmul(SSWU_A, fzero(tv2) ? SSWU_Z : fneg(tv2));
  tv2 = fsqr(tv3);
  Fp tv6 = fsqr(tv4);
  Fp tv5 = fmul(SSWU_A, tv6);
  tv2 = fmul(fadd(tv2, tv5), tv3);
  tv6 = fmul(tv6, tv4);
  tv5 = fmul(SSWU_B, tv6);
  tv2 = fadd(tv2, tv5);
  Fp x = fmul(tv1, tv3);
  // sqrt_ratio(tv2, tv6), p = 3 mod 4 (App. F.2.1.2)
  const Fp s1 = fmul(fsqr(tv6), fmul(tv2, tv6));
  Fp y1 = fmul(fpow(s1, E_SQRT_RATIO, NW(E_SQRT_RATIO)), fmul(tv2, tv6));
  const Fp y2 = fmul(y1, SQRT_MINUS_Z);
  const bool is_qr = feq(fmul(fsqr(y1), tv6), tv2);
  const Fp yr = is_qr ? y1 : y2;
  Fp y = fmul(fmul(tv1, u), yr);
  if (is_qr) x = tv3, y = yr;
  if (sgn0(u) != sgn0(y)) y = fneg(y);
  xo = fmul(x, finv(tv4));
  yo = y;
}
Fp horner(const Fp* c, int n, const Fp& x) {
  Fp acc = c[n - 1];
  for (int i = n - 2; i >= 0; i--) acc = fadd(fmul(acc, x), c[i]);
  return acc;
}
// 11-isogeny E' -> E; false when a denominator vanishes (identity)
bool iso_map(const Fp& x, const Fp& y, Fp& xo, Fp& yo) {
  const Fp xd = horner(ISO_XDEN_M, NW(ISO_XDEN_M), x), yd = horner(ISO_YDEN_M, NW(ISO_YDEN_M), x);
  if (fzero(xd) || fzero(yd)) return false;
  const Fp xn = horner(ISO_XNUM_M, NW(ISO_XNUM_M), x), yn = horner(ISO_YNUM_M, NW(ISO_YNUM_M), x);
  const Fp inv = finv(fmul(xd, yd));   // one inversion for both
  xo = fmul(xn, fmul(inv, yd));
  yo = fmul(fmul(y, yn), fmul(inv, xd));
  return true;
}
// hash_to_g1 (src/lib.rs:25-31): affine, inf on the identity
G1 hash_to_g1(const uint8_t* msg, size_t mlen) {
  uint8_t u[128];
  expand_xmd(msg, mlen, u);
  Jac<Fp> acc{ONE_M, ONE_M, Fp{}};
  for (int k = 0; k < 2; k++) {
    Fp x, y, ix, iy;
    sswu(field_elem(u + 64 * k), x, y);
    if (iso_map(x, y, ix, iy)) acc = jadd_aff<FpOps>(acc, ix, iy);
  }
  // clear cofactor: [1 - x] = [|x| + 1] (x < 0)
  if (FpOps::zero(acc.z)) return {Fp{}, Fp{}, true};
  const Fp zi = finv(acc.z), zi2 = fsqr(zi);
  const Fp ax = fmul(acc.x, zi2), ay = fmul(acc.y, fmul(zi2, zi));
  const Jac<Fp> r = jmul64<FpOps>(ax, ay, BLS_X + 1);
  if (FpOps::zero(r.z)) return {Fp{}, Fp{}, true};
  const Fp ri = finv(r.z), ri2 = fsqr(ri);
  return {fmul(r.x, ri2), fmul(r.y, fmul(ri2, ri)), false};
}

// ----------------------------------------------------------- pairing -------
struct Coeff {
  Fp2 c0, c1, c2;
};
constexpr int N_COEFFS = 68;
inline Fp2 f2muls(const Fp2& a, int s) {
  Fp2 r = a;
  for (int i = 1; i < s; i++) r = f2add(r, a);
  return r;
}
// oracle _doubling_step / _addition_step (Jacobian r)
Coeff dbl_step(Fp2& rx, Fp2& ry, Fp2& rz) {
  const Fp2 tmp0 = f2sqr(rx), tmp1 = f2sqr(ry), tmp2 = f2sqr(tmp1);
  Fp2 tmp3 = f2sub(f2sub(f2sqr(f2add(tmp1, rx)), tmp0), tmp2);
  tmp3 = f2dbl(tmp3);
  const Fp2 tmp4 = f2add(f2dbl(tmp0), tmp0);
  const Fp2 tmp6 = f2add(rx, tmp4);
  const Fp2 tmp5 = f2sqr(tmp4);
  const Fp2 zsq = f2sqr(rz);
  const Fp2 nx = f2sub(f2sub(tmp5, tmp3), tmp3);
  const Fp2 nz = f2sub(f2sub(f2sqr(f2add(rz, ry)), tmp1), zsq);
  Fp2 ny = f2mul(f2sub(tmp3, nx), tmp4);
  ny = f2sub(ny, f2muls(tmp2, 8));
  const Fp2 t3 = f2neg(f2dbl(f2mul(tmp4, zsq)));
  Fp2 t6 = f2sub(f2sub(f2sqr(tmp6), tmp0), tmp5);
  t6 = f2sub(t6, f2muls(tmp1, 4));
  const Fp2 t0 = f2dbl(f2mul(nz, zsq));
  rx = nx, ry = ny, rz = nz;
  return {t0, t3, t6};
}
Coeff add_step(Fp2& rx, Fp2& ry, Fp2& rz, const Fp2& qx, const Fp2& qy) {
  const Fp2 zsq = f2sqr(rz), ysq = f2sqr(qy);
  const Fp2 t0 = f2mul(zsq, qx);
  const Fp2 t1 = f2mul(f2sub(f2sub(f2sqr(f2add(qy, rz)), ysq), zsq), zsq);
  const Fp2 t2 = f2sub(t0, rx);
  const Fp2 t3 = f2sqr(t2);
  const Fp2 t4 = f2muls(t3, 4);
  const Fp2 t5 = f2mul(t4, t2);
  const Fp2 t6 = f2sub(f2sub(t1, ry), ry);
  Fp2 t9 = f2mul(t6, qx);
  const Fp2 t7 = f2mul(t4, rx);
  const Fp2 nx = f2sub(f2sub(f2sub(f2sqr(t6), t5), t7), t7);
  const Fp2 nz = f2sub(f2sub(f2sqr(f2add(rz, t2)), zsq), t3);
  Fp2 t10 = f2add(qy, nz);
  const Fp2 t8 = f2mul(f2sub(t7, nx), t6);
  const Fp2 ny = f2sub(t8, f2dbl(f2mul(ry, t5)));
  t10 = f2sub(f2sub(f2sqr(t10), ysq), f2sqr(nz));
  t9 = f2sub(f2dbl(t9), t10);
  t10 = f2dbl(nz);
  const Fp2 t1n = f2dbl(f2neg(t6));
  rx = nx, ry = ny, rz = nz;
  return {t10, t1n, t9};
}
// bits of |x| >> 1 below its leading one, MSB first (oracle _LOOP_BITS)
inline int loop_bit(int k) { return (int)(((BLS_X >> 1) >> (61 - k)) & 1); }   // k = 0..61
void g2_prepare(const Fp2& qx, const Fp2& qy, Coeff* out) {
  Fp2 rx = qx, ry = qy, rz{ONE_M, Fp{}};
  int idx = 0;
  for (int k = 0; k < 62; k++) {
    out[idx++] = dbl_step(rx, ry, rz);
    if (loop_bit(k)) out[idx++] = add_step(rx, ry, rz, qx, qy);
  }
  out[idx++] = dbl_step(rx, ry, rz);
}
inline Fp12 ell(const Fp12& f, const Coeff& c, const G1& p) {
  return f12mul014(f, c.c2, f2mulfp(c.c1, p.x), f2mulfp(c.c0, p.y));
}
Fp12 miller2(const G1& p0, const Coeff* c0, bool use0, const G1& p1, const Coeff* c1, bool use1) {
  Fp12 f{};
  f.c0.c0.c0 = ONE_M;
  int idx = 0;
  auto step = [&] {
    if (use0) f = ell(f, c0[idx], p0);
    if (use1) f = ell(f, c1[idx], p1);
    idx++;
  };
  for (int k = 0; k < 62; k++) {
    step();
    if (loop_bit(k)) step();
    f = f12sqr(f);
  }
  step();
  return f12conj(f);
}

Coeff g_neg_g2[N_COEFFS];
std::once_flag g_once;
void init() {
  g2_prepare(G2X_M, f2neg(G2Y_M), g_neg_g2);
}
bool is_one(const Fp12& f) {
  Fp12 one{};
  one.c0.c0.c0 = ONE_M;
  return memcmp(&f, &one, sizeof(Fp12)) == 0;
}

uint8_t verify_one(const uint8_t* sig, const uint8_t* msg, size_t mlen, const uint8_t* pk, Fp12* gt) {
  G1 s;
  if (!g1_decompress(sig, s)) return 2;
  G2 q;
  if (!g2_decompress(pk, q)) return 4;
  const G1 h = hash_to_g1(msg, mlen);
  Coeff pkc[N_COEFFS];
  g2_prepare(q.inf ? G2X_M : q.x, q.inf ? G2Y_M : q.y, pkc);
  const Fp12 f = final_exp(miller2(s, g_neg_g2, !s.inf, h, pkc, !q.inf && !h.inf));
  if (gt) *gt = f;
  return is_one(f) ? 0 : 5;
}
}  // namespace

extern "C" {
// n fixed-size records (48-B sigs, 96-B keys, messages with n + 1 offsets);
// codes_out[i] = 0..5 as cess_bls_verify_batch.  Returns 0.
int cpu64_verify_batch(uint64_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs,
                       const uint64_t* offs, uint8_t* codes_out, int threads) {
  std::call_once(g_once, init);
  if (threads < 1) threads = 1;
  std::atomic<uint64_t> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; t++)
    pool.emplace_back([&] {
      for (uint64_t i; (i = next.fetch_add(16)) < n;)
        for (uint64_t j = i; j < std::min<uint64_t>(n, i + 16); j++)
          codes_out[j] = verify_one(sigs + 48 * j, msgs + offs[j], offs[j + 1] - offs[j], pks + 96 * j, nullptr);
    });
  for (auto& th : pool) th.join();
  return 0;
}
// one record's code and Gt bytes (576, tower order, canonical big-endian)
int cpu64_gt(const uint8_t* sig, const uint8_t* msg, uint64_t mlen, const uint8_t* pk, uint8_t* gt_out) {
  std::call_once(g_once, init);
  Fp12 f;
  const uint8_t c = verify_one(sig, msg, mlen, pk, &f);
  if (c == 0 || c == 5) {
    const Fp6* h[2] = {&f.c0, &f.c1};
    int o = 0;
    for (int a = 0; a < 2; a++)
      for (const Fp2* e : {&h[a]->c0, &h[a]->c1, &h[a]->c2}) {
        to_be48(from_mont(e->c0), gt_out + 48 * o++);
        to_be48(from_mont(e->c1), gt_out + 48 * o++);
      }
  }
  return c;
}
// hash_to_g1 as 96 bytes x || y (canonical big-endian; zeros for the identity)
int cpu64_hash(const uint8_t* msg, uint64_t mlen, uint8_t* out96) {
  const G1 h = hash_to_g1(msg, mlen);
  memset(out96, 0, 96);
  if (h.inf) return 1;
  to_be48(from_mont(h.x), out96);
  to_be48(from_mont(h.y), out96 + 48);
  return 0;
}
}
