// G1 (y^2 = x^3 + 4 over Fp) and G2 (y^2 = x^3 + 4(1+u) over Fp2).
//
// Homogeneous projective coordinates with the complete a = 0 formulas of
// Renes-Costello-Batina (eprint 2015/1060, Alg. 7/8/9): exact on every input,
// including small-order points crafted by an adversary, which matters because
// subgroup checks run on attacker-chosen encodings.
//
// Reference call sites replaced (bls12_381 0.7.1):
//   G1Affine::from_compressed   utils/verify-bls-signatures/src/lib.rs:144
//   G2Affine::from_compressed   utils/verify-bls-signatures/src/lib.rs:74
//   to_compressed               src/lib.rs:64, :134
//   is_torsion_free (G1: phi(P) == -[x^2]P, G2: psi(P) == [x]P; eprint 2021/1130, 2022/352)
#pragma once
#include "field.hpp"

namespace bls {

template <class F>
struct proj {
  F x, y, z;
};
template <class F>
struct affine {
  F x, y;
  bool inf;
};
using g1p = proj<fp>;
using g2p = proj<fp2>;
using g1a = affine<fp>;
using g2a = affine<fp2>;

CESS_HD fp mul_b3(const fp& a) { return mul4(mul3(a)); }             // * 12
CESS_HD fp2 mul_b3(const fp2& a) { return mul4(mul3(mul_nr(a))); }   // * 12(1+u)
template <class F> CESS_HD F f_zero();
template <> CESS_HD fp f_zero<fp>() { return fp_zero(); }
template <> CESS_HD fp2 f_zero<fp2>() { return fp2_zero(); }
template <class F> CESS_HD F f_one();
template <> CESS_HD fp f_one<fp>() { return fp_one(); }
template <> CESS_HD fp2 f_one<fp2>() { return fp2_one(); }

template <class F>
CESS_HD proj<F> proj_identity() {
  return {f_zero<F>(), f_one<F>(), f_zero<F>()};
}
template <class F>
CESS_HD proj<F> proj_from_affine(const affine<F>& a) {
  if (a.inf) return proj_identity<F>();
  return {a.x, a.y, f_one<F>()};
}

// RCB Alg. 9 (doubling, a = 0)
template <class F>
CESS_HD proj<F> proj_dbl(const proj<F>& p) {
  F t0 = sqr(p.y);
  F z3 = mul8(t0);
  F t1 = mul(p.y, p.z);
  F t2 = sqr(p.z);
  t2 = mul_b3(t2);
  F x3 = mul(t2, z3);
  F y3 = add(t0, t2);
  z3 = mul(t1, z3);
  t1 = dbl(t2);
  t2 = add(t1, t2);
  t0 = sub(t0, t2);
  y3 = mul(t0, y3);
  y3 = add(x3, y3);
  t1 = mul(p.x, p.y);
  x3 = mul(t0, t1);
  x3 = dbl(x3);
  return {x3, y3, z3};
}

// RCB Alg. 7 (addition, a = 0)
template <class F>
CESS_HD proj<F> proj_add(const proj<F>& p, const proj<F>& q) {
  F t0 = mul(p.x, q.x);
  F t1 = mul(p.y, q.y);
  F t2 = mul(p.z, q.z);
  F t3 = mul(add(p.x, p.y), add(q.x, q.y));
  F t4 = add(t0, t1);
  t3 = sub(t3, t4);
  t4 = mul(add(p.y, p.z), add(q.y, q.z));
  F x3 = add(t1, t2);
  t4 = sub(t4, x3);
  x3 = mul(add(p.x, p.z), add(q.x, q.z));
  F y3 = add(t0, t2);
  y3 = sub(x3, y3);
  x3 = dbl(t0);
  t0 = add(x3, t0);
  t2 = mul_b3(t2);
  F z3 = add(t1, t2);
  t1 = sub(t1, t2);
  y3 = mul_b3(y3);
  x3 = mul(t4, y3);
  t2 = mul(t3, t1);
  x3 = sub(t2, x3);
  y3 = mul(y3, t0);
  t1 = mul(t1, z3);
  y3 = add(t1, y3);
  t0 = mul(t0, t3);
  z3 = mul(z3, t4);
  z3 = add(z3, t0);
  return {x3, y3, z3};
}

// RCB Alg. 8 (mixed addition, q affine and not the identity)
template <class F>
CESS_HD proj<F> proj_add_mixed(const proj<F>& p, const F& qx, const F& qy) {
  F t0 = mul(p.x, qx);
  F t1 = mul(p.y, qy);
  F t3 = mul(add(qx, qy), add(p.x, p.y));
  F t4 = add(t0, t1);
  t3 = sub(t3, t4);
  t4 = add(mul(qy, p.z), p.y);
  F y3 = add(mul(qx, p.z), p.x);
  F x3 = dbl(t0);
  t0 = add(x3, t0);
  F t2 = mul_b3(p.z);
  F z3 = add(t1, t2);
  t1 = sub(t1, t2);
  y3 = mul_b3(y3);
  x3 = mul(t4, y3);
  t2 = mul(t3, t1);
  x3 = sub(t2, x3);
  y3 = mul(y3, t0);
  t1 = mul(t1, z3);
  y3 = add(t1, y3);
  t0 = mul(t0, t3);
  z3 = mul(z3, t4);
  z3 = add(z3, t0);
  return {x3, y3, z3};
}

template <class F>
CESS_HD proj<F> proj_neg(const proj<F>& p) {
  return {p.x, neg(p.y), p.z};
}
template <class F>
CESS_HD bool proj_is_identity(const proj<F>& p) {
  return is_zero(p.z);
}
// projective equality (both may be the identity)
template <class F>
CESS_HD bool proj_eq(const proj<F>& p, const proj<F>& q) {
  bool pi = is_zero(p.z), qi = is_zero(q.z);
  if (pi || qi) return pi && qi;
  return eq(mul(p.x, q.z), mul(q.x, p.z)) && eq(mul(p.y, q.z), mul(q.y, p.z));
}
template <class F>
CESS_HD affine<F> proj_to_affine(const proj<F>& p) {
  affine<F> r;
  r.inf = is_zero(p.z);
  F zi = inv(p.z);
  r.x = mul(p.x, zi);
  r.y = mul(p.y, zi);
  if (r.inf) {
    r.x = f_zero<F>();
    r.y = f_one<F>();
  }
  return r;
}

// [k]P for a fixed 64-bit scalar k (MSB first, complete formulas)
template <class F>
CESS_HD proj<F> proj_mul_u64(const proj<F>& p, uint64_t k) {
  proj<F> acc = proj_identity<F>();
  bool started = false;
#pragma unroll 1
  for (int b = 63; b >= 0; b--) {
    if (started) acc = proj_dbl(acc);
    if ((k >> b) & 1u) {
      acc = started ? proj_add(acc, p) : p;
      started = true;
    }
  }
  return acc;
}
template <class F>
CESS_HD proj<F> proj_mul_u64_mixed(const F& px, const F& py, uint64_t k) {
  proj<F> acc = proj_identity<F>();
  bool started = false;
#pragma unroll 1
  for (int b = 63; b >= 0; b--) {
    if (started) acc = proj_dbl(acc);
    if ((k >> b) & 1u) {
      acc = started ? proj_add_mixed(acc, px, py) : proj<F>{px, py, f_one<F>()};
      started = true;
    }
  }
  return acc;
}

// as proj_mul_u64_mixed, with the affine base re-read through q(px, py) at
// each mixed addition instead of being held in registers across the doublings
template <class F, class QL>
CESS_HD proj<F> proj_mul_u64_mixed_ld(QL&& q, uint64_t k) {
  proj<F> acc = proj_identity<F>();
  bool started = false;
#pragma unroll 1
  for (int b = 63; b >= 0; b--) {
    if (started) acc = proj_dbl(acc);
    if ((k >> b) & 1u) {
      CESS_MEMBAR();
      F px, py;
      q(px, py);
      acc = started ? proj_add_mixed(acc, px, py) : proj<F>{px, py, f_one<F>()};
      started = true;
    }
  }
  return acc;
}

constexpr uint64_t BLS_X_ABS = 0xd201000000010000ull;   // x = -BLS_X_ABS
constexpr uint64_t H_EFF_G1 = 0xd201000000010001ull;    // 1 - x

// [k]P for a 256-bit scalar (little-endian 8 words), used by keygen/sign
template <class F>
CESS_HD proj<F> proj_mul_scalar_mixed(const F& px, const F& py, const uint32_t (&k)[8]) {
  proj<F> acc = proj_identity<F>();
#pragma unroll 1
  for (int w = 7; w >= 0; w--) {
#pragma unroll 1
    for (int b = 31; b >= 0; b--) {
      acc = proj_dbl(acc);
      if ((k[w] >> b) & 1u) acc = proj_add_mixed(acc, px, py);
    }
  }
  return acc;
}

// GLV split of a scalar for G1, where r = L^2 + L + 1 with L = x^2 - 1 (128
// bits) and [L]P = (beta^2 x, y) (beta: c::G1_BETA, phi = [-x^2] = [L^2];
// batch signing, k_sign.hip):
// k mod r = k1 + k2 L with 0 <= k1 < L and k2 < 2^128 -- plain long division
// by L (k is first reduced below r; a 32-byte key may exceed it).  Words
// little-endian.
CESS_CONST uint32_t R_LE[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                              0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
CESS_CONST uint32_t LAMBDA_LE[4] = {0xffffffffu, 0x00000000u, 0x0001a402u, 0xac45a401u};

CESS_HD void sub_r_if_ge(uint32_t (&k)[8]) {
  uint32_t t[8], br = 0;
#pragma unroll
  for (int w = 0; w < 8; w++) t[w] = subc32(k[w], R_LE[w], br, &br);
#pragma unroll
  for (int w = 0; w < 8; w++) k[w] = br ? k[w] : t[w];
}

CESS_HD void glv_split(const uint32_t (&k0)[8], uint32_t (&k1)[4], uint32_t (&k2)[4]) {
  uint32_t k[8];
#pragma unroll
  for (int w = 0; w < 8; w++) k[w] = k0[w];
  sub_r_if_ge(k);
  sub_r_if_ge(k);   // 2^256 < 3 r
  uint32_t rem[5] = {0, 0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
#pragma unroll 1
  for (int bit = 255; bit >= 0; bit--) {
    // rem = 2 rem + bit (rem < L before, so < 2^129), q <<= 1
#pragma unroll
    for (int w = 4; w > 0; w--) rem[w] = (rem[w] << 1) | (rem[w - 1] >> 31);
    rem[0] = (rem[0] << 1) | ((k[bit >> 5] >> (bit & 31)) & 1u);
#pragma unroll
    for (int w = 3; w > 0; w--) q[w] = (q[w] << 1) | (q[w - 1] >> 31);
    q[0] <<= 1;
    uint32_t t[5], br = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) t[w] = subc32(rem[w], LAMBDA_LE[w], br, &br);
    t[4] = subc32(rem[4], 0u, br, &br);
    const bool ge = br == 0;
#pragma unroll
    for (int w = 0; w < 5; w++) rem[w] = ge ? t[w] : rem[w];
    q[0] |= ge ? 1u : 0u;
  }
#pragma unroll
  for (int w = 0; w < 4; w++) k1[w] = rem[w], k2[w] = q[w];
}

// [k]P for affine P in G1 (not the identity): [k1]P + [k2]([L]P) by 2-bit
// joint windows over the affine table {P, 2P, 3P} (one inversion) and its
// image (beta^2 x, y): 128 doublings + 128 complete mixed additions, against
// 256 doublings + 256 additions for the bitwise ladder (some lane of a wave
// always adds).  The additions are computed every window and kept by a select
// (digits differ per lane).
CESS_HD g1p g1_mul_glv(const fp& px, const fp& py, const uint32_t (&k)[8]) {
  uint32_t k1[4], k2[4];
  glv_split(k, k1, k2);
  const g1p P2 = proj_dbl(g1p{px, py, fp_one()});
  const g1p P3 = proj_add_mixed(P2, px, py);
  const fp zi = inv(mul(P2.z, P3.z));
  const fp z2i = mul(zi, P3.z), z3i = mul(zi, P2.z);
  const fp x2 = mul(P2.x, z2i), y2 = mul(P2.y, z2i), x3 = mul(P3.x, z3i), y3 = mul(P3.y, z3i);
  const fp beta = fp_from(c::G1_BETA);
  const fp beta2 = mul(beta, beta);
  g1p acc = proj_identity<fp>();
#pragma unroll 1
  for (int w = 63; w >= 0; w--) {
    acc = proj_dbl(proj_dbl(acc));
    const int sh = 2 * (w & 15);
    const uint32_t d1 = (k1[w >> 4] >> sh) & 3u, d2 = (k2[w >> 4] >> sh) & 3u;
    {
      const fp tx = select(d1 == 1, px, select(d1 == 2, x2, x3)), ty = select(d1 == 1, py, select(d1 == 2, y2, y3));
      const g1p s = proj_add_mixed(acc, tx, ty);
      acc = {select(d1 != 0, s.x, acc.x), select(d1 != 0, s.y, acc.y), select(d1 != 0, s.z, acc.z)};
    }
    {
      const fp tx = mul(select(d2 == 1, px, select(d2 == 2, x2, x3)), beta2);
      const fp ty = select(d2 == 1, py, select(d2 == 2, y2, y3));
      const g1p s = proj_add_mixed(acc, tx, ty);
      acc = {select(d2 != 0, s.x, acc.x), select(d2 != 0, s.y, acc.y), select(d2 != 0, s.z, acc.z)};
    }
  }
  return acc;
}

// ---------------------------------------------------------------------------
// subgroup checks
// ---------------------------------------------------------------------------
// G1: phi(P) == -[x^2]P  with phi(x, y) = (beta x, y)   (P affine, not identity)
// Jacobian coordinates (x = X/Z^2, y = Y/Z^3) on y^2 = x^3 + b: dbl-2009-l
// (2M + 5S) and madd-2007-bl (7M + 4S), against 6M + 2S / 11M for the
// complete RCB formulas above.  Incomplete: doubling maps Z = 0 to Z = 0, and
// a mixed addition of T = +-Q or of T = O gives Z = 0, which then stays 0 --
// used only where that outcome means "reject" (g1_is_torsion_free).
CESS_HD g1p jac_dbl(const g1p& p) {
  const fp A = sqr(p.x), B = sqr(p.y), C = sqr(B);
  const fp D = dbl(sub(sub(sqr(add(p.x, B)), A), C));
  const fp E = mul3(A);
  const fp x3 = sub(sqr(E), dbl(D));
  const fp y3 = sub(mul(E, sub(D, x3)), mul8(C));
  const fp z3 = dbl(mul(p.y, p.z));
  return {x3, y3, z3};
}
CESS_HD g1p jac_add_mixed(const g1p& p, const fp& qx, const fp& qy) {
  const fp z1z1 = sqr(p.z);
  const fp u2 = mul(qx, z1z1), s2 = mul(qy, mul(p.z, z1z1));
  const fp h = sub(u2, p.x), hh = sqr(h);
  const fp i = mul4(hh), j = mul(h, i);
  const fp r = dbl(sub(s2, p.y));
  const fp v = mul(p.x, i);
  const fp x3 = sub(sub(sqr(r), j), dbl(v));
  const fp y3 = sub(mul(r, sub(v, x3)), dbl(mul(p.y, j)));
  const fp z3 = sub(sub(sqr(add(p.z, h)), z1z1), hh);
  return {x3, y3, z3};
}

// [a + b lambda]P for 32-bit a, b, where lambda is the eigenvalue of
// phi(x, y) = (beta x, y) on G1 (curve.hpp: phi = [-x^2]): 2-bit joint
// windows over the affine table {P, 2P, 3P} (one inversion) and its phi image
// (beta times the selected x): 32 doublings + 32 mixed additions, against 64 +
// 32 for a 64-bit scalar.  The distinct-key RLC mode's scalars (2^63 values:
// soundness 2^-63 per check).
// Jacobian coordinates with the incomplete dbl-2009-l / madd-2007-bl
// (jac_* above: 2M + 5S and 7M + 4S against 6M + 2S and 12M complete) and
// the identity tracked by a flag: P is in G1 (order r, not the identity), and
// no step adds +-T to T.  Before the a-digit addition the accumulator is
// [4 (A - B x^2)]P (A, B < 2^32 the digits so far, lambda = -x^2 mod r), and it
// adds [d]P, d in 1..3: 4 (A - B x^2) = +-d has no integer solution (|both|
// << r); before the b-digit addition it is [A' - 4 B x^2]P (A' < 2^34) and it
// adds [-d x^2]P: A' = (4 B -+ d) x^2 needs 4 B = +-d or A' >= x^2, neither
// possible -- so only the identity (no digit yet) is exceptional.
CESS_HD g1p g1_mul_glv32(const fp& px, const fp& py, uint32_t a, uint32_t b) {
  const g1p P2 = proj_dbl(g1p{px, py, fp_one()});
  const g1p P3 = proj_add_mixed(P2, px, py);
  const fp zi = inv(mul(P2.z, P3.z));
  const fp z2i = mul(zi, P3.z), z3i = mul(zi, P2.z);
  const fp x2 = mul(P2.x, z2i), y2 = mul(P2.y, z2i), x3 = mul(P3.x, z3i), y3 = mul(P3.y, z3i);
  const fp beta = fp_from(c::G1_BETA);
  g1p acc = {fp_zero(), fp_one(), fp_zero()};
  bool id = true;
#pragma unroll 1
  for (int bp = 30; bp >= 0; bp -= 2) {
    acc = jac_dbl(jac_dbl(acc));
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
      const uint32_t d = ((h ? b : a) >> bp) & 3u;
      fp tx = select(d == 1, px, select(d == 2, x2, x3));
      const fp ty = select(d == 1, py, select(d == 2, y2, y3));
      if (h) tx = mul(tx, beta);
      const g1p sum = jac_add_mixed(acc, tx, ty);
      const bool take = d != 0;
      acc = {select(take, select(id, tx, sum.x), acc.x), select(take, select(id, ty, sum.y), acc.y),
             select(take, select(id, fp_one(), sum.z), acc.z)};
      id = id && !take;
    }
  }
  if (id) return proj_identity<fp>();
  // Jacobian -> homogeneous (x = X / Z^2 = X Z / Z^3, y = Y / Z^3)
  return {mul(acc.x, acc.z), acc.y, mul(sqr(acc.z), acc.z)};
}

// phi(P) == -[x^2]P (phi(x, y) = (beta x, y) acts as [-x^2] on G1): one
// 128-bit ladder over x^2 = 0xac45a4010001a4020000000100000000 (17 set bits)
// in Jacobian coordinates with mixed additions of the affine P, then
// beta x Z^2 == X, y Z^3 == -Y, Z != 0.  A point of order below 2^128 (never
// in G1, whose order is the 255-bit prime r) drives some step into T = +-P or
// O, which leaves Z = 0 and is rejected, as it must be.
CESS_HD bool g1_is_torsion_free(const fp& px, const fp& py) {
  constexpr uint64_t X2_HI = 0xac45a4010001a402ull, X2_LO = 0x0000000100000000ull;
  g1p acc = {px, py, fp_one()};
#pragma unroll 1
  for (int b = 126; b >= 0; b--) {
    acc = jac_dbl(acc);
    const uint64_t w = b >= 64 ? X2_HI : X2_LO;
    if ((w >> (b & 63)) & 1u) acc = jac_add_mixed(acc, px, py);
  }
  const fp z2 = sqr(acc.z), z3 = mul(z2, acc.z);
  return !is_zero(acc.z) && eq(mul(mul(px, fp_from(c::G1_BETA)), z2), acc.x) && eq(mul(py, z3), neg(acc.y));
}
// the complete-formula form (two 64-bit ladders, RCB), kept as the host
// cross-check of the Jacobian one
CESS_HD bool g1_is_torsion_free_rcb(const fp& px, const fp& py) {
  g1p xp = proj_mul_u64_mixed(px, py, BLS_X_ABS);   // [|x|]P
  g1p x2p = proj_mul_u64(xp, BLS_X_ABS);           // [x^2]P
  g1p phi = {mul(px, fp_from(c::G1_BETA)), py, fp_one()};
  return proj_eq(phi, proj_neg(x2p));
}
// G2: psi(P) == [x]P = -[|x|]P
CESS_HD fp2 psi_x_coeff() { return {fp_from(c::PSI_X_C0), fp_from(c::PSI_X_C1)}; }
CESS_HD fp2 psi_y_coeff() { return {fp_from(c::PSI_Y_C0), fp_from(c::PSI_Y_C1)}; }
// `pk`: a store of two Fp2 (ld/st by index 0, 1) that holds the point during
// the scalar multiplication (LDS in k_decode_pk: 48 registers fewer live)
template <class Park>
CESS_HD bool g2_is_torsion_free(const fp2& px, const fp2& py, const Park& pk) {
  pk.st(0, px);
  pk.st(1, py);
  g2p xp = proj_mul_u64_mixed_ld<fp2>([&](fp2& x, fp2& y) { x = pk.ld(0), y = pk.ld(1); }, BLS_X_ABS);
  CESS_MEMBAR();
  g2p psi = {mul(conj(pk.ld(0)), psi_x_coeff()), mul(conj(pk.ld(1)), psi_y_coeff()), fp2_one()};
  return proj_eq(psi, proj_neg(xp));
}
struct RegPark2 {   // register-held store for g2_is_torsion_free (host emulation)
  fp2 v[2];
  CESS_HD fp2 ld(int k) const { return v[k]; }
  CESS_HD void st(int k, const fp2& a) const { const_cast<RegPark2*>(this)->v[k] = a; }
};

// ---------------------------------------------------------------------------
// ZCash compressed encodings
// ---------------------------------------------------------------------------
// Inputs are the encodings as big-endian 32-bit words (w[0] = bytes 0..3).
CESS_HD fp raw_from_be_words(const uint32_t* w) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = w[11 - i];
  return r;
}

// returns true if valid; out.inf set for the identity encoding
CESS_HD bool g1_decompress(const uint32_t* w, g1a& out) {
  uint32_t flags = w[0] >> 29;
  bool cflag = flags & 4, iflag = flags & 2, sflag = flags & 1;
  fp xr = raw_from_be_words(w);
  xr.v[11] &= 0x1fffffffu;
  out.inf = false;
  out.x = fp_zero();
  out.y = fp_one();
  if (!raw_lt_p(xr)) return false;
  if (iflag && cflag && !sflag && is_zero(xr)) {
    out.inf = true;
    return true;
  }
  if (iflag || !cflag) return false;   // (any such encoding is InvalidPoint)
  fp x = to_mont(xr);
  fp y;
  if (!sqrt(y, add(mul(sqr(x), x), fp_from(c::B1)))) return false;
  if (lex_largest(y) != sflag) y = neg(y);
  if (!g1_is_torsion_free(x, y)) return false;
  out.x = x;
  out.y = y;
  return true;
}

// psi(Q) == [x]Q = -T for T = [|x|]Q in homogeneous projective coordinates
// (X/Z, Y/Z): psi_x Z == X, psi_y Z == -Y, Z != 0.  k_prepare takes T from the
// G2Prepared iteration, which runs exactly the double-and-add of [|x|]Q
// (pairing.hpp g2_prepare), so the subgroup check costs ~4 Fp2 products
// instead of a second 63-doubling scalar multiplication in k_decode_pk.
CESS_HD bool g2_psi_is_neg_proj(const fp2& qx, const fp2& qy, const fp2& X, const fp2& Y, const fp2& Z) {
  const fp2 px = mul(conj(qx), psi_x_coeff()), py = mul(conj(qy), psi_y_coeff());
  return !is_zero(Z) && eq(mul(px, Z), X) && eq(mul(py, Z), neg(Y));
}

// subgroup = false: the on-curve point is returned without the psi check
// (k_decode_pk: k_prepare checks it, g2_psi_is_neg_jacobian)
template <class Park>
CESS_HD bool g2_decompress(const uint32_t* w, g2a& out, const Park& pk, bool subgroup = true) {
  uint32_t flags = w[0] >> 29;
  bool cflag = flags & 4, iflag = flags & 2, sflag = flags & 1;
  fp x1r = raw_from_be_words(w);
  x1r.v[11] &= 0x1fffffffu;
  fp x0r = raw_from_be_words(w + 12);
  out.inf = false;
  out.x = fp2_zero();
  out.y = fp2_one();
  if (!raw_lt_p(x1r) || !raw_lt_p(x0r)) return false;
  if (iflag && cflag && !sflag && is_zero(x1r) && is_zero(x0r)) {
    out.inf = true;
    return true;
  }
  if (iflag || !cflag) return false;
  fp2 x = {to_mont(x0r), to_mont(x1r)};
  fp2 b2 = {fp_from(c::B1), fp_from(c::B1)};   // 4(1 + u)
  fp2 y;
  if (!sqrt(y, add(mul(sqr(x), x), b2))) return false;
  if (lex_largest(y) != sflag) y = neg(y);
  if (!subgroup) {
    out.x = x;
    out.y = y;
    return true;
  }
  if (!g2_is_torsion_free(x, y, pk)) return false;
  CESS_MEMBAR();
  out.x = pk.ld(0);
  out.y = pk.ld(1);
  return true;
}
CESS_HD bool g2_decompress(const uint32_t* w, g2a& out) { return g2_decompress(w, out, RegPark2{}); }

CESS_HD void g1_compress(const g1a& p, uint8_t* out) {
  if (p.inf) {
    for (int i = 0; i < 48; i++) out[i] = 0;
    out[0] = 0xc0;
    return;
  }
  raw_to_be48(from_mont(p.x), out);
  out[0] |= 0x80;
  if (lex_largest(p.y)) out[0] |= 0x20;
}
CESS_HD void g2_compress(const g2a& p, uint8_t* out) {
  if (p.inf) {
    for (int i = 0; i < 96; i++) out[i] = 0;
    out[0] = 0xc0;
    return;
  }
  raw_to_be48(from_mont(p.x.c1), out);
  raw_to_be48(from_mont(p.x.c0), out + 48);
  out[0] |= 0x80;
  if (lex_largest(p.y)) out[0] |= 0x20;
}

}  // namespace bls
