// RFC 9380 hash_to_curve BLS12381G1_XMD:SHA-256_SSWU_RO_ with the CESS DST.
//
// Replaces reference hash_to_g1 (utils/verify-bls-signatures/src/lib.rs:25-31):
//   <G1Projective as HashToCurve<ExpandMsgXmd<Sha256>>>::hash_to_curve(msg, DST).to_affine()
// Pipeline per message (one lane):
//   expand_message_xmd (SHA-256; the 64-byte Z_pad block is a constant midstate;
//   b1..b4 share a constant second block) -> u0, u1 = OS2IP(64 B) mod p
//   -> simplified SWU on E' (RFC 9380 App. F.2 straight-line, sqrt_ratio for p = 3 mod 4)
//   -> Q0 + Q1 on E' (complete addition) -> ONE 11-isogeny evaluation
//   -> clear_cofactor [1 - x] (Jacobian ladder, complete-formula recompute
//   for the lanes that end with Z = 0) -> affine.
#pragma once
#include "curve.hpp"

namespace bls {

// ---------------------------------------------------------------------------
// SHA-256 compression
// ---------------------------------------------------------------------------
CESS_CONST uint32_t SHA_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
CESS_CONST uint32_t SHA_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

CESS_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

CESS_HD void sha256_compress(uint32_t (&st)[8], const uint32_t (&blk)[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], cc = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + SHA_K[i] + wi;
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & cc) ^ (b & cc);
    uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = cc;
    cc = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += cc;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

// byte `pos` of the stream  msg || 0x00 0x80 || 0x00 || DST'  || SHA padding,
// i.e. msg_prime of expand_message_xmd after the constant 64-byte Z_pad block.
CESS_HD uint32_t xmd_b0_byte(const uint8_t* msg, uint32_t len, uint32_t pos, uint32_t padded) {
  if (pos < len) return msg[pos];
  uint32_t q = pos - len;
  if (q == 0) return 0x00;   // I2OSP(128, 2)
  if (q == 1) return 0x80;
  if (q == 2) return 0x00;   // I2OSP(0, 1)
  if (q < 3 + 44) return c::DST_PRIME[q - 3];
  if (q == 47) return 0x80;  // SHA padding
  if (pos >= padded - 8) {
    uint64_t bits = (uint64_t)(64 + len + 47) * 8;
    return (uint32_t)(bits >> (8 * (padded - 1 - pos))) & 0xff;
  }
  return 0;
}

// expand_message_xmd(msg, DST, 128) -> 32 big-endian words (b1 || b2 || b3 || b4)
// SELECT: write b_idx through uniform selects instead of out[8 (idx - 1) + j]
// (a loop-variant index puts `out` in scratch; the selects keep it in VGPRs,
// which only pays where the caller has the registers: hash_to_g1_parked)
template <bool SELECT = false>
CESS_HD void expand_message_xmd_128(const uint8_t* msg, uint32_t len, uint32_t (&out)[32]) {
  uint32_t b0[8];
#pragma unroll
  for (int i = 0; i < 8; i++) b0[i] = c::SHA_ZPAD_MID[i];
  // bytes after the zero block: len + 47 data bytes + 1 + 8 padding, rounded to 64
  uint32_t padded = ((len + 47 + 9) + 63) & ~63u;
#pragma unroll 1
  for (uint32_t off = 0; off < padded; off += 64) {
    uint32_t blk[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint32_t p0 = off + 4 * j;
      blk[j] = (xmd_b0_byte(msg, len, p0, padded) << 24) | (xmd_b0_byte(msg, len, p0 + 1, padded) << 16) |
               (xmd_b0_byte(msg, len, p0 + 2, padded) << 8) | xmd_b0_byte(msg, len, p0 + 3, padded);
    }
    sha256_compress(b0, blk);
  }
  // b_i = H((b0 ^ b_{i-1}) || i || DST'), 77 bytes = 2 blocks; block 2 is constant.
  uint32_t blk2[16];
  {
    // DST'[31..44) (13 bytes) || 0x80 || 0... || bitlen 616
    uint8_t t[64];
#pragma unroll
    for (int j = 0; j < 64; j++) t[j] = 0;
#pragma unroll
    for (int j = 0; j < 13; j++) t[j] = c::DST_PRIME[31 + j];
    t[13] = 0x80;
    t[62] = (616 >> 8) & 0xff;
    t[63] = 616 & 0xff;
#pragma unroll
    for (int j = 0; j < 16; j++)
      blk2[j] = ((uint32_t)t[4 * j] << 24) | ((uint32_t)t[4 * j + 1] << 16) | ((uint32_t)t[4 * j + 2] << 8) | t[4 * j + 3];
  }
  uint32_t prev[8];
#pragma unroll
  for (int i = 0; i < 8; i++) prev[i] = 0;
#pragma unroll 1
  for (int idx = 1; idx <= 4; idx++) {
    uint32_t blk[16];
#pragma unroll
    for (int j = 0; j < 8; j++) blk[j] = b0[j] ^ prev[j];   // prev = 0 for b1
    // byte 32 = idx, bytes 33..63 = DST'[0..31)
    uint8_t t[32];
    t[0] = (uint8_t)idx;
#pragma unroll
    for (int j = 0; j < 31; j++) t[1 + j] = c::DST_PRIME[j];
#pragma unroll
    for (int j = 0; j < 8; j++)
      blk[8 + j] = ((uint32_t)t[4 * j] << 24) | ((uint32_t)t[4 * j + 1] << 16) | ((uint32_t)t[4 * j + 2] << 8) | t[4 * j + 3];
    uint32_t st[8];
#pragma unroll
    for (int j = 0; j < 8; j++) st[j] = SHA_IV[j];
    sha256_compress(st, blk);
    sha256_compress(st, blk2);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (SELECT) {
#pragma unroll
        for (int q = 0; q < 4; q++) out[8 * q + j] = idx == q + 1 ? st[j] : out[8 * q + j];
      } else {
        out[8 * (idx - 1) + j] = st[j];
      }
      prev[j] = st[j];
    }
  }
}

// 64 big-endian bytes (16 BE words) -> Montgomery(value mod p)
CESS_HD fp fp_from_be64_words(const uint32_t* w) {
  // value = H * 2^384 + L, H = words 0..3, L = words 4..15
  fp lo, hi = fp_zero();
#pragma unroll
  for (int i = 0; i < 12; i++) lo.v[i] = w[15 - i];
#pragma unroll
  for (int i = 0; i < 4; i++) hi.v[i] = w[3 - i];
  return add(mul(lo, fp_from(c::R2)), mul(hi, fp_from(c::R2_384)));
}

CESS_HD uint32_t sgn0(const fp& a) { return from_mont(a).v[0] & 1u; }

// simplified SWU onto E' : returns x = xn / xd and y (affine y)
CESS_HD void map_to_curve_sswu(const fp& u, fp& xn, fp& xd, fp& y) {
  const fp A = fp_from(c::ISO_A), B = fp_from(c::ISO_B), Z = fp_from(c::ISO_Z);
  fp tv1 = mul(Z, sqr(u));             // Z u^2
  fp tv2 = add(sqr(tv1), tv1);         // Z^2 u^4 + Z u^2
  fp tv3 = mul(B, add(tv2, fp_one()));
  fp tv4 = mul(A, select(is_zero(tv2), Z, neg(tv2)));
  fp tv6 = sqr(tv4);
  fp gxn = add(mul(add(sqr(tv3), mul(A, tv6)), tv3), mul(B, mul(tv6, tv4)));  // (tv3^2 + A tv6) tv3 + B tv6 tv4
  fp gxd = mul(tv6, tv4);
  // sqrt_ratio(gxn, gxd), q = 3 mod 4
  fp s1 = sqr(gxd);
  fp s2 = mul(gxn, gxd);
  s1 = mul(s1, s2);
  fp y1 = mul(pow_fixed(s1, c::EXP_SQRT_RATIO), s2);
  fp y2 = mul(y1, fp_from(c::SSWU_C2));
  bool is_qr = eq(mul(sqr(y1), gxd), gxn);
  fp yy = select(is_qr, y1, y2);
  fp x = mul(tv1, tv3);
  fp ycand = mul(mul(tv1, u), yy);
  xn = select(is_qr, tv3, x);
  y = select(is_qr, yy, ycand);
  if (sgn0(u) != sgn0(y)) y = neg(y);
  xd = tv4;
}

// 11-isogeny E' -> E on a homogeneous projective point (X : Y : Z) of E'
// (x = X/Z, y = Y/Z).  The four rational-map polynomials are evaluated
// together by homogeneous Horner steps in (X : Z), all padded to degree 15:
//   H_P = sum_i k_i X^i Z^(15-i),  acc_i = acc_(i+1) X + k_i Z^(15-i),
// so XN' = XNUM_h Z^4 and XD' = XDEN_h Z^5 = (XDEN_h Z) Z^4 carry the same
// factor, and the image is (XN' YD Z : Y YN XD' : XD' YD Z) -- the textbook
// point scaled by Z^5 (Z != 0 here: the caller maps O' to O itself).  Live
// state: four accumulators, Z^(15-i), X, Z, Y -- instead of 32 tabulated
// powers (384 dwords, which spilled).
CESS_HD g1p iso_map_proj(const fp& X, const fp& Y, const fp& Z) {
  fp aXN = fp_zero(), aXD = fp_zero(), aYN = fp_zero(), aYD = fp_zero(), D = fp_one();
#pragma unroll 1
  for (int i = 15; i >= 0; i--) {
    if (i < 15) {
      D = mul(D, Z);
      aYN = mul(aYN, X);
      aYD = mul(aYD, X);
      if (i < 11) aXN = mul(aXN, X);
      if (i < 10) aXD = mul(aXD, X);
    }
    aYN = add(aYN, mul(fp_from(c::ISO_YNUM[i]), D));
    aYD = add(aYD, mul(fp_from(c::ISO_YDEN[i]), D));
    if (i <= 11) aXN = add(aXN, mul(fp_from(c::ISO_XNUM[i]), D));
    if (i <= 10) aXD = add(aXD, mul(fp_from(c::ISO_XDEN[i]), D));
  }
  const fp yd = mul(aYD, Z);
  return {mul(aXN, yd), mul(mul(Y, aYN), aXD), mul(aXD, yd)};
}

// Complete addition on E': y^2 = x^3 + A'x + B' (a != 0), Renes-Costello-
// Batina eprint 2015/1060 Alg. 1 (12M + 3 m_a + 2 m_3b): exact for every pair
// of points, doubling and inverses included.
CESS_HD g1p iso_curve_add(const g1p& p, const g1p& q) {
  const fp A = fp_from(c::ISO_A), B3 = mul3(fp_from(c::ISO_B));
  fp t0 = mul(p.x, q.x), t1 = mul(p.y, q.y), t2 = mul(p.z, q.z);
  fp t3 = sub(mul(add_nr(p.x, p.y), add_nr(q.x, q.y)), add(t0, t1));
  fp t4 = sub(mul(add_nr(p.x, p.z), add_nr(q.x, q.z)), add(t0, t2));
  fp t5 = sub(mul(add_nr(p.y, p.z), add_nr(q.y, q.z)), add(t1, t2));
  fp z3 = add(mul(B3, t2), mul(A, t4));
  fp x3 = sub(t1, z3);
  z3 = add(t1, z3);
  fp y3 = mul(x3, z3);
  t1 = add(dbl(t0), t0);
  t2 = mul(A, t2);
  t4 = mul(B3, t4);
  t1 = add(t1, t2);
  t2 = mul(A, sub(t0, t2));
  t4 = add(t4, t2);
  y3 = add(y3, mul(t1, t4));
  x3 = sub(mul(t3, x3), mul(t5, t4));
  z3 = add(mul(t5, z3), mul(t3, t1));
  return {x3, y3, z3};
}

// [1 - x] R for an affine point R of E(Fp) (h_eff of RFC 9380 for G1),
// 1 - x = 0xd201000000010001: a Jacobian ladder with mixed additions of R
// (dbl-2009-l 2M + 5S against the complete projective doubling's 6M + 2S).
// Those formulas are incomplete, but an exceptional step (T = +-R or O) needs
// R of order dividing a number below 2^64, i.e. R with no component in G1,
// and it leaves Z = 0, which stays 0: a lane that ends with Z = 0 recomputes
// [1 - x]R with the complete formulas (divergent; never taken for a hash
// output in practice), so the result is exact for every R.
CESS_HD g1a clear_cofactor_g1(const fp& rx, const fp& ry) {
  g1p acc = {rx, ry, fp_one()};
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    acc = jac_dbl(acc);
    if ((H_EFF_G1 >> b) & 1u) acc = jac_add_mixed(acc, rx, ry);
  }
  if (is_zero(acc.z)) return proj_to_affine(proj_mul_u64_mixed(rx, ry, H_EFF_G1));
  const fp iz = inv(acc.z), iz2 = sqr(iz);
  g1a r;
  r.inf = false;
  r.x = mul(acc.x, iz2);
  r.y = mul(acc.y, mul(iz2, iz));
  return r;
}

// hash_to_g1 (RFC 9380 BLS12381G1_XMD:SHA-256_SSWU_RO_, the reference's
// hash_to_g1 at src/lib.rs:25-31):
//   * Q0 + Q1 is formed on E' (complete addition above) and the 11-isogeny
//     applied ONCE: the isogeny is a group homomorphism, so iso(Q0 + Q1) =
//     iso(Q0) + iso(Q1) -- one ~120-multiply map evaluation less;
//   * the cofactor clearing is clear_cofactor_g1 (Jacobian ladder, complete
//     recompute for the lanes that end with Z = 0).
CESS_HD g1a hash_to_g1(const uint8_t* msg, uint32_t len) {
  uint32_t uni[32];
  expand_message_xmd_128(msg, len, uni);
  // one SSWU body for both field elements; the sum accumulates in registers
  // (an array q[2] indexed by the loop counter, or uni indexed by it, would
  // live in scratch)
  g1p s;
#pragma unroll 1
  for (int j = 0; j < 2; j++) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = j ? uni[16 + k] : uni[k];
    fp xn, xd, y;
    map_to_curve_sswu(fp_from_be64_words(w), xn, xd, y);
    const g1p q = {xn, mul(y, xd), xd};   // (xn/xd, y), xd != 0
    s = j ? iso_curve_add(s, q) : q;
  }
  g1a r;
  r.inf = true;
  r.x = fp_zero();
  r.y = fp_one();
  if (is_zero(s.z)) return r;   // Q0 = -Q1: the sum is O', its image O
  const g1p t = iso_map_proj(s.x, s.y, s.z);
  if (is_zero(t.z)) return r;   // s in the isogeny's kernel: image O
  const fp zi = inv(t.z);
  return clear_cofactor_g1(mul(t.x, zi), mul(t.y, zi));
}

#if !defined(CESS_HOSTEMU)
// hash_to_g1 with the values that wait across an SSWU exponentiation parked
// in LDS (k_hash, CESS_HASH_PARK): the second field element u1 while the
// first is mapped, and the first image Q0 while the second is mapped -- 48
// dwords that otherwise stay in VGPRs beside the window-4 power table and
// make k_hash spill (76 VGPRs, 304 B/lane).  park: 48 rows x 256 lanes, row r
// of lane t at park[r][t].
CESS_HD void park_fp(uint32_t (*park)[256], int row, uint32_t t, const fp& a) {
#pragma unroll
  for (int i = 0; i < 12; i++) park[row + i][t] = a.v[i];
}
CESS_HD fp unpark_fp(uint32_t (*park)[256], int row, uint32_t t) {
  fp a;
#pragma unroll
  for (int i = 0; i < 12; i++) a.v[i] = park[row + i][t];
  return a;
}
CESS_HD g1a hash_to_g1_parked(const uint8_t* msg, uint32_t len, uint32_t (*park)[256], uint32_t t) {
  fp u0;
  {
    uint32_t uni[32];
    expand_message_xmd_128<true>(msg, len, uni);
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = uni[16 + k];
    park_fp(park, 36, t, fp_from_be64_words(w));
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = uni[k];
    u0 = fp_from_be64_words(w);
  }
  {
    fp xn, xd, y;
    map_to_curve_sswu(u0, xn, xd, y);
    park_fp(park, 0, t, xn);
    park_fp(park, 12, t, mul(y, xd));
    park_fp(park, 24, t, xd);
  }
  CESS_MEMBAR();
  g1p s;
  {
    fp xn, xd, y;
    map_to_curve_sswu(unpark_fp(park, 36, t), xn, xd, y);
    const g1p q = {xn, mul(y, xd), xd};
    CESS_MEMBAR();
    const g1p q0 = {unpark_fp(park, 0, t), unpark_fp(park, 12, t), unpark_fp(park, 24, t)};
    s = iso_curve_add(q0, q);
  }
  g1a r;
  r.inf = true;
  r.x = fp_zero();
  r.y = fp_one();
  if (is_zero(s.z)) return r;   // Q0 = -Q1: the sum is O', its image O
  const g1p tt = iso_map_proj(s.x, s.y, s.z);
  if (is_zero(tt.z)) return r;   // s in the isogeny's kernel: image O
  const fp zi = inv(tt.z);
  return clear_cofactor_g1(mul(tt.x, zi), mul(tt.y, zi));
}
#endif

}  // namespace bls
