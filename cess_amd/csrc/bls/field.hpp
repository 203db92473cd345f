// BLS12-381 field tower for CDNA4 (gfx950): Fp, Fp2, Fp6, Fp12.
//
// Representation: 12 x u32 little-endian limbs (cheap carry-chain add/sub),
// Montgomery form with R = 2^392, values kept in the redundant range [0, 2p):
// a Montgomery product of inputs < 8p is already < 2p, so no multiply pays for a
// final conditional subtraction; add/sub/neg work modulo 2p with the same
// instruction count as modulo p, and only eq/is_zero/from_mont (comparisons and
// serialisation) bring a value to its canonical form < p.
//
// Hot primitive: product-scanning (Comba) Montgomery multiplication computed in
// 14 x 28-bit limbs.  Each column of 28-bit products fits a 64-bit accumulator
// with headroom, so one limb product is exactly one `v_mad_u64_u32` with the
// running column as its 64-bit addend -- no carry flags, no SGPR round trips.
// Measured on MI355X (tools/mad_peak.hip): v_mad_u64_u32 peaks at ~32.5 T/s;
// this carry-free multiply runs 1.17x (8 waves/SIMD) to 1.8x (1 wave/SIMD) the
// rate of the 12 x 32-bit carry-chain multiply.  392 mads per multiply (196 a*b +
// 196 m*p), 301 per square.
//
// Replaces the arithmetic of the `bls12_381` 0.7.1 crate (Fp/Fp2/Fp6/Fp12) that
// the reference calls from utils/verify-bls-signatures/src/lib.rs:14-16.
//
// The same source compiles for the host only inside the test harness
// (tests/hostemu, macro CESS_HOSTEMU) so that the device algorithms can be
// checked against the oracle on a machine without a GPU; the product library
// is built for gfx950 only.
#pragma once
#include <stdint.h>

#if defined(CESS_HOSTEMU)
#define CESS_HD inline
#define CESS_NOINLINE inline
#define CESS_CONST static constexpr
#else
#include <hip/hip_runtime.h>
#define CESS_HD __device__ __forceinline__
#define CESS_CONST static constexpr
#endif

#include "consts.hpp"

#if defined(CESS_HOSTEMU)
#define CESS_MEMBAR() ((void)0)
#else
// compiler-only barrier: LDS/HBM operands are re-read after it instead of being
// kept live in registers across phases (register working set control)
#define CESS_MEMBAR() asm volatile("" ::: "memory")
#endif

namespace bls {

#if defined(CESS_COUNT_OPS)
// host test harness only: Fp multiply / square counters (algorithmic work)
// (g_mul2_count: lazily reduced Fp2 products = 3 half-products + 2 reductions,
// i.e. 2.5 Fp multiplies of work; g_half_count: other lazily reduced forms in
// half-multiply units, one per 196-mad half-product or reduction: dot2 = 8)
inline uint64_t g_mul_count = 0, g_sqr_count = 0, g_mul2_count = 0, g_half_count = 0;
#define CESS_COUNT_MUL() (++g_mul_count)
#define CESS_COUNT_SQR() (++g_sqr_count)
#define CESS_COUNT_MUL2() (++g_mul2_count)
#define CESS_COUNT_HALVES(n) (g_half_count += (n))
#else
#define CESS_COUNT_MUL() ((void)0)
#define CESS_COUNT_SQR() ((void)0)
#define CESS_COUNT_MUL2() ((void)0)
#define CESS_COUNT_HALVES(n) ((void)0)
#endif

struct fp {
  uint32_t v[12];
};
struct fp2 {
  fp c0, c1;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ---------------------------------------------------------------------------
// Fp
// ---------------------------------------------------------------------------
CESS_HD fp fp_from(const uint32_t (&k)[12]) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = k[i];
  return r;
}
CESS_HD fp fp_zero() {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = 0;
  return r;
}
CESS_HD fp fp_one() { return fp_from(c::ONE); }

// 32-bit add/sub with carry: __builtin_addc/__builtin_subc lower to
// v_add_co_u32 / v_addc_co_u32 (v_sub_co / v_subb_co) chains on gfx950 -- one
// instruction per limb.  (A 64-bit "(uint64_t)a - b - borrow" formulation
// compiles to ~8 VALU per limb.)
#if defined(CESS_HOSTEMU) && !defined(__clang__)
CESS_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
CESS_HD uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
}
#else
CESS_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  unsigned c;
  uint32_t r = __builtin_addc(a, b, cin, &c);
  *cout = c;
  return r;
}
CESS_HD uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  unsigned c;
  uint32_t r = __builtin_subc(a, b, bin, &c);
  *bout = c;
  return r;
}
#endif

// r = t - p if t >= p  (t < 2p): canonical form
CESS_HD fp fp_reduce_once(const fp& t) {
  fp s;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.v[i] = subc32(t.v[i], c::P_RAW[i], borrow, &borrow);
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = borrow ? t.v[i] : s.v[i];
  return r;
}

// r = t - 2p if t >= 2p  (t < 4p): back into [0, 2p)
CESS_HD fp fp_reduce2(const fp& t) {
  fp s;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.v[i] = subc32(t.v[i], c::P2_RAW[i], borrow, &borrow);
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = borrow ? t.v[i] : s.v[i];
  return r;
}

// a + b < 4p < 2^383 (no carry out of limb 11), then - 2p if >= 2p.  The sum
// and the trial subtraction run as two chains interleaved limb by limb (the
// subtraction's limb i needs only the sum's limb i): one chain alone waits two
// states on its carry register between links (s_nop 1 per link on gfx950),
// two interleaved chains one.
#ifndef CESS_ADD_ILV
#define CESS_ADD_ILV 1
#endif
CESS_HD fp add(const fp& a, const fp& b) {
#if CESS_ADD_ILV
  fp t, s;
  uint32_t carry = 0, borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    t.v[i] = addc32(a.v[i], b.v[i], carry, &carry);
    s.v[i] = subc32(t.v[i], c::P2_RAW[i], borrow, &borrow);
  }
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = borrow ? t.v[i] : s.v[i];
  return r;
#else
  fp t;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) t.v[i] = addc32(a.v[i], b.v[i], carry, &carry);
  return fp_reduce2(t);
#endif
}

CESS_HD fp sub(const fp& a, const fp& b) {
#if CESS_ADD_ILV
  // a - b and a - b + 2p as two interleaved chains (as add), the second kept
  // if the first borrows (a - b > -2p)
  fp t, u;
  uint32_t borrow = 0, carry = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    t.v[i] = subc32(a.v[i], b.v[i], borrow, &borrow);
    u.v[i] = addc32(t.v[i], c::P2_RAW[i], carry, &carry);
  }
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = borrow ? u.v[i] : t.v[i];
  return r;
#else
  fp t;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) t.v[i] = subc32(a.v[i], b.v[i], borrow, &borrow);
  // if borrow: add 2p back (a - b > -2p)
  const uint32_t mask = 0u - borrow;
  uint32_t carry = 0;
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = addc32(t.v[i], c::P2_RAW[i] & mask, carry, &carry);
  return r;
#endif
}

// Unreduced sum (no conditional subtraction): a + b < 4p for a, b < 2p.
// ONLY for values consumed by mul(): the Montgomery product accepts inputs up to
// 8p (a*b < 64 p^2 < p R, R = 2^392) and returns a value < 2p.  Never
// feed an unreduced value to sub/neg/sqr/eq or store it.
CESS_HD fp add_nr(const fp& a, const fp& b) {
  fp t;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) t.v[i] = addc32(a.v[i], b.v[i], carry, &carry);
  return t;
}

CESS_HD fp dbl(const fp& a) { return add(a, a); }

// a = 0 mod p, for a in [0, 2p): a is 0 or p
CESS_HD bool is_zero(const fp& a) {
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) z |= a.v[i], q |= a.v[i] ^ c::P_RAW[i];
  return z == 0 || q == 0;
}

CESS_HD fp neg(const fp& a) {
  // 2p - a, and 0 -> 0 (p stays p: both represent 0)
  fp r;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = subc32(c::P2_RAW[i], a.v[i], borrow, &borrow);
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) z |= a.v[i];
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = z == 0 ? 0u : r.v[i];
  return r;
}

CESS_HD bool eq(const fp& a0, const fp& b0) {
  const fp a = fp_reduce_once(a0), b = fp_reduce_once(b0);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

CESS_HD fp select(bool c, const fp& a, const fp& b) {  // c ? a : b
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// --- sequencing ---------------------------------------------------------------
// seq(x): an empty volatile asm that "rewrites" x in VGPRs.  Volatile asms keep
// their program order, so routing every multiply's operands and result through
// one serialises the Fp multiplies: LLVM otherwise interleaves the independent
// multiplies of an Fp2/Fp6 product for ILP and needs 512+ registers for an Fp6
// multiply (measured), spilling to scratch.  Within one multiply the column
// accumulation keeps enough independent work for a wave.
#if defined(CESS_HOSTEMU)
CESS_HD void seq(fp&) {}
#else
CESS_HD void seq(fp& a) {
  asm volatile(""
               : "+v"(a.v[0]), "+v"(a.v[1]), "+v"(a.v[2]), "+v"(a.v[3]), "+v"(a.v[4]), "+v"(a.v[5]),
                 "+v"(a.v[6]), "+v"(a.v[7]), "+v"(a.v[8]), "+v"(a.v[9]), "+v"(a.v[10]), "+v"(a.v[11]));
}
#endif

// zero_after(x): 0, data-dependent on x (orders a new accumulation chain after x)
#if defined(CESS_HOSTEMU)
CESS_HD uint64_t zero_after(uint64_t) { return 0; }
#else
CESS_HD uint64_t zero_after(uint64_t x) {
  uint32_t z;
  asm volatile("" : "=v"(z) : "0"(0u), "v"((uint32_t)x));
  return z;
}
#endif

// opaque(x): an empty NON-volatile asm on a partial column sum, so LLVM can
// neither reassociate it back into the carried accumulator chain nor is it
// pinned in program order (it moves with its operand)
#if defined(CESS_HOSTEMU)
CESS_HD void opaque(uint64_t&) {}
#else
CESS_HD void opaque(uint64_t& x) { asm("" : "+v"(x)); }
#endif

// --- 28-bit compute domain ---------------------------------------------------
constexpr uint32_t M28 = 0x0fffffffu;

// The digit mask as an operand: a literal makes every v_and_b32 an 8-byte
// instruction; held in an SGPR (CESS_M28_SGPR, a CSE-able non-volatile asm)
// the AND is the 4-byte VOP2 form (one wave issues 4-byte instructions every
// 4.04 cycles against 4.53 for 8-byte ones, profiles/round5_o_lat_probe.txt).
// Measured, not adopted: k_miller +1.7-2.1 ms, k_final +1 ms (+788
// instructions in k_miller's step; profiles/round5_aa_sweep.txt).
#ifndef CESS_M28_SGPR
#define CESS_M28_SGPR 0
#endif
#if CESS_M28_SGPR && !defined(CESS_HOSTEMU)
CESS_HD uint32_t m28_sgpr() {
  uint32_t m;
  asm("s_mov_b32 %0, 0xfffffff" : "=s"(m));
  return m;
}
#define M28V m28_sgpr()
#else
#define M28V M28
#endif

// acc += x * y (one v_mad_u64_u32; column sums stay below 2^64)
CESS_HD void mac(uint64_t& acc, uint32_t x, uint32_t y) { acc += (uint64_t)x * y; }

// 384-bit value (12 x 32) -> 14 x 28-bit limbs
CESS_HD void unpack28(const fp& a, uint32_t (&l)[14]) {
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int off = 28 * k, i = off >> 5, sh = off & 31;
    uint32_t lo = a.v[i] >> sh;
    if (sh > 4 && i + 1 < 12) lo |= a.v[i + 1] << (32 - sh);
    l[k] = lo & M28V;
  }
}
// 14 x 28-bit normalised limbs (value < 2^384) -> 12 x 32
CESS_HD fp pack28(const uint32_t (&l)[14]) {
  fp r;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const int off = 32 * j, k = off / 28, sh = off - 28 * k;
    uint32_t w = l[k] >> sh;
    w |= l[k + 1] << (28 - sh);
    if (28 - sh + 28 < 32 && k + 2 < 14) w |= l[k + 2] << (56 - sh);
    r.v[j] = w;
  }
  return r;
}

// Montgomery reduction tail shared by mul and sqr:
//   columns k of the double-width product are accumulated by
//   `col(k, h, acc)`, which adds the column's products a_i b_j with i of
//   parity h (h = -1: all of them); the result (< 2p) is left in 14 x 28-bit
//   digits t.
// CESS_MONT_SEP: each column's products go to two fresh partial sums (by the
// parity of i; the known m * p terms continue the second), and only their
// merge, m_k and the shift stay on the carried chain -- the wave then has
// independent mads to issue while the chain's mul_lo / and / mad / shift
// steps complete.  A lazy Fp2 product in a dependent loop: 7,476 -> 6,524
// cycles at one wave per SIMD, 13,085 -> 12,700 at two
// (profiles/round5_j_fp_probe.txt, mul_sep<2,noq>).
#ifndef CESS_MONT_SEP
#define CESS_MONT_SEP 0
#endif
template <class Col>
CESS_HD void mont28_d(Col&& col, uint32_t (&t)[14]) {
  uint32_t m[14];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
#if CESS_MONT_SEP
    uint64_t sa = 0, sb = 0;
    col(k, 0, sa);
    col(k, 1, sb);
#pragma unroll
    for (int i = k < 14 ? 0 : k - 13; i < (k < 14 ? k : 14); i++) mac(sb, m[i], c::P28[k - i]);
    opaque(sa);
    opaque(sb);
    sa += sb;
    opaque(sa);
    acc += sa;
#else
    col(k, -1, acc);
#pragma unroll
    for (int i = k < 14 ? 0 : k - 13; i < (k < 14 ? k : 14); i++) mac(acc, m[i], c::P28[k - i]);
#endif
    if (k < 14) {
      m[k] = ((uint32_t)acc * c::PINV28) & M28V;
      mac(acc, m[k], c::P28[0]);
    } else {
      t[k - 14] = (uint32_t)acc & M28V;
    }
    acc >>= 28;
  }
  t[13] = (uint32_t)acc;   // result < 2p < 2^382: fits
}
template <class Col>
CESS_HD fp mont28(Col&& col) {
  uint32_t t[14];
  mont28_d(col, t);
  return pack28(t);
}

// Two Montgomery reductions side by side (lazy Fp2 product):
//   `col(k, h, acc0, acc1)` adds column k of each combined double-width
//   value, products a_i b_j with i of parity h (h = -1: all); CESS_MONT_SEP
//   as mont28_d.
template <class Col>
CESS_HD void mont28x2(Col&& col, fp& out0, fp& out1) {
  uint32_t m0[14], m1[14], t0[14], t1[14];
  uint64_t acc0 = 0, acc1 = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
#if CESS_MONT_SEP
    uint64_t s0a = 0, s1a = 0, s0b = 0, s1b = 0;
    col(k, 0, s0a, s1a);
    col(k, 1, s0b, s1b);
#pragma unroll
    for (int i = k < 14 ? 0 : k - 13; i < (k < 14 ? k : 14); i++) {
      mac(s0b, m0[i], c::P28[k - i]);
      mac(s1b, m1[i], c::P28[k - i]);
    }
    opaque(s0a);
    opaque(s1a);
    opaque(s0b);
    opaque(s1b);
    s0a += s0b;
    s1a += s1b;
    opaque(s0a);
    opaque(s1a);
    acc0 += s0a;
    acc1 += s1a;
#else
    col(k, -1, acc0, acc1);
#pragma unroll
    for (int i = k < 14 ? 0 : k - 13; i < (k < 14 ? k : 14); i++) {
      mac(acc0, m0[i], c::P28[k - i]);
      mac(acc1, m1[i], c::P28[k - i]);
    }
#endif
    if (k < 14) {
      m0[k] = ((uint32_t)acc0 * c::PINV28) & M28V;
      m1[k] = ((uint32_t)acc1 * c::PINV28) & M28V;
      mac(acc0, m0[k], c::P28[0]);
      mac(acc1, m1[k], c::P28[0]);
    } else {
      t0[k - 14] = (uint32_t)acc0 & M28V;
      t1[k - 14] = (uint32_t)acc1 & M28V;
    }
    acc0 >>= 28;
    acc1 >>= 28;
  }
  t0[13] = (uint32_t)acc0;
  t1[13] = (uint32_t)acc1;
  out0 = pack28(t0);
  out1 = pack28(t1);
}

// Four Montgomery reductions side by side (two independent lazy Fp2
// products, mul2): four accumulation chains per column instead of two, so a
// single wave per SIMD has independent work to issue while one chain's
// reduction step (m = acc * p' -> m * p[0] -> shift) completes.
template <class Col>
CESS_HD void mont28x4(Col&& col, fp& out0, fp& out1, fp& out2, fp& out3) {
  uint32_t m0[14], m1[14], m2[14], m3[14], t0[14], t1[14], t2[14], t3[14];
  uint64_t acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    col(k, -1, acc0, acc1, acc2, acc3);
#pragma unroll
    for (int i = 0; i < k; i++) {
      mac(acc0, m0[i], c::P28[k - i]);
      mac(acc1, m1[i], c::P28[k - i]);
      mac(acc2, m2[i], c::P28[k - i]);
      mac(acc3, m3[i], c::P28[k - i]);
    }
    m0[k] = ((uint32_t)acc0 * c::PINV28) & M28V;
    m1[k] = ((uint32_t)acc1 * c::PINV28) & M28V;
    m2[k] = ((uint32_t)acc2 * c::PINV28) & M28V;
    m3[k] = ((uint32_t)acc3 * c::PINV28) & M28V;
    mac(acc0, m0[k], c::P28[0]);
    mac(acc1, m1[k], c::P28[0]);
    mac(acc2, m2[k], c::P28[0]);
    mac(acc3, m3[k], c::P28[0]);
    acc0 >>= 28;
    acc1 >>= 28;
    acc2 >>= 28;
    acc3 >>= 28;
  }
#pragma unroll
  for (int k = 14; k < 27; k++) {
    col(k, -1, acc0, acc1, acc2, acc3);
#pragma unroll
    for (int i = k - 13; i < 14; i++) {
      mac(acc0, m0[i], c::P28[k - i]);
      mac(acc1, m1[i], c::P28[k - i]);
      mac(acc2, m2[i], c::P28[k - i]);
      mac(acc3, m3[i], c::P28[k - i]);
    }
    t0[k - 14] = (uint32_t)acc0 & M28V;
    t1[k - 14] = (uint32_t)acc1 & M28V;
    t2[k - 14] = (uint32_t)acc2 & M28V;
    t3[k - 14] = (uint32_t)acc3 & M28V;
    acc0 >>= 28;
    acc1 >>= 28;
    acc2 >>= 28;
    acc3 >>= 28;
  }
  t0[13] = (uint32_t)acc0;
  t1[13] = (uint32_t)acc1;
  t2[13] = (uint32_t)acc2;
  t3[13] = (uint32_t)acc3;
  out0 = pack28(t0);
  out1 = pack28(t1);
  out2 = pack28(t2);
  out3 = pack28(t3);
}

// a * b * 2^-392 mod p
CESS_HD fp mul(const fp& a0, const fp& b0) {
  CESS_COUNT_MUL();
  fp a = a0, b = b0;
  seq(a);
  seq(b);
  uint32_t x[14], y[14];
  unpack28(a, x);
  unpack28(b, y);
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++)
      if (k - i >= 0 && k - i < 14 && (h < 0 || (i & 1) == h)) mac(acc, x[i], y[k - i]);
  });
  seq(r);
  return r;
}

// a^2 * 2^-392 mod p: off-diagonal products once against a doubled operand
CESS_HD fp sqr(const fp& a0) {
  CESS_COUNT_SQR();
  fp a = a0;
  seq(a);
  uint32_t x[14], x2[14];
  unpack28(a, x);
#pragma unroll
  for (int i = 0; i < 14; i++) x2[i] = x[i] << 1;
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j > i && j < 14 && (h < 0 || (i & 1) == h)) mac(acc, x[i], x2[j]);
    }
    if ((k & 1) == 0 && (k >> 1) < 14 && (h < 0 || ((k >> 1) & 1) == h)) mac(acc, x[k >> 1], x[k >> 1]);
  });
  seq(r);
  return r;
}

// a * 2^k-ish small multiples by repeated addition
CESS_HD fp mul3(const fp& a) { return add(dbl(a), a); }
CESS_HD fp mul4(const fp& a) { return dbl(dbl(a)); }
CESS_HD fp mul8(const fp& a) { return dbl(dbl(dbl(a))); }

// canonical integer <-> Montgomery (a * 1 / R <= p: one subtraction canonicalises)
CESS_HD fp from_mont(const fp& a) {
  fp one_raw = fp_zero();
  one_raw.v[0] = 1;
  return fp_reduce_once(mul(a, one_raw));
}
CESS_HD fp to_mont(const fp& a_raw) { return mul(a_raw, fp_from(c::R2)); }

// a^e for a fixed 12-word exponent: MSB-first sliding window of width W
// (CESS_POW_W, default 4: decode/hash kernels 1-3 % faster than width 3 on
// one MI355X, width 5 spills -- profiles/round4_d_sweep.txt) over the odd
// powers a, a^3, .., a^(2^W - 1) (table held in registers; the window's entry
// is copied under a wave-uniform branch, CESS_POW_SWITCH, not read through a
// dynamically indexed array, so nothing goes to scratch).  For the 379-381-bit exponents used here (p-2, (p+1)/4,
// (p-3)/4; ~229 set bits) this is ~110 multiplies instead of ~229.  All
// branches depend on the exponent only, so they are wave-uniform.
// The chain runs in the 28-bit digit domain: a Montgomery product's digits
// (< 2^28, value < 2p) are a valid operand of the next product as they are, so
// the 12 x 32-bit pack / unpack of every multiply (~70 instructions) is paid
// once per exponentiation.
#if defined(CESS_HOSTEMU)
CESS_HD void seq14(uint32_t (&)[14]) {}
#else
CESS_HD void seq14(uint32_t (&x)[14]) {
  asm volatile(""
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                 "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]));
}
#endif
// r = x y / R on digits (r may alias x or y)
CESS_HD void mul_d(uint32_t (&r)[14], const uint32_t (&x)[14], const uint32_t (&y)[14]) {
  CESS_COUNT_MUL();
  uint32_t t[14];
  mont28_d(
      [&](int k, int h, uint64_t& acc) {
#pragma unroll
        for (int i = 0; i < 14; i++)
          if (k - i >= 0 && k - i < 14 && (h < 0 || (i & 1) == h)) mac(acc, x[i], y[k - i]);
      },
      t);
#pragma unroll
  for (int i = 0; i < 14; i++) r[i] = t[i];
  seq14(r);
}
// x = x^2 / R on digits
CESS_HD void sqr_d(uint32_t (&x)[14]) {
  CESS_COUNT_SQR();
  uint32_t x2[14], t[14];
#pragma unroll
  for (int i = 0; i < 14; i++) x2[i] = x[i] << 1;
  mont28_d(
      [&](int k, int h, uint64_t& acc) {
#pragma unroll
        for (int i = 0; i < 14; i++) {
          const int j = k - i;
          if (j > i && j < 14 && (h < 0 || (i & 1) == h)) mac(acc, x[i], x2[j]);
        }
        if ((k & 1) == 0 && (k >> 1) < 14 && (h < 0 || ((k >> 1) & 1) == h)) mac(acc, x[k >> 1], x[k >> 1]);
      },
      t);
#pragma unroll
  for (int i = 0; i < 14; i++) x[i] = t[i];
  seq14(x);
}
CESS_HD uint32_t exp_bit(const uint32_t (&e)[12], int i) { return (e[i >> 5] >> (i & 31)) & 1u; }
#ifndef CESS_POW_W
#define CESS_POW_W 4
#endif
#ifndef CESS_POW_SWITCH
#define CESS_POW_SWITCH 1
#endif
CESS_HD fp pow_fixed(const fp& a0, const uint32_t (&e)[12]) {
  constexpr int W = CESS_POW_W, NT = 1 << (W - 1);   // odd powers a, a^3, .., a^(2^W - 1)
  fp a = a0;
  seq(a);
  uint32_t t[NT][14], a2[14], r[14], w[14];
  unpack28(a, t[0]);
#pragma unroll
  for (int q = 0; q < 14; q++) a2[q] = t[0][q];
  sqr_d(a2);
#pragma unroll
  for (int j = 1; j < NT; j++) mul_d(t[j], t[j - 1], a2);
  bool started = false;
  int i = 383;
#pragma unroll 1
  while (i >= 0) {
    if (!exp_bit(e, i)) {
      if (started) sqr_d(r);
      i--;
      continue;
    }
    int j = i >= W - 1 ? i - (W - 1) : 0;   // window e[i..j], j the lowest set bit in it
    while (!exp_bit(e, j)) j++;
    uint32_t v = 0;
#pragma unroll 1
    for (int k = i; k >= j; k--) {
      v = 2 * v + exp_bit(e, k);
      if (started) sqr_d(r);
    }
#if CESS_POW_SWITCH
    // v is wave-uniform: a scalar branch to one copy of the table entry (14
    // moves) instead of NT - 1 selects per digit
#if defined(CESS_HOSTEMU)
    const uint32_t m0 = v >> 1;
#else
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(v >> 1);
#endif
#pragma unroll
    for (int m = 0; m < NT; m++)
      if (m0 == (uint32_t)m) {
#pragma unroll
        for (int q = 0; q < 14; q++) w[q] = t[m][q];
      }
#else
    // uniform selects (v is wave-uniform): no dynamically indexed table
#pragma unroll
    for (int q = 0; q < 14; q++) {
      uint32_t x = t[0][q];
#pragma unroll
      for (int m = 1; m < NT; m++) x = v == (uint32_t)(2 * m + 1) ? t[m][q] : x;
      w[q] = x;
    }
#endif
    if (started) {
      mul_d(r, r, w);
    } else {
#pragma unroll
      for (int q = 0; q < 14; q++) r[q] = w[q];
    }
    started = true;
    i = j - 1;
  }
  return pack28(r);
}

// --- inversion: Bernstein-Yang safegcd (eprint 2019/266) ----------------------
// Integers in 13 signed 30-bit limbs (two's complement digits: limbs 0..11 in
// [0, 2^30), limb 12 carries the sign).  Each outer step runs 30 divsteps on
// the low 30 bits of f, g (32-bit VALU only, no branches: every lane follows the
// same instruction stream), then applies the 2x2 transition matrix to the full
// f, g and to the Bezout coefficients d, e (mod p, exact division by 2^30 via a
// multiple of p).  37 x 30 = 1,110 divsteps >= floor((49 d + 57) / 17) = 1,101
// for d = 381 bits, the paper's bound (Theorem 11.2), so g reaches 0 for every
// input.  Since round 6 the steps are the half-delta variant (delta starts at
// 1/2; libsecp256k1's safegcd analysis puts its worst case lower, ~880
// divsteps for 381 bits, so the 37-iteration cap stays a safe bound), and the
// loop leaves as soon as g = 0 in every lane of the wave: once g = 0 further
// divsteps leave f and d unchanged, so the early exit is exact.  Random inputs
// need 26-28 iterations (half-delta 26-27; 200,000 samples,
// tools/divsteps_sim.c), not 37.  Cost ~1,240 VALU per iteration (~3.3 x 10^4
// per inversion), about 60 Montgomery products, against ~490 for a^(p-2).
struct s30 {
  int32_t v[13];
};
constexpr int32_t M30 = 0x3fffffff;

// 30 divsteps (half-delta form: zeta = -(delta + 1/2), delta starts at 1/2,
// so zeta starts at -1; a swap step sets delta to 1 - delta, i.e. zeta to
// -zeta - 2, any other step delta to 1 + delta, zeta to zeta - 1) on the low
// bits f0 (odd), g0; returns zeta and the matrix [u v; q r] with
// 2^30 [f'; g'] = [u v; q r] [f; g]
CESS_HD int32_t divsteps30(int32_t zeta, uint32_t f, uint32_t g, int32_t& ou, int32_t& ov, int32_t& oq,
                           int32_t& orr) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    uint32_t c1 = (uint32_t)(zeta >> 31);   // delta > 0
    const uint32_t c2 = 0u - (g & 1u);        // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    c1 &= c2;   // swap step: delta > 0 and g odd
    zeta = (int32_t)(((uint32_t)zeta ^ c1) - 1u);   // swap: -zeta - 2, else zeta - 1
    f += g & c1;
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  ou = (int32_t)u, ov = (int32_t)v, oq = (int32_t)q, orr = (int32_t)r;
  return zeta;
}

// [d; e] <- [u v; q r] [d; e] / 2^30 mod p, keeping d, e in (-2p, p)
CESS_HD void update_de30(s30& d, s30& e, int32_t u, int32_t v, int32_t q, int32_t r) {
  const int32_t sd = d.v[12] >> 31, se = e.v[12] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((c::PINV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((c::PINV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)c::P30[0] * md;
  ce += (int64_t)c::P30[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 13; i++) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)c::P30[i] * md;
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)c::P30[i] * me;
    d.v[i - 1] = (int32_t)cd & M30;
    e.v[i - 1] = (int32_t)ce & M30;
    cd >>= 30;
    ce >>= 30;
  }
  d.v[12] = (int32_t)cd;
  e.v[12] = (int32_t)ce;
}

// [f; g] <- [u v; q r] [f; g] / 2^30 (exact)
CESS_HD void update_fg30(s30& f, s30& g, int32_t u, int32_t v, int32_t q, int32_t r) {
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 13; i++) {
    cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
    cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
    f.v[i - 1] = (int32_t)cf & M30;
    g.v[i - 1] = (int32_t)cg & M30;
    cf >>= 30;
    cg >>= 30;
  }
  f.v[12] = (int32_t)cf;
  g.v[12] = (int32_t)cg;
}

// r in (-2p, p) -> sign * r mod p in [0, p) (sign < 0: negate), limbs normalised
CESS_HD void normalize30(s30& r, int32_t sign) {
  int32_t ca = r.v[12] >> 31;
#pragma unroll
  for (int i = 0; i < 13; i++) r.v[i] += c::P30[i] & ca;
  const int32_t cn = sign >> 31;
#pragma unroll
  for (int i = 0; i < 13; i++) r.v[i] = (r.v[i] ^ cn) - cn;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i + 1] += r.v[i] >> 30, r.v[i] &= M30;
  ca = r.v[12] >> 31;
#pragma unroll
  for (int i = 0; i < 13; i++) r.v[i] += c::P30[i] & ca;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i + 1] += r.v[i] >> 30, r.v[i] &= M30;
}

// a^-1 in Montgomery form (inv(0) = 0)
CESS_HD fp inv(const fp& a0) {
  const fp a = fp_reduce_once(a0);   // canonical aR mod p
  s30 f, g, d, e;
#pragma unroll
  for (int k = 0; k < 13; k++) {
    const int off = 30 * k, i = off >> 5, sh = off & 31;
    uint32_t w = i < 12 ? a.v[i] >> sh : 0u;
    if (sh > 2 && i + 1 < 12) w |= a.v[i + 1] << (32 - sh);
    g.v[k] = (int32_t)(w & (uint32_t)M30);
    f.v[k] = c::P30[k];
    d.v[k] = 0;
    e.v[k] = 0;
  }
  e.v[0] = 1;
  int32_t zeta = -1;
#pragma unroll 1
  for (int it = 0; it < 37; it++) {
    if (it >= 25) {   // leave once g = 0 in every lane of the wave (uniform)
      uint32_t nz = 0;
#pragma unroll
      for (int k = 0; k < 13; k++) nz |= (uint32_t)g.v[k];
#if defined(CESS_HOSTEMU)
      if (nz == 0) break;
#else
      if (__ballot(nz != 0) == 0) break;
#endif
    }
    int32_t u, v, q, r;
    zeta = divsteps30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], u, v, q, r);
    update_de30(d, e, u, v, q, r);
    update_fg30(f, g, u, v, q, r);
  }
  // f = +-1 (or p when a = 0, with d = 0): d a = f mod p
  normalize30(d, f.v[12]);
  fp x;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const int off = 32 * j, k = off / 30, sh = off - 30 * k;
    uint32_t w = (uint32_t)d.v[k] >> sh;
    w |= (uint32_t)d.v[k + 1] << (30 - sh);
    if (sh > 28 && k + 2 < 13) w |= (uint32_t)d.v[k + 2] << (60 - sh);
    x.v[j] = w;
  }
  return mul(x, fp_from(c::R3));   // (aR)^-1 R^3 / R = a^-1 R
}

// returns true and a root if a is a square
CESS_HD bool sqrt(fp& r, const fp& a) {
  r = pow_fixed(a, c::EXP_SQRT);
  return eq(sqr(r), a);
}

// canonical compare: raw (non-Montgomery) a > (p-1)/2
CESS_HD bool raw_gt_half(const fp& a_raw) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)subc32(c::P_HALF_RAW[i], a_raw.v[i], borrow, &borrow);
  return borrow != 0;  // (p-1)/2 - a < 0
}
CESS_HD bool lex_largest(const fp& a) { return raw_gt_half(from_mont(a)); }

// raw a < p ?
CESS_HD bool raw_lt_p(const fp& a_raw) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)subc32(a_raw.v[i], c::P_RAW[i], borrow, &borrow);
  return borrow != 0;
}

// 48 big-endian bytes -> raw limbs
CESS_HD fp raw_from_be48(const uint8_t* b) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  return r;
}
CESS_HD void raw_to_be48(const fp& a, uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = a.v[i] >> 24;
    q[1] = a.v[i] >> 16;
    q[2] = a.v[i] >> 8;
    q[3] = a.v[i];
  }
}

// ---------------------------------------------------------------------------
// Fp2 = Fp[u]/(u^2 + 1)
// ---------------------------------------------------------------------------
CESS_HD fp2 fp2_zero() { return {fp_zero(), fp_zero()}; }
CESS_HD fp2 fp2_one() { return {fp_one(), fp_zero()}; }
// Fp2 add/sub with the two components' carry chains interleaved limb by limb
// (one chain alone stalls on the VCC carry hazard between dependent links).
CESS_HD fp2 add(const fp2& a, const fp2& b) {
  fp t0, t1, s0, s1;
  uint32_t c0 = 0, c1 = 0, b0 = 0, b1 = 0;
#if CESS_ADD_ILV
  // the two sums and their trial subtractions: four chains, no wait states
#pragma unroll
  for (int i = 0; i < 12; i++) {
    t0.v[i] = addc32(a.c0.v[i], b.c0.v[i], c0, &c0);
    t1.v[i] = addc32(a.c1.v[i], b.c1.v[i], c1, &c1);
    s0.v[i] = subc32(t0.v[i], c::P2_RAW[i], b0, &b0);
    s1.v[i] = subc32(t1.v[i], c::P2_RAW[i], b1, &b1);
  }
#else
#pragma unroll
  for (int i = 0; i < 12; i++) {
    t0.v[i] = addc32(a.c0.v[i], b.c0.v[i], c0, &c0);
    t1.v[i] = addc32(a.c1.v[i], b.c1.v[i], c1, &c1);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) {
    s0.v[i] = subc32(t0.v[i], c::P2_RAW[i], b0, &b0);
    s1.v[i] = subc32(t1.v[i], c::P2_RAW[i], b1, &b1);
  }
#endif
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.v[i] = b0 ? t0.v[i] : s0.v[i];
    r.c1.v[i] = b1 ? t1.v[i] : s1.v[i];
  }
  return r;
}
CESS_HD fp2 sub(const fp2& a, const fp2& b) {
#if CESS_ADD_ILV
  // the two differences and the same plus 2p: four chains, no wait states
  fp t0, t1, u0, u1;
  uint32_t b0 = 0, b1 = 0, c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    t0.v[i] = subc32(a.c0.v[i], b.c0.v[i], b0, &b0);
    t1.v[i] = subc32(a.c1.v[i], b.c1.v[i], b1, &b1);
    u0.v[i] = addc32(t0.v[i], c::P2_RAW[i], c0, &c0);
    u1.v[i] = addc32(t1.v[i], c::P2_RAW[i], c1, &c1);
  }
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.v[i] = b0 ? u0.v[i] : t0.v[i];
    r.c1.v[i] = b1 ? u1.v[i] : t1.v[i];
  }
  return r;
#else
  fp t0, t1;
  uint32_t b0 = 0, b1 = 0, c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    t0.v[i] = subc32(a.c0.v[i], b.c0.v[i], b0, &b0);
    t1.v[i] = subc32(a.c1.v[i], b.c1.v[i], b1, &b1);
  }
  const uint32_t m0 = 0u - b0, m1 = 0u - b1;
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.v[i] = addc32(t0.v[i], c::P2_RAW[i] & m0, c0, &c0);
    r.c1.v[i] = addc32(t1.v[i], c::P2_RAW[i] & m1, c1, &c1);
  }
  return r;
#endif
}
// unreduced, for mul() operands only (see add_nr(fp, fp))
CESS_HD fp2 add_nr(const fp2& a, const fp2& b) {
  fp2 r;
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.v[i] = addc32(a.c0.v[i], b.c0.v[i], c0, &c0);
    r.c1.v[i] = addc32(a.c1.v[i], b.c1.v[i], c1, &c1);
  }
  return r;
}
CESS_HD fp2 dbl(const fp2& a) { return {dbl(a.c0), dbl(a.c1)}; }
// a + xi b unreduced, xi = 1 + u: (a0 + b0 + (2p - b1), a1 + b0 + b1), each
// component < 6p < 2^384 for a, b < 2p -- for mul() operands only (see
// add_nr).  Four interleaved carry chains and no conditional subtraction,
// against mul_nr's two reduced chains plus add_nr.
CESS_HD fp2 add_xi_nr(const fp2& a, const fp2& b) {
  fp2 r;
  uint32_t bn = 0, k0 = 0, k1 = 0, k2 = 0, k3 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t nb1 = subc32(c::P2_RAW[i], b.c1.v[i], bn, &bn);
    const uint32_t s0 = addc32(a.c0.v[i], b.c0.v[i], k0, &k0);
    const uint32_t s1 = addc32(a.c1.v[i], b.c0.v[i], k1, &k1);
    r.c0.v[i] = addc32(s0, nb1, k2, &k2);
    r.c1.v[i] = addc32(s1, b.c1.v[i], k3, &k3);
  }
  return r;
}

CESS_HD fp2 neg(const fp2& a) { return {neg(a.c0), neg(a.c1)}; }
CESS_HD fp2 conj(const fp2& a) { return {a.c0, neg(a.c1)}; }
CESS_HD bool is_zero(const fp2& a) { return is_zero(a.c0) && is_zero(a.c1); }
CESS_HD bool eq(const fp2& a, const fp2& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
CESS_HD fp2 select(bool c, const fp2& a, const fp2& b) { return {select(c, a.c0, b.c0), select(c, a.c1, b.c1)}; }
CESS_HD fp2 mul3(const fp2& a) { return {mul3(a.c0), mul3(a.c1)}; }
CESS_HD fp2 mul4(const fp2& a) { return {mul4(a.c0), mul4(a.c1)}; }
CESS_HD fp2 mul8(const fp2& a) { return {mul8(a.c0), mul8(a.c1)}; }

// Inputs may be unreduced (each component < 2^384, e.g. add_nr sums): only
// mul() and add_nr() touch them, and every output is reduced.
#ifndef CESS_FP2_MUL_LAZY
#define CESS_FP2_MUL_LAZY 1
#endif
#if !CESS_FP2_MUL_LAZY
// Karatsuba with three separately reduced products (fewer live registers than
// the lazy form below: for kernels that run two waves per SIMD)
CESS_HD fp2 mul(const fp2& a, const fp2& b) {
  fp v0 = mul(a.c0, b.c0), v1 = mul(a.c1, b.c1);
  fp t = mul(add_nr(a.c0, a.c1), add_nr(b.c0, b.c1));
  return {sub(v0, v1), sub(sub(t, v0), v1)};
}
#else
// Lazily reduced schoolbook form: c0 = a0 b0 + a1 (K - b1) and
// c1 = a0 b1 + a1 b0 (K = c::NEG_K28, digit-wise -b1 mod p), four
// half-products accumulated straight into the two reduction columns -- no
// per-column combination of separate sums (64-bit subtractions, each with a
// carry hazard on gfx950) and no operand digit sums.  Columns stay below
// 14 x 2^56 x 4 + 2^36 < 2^62; c0 < 2^768 + 2^769 < p R, so each reduction
// returns < 2p.  1,176 mads against 980 for the lazily reduced Karatsuba form
// (v0 = a0 b0, v1 = a1 b1, t = (a0 + a1)(b0 + b1) combined per column), but
// 1,529 VALU instructions against 1,756: k_miller 180.4 -> 170.4, k_final
// 188.4 -> 183.9 ms per 1 M (profiles/r02o_sweep.txt).
// mul_scaled<S>(a, b) = S a b, S <= 3, with a's digits scaled after the unpack
// (digits < 3 x 2^28: columns < 14 (2^57.6 + 2^58.6) + 2^59.8 < 2^63.3, and
// S a b < 9 x 2^769 < p R, so the reduction still returns < 2p): the small
// multiple costs one instruction per digit instead of Fp2 additions.
template <uint32_t S>
CESS_HD fp2 mul_scaled(const fp2& a, const fp2& b) {
  static_assert(S >= 1 && S <= 3, "digit bound");
  CESS_COUNT_MUL2();
  fp a0 = a.c0, a1 = a.c1, b0 = b.c0, b1 = b.c1;
  seq(a0);
  seq(a1);
  seq(b0);
  seq(b1);
  uint32_t x0[14], x1[14], y0[14], y1[14], y1n[14];
  unpack28(a0, x0);
  unpack28(a1, x1);
  unpack28(b0, y0);
  unpack28(b1, y1);
#pragma unroll
  for (int i = 0; i < 14; i++) {
    y1n[i] = c::NEG_K28[i] - y1[i];
    x0[i] *= S;
    x1[i] *= S;
  }
  fp2 r;
  mont28x2(
      [&](int k, int h, uint64_t& acc0, uint64_t& acc1) {
#pragma unroll
        for (int i = 0; i < 14; i++) {
          const int j = k - i;
          if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
          mac(acc0, x0[i], y0[j]);
          mac(acc1, x0[i], y1[j]);
          mac(acc0, x1[i], y1n[j]);
          mac(acc1, x1[i], y0[j]);
        }
      },
      r.c0, r.c1);
  seq(r.c0);
  seq(r.c1);
  return r;
}
CESS_HD fp2 mul(const fp2& a, const fp2& b) { return mul_scaled<1>(a, b); }
// Two independent lazy products r = S a b, q = S c d in ONE column loop
// (mont28x4): the same mads and bounds as two mul_scaled<S> calls, but four
// accumulation chains for the wave to interleave (a lone product measured
// 4.9 cycles per instruction at one wave per SIMD against 4.0 for dot2's
// denser columns, profiles/round5_e_fp_probe.txt).  For kernels with the
// register room (working set ~260 VGPRs: k_miller).
template <uint32_t S>
CESS_HD void mul2_scaled(const fp2& a, const fp2& b, const fp2& c, const fp2& d, fp2& r, fp2& q) {
  static_assert(S >= 1 && S <= 3, "digit bound");
  CESS_COUNT_MUL2();
  CESS_COUNT_MUL2();
  fp a0 = a.c0, a1 = a.c1, b0 = b.c0, b1 = b.c1, c0 = c.c0, c1 = c.c1, d0 = d.c0, d1 = d.c1;
  seq(a0);
  seq(a1);
  seq(b0);
  seq(b1);
  seq(c0);
  seq(c1);
  seq(d0);
  seq(d1);
  uint32_t x0[14], x1[14], y0[14], y1[14], y1n[14], u0[14], u1[14], w0[14], w1[14], w1n[14];
  unpack28(a0, x0);
  unpack28(a1, x1);
  unpack28(b0, y0);
  unpack28(b1, y1);
  unpack28(c0, u0);
  unpack28(c1, u1);
  unpack28(d0, w0);
  unpack28(d1, w1);
#pragma unroll
  for (int i = 0; i < 14; i++) {
    y1n[i] = c::NEG_K28[i] - y1[i];
    w1n[i] = c::NEG_K28[i] - w1[i];
    x0[i] *= S;
    x1[i] *= S;
    u0[i] *= S;
    u1[i] *= S;
  }
  mont28x4(
      [&](int k, int, uint64_t& acc0, uint64_t& acc1, uint64_t& acc2, uint64_t& acc3) {
#pragma unroll
        for (int i = 0; i < 14; i++) {
          const int j = k - i;
          if (j < 0 || j >= 14) continue;
          mac(acc0, x0[i], y0[j]);
          mac(acc1, x0[i], y1[j]);
          mac(acc2, u0[i], w0[j]);
          mac(acc3, u0[i], w1[j]);
          mac(acc0, x1[i], y1n[j]);
          mac(acc1, x1[i], y0[j]);
          mac(acc2, u1[i], w1n[j]);
          mac(acc3, u1[i], w0[j]);
        }
      },
      r.c0, r.c1, q.c0, q.c1);
  seq(r.c0);
  seq(r.c1);
  seq(q.c0);
  seq(q.c1);
}
CESS_HD void mul2(const fp2& a, const fp2& b, const fp2& c, const fp2& d, fp2& r, fp2& q) {
  mul2_scaled<1>(a, b, c, d, r, q);
}
#endif
// a*b + c*d over Fp2 with ONE Montgomery reduction per output component:
// the schoolbook form of mul(fp2, fp2) above, 8 half-products straight into
// the two reduction columns (columns < 14 x 2^56 x 7 + 2^36 < 2^63,
// c0 < 2^770.6 < p R, so each reduction returns < 2p), against two products
// (2,352 mads) and an Fp2 addition.  Same input contract as mul(fp2, fp2).
CESS_HD fp2 dot2(const fp2& a, const fp2& b, const fp2& c, const fp2& d) {
  CESS_COUNT_HALVES(8);   // algorithmic work: the Karatsuba form's 6 half-products + 2 reductions
  fp a0 = a.c0, a1 = a.c1, b0 = b.c0, b1 = b.c1, c0 = c.c0, c1 = c.c1, d0 = d.c0, d1 = d.c1;
  seq(a0);
  seq(a1);
  seq(b0);
  seq(b1);
  seq(c0);
  seq(c1);
  seq(d0);
  seq(d1);
  uint32_t xa0[14], xa1[14], yb0[14], yb1[14], xc0[14], xc1[14], yd0[14], yd1[14], yb1n[14], yd1n[14];
  unpack28(a0, xa0);
  unpack28(a1, xa1);
  unpack28(b0, yb0);
  unpack28(b1, yb1);
  unpack28(c0, xc0);
  unpack28(c1, xc1);
  unpack28(d0, yd0);
  unpack28(d1, yd1);
#pragma unroll
  for (int i = 0; i < 14; i++) yb1n[i] = c::NEG_K28[i] - yb1[i], yd1n[i] = c::NEG_K28[i] - yd1[i];
  fp2 r;
  mont28x2(
      [&](int k, int h, uint64_t& acc0, uint64_t& acc1) {
#pragma unroll
        for (int i = 0; i < 14; i++) {
          const int j = k - i;
          if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
          mac(acc0, xa0[i], yb0[j]);
          mac(acc1, xa0[i], yb1[j]);
          mac(acc0, xa1[i], yb1n[j]);
          mac(acc1, xa1[i], yb0[j]);
          mac(acc0, xc0[i], yd0[j]);
          mac(acc1, xc0[i], yd1[j]);
          mac(acc0, xc1[i], yd1n[j]);
          mac(acc1, xc1[i], yd0[j]);
        }
      },
      r.c0, r.c1);
  seq(r.c0);
  seq(r.c1);
  return r;
}

// a^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u as two half-products over ONE unpack of
// a0, a1: -a1 is the digit vector K - a1 (c::NEG_K28, K = 0 mod p, digits at
// least those of any value < 2^384), 2 a1 a doubled digit vector, so neither
// needs a modular subtraction or doubling.  Columns of (a0 + a1)(a0 + K - a1)
// stay below 14 x 2^58.6 + 14 x 2^56 < 2^62.6 and its value below
// 2^385 x 2^385.1 < p R, so each reduction returns < 2p.  Inputs < 2^384.
// (k_final 210.2 -> 207.2 ms per 1 M against two separate products,
// profiles/r02i_sweep.txt.)
CESS_HD fp2 sqr(const fp2& a) {
  CESS_COUNT_MUL();
  CESS_COUNT_MUL();
  fp a0 = a.c0, a1 = a.c1;
  seq(a0);
  seq(a1);
  uint32_t x0[14], x1[14], s[14], d[14], x1d[14];
  unpack28(a0, x0);
  unpack28(a1, x1);
#pragma unroll
  for (int i = 0; i < 14; i++) {
    s[i] = x0[i] + x1[i];
    d[i] = x0[i] + (c::NEG_K28[i] - x1[i]);
    x1d[i] = x1[i] << 1;
  }
  fp2 r;
  mont28x2(
      [&](int k, int h, uint64_t& acc0, uint64_t& acc1) {
#pragma unroll
        for (int i = 0; i < 14; i++) {
          const int j = k - i;
          if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
          mac(acc0, s[i], d[j]);
          mac(acc1, x0[i], x1d[j]);
        }
      },
      r.c0, r.c1);
  seq(r.c0);
  seq(r.c1);
  return r;
}

CESS_HD fp2 mul_fp(const fp2& a, const fp& s) { return {mul(a.c0, s), mul(a.c1, s)}; }
// * xi = (1 + u)
CESS_HD fp2 mul_nr(const fp2& a) { return {sub(a.c0, a.c1), add(a.c0, a.c1)}; }
CESS_HD fp2 inv(const fp2& a) {
  fp t = inv(add(sqr(a.c0), sqr(a.c1)));
  return {mul(a.c0, t), neg(mul(a.c1, t))};
}
CESS_HD bool lex_largest(const fp2& a) {
  fp c1 = from_mont(a.c1);
  if (!is_zero(c1)) return raw_gt_half(c1);
  return raw_gt_half(from_mont(a.c0));
}

// Square root in Fp2 via the norm (p = 3 mod 4): returns false if a is not a square.
// Any root is acceptable: callers normalise the sign (lexicographic rule).
CESS_HD bool sqrt(fp2& r, const fp2& a) {
  if (is_zero(a.c1)) {
    // a real: sqrt(a0) if a0 is a QR, else sqrt(-a0) * u
    fp s;
    if (sqrt(s, a.c0)) {
      r = {s, fp_zero()};
      return true;
    }
    bool ok = sqrt(s, neg(a.c0));
    r = {fp_zero(), s};
    return ok;
  }
  fp n = add(sqr(a.c0), sqr(a.c1));
  fp s;
  if (!sqrt(s, n)) return false;
  // exactly one of al = (a0 + s)/2, al' = (a0 - s)/2 is a nonzero square
  // (a1 != 0), and al * al' = -a1^2/4.  With t = al^((p-3)/4):
  //   al square:     x = (t al, a1 t / 2)
  //   al non-square: t^2 al = -1, so sqrt(al') = -a1 t / 2 and a1 / (2 sqrt(al'))
  //                  = -1/t = t al:  x = (-a1 t / 2, t al)
  // (p = 3 mod 8).  One exponentiation instead of a second one on al'; the
  // final check below covers both branches.
  const fp half = fp_from(c::HALF);
  const fp al = mul(add(a.c0, s), half);
  const fp t = pow_fixed(al, c::EXP_SQRT_RATIO);  // al^((p-3)/4)
  const fp u = mul(t, al);                        // sqrt(al) if al is a square
  const fp w = mul(mul(a.c1, t), half);           // a1 t / 2
  const bool sq = eq(mul(u, t), fp_one());        // t^2 al == 1
  r = {select(sq, u, neg(w)), select(sq, w, u)};
  return eq(sqr(r), a);
}

// ---------------------------------------------------------------------------
// Fp6 = Fp2[v]/(v^3 - xi)
// ---------------------------------------------------------------------------
CESS_HD fp6 fp6_zero() { return {fp2_zero(), fp2_zero(), fp2_zero()}; }
CESS_HD fp6 fp6_one() { return {fp2_one(), fp2_zero(), fp2_zero()}; }
CESS_HD fp6 add(const fp6& a, const fp6& b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
CESS_HD fp6 sub(const fp6& a, const fp6& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1), sub(a.c2, b.c2)}; }
CESS_HD fp6 neg(const fp6& a) { return {neg(a.c0), neg(a.c1), neg(a.c2)}; }
CESS_HD fp6 dbl(const fp6& a) { return {dbl(a.c0), dbl(a.c1), dbl(a.c2)}; }
CESS_HD bool eq(const fp6& a, const fp6& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1) && eq(a.c2, b.c2); }
// * v
CESS_HD fp6 mul_v(const fp6& a) { return {mul_nr(a.c2), a.c0, a.c1}; }
// unreduced, for mul() operands only
CESS_HD fp6 add_nr(const fp6& a, const fp6& b) { return {add_nr(a.c0, b.c0), add_nr(a.c1, b.c1), add_nr(a.c2, b.c2)}; }

#ifndef CESS_MUL2
#define CESS_MUL2 0
#endif
CESS_HD fp6 mul(const fp6& a, const fp6& b) {
#if CESS_MUL2
  // the six Karatsuba products as three independent pairs (mul2)
  fp2 t0, t1, t2, u0, u1, u2;
  mul2(a.c0, b.c0, a.c1, b.c1, t0, t1);
  mul2(a.c2, b.c2, add_nr(a.c1, a.c2), add_nr(b.c1, b.c2), t2, u0);
  mul2(add_nr(a.c0, a.c1), add_nr(b.c0, b.c1), add_nr(a.c0, a.c2), add_nr(b.c0, b.c2), u1, u2);
  fp2 c0 = add(mul_nr(sub(sub(u0, t1), t2)), t0);
  fp2 c1 = add(sub(sub(u1, t0), t1), mul_nr(t2));
  fp2 c2 = add(sub(sub(u2, t0), t2), t1);
  return {c0, c1, c2};
#else
  fp2 t0 = mul(a.c0, b.c0);
  fp2 t1 = mul(a.c1, b.c1);
  fp2 t2 = mul(a.c2, b.c2);
  // inputs may be unreduced (< 2p per Fp component); sums feed mul() only
  fp2 c0 = add(mul_nr(sub(sub(mul(add_nr(a.c1, a.c2), add_nr(b.c1, b.c2)), t1), t2)), t0);
  fp2 c1 = add(sub(sub(mul(add_nr(a.c0, a.c1), add_nr(b.c0, b.c1)), t0), t1), mul_nr(t2));
  fp2 c2 = add(sub(sub(mul(add_nr(a.c0, a.c2), add_nr(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
#endif
}
CESS_HD fp6 sqr(const fp6& a) {
  // CH-SQR2
  fp2 s0 = sqr(a.c0);
  fp2 ab = mul(a.c0, a.c1);
  fp2 s1 = dbl(ab);
  fp2 s2 = sqr(add(sub(a.c0, a.c1), a.c2));
  fp2 bc = mul(a.c1, a.c2);
  fp2 s3 = dbl(bc);
  fp2 s4 = sqr(a.c2);
  fp2 c0 = add(mul_nr(s3), s0);
  fp2 c1 = add(mul_nr(s4), s1);
  fp2 c2 = sub(sub(add(add(s1, s2), s3), s0), s4);
  return {c0, c1, c2};
}
// a * (b0 + b1 v)
CESS_HD fp6 mul_by_01(const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0 = mul(a.c0, b0);
  fp2 t1 = mul(a.c1, b1);
  fp2 c0 = add(mul_nr(mul(a.c2, b1)), t0);
  fp2 c1 = sub(sub(mul(add_nr(a.c0, a.c1), add_nr(b0, b1)), t0), t1);
  fp2 c2 = add(mul(a.c2, b0), t1);
  return {c0, c1, c2};
}
// a * (b1 v)
CESS_HD fp6 mul_by_1(const fp6& a, const fp2& b1) {
#if CESS_MUL2
  fp2 p2, p0;
  mul2(a.c2, b1, a.c0, b1, p2, p0);
  return {mul_nr(p2), p0, mul(a.c1, b1)};
#else
  return {mul_nr(mul(a.c2, b1)), mul(a.c0, b1), mul(a.c1, b1)};
#endif
}
CESS_HD fp6 inv(const fp6& a) {
  fp2 c0 = sub(sqr(a.c0), mul_nr(mul(a.c1, a.c2)));
  fp2 c1 = sub(mul_nr(sqr(a.c2)), mul(a.c0, a.c1));
  fp2 c2 = sub(sqr(a.c1), mul(a.c0, a.c2));
  fp2 t = add(mul(a.c0, c0), mul_nr(add(mul(a.c2, c1), mul(a.c1, c2))));
  t = inv(t);
  return {mul(c0, t), mul(c1, t), mul(c2, t)};
}

// ---------------------------------------------------------------------------
// Fp12 = Fp6[w]/(w^2 - v)
// ---------------------------------------------------------------------------
CESS_HD fp12 fp12_one() { return {fp6_one(), fp6_zero()}; }
CESS_HD bool eq(const fp12& a, const fp12& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
CESS_HD bool is_one(const fp12& a) { return eq(a, fp12_one()); }
CESS_HD fp12 conj(const fp12& a) { return {a.c0, neg(a.c1)}; }

CESS_HD fp12 mul(const fp12& a, const fp12& b) {
  fp6 t0 = mul(a.c0, b.c0);
  fp6 t1 = mul(a.c1, b.c1);
  fp6 c1 = sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1);
  fp6 c0 = add(t0, mul_v(t1));
  return {c0, c1};
}
CESS_HD fp12 sqr(const fp12& a) {
  fp6 ab = mul(a.c0, a.c1);
  fp6 c0 = sub(sub(mul(add(a.c0, a.c1), add(a.c0, mul_v(a.c1))), ab), mul_v(ab));
  return {c0, dbl(ab)};
}
// f * (c0 + c1 v + c4 v w)   (bls12_381 Fp12::mul_by_014)
CESS_HD fp12 mul_by_014(const fp12& f, const fp2& c0, const fp2& c1, const fp2& c4) {
  fp6 aa = mul_by_01(f.c0, c0, c1);
  fp6 bb = mul_by_1(f.c1, c4);
  fp2 o = add(c1, c4);
  fp6 t = mul_by_01(add(f.c1, f.c0), c0, o);
  fp6 r1 = sub(sub(t, aa), bb);
  fp6 r0 = add(mul_v(bb), aa);
  return {r0, r1};
}
CESS_HD fp12 inv(const fp12& a) {
  fp6 t = sub(mul(a.c0, a.c0), mul_v(mul(a.c1, a.c1)));
  t = inv(t);
  return {mul(a.c0, t), neg(mul(a.c1, t))};
}

// Frobenius^k (k = 1, 2, 3): coefficient of w^i is conj^k(a_i) * gamma_{k,i}
// w-basis order: c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2  (i = 0..5)
CESS_HD fp2 frob_coeff(int k, int i) {
  return {fp_from(c::FROB[k - 1][i][0]), fp_from(c::FROB[k - 1][i][1])};
}
template <int K>
CESS_HD fp12 frobenius(const fp12& a) {
  auto f = [](const fp2& x, int i) -> fp2 {
    fp2 y = (K & 1) ? conj(x) : x;
    if (i == 0) return y;
    return mul(y, frob_coeff(K, i));
  };
  fp12 r;
  r.c0.c0 = f(a.c0.c0, 0);
  r.c1.c0 = f(a.c1.c0, 1);
  r.c0.c1 = f(a.c0.c1, 2);
  r.c1.c1 = f(a.c1.c1, 3);
  r.c0.c2 = f(a.c0.c2, 4);
  r.c1.c2 = f(a.c1.c2, 5);
  return r;
}

// Granger-Scott squaring in the cyclotomic subgroup (eprint 2009/565)
// (a + b s)^2 in Fp4 = Fp2[s]/(s^2 - xi): c0 = a^2 + xi b^2, c1 = 2ab.
// (A single-reduction form of c0 -- five half-products accumulated with
// digit-negated operands, two reductions -- issues 8 % fewer instructions in
// the square run but needs ~190 registers and spills at two waves per SIMD:
// k_final 221.7 vs 211.9 ms per 1 M, profiles/r02g_sweep.txt.)
CESS_HD void fp4_square(fp2& c0, fp2& c1, const fp2& a, const fp2& b) {
  fp2 t0 = sqr(a);
  fp2 t1 = sqr(b);
  c0 = add(mul_nr(t1), t0);
  c1 = sub(sub(sqr(add(a, b)), t0), t1);
}
CESS_HD fp12 cyclotomic_square(const fp12& f) {
  fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2;
  fp2 z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fp2 t0, t1, t2, t3;
  fp4_square(t0, t1, z0, z1);
  z0 = sub(t0, z0);
  z0 = add(dbl(z0), t0);
  z1 = add(t1, z1);
  z1 = add(dbl(z1), t1);
  fp4_square(t0, t1, z2, z3);
  fp4_square(t2, t3, z4, z5);
  z4 = sub(t0, z4);
  z4 = add(dbl(z4), t0);
  z5 = add(t1, z5);
  z5 = add(dbl(z5), t1);
  t0 = mul_nr(t3);
  z2 = add(t0, z2);
  z2 = add(dbl(z2), t0);
  z3 = sub(t2, z3);
  z3 = add(dbl(z3), t2);
  fp12 r;
  r.c0 = {z0, z4, z3};
  r.c1 = {z2, z1, z5};
  return r;
}

// f^x for x = -0xd201000000010000 in the cyclotomic subgroup
CESS_HD fp12 cyclotomic_exp(const fp12& f) {
  // |x| bits below the leading one (bit 63): 62, 60, 57, 48, 16
  fp12 t = f;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    t = cyclotomic_square(t);
    if (b == 62 || b == 60 || b == 57 || b == 48 || b == 16) t = mul(t, f);
  }
  return conj(t);
}

}  // namespace bls
