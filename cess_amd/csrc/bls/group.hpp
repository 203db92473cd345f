// One lane's operation of a lane-group program round (gen_group.py encoding;
// bls/group_prog.hpp), shared by the kernel (k_group.hip, LDS register file)
// and the host emulation of the test harness (tests/hostemu/group_emu.cpp).
// group_eval returns the value and its destination slot; the caller stores it
// after every lane of the round has read its operands (lockstep in a wave).
#pragma once
#include "field.hpp"
#include "group_prog.hpp"

namespace bls {

enum : uint32_t { GRP_MUL = 0, GRP_SQR = 1, GRP_LIN = 2, GRP_INV = 3 };

// pool constant k (Montgomery form)
CESS_HD fp2 grp_const(uint32_t k) {
  fp2 r;
#pragma unroll
  for (int l = 0; l < 12; l++) r.c0.v[l] = grp::kConsts[k][l], r.c1.v[l] = grp::kConsts[k][12 + l];
  return r;
}

// byte p (0..15) of a 16-byte entry
CESS_HD uint32_t grp_byte(uint32_t ex, uint32_t ey, uint32_t ez, uint32_t ew, uint32_t p) {
  const uint32_t w = p < 4 ? ex : p < 8 ? ey : p < 12 ? ez : ew;
  return (w >> (8 * (p & 3))) & 0xffu;
}

// MUL/SQR operand: a slot or a constant, optionally +- a second slot
template <class Regs>
CESS_HD fp2 grp_operand(const Regs& R, uint32_t x0, uint32_t x1, uint32_t fl, uint32_t present, uint32_t subtract,
                        uint32_t is_const) {
  fp2 v = (fl & is_const) ? grp_const(x0) : R.ld(x0);
  if (fl & present) {
    const fp2 t = R.ld(x1);
    v = (fl & subtract) ? sub(v, t) : add_nr(v, t);
  }
  return v;
}

// ---------------------------------------------------------------------------
// Two lanes per operation: lane (2 op + comp) computes component `comp` of
// op's result.  Both components of a lazy Fp2 product are sums of two
// half-products over the same digits (c0 = a0 b0 + a1 (K - b1), c1 = a0 b1 +
// a1 b0; field.hpp mul_scaled), and of a square one half-product each (c0 =
// (a0 + a1)(a0 + K - a1), c1 = a0 (2 a1)); a lane selects its operand digits
// and runs ONE reduction, so the wave issues half a product's instructions --
// the latency of a round halves (a lone wave is issue-bound).
// ---------------------------------------------------------------------------
CESS_HD fp grp_mul_comp(const fp2& a, const fp2& b, uint32_t comp) {
  CESS_COUNT_HALVES(3);
  fp a0 = a.c0, a1 = a.c1, b0 = b.c0, b1 = b.c1;
  seq(a0);
  seq(a1);
  seq(b0);
  seq(b1);
  uint32_t x0[14], x1[14], u0[14], u1[14], y0[14], y1[14];
  unpack28(a0, x0);
  unpack28(a1, x1);
  unpack28(b0, u0);
  unpack28(b1, u1);
#pragma unroll
  for (int i = 0; i < 14; i++) {
    y0[i] = comp ? u1[i] : u0[i];
    y1[i] = comp ? u0[i] : c::NEG_K28[i] - u1[i];
  }
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      const int j = k - i;
      if (j < 0 || j >= 14 || (h >= 0 && (i & 1) != h)) continue;
      mac(acc, x0[i], y0[j]);
      mac(acc, x1[i], y1[j]);
    }
  });
  seq(r);
  return r;
}

CESS_HD fp grp_sqr_comp(const fp2& a, uint32_t comp) {
  CESS_COUNT_HALVES(2);
  fp a0 = a.c0, a1 = a.c1;
  seq(a0);
  seq(a1);
  uint32_t x0[14], x1[14], xs[14], ys[14];
  unpack28(a0, x0);
  unpack28(a1, x1);
#pragma unroll
  for (int i = 0; i < 14; i++) {
    xs[i] = comp ? x0[i] : x0[i] + x1[i];
    ys[i] = comp ? (x1[i] << 1) : x0[i] + (c::NEG_K28[i] - x1[i]);
  }
  fp r = mont28([&](int k, int h, uint64_t& acc) {
#pragma unroll
    for (int i = 0; i < 14; i++)
      if (k - i >= 0 && k - i < 14 && (h < 0 || (i & 1) == h)) mac(acc, xs[i], ys[k - i]);
  });
  seq(r);
  return r;
}

// component `comp` of an operation's result (register file: < 2p per component)
template <class Regs>
CESS_HD fp group_eval_comp(const Regs& R, uint32_t kind, uint32_t ex, uint32_t ey, uint32_t ez, uint32_t ew,
                           uint32_t comp, uint32_t* dest) {
  *dest = ex & 0xffu;
  if (kind == GRP_MUL || kind == GRP_SQR) {
    const uint32_t a0 = (ex >> 8) & 0xffu, a1 = (ex >> 16) & 0xffu, b0 = ex >> 24;
    const uint32_t b1 = ey & 0xffu, f = (ey >> 8) & 0xffu;
    fp2 A = grp_operand(R, a0, a1, f, 1, 2, 16);
    if (f & 64) A = conj(A);   // only on a plain operand (gen_group.py)
    if (kind == GRP_SQR) return grp_sqr_comp(A, comp);
    const fp2 B = grp_operand(R, b0, b1, f, 4, 8, 32);
    return grp_mul_comp(A, B, comp);
  }
  if (kind == GRP_LIN) {
    // plain terms: this lane's component only; xi terms: both (xi mixes them)
    const uint32_t n0 = (ex >> 8) & 15u, n1 = (ex >> 12) & 15u, n2 = (ex >> 16) & 15u, n3 = (ex >> 20) & 15u;
    uint32_t p = 3;
    fp acc = fp_zero();
    fp2 accx = fp2_zero();
#pragma unroll 1
    for (uint32_t t = 0; t < n0; t++) acc = add(acc, R.ld_comp(grp_byte(ex, ey, ez, ew, p++), comp));
#pragma unroll 1
    for (uint32_t t = 0; t < n1; t++) acc = sub(acc, R.ld_comp(grp_byte(ex, ey, ez, ew, p++), comp));
#pragma unroll 1
    for (uint32_t t = 0; t < n2; t++) accx = add(accx, R.ld(grp_byte(ex, ey, ez, ew, p++)));
#pragma unroll 1
    for (uint32_t t = 0; t < n3; t++) accx = sub(accx, R.ld(grp_byte(ex, ey, ez, ew, p++)));
    if (n2 + n3) acc = add(acc, comp ? add(accx.c0, accx.c1) : sub(accx.c0, accx.c1));   // xi = 1 + u
    return acc;
  }
  const fp2 v = inv(R.ld((ex >> 8) & 0xffu));   // GRP_INV (both lanes, one component each)
  return comp ? v.c1 : v.c0;
}

// values in the register file are < 2p per component; sums feed products only
template <class Regs>
CESS_HD fp2 group_eval(const Regs& R, uint32_t kind, uint32_t ex, uint32_t ey, uint32_t ez, uint32_t ew,
                       uint32_t* dest) {
  *dest = ex & 0xffu;
  if (kind == GRP_MUL || kind == GRP_SQR) {
    const uint32_t a0 = (ex >> 8) & 0xffu, a1 = (ex >> 16) & 0xffu, b0 = ex >> 24;
    const uint32_t b1 = ey & 0xffu, f = (ey >> 8) & 0xffu;
    fp2 A = grp_operand(R, a0, a1, f, 1, 2, 16);
    if (f & 64) A = conj(A);   // only on a plain operand (gen_group.py)
    if (kind == GRP_SQR) return sqr(A);
    const fp2 B = grp_operand(R, b0, b1, f, 4, 8, 32);
    return mul(A, B);
  }
  if (kind == GRP_LIN) {
    const uint32_t n0 = (ex >> 8) & 15u, n1 = (ex >> 12) & 15u, n2 = (ex >> 16) & 15u, n3 = (ex >> 20) & 15u;
    uint32_t p = 3;
    fp2 acc = fp2_zero(), accx = fp2_zero();
#pragma unroll 1
    for (uint32_t t = 0; t < n0; t++) acc = add(acc, R.ld(grp_byte(ex, ey, ez, ew, p++)));
#pragma unroll 1
    for (uint32_t t = 0; t < n1; t++) acc = sub(acc, R.ld(grp_byte(ex, ey, ez, ew, p++)));
#pragma unroll 1
    for (uint32_t t = 0; t < n2; t++) accx = add(accx, R.ld(grp_byte(ex, ey, ez, ew, p++)));
#pragma unroll 1
    for (uint32_t t = 0; t < n3; t++) accx = sub(accx, R.ld(grp_byte(ex, ey, ez, ew, p++)));
    if (n2 + n3) acc = add(acc, mul_nr(accx));
    return acc;
  }
  return inv(R.ld((ex >> 8) & 0xffu));   // GRP_INV
}

}  // namespace bls
