// CDNA4 (gfx950) batch RSA PKCS#1 v1.5 raw signature verification -- SURVEY
// §8(f) rank 4: cp_enclave_verify::verify_rsa (reference
// primitives/enclave-verify/src/lib.rs:221-228) =
// RsaPublicKey::verify(Pkcs1v15Sign::new_raw(), msg, sig) of rsa 0.8.2:
//   s = OS2IP(sig) (< n), m = s^e mod n, EM = I2OSP(m, k) must equal
//   0x00 0x01 0xff..0xff 0x00 || msg.
// One lane = one signature.  The modulus is held in 28-bit limbs (L of them,
// R = 2^(28 L) >= 4n) so every limb product is one v_mad_u64_u32 into a 64-bit
// column accumulator (product scanning, no carry flags; a column holds at most
// 2L products < 2^56: 2L * 2^56 < 2^64 for L <= 110).  Values stay in [0, 2n)
// between Montgomery products (no conditional subtraction until the end).
// Squarings accumulate the off-diagonal products once and double the column.
// The host has already rejected wrong signature / message lengths (codes 1, 3);
// the kernel returns 0 OK, 2 SIG_RANGE (s >= n), 4 MISMATCH.
#pragma once
#include <hip/hip_runtime.h>

#include <utility>

#include "kernels.hpp"
#include "rsa.hpp"

namespace rsa_detail {

constexpr uint32_t M28 = 0x0fffffffu;

// 0, data-dependent on x: each column's products start after the previous
// column is complete, so the scheduler cannot hoist a fully unrolled
// product scan's independent columns and run out of registers
__device__ __forceinline__ uint64_t zero_after(uint64_t x) {
  uint32_t z;
  asm volatile("" : "=v"(z) : "0"(0u), "v"((uint32_t)x));
  return z;
}

template <int L>
struct Big {
  uint32_t v[L];
};

// out = a * b * R^-1 mod n (in [0, 2n) for a, b < 2n).  out may alias a or b:
// out[j] is written at column L + j, after the last use of a[j] and b[j]
// (column j + L - 1).  The column loop and its product sums are expanded by
// templates (ColStep<K> / fold expressions), so the scan is straight-line code
// with compile-time limb indices at any L (a `#pragma unroll` of the 2L - 1
// columns is not honoured at L = 37+, which sends the limb arrays to scratch).
template <int L>
struct MontCtx {
  const uint32_t (&a)[L];
  const uint32_t (&b)[L];
  const uint32_t (&n)[L];
  uint32_t ninv;
  uint32_t (&m)[L];
  uint32_t (&out)[L];
  uint64_t acc;
};

// column K of a * b (SQR: of a^2, off-diagonal products once, then doubled)
template <int L, bool SQR, int K, int I>
__device__ __forceinline__ void ab_term(MontCtx<L>& c, uint64_t& col) {
  constexpr int J = K - I;
  if constexpr (SQR) {
    if constexpr (J > I && J < L) col += (uint64_t)c.a[I] * c.a[J];
  } else {
    if constexpr (J >= 0 && J < L) col += (uint64_t)c.a[I] * c.b[J];
  }
}
template <int L, int K, int I>
__device__ __forceinline__ void mn_term(MontCtx<L>& c) {
  constexpr int J = K - I;
  if constexpr (I < K && J >= 0 && J < L) c.acc += (uint64_t)c.m[I] * c.n[J];
}
template <int L, bool SQR, int K, int... I>
__device__ __forceinline__ void column(MontCtx<L>& c, std::integer_sequence<int, I...>) {
  uint64_t col = zero_after(c.acc);
  (ab_term<L, SQR, K, I>(c, col), ...);
  if constexpr (SQR) {
    col <<= 1;
    if constexpr ((K & 1) == 0 && (K >> 1) < L) col += (uint64_t)c.a[K >> 1] * c.a[K >> 1];
  }
  c.acc += col;
  (mn_term<L, K, I>(c), ...);
  if constexpr (K < L) {
    c.m[K] = ((uint32_t)c.acc * c.ninv) & M28;
    c.acc += (uint64_t)c.m[K] * c.n[0];
  } else {
    c.out[K - L] = (uint32_t)c.acc & M28;
  }
  c.acc >>= 28;
}
template <int L, bool SQR, int K>
__device__ __forceinline__ void columns(MontCtx<L>& c) {
  column<L, SQR, K>(c, std::make_integer_sequence<int, L>{});
  if constexpr (K + 1 < 2 * L - 1) columns<L, SQR, K + 1>(c);
}

template <int L, bool SQR>
__device__ __forceinline__ void mont(const uint32_t (&a)[L], const uint32_t (&b)[L], const uint32_t (&n)[L],
                                     uint32_t ninv, uint32_t (&out)[L]) {
  uint32_t m[L];
  MontCtx<L> c{a, b, n, ninv, m, out, 0};
  columns<L, SQR, 0>(c);
  out[L - 1] = (uint32_t)c.acc;   // < 2n < R: the top limb holds the rest
}

// a - n if a >= n (a < 2n)
template <int L>
__device__ __forceinline__ void canon(uint32_t (&a)[L], const uint32_t (&n)[L]) {
  uint32_t d[L];
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int32_t t = (int32_t)a[i] - (int32_t)n[i] - borrow;
    borrow = t < 0;
    d[i] = (uint32_t)t & M28;
  }
#pragma unroll
  for (int i = 0; i < L; i++) a[i] = borrow ? a[i] : d[i];
}

// 28-bit limbs -> W 32-bit words (compile-time shifts)
template <int L, int W>
__device__ __forceinline__ void to_words(const uint32_t (&a)[L], uint32_t (&w)[W]) {
#pragma unroll
  for (int j = 0; j < W; j++) {
    uint32_t r = 0;
#pragma unroll
    for (int t = 0; t < L; t++) {
      const int lo = 28 * t;
      if (lo < 32 * j + 32 && lo + 28 > 32 * j) {
        const int sh = lo - 32 * j;
        r |= sh >= 0 ? (a[t] << sh) : (a[t] >> -sh);
      }
    }
    w[j] = r;
  }
}

}  // namespace rsa_detail
using namespace rsa_detail;

// One size class: L 28-bit limbs.  rec[t] = record of lane t; keys[] rows of
// the distinct-key table (rsa.hpp RsaKeyDev).  base: SoA scratch (L words per
// lane, stride `cnt` = the launch's n_max) for s R mod n, re-read for the final multiply of each
// exponent bit, so the exponentiation keeps 3 L values live (x, n, m).
// UNI: the wave's records share one key (key-sorted, wave-padded lists of
// k_rsa_scatter), so the key row is read through a wave-uniform index and the
// modulus limbs live in SGPRs: the exponentiation keeps 2 L values (x, m) in
// VGPRs instead of 3 L.  PAD list entries (0xffffffff) are inactive lanes.
template <int L, bool UNI = false>
__device__ __forceinline__ void rsa_verify_lane(uint32_t t, uint32_t cnt, const uint32_t* __restrict__ rec,
                                                const uint32_t* __restrict__ key_idx,
                                                const RsaKeyDev* __restrict__ keys, const uint8_t* __restrict__ sigs,
                                                const uint64_t* __restrict__ sig_offs, const uint8_t* __restrict__ msgs,
                                                const uint64_t* __restrict__ msg_offs, uint32_t* __restrict__ base,
                                                uint8_t* __restrict__ codes) {
  const uint32_t r = rec[t];
  if (r == RSA_PAD) return;
  const uint32_t ki = key_idx[r];
  const RsaKeyDev& K = keys[UNI ? __builtin_amdgcn_readfirstlane(ki) : ki];
  const int kb = (int)K.k_bytes;
  uint32_t n[L], x[L];
#pragma unroll
  for (int i = 0; i < L; i++) n[i] = K.n28[i];
  // s = OS2IP(sig): big-endian bytes -> 28-bit limbs (limb q takes the bytes
  // whose bits meet [28 q, 28 q + 28); byte i counted from the least significant)
  const uint8_t* sg = sigs + sig_offs[r];
#pragma unroll
  for (int q = 0; q < L; q++) {
    uint32_t v = 0;
#pragma unroll
    for (int i = (28 * q) / 8; i <= (28 * q + 27) / 8; i++) {
      const uint32_t byte = i < kb ? (uint32_t)sg[kb - 1 - i] : 0u;
      const int sh = 8 * i - 28 * q;
      v |= sh >= 0 ? (byte << sh) : (byte >> -sh);
    }
    x[q] = v & M28;
  }
  // s < n (RSAVP1 step 1)
  {
    int32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int32_t d = (int32_t)x[i] - (int32_t)n[i] - borrow;
      borrow = d < 0;
    }
    if (!borrow) {
      codes[r] = RSA_SIG_RANGE;
      return;
    }
  }
  // x = s R mod n (Montgomery form), kept as the exponentiation's base
  {
    uint32_t r2[L];
#pragma unroll
    for (int i = 0; i < L; i++) r2[i] = K.r2_28[i];
    mont<L, false>(x, r2, n, K.ninv, x);
  }
#pragma unroll
  for (int i = 0; i < L; i++) base[(uint64_t)i * cnt + t] = x[i];
  // left-to-right binary exponentiation by e (e = 65537: 16 squarings, 1 product)
  const uint64_t e = K.e;
  const int top = 63 - __builtin_clzll(e);
#pragma unroll 1
  for (int bit = top - 1; bit >= 0; bit--) {
    mont<L, true>(x, x, n, K.ninv, x);
    if ((e >> bit) & 1) {
      uint32_t y[L];
#pragma unroll
      for (int i = 0; i < L; i++) y[i] = base[(uint64_t)i * cnt + t];
      mont<L, false>(x, y, n, K.ninv, x);
    }
  }
  // out of Montgomery form, canonical
  {
    uint32_t one[L];
#pragma unroll
    for (int i = 0; i < L; i++) one[i] = i == 0;
    mont<L, false>(x, one, n, K.ninv, x);
  }
  canon<L>(x, n);
  // EM = I2OSP(m, k) == 0x00 0x01 0xff.. 0x00 || msg, compared byte by byte
  // from the least significant end (byte i is EM[k - 1 - i])
  const uint8_t* msg = msgs + msg_offs[r];
  const int tl = (int)(msg_offs[r + 1] - msg_offs[r]);
  constexpr int W = (28 * L + 31) / 32;
  uint32_t w[W];
  to_words<L, W>(x, w);
  bool ok = true;
#pragma unroll
  for (int j = 0; j < W; j++) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t got = (w[j] >> (8 * q)) & 0xff;
      const int b = kb - 1 - (4 * j + q);   // big-endian position
      uint32_t want;
      if (b < 0) want = 0;
      else if (b == 0) want = 0x00;
      else if (b == 1) want = 0x01;
      else if (b < kb - tl - 1) want = 0xff;
      else if (b == kb - tl - 1) want = 0x00;
      else want = msg[b - (kb - tl)];
      ok = ok && got == want;
    }
  }
  codes[r] = ok ? RSA_OK : RSA_MISMATCH;
}

// rec: this class's record list (its length at *cnt, filled by
// k_rsa_classify or k_rsa_scatter); base: SoA scratch of stride n_max.
#define CESS_RSA_KERNEL(NAME, L, WAVES)                                                                              \
  __global__ __launch_bounds__(256, WAVES) void NAME(                                                                \
      uint32_t n_max, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ rec,                            \
      const uint32_t* __restrict__ key_idx, const RsaKeyDev* __restrict__ keys, const uint8_t* __restrict__ sigs,   \
      const uint64_t* __restrict__ sig_offs, const uint8_t* __restrict__ msgs,                                      \
      const uint64_t* __restrict__ msg_offs, uint32_t* __restrict__ base, uint8_t* __restrict__ codes) {            \
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;                                                        \
    if (t >= *cnt) return;                                                                                           \
    rsa_verify_lane<L>(t, n_max, rec, key_idx, keys, sigs, sig_offs, msgs, msg_offs, base, codes);                  \
  }
#define CESS_RSA_KERNEL_U(NAME, L, WAVES)                                                                            \
  __global__ __launch_bounds__(256, WAVES) void NAME(                                                                \
      uint32_t n_max, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ rec,                            \
      const uint32_t* __restrict__ key_idx, const RsaKeyDev* __restrict__ keys, const uint8_t* __restrict__ sigs,   \
      const uint64_t* __restrict__ sig_offs, const uint8_t* __restrict__ msgs,                                      \
      const uint64_t* __restrict__ msg_offs, uint32_t* __restrict__ base, uint8_t* __restrict__ codes) {            \
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;                                                        \
    if (t >= *cnt) return;                                                                                           \
    rsa_verify_lane<L, true>(t, n_max, rec, key_idx, keys, sigs, sig_offs, msgs, msg_offs, base, codes);            \
  }
