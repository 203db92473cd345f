// Montgomery product of the loop-form RSA class (k_rsa_big.hip): run-time
// limb count, 28-bit digits.  Host-compilable with -DCESS_HOSTEMU for the CPU
// test of the systolic row schedule (tests/test_rsa.py).
#pragma once
#include <stdint.h>

#include "rsa.hpp"

#if defined(CESS_HOSTEMU)
#define CESS_RSA_HD inline
#else
#include <hip/hip_runtime.h>
#define CESS_RSA_HD __device__ inline
#endif

namespace rsa_big {

constexpr uint32_t M28 = 0x0fffffffu;

// out = a b R^-1 mod n, in [0, 2n) for a, b < 2n (4n <= R = 2^(28 L)); out
// (L + 1 words) must not alias a or b.  FIOS rows (one per digit a_i: m_i from
// the running low word, then t <- (t + a_i b + m_i n) / 2^28), RSA_BIG_ROWS
// of them per pass over the columns: the rows of a pass run as a systolic
// chain, row r one column behind row r - 1 and fed its output word in a
// register, so one pass reads t, b and n and writes t once per column for
// RSA_BIG_ROWS rows (the one-row form moved 3 L^2 private words per product).
// The host pads L to a multiple of RSA_BIG_ROWS (rsa.hpp), so the first and
// last chunk of RSA_BIG_ROWS steps have compile-time column offsets and the
// chunks between them run every row on an interior column.
CESS_RSA_HD void mont_rt(const uint32_t* a, const uint32_t* b, const uint32_t* __restrict__ n, uint32_t ninv, int L,
                        uint32_t* t) {
  constexpr int KR = RSA_BIG_ROWS;
  for (int j = 0; j <= L; j++) t[j] = 0;
#pragma unroll 1
  for (int i0 = 0; i0 < L; i0 += KR) {
    uint32_t ar[KR], m[KR], c[KR], top[KR], bw[KR], nw[KR];
#pragma unroll
    for (int r = 0; r < KR; r++) ar[r] = a[i0 + r], c[r] = 0, top[r] = 0, m[r] = 0;
    // interior column of row r: window slot w holds column col's b and n
    auto mid = [&](int r, int w, uint32_t in) -> uint32_t {
      const uint64_t u = (uint64_t)in + (uint64_t)ar[r] * bw[w] + (uint64_t)m[r] * nw[w] + c[r];
      c[r] = (uint32_t)(u >> 28);
      return (uint32_t)u & M28;
    };
    // first chunk: steps s = q, row r on column q - r (column 0: m_r)
#pragma unroll
    for (int q = 0; q < KR; q++) {
      bw[q] = b[q];
      nw[q] = n[q];
      uint32_t pass = t[q];
#pragma unroll
      for (int r = 0; r <= q; r++) {
        if (r == q) {   // column 0
          uint64_t u = (uint64_t)pass + (uint64_t)ar[r] * bw[0];
          m[r] = ((uint32_t)u * ninv) & M28;
          u += (uint64_t)m[r] * nw[0];
          c[r] = (uint32_t)(u >> 28);   // the low 28 bits are zero
        } else {
          pass = mid(r, q - r, pass);
        }
      }
    }
    // interior chunks: every row on a column in [1, L - 1]; row KR - 1 writes
    // column s - KR of the result in place (row 0 read it KR steps earlier)
#pragma unroll 1
    for (int s0 = KR; s0 < L; s0 += KR) {
#pragma unroll
      for (int q = 0; q < KR; q++) {
        const int s = s0 + q;
        bw[q] = b[s];
        nw[q] = n[s];
        uint32_t pass = t[s];
#pragma unroll
        for (int r = 0; r < KR; r++) pass = mid(r, (q - r + KR) % KR, pass);
        t[s - KR] = pass;
      }
    }
    // last chunk: steps s = L + q; row r reaches column L (the carry word) at
    // q == r and hands its top word to row r + 1 one step later
#pragma unroll
    for (int q = 0; q < KR; q++) {
      uint32_t pass = q == 0 ? t[L] : 0;
#pragma unroll
      for (int r = 0; r < KR; r++) {
        if (q < r) {
          pass = mid(r, (q - r + KR) % KR, pass);
        } else if (q == r) {
          const uint64_t u = (uint64_t)pass + c[r];
          pass = (uint32_t)u & M28;
          top[r] = (uint32_t)(u >> 28);
        } else if (q == r + 1) {
          pass = top[r];
        }
      }
      t[L + q - KR] = pass;   // row KR - 1 on column L + q - (KR - 1)
    }
    t[L] = top[KR - 1];
  }
}

}  // namespace rsa_big
