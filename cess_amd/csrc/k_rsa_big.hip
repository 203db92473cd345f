// RSA PKCS#1 v1.5 verify for moduli of 2049-4096 bits (rsa.hpp: the loop-form
// size class).  Same verification as k_rsa.hpp (reference:
// primitives/enclave-verify/src/lib.rs:221-228, rsa 0.8.2
// RsaPublicKey::verify(Pkcs1v15Sign::new_raw(), msg, sig)) with the limb count
// L = K.limbs a run-time value: Montgomery products in finely integrated
// operand-scanning form (FIOS, 28-bit digits, 64-bit column values never above
// 2^58), RSA_BIG_ROWS rows per pass as a systolic chain (rsa_mont.hpp), over
// per-lane arrays in private memory.
// Keys of these sizes are rare (Podr2Key is 2048-bit,
// primitives/common/src/lib.rs:54): the kernel exists so that every key the
// reference verifies gets a GPU verdict, not for throughput.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "rsa.hpp"
#include "rsa_mont.hpp"

using namespace rsa_big;

// rec: this class's record list (its length at *cnt), key_idx / keys / the
// record buffers as k_rsa_verify_2048.  One lane per record.
__global__ __launch_bounds__(256) void k_rsa_verify_big(uint32_t n_max, const uint32_t* __restrict__ cnt,
                                                        const uint32_t* __restrict__ rec,
                                                        const uint32_t* __restrict__ key_idx,
                                                        const RsaKeyDev* __restrict__ keys,
                                                        const uint8_t* __restrict__ sigs,
                                                        const uint64_t* __restrict__ sig_offs,
                                                        const uint8_t* __restrict__ msgs,
                                                        const uint64_t* __restrict__ msg_offs,
                                                        uint8_t* __restrict__ codes) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= *cnt || t >= n_max) return;
  const uint32_t r = rec[t];
  if (r == RSA_PAD) return;
  const RsaKeyDev& K = keys[key_idx[r]];
  const int L = (int)K.limbs, kb = (int)K.k_bytes;
  if (L <= 0 || L > RSA_LMAX) return;   // the host never builds such a row
  const uint32_t* n = K.n28;
  uint32_t x[RSA_LMAX + 1], base[RSA_LMAX + 1], y[RSA_LMAX + 1];
  // s = OS2IP(sig) -> 28-bit limbs (bit k of s = bit k % 8 of byte kb - 1 - k / 8)
  const uint8_t* sg = sigs + sig_offs[r];
  for (int q = 0; q < L; q++) x[q] = 0;
  for (int i = 0; i < kb; i++) {
    const uint32_t v = sg[kb - 1 - i];
    const int bit = 8 * i, li = bit / 28, sh = bit % 28;
    x[li] |= (v << sh) & M28;
    if (sh > 20 && li + 1 < L) x[li + 1] |= v >> (28 - sh);
  }
  // s < n (RSAVP1 step 1)
  int32_t borrow = 0;
  for (int i = 0; i < L; i++) {
    const int32_t d = (int32_t)x[i] - (int32_t)n[i] - borrow;
    borrow = d < 0;
  }
  if (!borrow) {
    codes[r] = RSA_SIG_RANGE;
    return;
  }
  // Montgomery form, then left-to-right binary exponentiation by e
  mont_rt(x, K.r2_28, n, K.ninv, L, base);
  for (int i = 0; i < L; i++) x[i] = base[i];
  const uint64_t e = K.e;
  const int top = 63 - __builtin_clzll(e);
  for (int bit = top - 1; bit >= 0; bit--) {
    mont_rt(x, x, n, K.ninv, L, y);
    if ((e >> bit) & 1)
      mont_rt(y, base, n, K.ninv, L, x);
    else
      for (int i = 0; i < L; i++) x[i] = y[i];
  }
  // out of Montgomery form (x * 1 / R <= n), canonical
  for (int i = 0; i < L; i++) base[i] = i == 0;
  mont_rt(x, base, n, K.ninv, L, y);
  {
    int32_t br = 0;
    for (int i = 0; i < L; i++) {
      const int32_t d = (int32_t)y[i] - (int32_t)n[i] - br;
      br = d < 0;
      x[i] = (uint32_t)d & M28;
    }
    if (br)
      for (int i = 0; i < L; i++) x[i] = y[i];
  }
  // EM = I2OSP(m, k) == 0x00 0x01 0xff.. 0x00 || msg: byte i from the least
  // significant end is EM[kb - 1 - i]; every bit of m above 8 kb must be zero
  const uint8_t* msg = msgs + msg_offs[r];
  const int tl = (int)(msg_offs[r + 1] - msg_offs[r]);
  bool ok = true;
  for (int i = 0; i < (28 * L + 7) / 8; i++) {
    const int bit = 8 * i, li = bit / 28, sh = bit % 28;
    uint32_t got = x[li] >> sh;
    if (sh > 20 && li + 1 < L) got |= x[li + 1] << (28 - sh);
    got &= 0xff;
    const int b = kb - 1 - i;   // big-endian position
    uint32_t want;
    if (b < 0) want = 0;
    else if (b == 0) want = 0x00;
    else if (b == 1) want = 0x01;
    else if (b < kb - tl - 1) want = 0xff;
    else if (b == kb - tl - 1) want = 0x00;
    else want = msg[b - (kb - tl)];
    ok = ok && got == want;
  }
  codes[r] = ok ? RSA_OK : RSA_MISMATCH;
}
