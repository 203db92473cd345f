// RSA batch front end (see k_rsa.hpp): per record, the length checks of
// rsa 0.8.2's pkcs1v15 verify (sig.len() == k, k >= msg.len() + 11) and the
// key lookup; records that pass are appended to their size class's list
// (1024 / 2048-bit moduli), the others get their final code here.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "rsa.hpp"

__global__ __launch_bounds__(256) void k_rsa_classify(uint64_t n, const uint32_t* __restrict__ key_idx, uint32_t nkeys,
                                                      const RsaKeyDev* __restrict__ keys,
                                                      const uint8_t* __restrict__ key_ok,
                                                      const uint64_t* __restrict__ sig_offs,
                                                      const uint64_t* __restrict__ msg_offs,
                                                      uint8_t* __restrict__ codes, uint32_t* __restrict__ lists,
                                                      uint32_t* __restrict__ counts) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t j = key_idx[r];
  if (j >= nkeys || !key_ok[j]) {   // no such key / the key did not load
    codes[r] = RSA_KEY;
    return;
  }
  const RsaKeyDev& K = keys[j];
  const uint64_t sl = sig_offs[r + 1] - sig_offs[r], ml = msg_offs[r + 1] - msg_offs[r];
  if (sl != K.k_bytes) {
    codes[r] = RSA_SIG_LEN;
    return;
  }
  if ((uint64_t)K.k_bytes < ml + 11) {
    codes[r] = RSA_MSG_LEN;
    return;
  }
  const int cls = K.limbs == RSA_L1024 ? 0 : 1;
  const uint32_t pos = atomicAdd(&counts[cls], 1u);
  lists[(uint64_t)cls * n + pos] = (uint32_t)r;
}
