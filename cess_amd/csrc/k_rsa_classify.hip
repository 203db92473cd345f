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
  int cls = -1;   // size class of a record that goes on to the verify kernels
  if (r < n) {
    const uint32_t j = key_idx[r];
    if (j >= nkeys || !key_ok[j]) {   // no such key / the key did not load
      codes[r] = RSA_KEY;
    } else {
      const RsaKeyDev& K = keys[j];
      const uint64_t sl = sig_offs[r + 1] - sig_offs[r], ml = msg_offs[r + 1] - msg_offs[r];
      if (sl != K.k_bytes) codes[r] = RSA_SIG_LEN;
      else if ((uint64_t)K.k_bytes < ml + 11) codes[r] = RSA_MSG_LEN;
      else cls = K.limbs == RSA_L1024 ? 0 : 1;
    }
  }
  // wave-aggregated append: one atomic per wave and class (a per-lane atomic on
  // one counter serialises the whole batch in L2: 47.5 ms for 4 M records,
  // more than the 2048-bit verification itself, profiles/round3_rsa_a_*)
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint64_t mask = __ballot(cls == c);
    if (!mask) continue;
    const int leader = __ffsll((unsigned long long)mask) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&counts[c], (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    if (cls == c) lists[(uint64_t)c * n + base + __popcll(mask & below)] = (uint32_t)r;
  }
}
