// RSA batch front end (see k_rsa.hpp): per record, the length checks of
// rsa 0.8.2's pkcs1v15 verify (sig.len() == k, k >= msg.len() + 11) and the
// key lookup; records that pass are appended to their size class's list
// (1024 / 2048-bit moduli, and 2049-4096 for the loop-form kernel), the
// others get their final code here.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "rsa.hpp"

// the length checks and key lookup of one record: its size class (0: 1024,
// 1: 2048-bit modulus, 2: larger) or -1 with its final code written (codes may
// be null)
__device__ __forceinline__ int rsa_class(uint64_t r, uint64_t n, const uint32_t* __restrict__ key_idx, uint32_t nkeys,
                                         const RsaKeyDev* __restrict__ keys, const uint8_t* __restrict__ key_ok,
                                         const uint64_t* __restrict__ sig_offs, const uint64_t* __restrict__ msg_offs,
                                         uint8_t* __restrict__ codes) {
  if (r >= n) return -1;
  const uint32_t j = key_idx[r];
  if (j >= nkeys || !key_ok[j]) {   // no such key / the key did not load
    if (codes) codes[r] = RSA_KEY;
    return -1;
  }
  const RsaKeyDev& K = keys[j];
  const uint64_t sl = sig_offs[r + 1] - sig_offs[r], ml = msg_offs[r + 1] - msg_offs[r];
  if (sl != K.k_bytes) {
    if (codes) codes[r] = RSA_SIG_LEN;
    return -1;
  }
  if ((uint64_t)K.k_bytes < ml + 11) {
    if (codes) codes[r] = RSA_MSG_LEN;
    return -1;
  }
  return K.limbs == RSA_L1024 ? 0 : K.limbs == RSA_L2048 ? 1 : 2;
}

// wave-aggregated atomicAdd(&ctr[slot], 1) for the lanes with slot >= 0; returns
// each such lane's old value (one atomic per distinct slot of the wave when the
// slots agree, per-lane atomics otherwise)
__device__ __forceinline__ uint32_t wave_append(uint32_t* __restrict__ ctr, int64_t slot) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t act = __ballot(slot >= 0);
  if (!act) return 0;
  const int leader = __ffsll((unsigned long long)act) - 1;
  const int64_t s0 = __shfl(slot, leader);
  if (__ballot(slot >= 0 && slot != s0) == 0) {
    uint32_t b = 0;
    if ((int)lane == leader) b = atomicAdd(&ctr[s0], (uint32_t)__popcll(act));
    b = __shfl(b, leader);
    return b + (uint32_t)__popcll(act & ((1ull << lane) - 1));
  }
  return slot >= 0 ? atomicAdd(&ctr[slot], 1u) : 0u;
}

// Key-uniform path (few keys, many records each): records of each (class,
// key) are placed in a segment of the class list whose start is a multiple of
// 64, so every wave of the verification kernel sees one key (k_rsa_2048u).
// Only taken for tables without keys of the loop-form class (classes 0, 1).
// count -> scan -> scatter; slots are cls * nkeys + key.
__global__ __launch_bounds__(256) void k_rsa_count(uint64_t n, const uint32_t* __restrict__ key_idx, uint32_t nkeys,
                                                   const RsaKeyDev* __restrict__ keys,
                                                   const uint8_t* __restrict__ key_ok,
                                                   const uint64_t* __restrict__ sig_offs,
                                                   const uint64_t* __restrict__ msg_offs, uint8_t* __restrict__ codes,
                                                   uint32_t* __restrict__ cnt) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cls = rsa_class(r, n, key_idx, nkeys, keys, key_ok, sig_offs, msg_offs, codes);
  (void)wave_append(cnt, cls < 0 ? -1 : (int64_t)cls * nkeys + key_idx[r]);
}
// one thread: 64-aligned exclusive prefix of the counts per class; totals[c]
// = the padded length of class c's list
__global__ void k_rsa_scan(uint32_t nkeys, const uint32_t* __restrict__ cnt, uint32_t* __restrict__ segbase,
                           uint32_t* __restrict__ totals) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (uint32_t c = 0; c < 2; c++) {
    uint32_t off = 0;
    for (uint32_t k = 0; k < nkeys; k++) {
      segbase[c * nkeys + k] = off;
      off += (cnt[c * nkeys + k] + 63u) & ~63u;
    }
    totals[c] = off;
  }
}
__global__ __launch_bounds__(256) void k_rsa_scatter(uint64_t n, const uint32_t* __restrict__ key_idx, uint32_t nkeys,
                                                     const RsaKeyDev* __restrict__ keys,
                                                     const uint8_t* __restrict__ key_ok,
                                                     const uint64_t* __restrict__ sig_offs,
                                                     const uint64_t* __restrict__ msg_offs,
                                                     const uint32_t* __restrict__ segbase, uint32_t* __restrict__ cur,
                                                     uint32_t* __restrict__ lists, uint64_t cap) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // (codes were written by k_rsa_count)
  const int cls = rsa_class(r, n, key_idx, nkeys, keys, key_ok, sig_offs, msg_offs, nullptr);
  const int64_t slot = cls < 0 ? -1 : (int64_t)cls * nkeys + key_idx[r];
  const uint32_t pos = wave_append(cur, slot);
  if (slot >= 0) lists[(uint64_t)cls * cap + segbase[slot] + pos] = (uint32_t)r;
}

__global__ __launch_bounds__(256) void k_rsa_classify(uint64_t n, const uint32_t* __restrict__ key_idx, uint32_t nkeys,
                                                      const RsaKeyDev* __restrict__ keys,
                                                      const uint8_t* __restrict__ key_ok,
                                                      const uint64_t* __restrict__ sig_offs,
                                                      const uint64_t* __restrict__ msg_offs,
                                                      uint8_t* __restrict__ codes, uint32_t* __restrict__ lists,
                                                      uint32_t* __restrict__ counts) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // size class of a record that goes on to the verify kernels
  const int cls = rsa_class(r, n, key_idx, nkeys, keys, key_ok, sig_offs, msg_offs, codes);
  // wave-aggregated append: one atomic per wave and class (a per-lane atomic on
  // one counter serialises the whole batch in L2: 47.5 ms for 4 M records,
  // more than the 2048-bit verification itself, profiles/round3_rsa_a_*)
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const uint64_t mask = __ballot(cls == c);
    if (!mask) continue;
    const int leader = __ffsll((unsigned long long)mask) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&counts[c], (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    if (cls == c) lists[(uint64_t)c * n + base + __popcll(mask & below)] = (uint32_t)r;
  }
}
