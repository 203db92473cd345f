// CDNA4 (gfx950) generator-side kernels (PrivateKey, reference src/lib.rs:166-236, A15):
//   k_keygen : pk = compress([sk] G2)          PrivateKey::public_key   src/lib.rs:226-228
//   k_sign   : sig = compress([sk] H(msg))     PrivateKey::sign         src/lib.rs:233-236
//   k_hash_out: compress(H(msg))               hash_to_g1               src/lib.rs:25-31
// Secret keys are 32-byte big-endian scalars < r (PrivateKey::deserialize, :208-223).
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

namespace {
__device__ void load_sk(const uint8_t* sk, uint32_t (&k)[8]) {
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const uint8_t* q = sk + 28 - 4 * w;
    k[w] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
__device__ void store_bytes(uint8_t* dst, const uint8_t* src, int n) {
  for (int j = 0; j < n; j++) dst[j] = src[j];
}

}  // namespace

__global__ CESS_LB void k_keygen(uint64_t n, const uint8_t* __restrict__ sks, uint8_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_sk(sks + 32 * i, k);
  fp2 gx = {fp_from(c::G2_GEN_X0), fp_from(c::G2_GEN_X1)};
  fp2 gy = {fp_from(c::G2_GEN_Y0), fp_from(c::G2_GEN_Y1)};
  g2a p = proj_to_affine(proj_mul_scalar_mixed(gx, gy, k));
  uint8_t b[96];
  g2_compress(p, b);
  store_bytes(out + 96 * i, b, 96);
}

__global__ CESS_LB void k_sign(uint64_t n, const uint8_t* __restrict__ sks, const uint8_t* __restrict__ msgs,
                                               const uint64_t* __restrict__ offs, uint8_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  load_sk(sks + 32 * i, k);
  uint64_t o = offs[i];
  __shared__ uint32_t park[48][256];   // SSWU values parked in LDS (k_hash.hip)
  g1a h = hash_to_g1_parked(msgs + o, (uint32_t)(offs[i + 1] - o), park, threadIdx.x);
  g1a s;
  if (h.inf) {
    s = h;
  } else {
    s = proj_to_affine(g1_mul_glv(h.x, h.y, k));
  }
  uint8_t b[48];
  g1_compress(s, b);
  store_bytes(out + 48 * i, b, 48);
}

__global__ CESS_LB void k_hash_out(uint64_t n, const uint8_t* __restrict__ msgs,
                                                   const uint64_t* __restrict__ offs, uint8_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t o = offs[i];
  __shared__ uint32_t park[48][256];
  g1a h = hash_to_g1_parked(msgs + o, (uint32_t)(offs[i + 1] - o), park, threadIdx.x);
  uint8_t b[48];
  g1_compress(h, b);
  store_bytes(out + 48 * i, b, 48);
}
