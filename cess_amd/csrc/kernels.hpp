// Shared definitions between the HIP kernels and the host runtime.
#pragma once
#include <stdint.h>

// Register budget of the stage kernels: 256-thread blocks, at least
// CESS_MIN_WAVES waves per SIMD (512 / CESS_MIN_WAVES VGPR+AGPR per lane).
#ifndef CESS_MIN_WAVES
#define CESS_MIN_WAVES 1
#endif
#define CESS_LB __launch_bounds__(256, CESS_MIN_WAVES)

// verdict codes; precedence: signature, then key, then pairing
enum : uint8_t {
  CODE_OK = 0,
  CODE_SIG_LEN = 1,
  CODE_SIG_POINT = 2,
  CODE_PK_LEN = 3,
  CODE_PK_POINT = 4,
  CODE_PAIRING = 5,
};
// host-side pre-validation flags (variable-length API)
enum : uint8_t { PRE_SIG_LEN_BAD = 1, PRE_PK_LEN_BAD = 2 };
// identity flags
enum : uint8_t { INF_SIG = 1, INF_PK = 2 };

// words per signature of each SoA stage buffer
#define CESS_W_G1 24u          // affine G1
#define CESS_W_G2 48u          // affine G2
#define CESS_W_COEFFS 4896u    // 68 x 3 Fp2
#define CESS_W_FP12 144u
#define CESS_FE_SLOTS 16u      // HBM Fp12 slots of the final-exponentiation program (bls/staged.hpp):
                               // 7 temporaries, 6 powers of FE_CHAIN, FE_MUL's Fp6 temporary (SL_TM),
                               // 2 ping-pong accumulators

// RLC bucket sums (k_rlc.hip k_msm_*): 16 windows x 256 digit buckets per
// segment; a bucket of cnt entries is summed in chunks of msm_chunk(cnt)
// entries (at least 64, at most 32 chunks), one work item per chunk
#define CESS_MSM_SEG_BUCKETS 4096u
// records per lane of the distinct-key RLC's Miller values (k_miller_rr): a
// lane's value is the product of its records' Miller values
// threads per block of the lane-pair kernels (k_miller2, k_final2): two lanes
// per signature, an 18 x CESS_PAIR_THREADS uint4 LDS image per block, two
// waves per SIMD whatever the block size
#ifndef CESS_PAIR_THREADS
#define CESS_PAIR_THREADS 256
#endif
#ifndef CESS_RLCD_PER
#define CESS_RLCD_PER 4
#endif
#define CESS_MSM_MAX_SEGS 256u    // segments of one bucket pass (bucket tables <= 1 M entries, ~190 MB)
// Segments of one bucket pass (kernel argument): parts (perm-position ranges;
// their signatures) are segments 0 .. nparts - 1, terms (part x key group
// ranges; their hashes) nparts + t.  pos == nullptr: the batch's first check
// (one part = the whole batch, term g = key group g: segment 1 + grp[i]); else
// pos[i] = record i's perm position, looked up in the sorted bounds.
struct MsmSegs {
  const uint32_t *grp, *pos, *plo, *phi, *tlo, *thi;
  uint32_t nparts, nterms;
};
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t msm_chunk(uint32_t cnt) {
  const uint32_t c = (cnt + 31u) / 32u;
  return c > 64u ? c : 64u;
}
