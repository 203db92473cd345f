// k_final2: final exponentiation -> code 0/5 + verdict bitmap
// (MillerLoopResult::final_exponentiation().is_identity(), src/lib.rs:93-99,
// SURVEY §8(a) A13/A14) on a lane PAIR per signature (bls/pair_fe.hpp):
// 256-thread blocks of 128 signatures, the accumulator in LDS (G[18][256],
// 72 KiB per block, two blocks per CU: two waves per SIMD), every opcode of
// the staged.hpp program in place on it; HBM slots hold the cold Fp12
// temporaries (same rows as k_final's).  Same arguments and outputs as
// k_final (k_final.hip): codes, the LSB-first bitmap, optional Gt bytes.
#include <hip/hip_runtime.h>
#include "soa.hpp"
#include "bls/pair_fe.hpp"

using namespace bls;
using namespace cess;

__constant__ uint8_t kFeProgramPair[][2] = {CESS_FE_PROGRAM};
__constant__ uint8_t kFeProgramPairVerify[][2] = {CESS_FE_PROGRAM_VERIFY};

__global__ __launch_bounds__(CESS_PAIR_THREADS, 2) void k_final2(uint64_t n, uint8_t* __restrict__ code, uint4* __restrict__ fin,
                                                   uint4* __restrict__ slots, uint64_t* __restrict__ bitmap,
                                                   uint8_t* __restrict__ gt_out, uint64_t stride) {
  // signature of the pair; both lanes of a pair take every branch together
  const uint32_t i = blockIdx.x * (blockDim.x >> 1) + (threadIdx.x >> 1);
  const uint32_t h = threadIdx.x & 1u;
  uint8_t c = CODE_SIG_LEN;
  if (i < n) {
    c = code[i];
    if (c == 0) {
      // slot views start at the wave's first signature (uniform)
      const uint32_t s0 = blockIdx.x * (blockDim.x >> 1) + (wave_first_thread() >> 1);
      __shared__ uint4 G[18][CESS_PAIR_THREADS];
      const LdsPair acc{G, wave_first_thread()};
      auto slot = [&](int s) {
        return GlobPair{(s == SL_F ? fin : slots + (uint64_t)(s - 1) * 36 * stride) + s0, stride};
      };
      // f = 1 ((O, O) records) has f^e = 1 (k_final.hip)
      if (gt_out || !pis_one12(slot(SL_F))) {
        final_exp_pair(acc, gt_out ? kFeProgramPair : kFeProgramPairVerify, slot);
        if (!(gt_out ? pis_one12(acc) : pis_conj12(acc, slot(SL_T4)))) c = CODE_PAIRING;
        if (gt_out) {   // 576 B per signature: Fp 2k + h of tower order from lane h
#pragma unroll 1
          for (int k = 0; k < 6; k++) {
            const fph e = acc.ld(k);
            uint8_t b[48];
            raw_to_be48(from_mont(e.v), b);
            for (int t = 0; t < 48; t++) gt_out[576 * (uint64_t)i + 96 * k + 48 * h + t] = b[t];
          }
        }
      }
      if (h == 0) code[i] = c;
    }
  }
  // 32 signatures per wave: the ballot's even bits, bit (i mod 32) of the
  // 32-bit half word i / 32 of the LSB-first bitmap; every half of a 64-bit
  // word that holds a record is written (zero bits past the last record, as
  // k_final's whole-word ballot)
  uint64_t x = __ballot(c == 0) & 0x5555555555555555ull;
  x = (x | (x >> 1)) & 0x3333333333333333ull;
  x = (x | (x >> 2)) & 0x0f0f0f0f0f0f0f0full;
  x = (x | (x >> 4)) & 0x00ff00ff00ff00ffull;
  x = (x | (x >> 8)) & 0x0000ffff0000ffffull;
  x = (x | (x >> 16)) & 0x00000000ffffffffull;
  if ((threadIdx.x & 63) == 0 && n > 0 && (i >> 6) <= ((n - 1) >> 6))
    reinterpret_cast<uint32_t*>(bitmap)[i >> 5] = (uint32_t)x;
}
