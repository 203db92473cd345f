// CDNA4 (gfx950) kernels for batch BLS12-381 verification — one lane = one signature.
// k_final: final exponentiation -> code 0/5 + verdict bitmap (src/lib.rs:93-99, A13/A14)
//
// The exponentiation runs as a short program (bls/staged.hpp CESS_FE_PROGRAM)
// over two ping-pong accumulators (HBM slots 8 and 9) and seven HBM slots
// (uint4 SoA, stride = context capacity) for the cold Fp12 temporaries; the
// Miller-loop output is slot SL_F.  Cyclotomic square runs hold the accumulator in
// registers, with a third of it parked in LDS (two waves per SIMD).
#include <hip/hip_runtime.h>
#include "soa.hpp"

using namespace bls;
using namespace cess;

__constant__ uint8_t kFeProgram[][2] = {CESS_FE_PROGRAM};
// verdict only (no Gt bytes requested): one Fp12 multiply less (staged.hpp)
__constant__ uint8_t kFeProgramVerify[][2] = {CESS_FE_PROGRAM_VERIFY};

// two waves per SIMD (one wave with 512 registers and no scratch measured
// slower: 245 vs 212 ms per 1 M, profiles/r02g_sweep.txt)
#define CESS_LB_F12 __launch_bounds__(256, 2)

#if defined(CESS_DIAG)
CESS_DIAG_TABLE(k_final)
#endif

__global__ CESS_LB_F12 void k_final(uint64_t n, uint8_t* __restrict__ code, uint4* __restrict__ fin,
                                    uint4* __restrict__ slots, uint64_t* __restrict__ bitmap,
                                    uint8_t* __restrict__ gt_out, uint64_t stride) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t c = CODE_SIG_LEN;
  if (i < n) {
    c = code[i];
    if (c == 0) {
      // two HBM accumulators (slots SL_N - 1 and SL_N): FE_MUL ping-pongs.
      // Slot views start at the wave's first record (uniform) and add the
      // lane id per access (staged.hpp GlobF12W).
#if defined(CESS_FE_L2PROBE)
      // TIMING PROBE ONLY (wrong verdicts): every block's slot views alias the
      // first block's records, so the slots' working set (~2.4 MB) stays in
      // L2 -- k_final with its HBM latency removed
      const uint32_t w0 = wave_first_thread();
#else
      const uint32_t w0 = blockIdx.x * blockDim.x + wave_first_thread();
#endif
      GlobF12W acc0{slots + (uint64_t)(SL_N - 1) * 36 * stride + w0, stride};
      GlobF12W acc1{slots + (uint64_t)SL_N * 36 * stride + w0, stride};
      // 18 uint4 rows x 256 lanes = 72 KiB per block: two blocks per CU
      __shared__ uint4 park[18][256];
      auto slot = [&](int s) {
        return GlobF12W{(s == SL_F ? fin : slots + (uint64_t)(s - 1) * 36 * stride) + w0, stride};
      };
      // f = 1 (an (O, O) record: both Miller terms skipped) has f^e = 1: the
      // verdict is OK without the exponentiation, and the lane does not take
      // the Karabina fallback (z2 = z3 = 0 redoes every chain in Granger-Scott
      // form, for its whole wave).  (Gt bytes requested: the full program.)
#if defined(CESS_DIAG)
      // regions: 0 other opcodes, 1 FE_MUL, 2 FE_INV, 3 compressed squarings,
      // 4 decompression, 5 verdict
      Diag dg;
      dg.begin();
      Diag* dgp = &dg;
#else
      NoDiag* dgp = nullptr;
#endif
      if (gt_out || !is_one12(slot(SL_F))) {
        const int which = final_exp_staged(acc0, acc1, gt_out ? kFeProgram : kFeProgramVerify, slot,
                                           LdsF12{park, wave_first_thread()}, dgp);
        const GlobF12W acc = which ? acc1 : acc0;
        if (!(gt_out ? is_one12(acc) : is_conj12(acc, slot(SL_T4)))) c = CODE_PAIRING;
        if (gt_out) {   // optional Gt bytes for parity tests (576 B per signature)
#pragma unroll 1
          for (int k = 0; k < 6; k++) {
            fp2 e = acc.ld(k);
            uint8_t b[48];
            raw_to_be48(from_mont(e.c0), b);
            for (int t = 0; t < 48; t++) gt_out[576 * (uint64_t)i + 96 * k + t] = b[t];
            raw_to_be48(from_mont(e.c1), b);
            for (int t = 0; t < 48; t++) gt_out[576 * (uint64_t)i + 96 * k + 48 + t] = b[t];
          }
        }
      }
#if defined(CESS_DIAG)
      dg.mark<5>();
      dg.end(cess_diag_tab);
#endif
      code[i] = c;
    }
  }
  // one bitmap word per wave: bit (i mod 64) of word i/64 = (code == 0)
  uint64_t ball = __ballot(c == 0);
  if ((threadIdx.x & 63) == 0 && i < n) bitmap[i >> 6] = ball;
}
