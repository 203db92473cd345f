// In-kernel cycle stamps for DIAGNOSTIC builds only (-DCESS_DIAG, built as a
// variant by tools/build_variant.sh; never in the product library).
//
// A wave-uniform s_memtime is taken at each mark; the cycles since the
// previous mark are added to the region's accumulator (compile-time index,
// SGPRs).  At the end one lane per wave adds the accumulators, the wave's
// total s_memtime / s_memrealtime spans and a wave count into a per-
// translation-unit __device__ table (vector-memory atomics), which the TU's
// host function `cess_diag_read_<tu>` copies out.  The in-kernel clock is
// d(s_memtime) / d(s_memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
// Table layout: [0, 12) region cycles, [12] waves, [13] total cycles,
// [14] total realtime ticks, [15] unused.
#pragma once
#include <stdint.h>

namespace bls {

// the no-op form the product kernels instantiate
struct NoDiag {
  template <int R>
  CESS_HD void mark() {}
};

#if defined(CESS_DIAG) && !defined(CESS_HOSTEMU)
#define CESS_DIAG_SLOTS 16
CESS_HD uint64_t diag_memtime() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
CESS_HD uint64_t diag_realtime() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
struct Diag {
  uint64_t acc[12];
  uint64_t t, t0, r0;
  CESS_HD void begin() {
#pragma unroll
    for (int r = 0; r < 12; r++) acc[r] = 0;
    t0 = t = diag_memtime();
    r0 = diag_realtime();
  }
  template <int R>
  CESS_HD void mark() {
    const uint64_t n = diag_memtime();
    acc[R] += n - t;
    t = n;
  }
  // one lane of the calling wave adds the wave's figures to tab
  CESS_HD void end(unsigned long long* tab) {
    const uint64_t t1 = diag_memtime(), r1 = diag_realtime();
    const uint64_t ex = __builtin_amdgcn_read_exec();
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    if (lane == (uint32_t)__builtin_ctzll(ex)) {
#pragma unroll
      for (int r = 0; r < 12; r++) atomicAdd(&tab[r], (unsigned long long)acc[r]);
      atomicAdd(&tab[12], 1ull);
      atomicAdd(&tab[13], (unsigned long long)(t1 - t0));
      atomicAdd(&tab[14], (unsigned long long)(r1 - r0));
    }
  }
};
// per-TU table and its reader (the host function is compiled into the TU that
// defines the kernels: CESS_DIAG_TU names it)
#define CESS_DIAG_TABLE(TU)                                                                \
  static __device__ unsigned long long cess_diag_tab[CESS_DIAG_SLOTS];                     \
  extern "C" int cess_diag_read_##TU(unsigned long long* out, int reset) {                 \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cess_diag_tab), sizeof(cess_diag_tab), 0,      \
                            hipMemcpyDeviceToHost) != hipSuccess)                          \
      return -1;                                                                           \
    if (reset) {                                                                           \
      static const unsigned long long z[CESS_DIAG_SLOTS] = {};                             \
      if (hipMemcpyToSymbol(HIP_SYMBOL(cess_diag_tab), z, sizeof(z), 0,                    \
                            hipMemcpyHostToDevice) != hipSuccess)                          \
        return -1;                                                                         \
    }                                                                                      \
    return CESS_DIAG_SLOTS;                                                                \
  }
#endif

}  // namespace bls
