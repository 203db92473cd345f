// Microbenchmark: issue cost of the VALU instructions the field arithmetic
// uses (gfx950).  Each kernel runs 8 independent chains of one instruction
// per wave (inline asm, so the compiler cannot fold them), 256-thread blocks,
// CUs x W blocks for W waves per SIMD.  Reports cycles per wave-instruction
// per SIMD at 2.4 GHz: 4.0 = full rate (16 lanes/clk), 16 = quarter rate.
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);           \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint64_t* out, int iters, uint32_t s) {
  extern __shared__ uint32_t pad[];   // dynamic LDS pins the blocks per CU (see main)
  if (iters < 0) pad[threadIdx.x] = s;
  uint32_t a = threadIdx.x * 77 + s, b = blockIdx.x * 31 + s;
  uint32_t x[8];
  uint64_t y[8], z[8];
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = a + j, y[j] = ((uint64_t)b << 32) + j, z[j] = y[j] ^ a;
  for (int it = 0; it < iters; it++) {
#define U32(j) asm volatile(INS : "+v"(x[j]) : "v"(a), "v"(b));
#define U64(j) asm volatile(INS : "+v"(y[j]) : "v"(a), "v"(b));
#define U64C(j) asm volatile(INS : "+v"(y[j]) : "v"(a), "v"(b) : "vcc");
    if (OP == 0) {
#define INS "v_mad_u64_u32 %0, vcc, %1, %2, %0"
      R8(U64C)
#undef INS
    } else if (OP == 1) {
#define INS "v_mul_lo_u32 %0, %0, %1"
      R8(U32)
#undef INS
    } else if (OP == 2) {
#define INS "v_lshrrev_b64 %0, 28, %0"
      R8(U64)
#undef INS
    } else if (OP == 3) {
#define INS "v_lshl_add_u64 %0, %0, 0, %0"
      R8(U64)
#undef INS
    } else if (OP == 4) {
#define INS "v_alignbit_b32 %0, %0, %1, 28"
      R8(U32)
#undef INS
    } else if (OP == 5) {
#define INS "v_and_b32 %0, %0, %1"
      R8(U32)
#undef INS
    } else if (OP == 6) {
#define INS "v_mul_hi_u32 %0, %0, %1"
      R8(U32)
#undef INS
    } else if (OP == 7) {
#define INS "v_mov_b64 %0, %0"
      R8(U64)
#undef INS
    } else if (OP == 8) {
#define U32C(j) asm volatile(INS : "+v"(x[j]) : "v"(a), "v"(b) : "vcc");
#define INS "v_add_co_u32 %0, vcc, %0, %1"
      R8(U32C)
#undef INS
    } else if (OP == 9) {
#define INS "v_mad_i64_i32 %0, vcc, %1, %2, %0"
      R8(U64C)
#undef INS
    } else if (OP == 10) {
#define INS "v_perm_b32 %0, %0, %1, %2"
      R8(U32)
#undef INS
    } else if (OP == 11) {
#define INS "v_add3_u32 %0, %0, %1, %2"
      R8(U32)
#undef INS
    } else if (OP == 12) {
#define INS "v_mul_u32_u24 %0, %0, %1"
      R8(U32)
#undef INS
    } else if (OP == 13) {
#define INS "v_lshl_or_b32 %0, %0, 4, %1"
      R8(U32)
#undef INS
    } else if (OP == 14) {
      // carry chain: 8 links, each reading the previous link's vcc
      asm volatile(
          "v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n"
          "v_addc_co_u32 %2, vcc, %2, %8, vcc\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
          "v_addc_co_u32 %4, vcc, %4, %8, vcc\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n"
          "v_addc_co_u32 %6, vcc, %6, %8, vcc\n v_addc_co_u32 %7, vcc, %7, %8, vcc\n"
          : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
          : "v"(a)
          : "vcc");
    } else if (OP == 15) {
#define INS "v_cndmask_b32 %0, %0, %1, vcc"
      R8(U32)
#undef INS
    } else if (OP == 16) {
#define INS "v_sub_u32 %0, %0, %1"
      R8(U32)
#undef INS
    } else if (OP == 17) {
#define INS "v_ashrrev_i32 %0, 28, %0"
      R8(U32)
#undef INS
    } else if (OP == 19) {
#define INS "v_cndmask_b32_e32 %0, %1, %0, vcc"
      R8(U32)
#undef INS
    } else if (OP == 20) {
      // select after a borrow-producing subtract (the fp_reduce pattern)
#define SUBSEL(j) asm volatile("v_sub_co_u32 %1, vcc, %0, %2\n v_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"(x[j]), "=&v"(t) : "v"(a) : "vcc");
      uint32_t t;
      R8(SUBSEL)
#undef SUBSEL
    } else if (OP == 21) {
#define INS "v_cndmask_b32_e64 %0, %0, %1, s[40:41]"
#define U32S(j) asm volatile(INS : "+v"(x[j]) : "v"(a), "v"(b) : "s40", "s41");
      R8(U32S)
#undef INS
    } else if (OP == 22) {   // mixed: 8 mads + 8 ands (counted as 16 instructions)
#define MIX1(j) asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_and_b32 %1, %1, %2" : "+v"(y[j]), "+v"(x[j]) : "v"(a), "v"(b) : "vcc");
      R8(MIX1)
#undef MIX1
    } else if (OP == 23) {   // mixed: 8 mads + 16 ands (24 instructions)
#define MIX2(j) asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_and_b32 %1, %1, %2\n v_xor_b32 %1, %1, %3" : "+v"(y[j]), "+v"(x[j]) : "v"(a), "v"(b) : "vcc");
      R8(MIX2)
#undef MIX2
    } else if (OP == 24) {   // mixed: 8 mads + 8 v_lshl_add_u64 (16 instructions)
#define MIX3(j) asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_lshl_add_u64 %1, %1, 0, %1" : "+v"(y[j]), "+v"(z[j]) : "v"(a), "v"(b) : "vcc");
      R8(MIX3)
#undef MIX3
    } else if (OP == 18) {
#define INS "v_mad_u32_u24 %0, %0, %1, %2"
      R8(U32)
#undef INS
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= x[j] ^ y[j] ^ z[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kfn)(uint64_t*, int, uint32_t);
static const struct {
  kfn f;
  const char* name;
} kOps[] = {
    {k_rate<0>, "v_mad_u64_u32"},   {k_rate<1>, "v_mul_lo_u32"},    {k_rate<2>, "v_lshrrev_b64"},
    {k_rate<3>, "v_lshl_add_u64"},  {k_rate<4>, "v_alignbit_b32"},  {k_rate<5>, "v_and_b32"},
    {k_rate<6>, "v_mul_hi_u32"},    {k_rate<7>, "v_mov_b64"},       {k_rate<8>, "v_add_co_u32(vcc)"},
    {k_rate<9>, "v_mad_i64_i32"},   {k_rate<10>, "v_perm_b32"},     {k_rate<11>, "v_add3_u32"},
    {k_rate<12>, "v_mul_u32_u24"},  {k_rate<13>, "v_lshl_or_b32"},  {k_rate<14>, "addc chain(vcc)"},
    {k_rate<15>, "v_cndmask_b32"},  {k_rate<16>, "v_sub_u32"},      {k_rate<17>, "v_ashrrev_i32"},
    {k_rate<18>, "v_mad_u32_u24"},  {k_rate<19>, "v_cndmask_b32_e32"}, {k_rate<20>, "sub_co+cndmask"},
    {k_rate<21>, "v_cndmask_e64 sgpr"}, {k_rate<22>, "mad+and (per pair)"}, {k_rate<23>, "mad+2 alu (per trio)"},
    {k_rate<24>, "mad+lshl_add_u64 (pair)"},
};

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 8192;
  const double clk = 2.4e9;
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 8));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  printf("# cycles per wave-instruction per SIMD (8 independent chains/wave), %d CUs @2.4GHz\n", cus);
  printf("%-20s %8s %8s %8s %8s\n", "instruction", "W=1", "W=2", "W=4", "W=8");
  for (const auto& op : kOps) CHK(hipFuncSetAttribute((const void*)op.f, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  for (const auto& op : kOps) {
    printf("%-20s", op.name);
    for (int w : {1, 2, 4, 8}) {
      // (160 KiB / w) - 1 KiB of LDS per block: exactly w blocks (w waves per SIMD) fit a CU, so the
      // dispatcher cannot stack blocks on some CUs and leave others idle
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      hipLaunchKernelGGL(op.f, dim3(cus * w), dim3(256), lds, 0, out, 64, 1u);   // warm
      CHK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(op.f, dim3(cus * w), dim3(256), lds, 0, out, iters, 1u);
      CHK(hipEventRecord(e1, 0));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      // per SIMD: w waves x iters x 8 instructions
      const double cyc = ms * 1e-3 * clk / ((double)w * iters * 8);
      printf(" %8.2f", cyc);
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
