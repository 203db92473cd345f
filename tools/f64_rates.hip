// Microbenchmark (gfx950): issue cost of FP64 FMA against v_mad_u64_u32, the
// question behind a floating-point limb scheme for the field arithmetic
// (52-bit limbs, exact products as hi = fma(a, b, 0), lo = fma(a, b, -hi)).
// Same method as tools/valu_rates.hip: 8 independent chains per wave in
// inline asm, 256-thread blocks, exactly W blocks per CU (LDS-pinned);
// cycles per wave-instruction per SIMD at 2.4 GHz (4.0 = 16 lanes/clock).
// Build: hipcc -O3 --offload-arch=gfx950 tools/f64_rates.hip -o tools/f64_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                         \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(2);                                                         \
    }                                                                  \
  } while (0)

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void k_rate(double* out, int iters, double s) {
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = (uint32_t)s;
  const double a = 1.0 + threadIdx.x * 1e-6, b = 0.999999 - blockIdx.x * 1e-9;
  const uint32_t ia = threadIdx.x * 77 + 1, ib = blockIdx.x * 31 + 3;
  double x[8];
  uint64_t y[8];
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = s + j, y[j] = ((uint64_t)ib << 32) + j;
  for (int it = 0; it < iters; it++) {
#define F64(j) asm volatile(INS : "+v"(x[j]) : "v"(a), "v"(b));
    if (OP == 0) {
#define INS "v_mad_u64_u32 %0, vcc, %1, %2, %0"
#define U64C(j) asm volatile(INS : "+v"(y[j]) : "v"(ia), "v"(ib) : "vcc");
      R8(U64C)
#undef INS
    } else if (OP == 1) {
#define INS "v_fma_f64 %0, %1, %2, %0"
      R8(F64)
#undef INS
    } else if (OP == 2) {
#define INS "v_mul_f64 %0, %0, %1"
      R8(F64)
#undef INS
    } else if (OP == 3) {
#define INS "v_add_f64 %0, %0, %1"
      R8(F64)
#undef INS
    } else if (OP == 4) {   // fma + mad interleaved (16 instructions)
#define MIX(j) asm volatile("v_fma_f64 %0, %2, %3, %0\n v_mad_u64_u32 %1, vcc, %4, %5, %1" : "+v"(x[j]), "+v"(y[j]) : "v"(a), "v"(b), "v"(ia), "v"(ib) : "vcc");
      R8(MIX)
#undef MIX
    } else if (OP == 5) {
#define INS "v_pk_fma_f32 %0, %1, %2, %0"
      R8(F64)
#undef INS
    }
  }
  double r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r += x[j] + (double)y[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kfn)(double*, int, double);
static const struct {
  kfn f;
  const char* name;
  int per;   // instructions per chain link
} kOps[] = {
    {k_rate<0>, "v_mad_u64_u32", 1}, {k_rate<1>, "v_fma_f64", 1},        {k_rate<2>, "v_mul_f64", 1},
    {k_rate<3>, "v_add_f64", 1},     {k_rate<4>, "fma_f64+mad_u64", 2}, {k_rate<5>, "v_pk_fma_f32", 1},
};

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, iters = 8192;
  const double clk = 2.4e9;
  double* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 8));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  printf("# cycles per wave-instruction per SIMD (8 independent chains/wave), %d CUs @2.4GHz\n", cus);
  printf("%-20s %8s %8s %8s\n", "instruction", "W=1", "W=2", "W=4");
  for (const auto& op : kOps) CHK(hipFuncSetAttribute((const void*)op.f, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024));
  for (const auto& op : kOps) {
    printf("%-20s", op.name);
    for (int w : {1, 2, 4}) {
      const size_t lds = (size_t)(160 / w - 1) * 1024;
      hipLaunchKernelGGL(op.f, dim3(cus * w), dim3(256), lds, 0, out, 64, 1.0);
      CHK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(op.f, dim3(cus * w), dim3(256), lds, 0, out, iters, 1.0);
      CHK(hipEventRecord(e1, 0));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double cyc = ms * 1e-3 * clk / ((double)w * iters * 8 * op.per);
      printf(" %8.2f", cyc);
    }
    printf("\n");
  }
  CHK(hipDeviceSynchronize());
  return 0;
}
