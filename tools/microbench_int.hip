// Integer/FP64 VALU throughput microbenchmark for gfx950 (MI355X).
// Measures wave-instruction throughput of the instructions the 128-bit
// prime-field and Blake2b kernels are built from. Each thread runs 8
// independent dependency chains so issue rate, not latency, is measured.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 2048
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define BODY8(ASM) ASM(0) ASM(1) ASM(2) ASM(3) ASM(4) ASM(5) ASM(6) ASM(7)

__global__ void k_add_u32(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(A)
#undef A
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_lo(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(A)
#undef A
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_hi(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(A)
#undef A
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_u24(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(A)
#undef A
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad_u64(uint32_t* out, uint32_t seed) {
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1, c = seed ^ 0x55;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
    BODY8(A)
#undef A
  }
  uint64_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
__global__ void k_lshl_add_u64(uint32_t* out, uint32_t seed) {
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint64_t b = seed * 3ull + 1;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(b));
    BODY8(A)
#undef A
  }
  uint64_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
__global__ void k_add_co(uint32_t* out, uint32_t seed) {
  // 64-bit add as v_add_co_u32 + v_addc_co_u32 pair (counts 2 instr per chain step)
  uint32_t lo[8], hi[8]; for (int i = 0; i < 8; ++i) { lo[i] = seed + threadIdx.x + i; hi[i] = i; }
  uint32_t bl = seed * 3 + 1, bh = seed;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n v_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(lo[i]), "+v"(hi[i]) : "v"(bl), "v"(bh) : "vcc");
    BODY8(A)
#undef A
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= lo[i] ^ hi[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(a[i]) : "v"(b));
    BODY8(A)
#undef A
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_xor3(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1, c = seed ^ 7;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
    BODY8(A)
#undef A
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma_f64(uint32_t* out, uint32_t seed) {
  double a[8]; for (int i = 0; i < 8; ++i) a[i] = 1.0 + 1e-9 * (threadIdx.x + i);
  double b = 0.999999 + 1e-12 * seed, c = 1e-7;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    BODY8(A)
#undef A
  }
  double s = 0; for (int i = 0; i < 8; ++i) s += a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s * 1000);
}
__global__ void k_pk_fma_f32(uint32_t* out, uint32_t seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a[8]; for (int i = 0; i < 8; ++i) { a[i].x = 1.0f + i; a[i].y = 2.0f + threadIdx.x; }
  f2 b; b.x = 0.9999f; b.y = 0.9998f + seed * 1e-9f; f2 c; c.x = 1e-3f; c.y = 2e-3f;
  for (int it = 0; it < ITERS; ++it) {
#define A(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    BODY8(A)
#undef A
  }
  float s = 0; for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

typedef void (*kfn)(uint32_t*, uint32_t);
static int run(const char* name, kfn k, int instr_per_step) {
  const int threads = 256, blocks = 256 * 8;
  uint32_t* out; CHK(hipMalloc(&out, sizeof(uint32_t) * threads * blocks));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, (uint32_t)r);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double waves = (double)blocks * threads / 64.0 * 5;
  double winstr = waves * ITERS * 8 * instr_per_step;
  double s = ms * 1e-3;
  // wave-instructions per CU per cycle assuming 2.4 GHz
  double per_cu_cycle = winstr / s / 256.0 / 2.4e9;
  printf("%-16s %8.3f ms  %8.2f T lane-instr/s  %6.3f wave-instr/CU/clk(@2.4GHz)\n", name, ms / 5, winstr * 64 / s / 1e12, per_cu_cycle);
  CHK(hipFree(out));
  return 0;
}
int main() {
  run("v_add_u32", k_add_u32, 1);
  run("v_mul_lo_u32", k_mul_lo, 1);
  run("v_mul_hi_u32", k_mul_hi, 1);
  run("v_mul_u32_u24", k_mul_u24, 1);
  run("v_mad_u64_u32", k_mad_u64, 1);
  run("v_lshl_add_u64", k_lshl_add_u64, 1);
  run("add_co+addc", k_add_co, 2);
  run("v_alignbit_b32", k_alignbit, 1);
  run("v_bitop3_b32", k_xor3, 1);
  run("v_fma_f64", k_fma_f64, 1);
  run("v_pk_fma_f32", k_pk_fma_f32, 1);
  return 0;
}
