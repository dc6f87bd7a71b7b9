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


#define K1(NAME, ASMSTR) \
__global__ void NAME(uint32_t* out, uint32_t seed) { \
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i; \
  uint32_t b = seed * 3 + 1, c = seed ^ 0x0c0d0e0f; \
  for (int it = 0; it < ITERS; ++it) { \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASMSTR : "+v"(a[i]) : "v"(b), "v"(c)); \
  } \
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s; }
K1(k_perm, "v_perm_b32 %0, %0, %1, %2")
K1(k_xor, "v_xor_b32 %0, %0, %1")
K1(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
K1(k_add_e64, "v_add_u32_e64 %0, %0, %1")
K1(k_lshl_e64, "v_lshlrev_b32_e64 %0, 7, %0")
K1(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
K1(k_sub_u32, "v_sub_u32 %0, %1, %0")
K1(k_mov_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K1(k_add_sdwa, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")
K1(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
K1(k_lshl_or, "v_lshl_or_b32 %0, %0, 1, %1")
K1(k_add3, "v_add3_u32 %0, %0, %1, %2")
K1(k_lshr, "v_lshrrev_b32 %0, 7, %0")
K1(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 3")
K1(k_xad, "v_xad_u32 %0, %0, %1, %2")
__global__ void k_add64_pair(uint32_t* out, uint32_t seed) {
  // 64-bit add as co/addc pairs with a distinct SGPR-pair carry per chain
  uint32_t lo[8], hi[8]; for (int i = 0; i < 8; ++i) { lo[i] = seed + threadIdx.x + i; hi[i] = i; }
  uint32_t bl = seed * 3 + 1, bh = seed;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t cy;
      asm volatile("v_add_co_u32 %0, %2, %0, %3\n v_addc_co_u32 %1, %2, %1, %4, %2" : "+v"(lo[i]), "+v"(hi[i]), "=&s"(cy) : "v"(bl), "v"(bh));
    }
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= lo[i] ^ hi[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_lshlrev64(uint32_t* out, uint32_t seed) {
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(a[i]));
  }
  uint64_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
__global__ void k_mix_xor_perm(uint32_t* out, uint32_t seed) {
  // interleaved xor + perm (dual-issue check)
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1, c = seed ^ 0x0c0d0e0f;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i & 1) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    }
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mix_xor_align(uint32_t* out, uint32_t seed) {
  uint32_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint32_t b = seed * 3 + 1;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i & 1) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(a[i]) : "v"(b));
      else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    }
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mix_xor_lshladd(uint32_t* out, uint32_t seed) {
  uint64_t a[8]; for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x + i;
  uint64_t b = seed * 3ull + 1;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i & 1) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(b));
      else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(((uint32_t*)&a[i])[0]) : "v"((uint32_t)b));
    }
  }
  uint64_t s = 0; for (int i = 0; i < 8; ++i) s ^= a[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
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
  run("v_perm_b32", k_perm, 1);
  run("v_xor_b32", k_xor, 1);
  run("v_xor_b32_e64", k_xor_e64, 1);
  run("v_add_u32_e64", k_add_e64, 1);
  run("v_lshlrev_b32_e64", k_lshl_e64, 1);
  run("v_and_or_b32", k_and_or, 1);
  run("v_sub_u32", k_sub_u32, 1);
  run("v_mov_b32_dpp", k_mov_dpp, 1);
  run("v_add_u32_sdwa", k_add_sdwa, 1);
  run("v_pk_add_u16", k_pk_add_u16, 1);
  run("v_lshl_or_b32", k_lshl_or, 1);
  run("v_add3_u32", k_add3, 1);
  run("v_lshrrev_b32", k_lshr, 1);
  run("v_alignbyte_b32", k_alignbyte, 1);
  run("v_xad_u32", k_xad, 1);
  run("add64 pair(sgpr)", k_add64_pair, 2);
  run("v_lshlrev_b64", k_lshlrev64, 1);
  run("xor+perm mix", k_mix_xor_perm, 1);
  run("xor+alignbit mix", k_mix_xor_align, 1);
  run("xor+lshladd mix", k_mix_xor_lshladd, 1);
  return 0;
}
