// BLAKE2b single-block compression throughput on gfx950: rotation/add lowering variants.
// Each thread chains ITERS compressions (output feeds the next message) so the
// measurement is the compression's VALU cost, not memory.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 64
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct u2 { uint32_t lo, hi; };

// ---- variant 0: plain C (compiler lowering)
__device__ __forceinline__ uint64_t rotr_c(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
// ---- variant 1: alignbit
__device__ __forceinline__ uint64_t rotr_ab(uint64_t x, int n) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return ((uint64_t)lo << 32) | hi;
  if (n > 32) { uint32_t t = lo; lo = hi; hi = t; n -= 32; }
  uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, n);
  uint32_t nhi = __builtin_amdgcn_alignbit(lo, hi, n);
  return ((uint64_t)nhi << 32) | nlo;
}
// ---- variant 3: perm for 16/24, rotl1 via lshl_add_u64 for 63
__device__ __forceinline__ uint64_t rotr_pm2(uint64_t x, int n) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return ((uint64_t)lo << 32) | hi;
  if (n == 16 || n == 24) {
    uint32_t sel = n == 16 ? 0x05040302u : 0x06050403u;
    uint32_t nlo = __builtin_amdgcn_perm(hi, lo, sel);
    uint32_t nhi = __builtin_amdgcn_perm(lo, hi, sel);
    return ((uint64_t)nhi << 32) | nlo;
  }
  // n == 63: rotl 1 = (x << 1) + (x >> 63)
  return (x << 1) + (uint64_t)(hi >> 31);
}
// ---- variant 2: v_perm_b32 for byte rotations (16, 24), alignbit for 63
__device__ __forceinline__ uint64_t rotr_pm(uint64_t x, int n) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return ((uint64_t)lo << 32) | hi;
  if (n == 16 || n == 24) {
    // perm(s0, s1, sel): bytes {s0: 7..4, s1: 3..0}
    uint32_t sel = n == 16 ? 0x05040302u : 0x06050403u;
    uint32_t nlo = __builtin_amdgcn_perm(hi, lo, sel);
    uint32_t nhi = __builtin_amdgcn_perm(lo, hi, sel);
    return ((uint64_t)nhi << 32) | nlo;
  }
  return rotr_ab(x, n);
}

// ---- variant 4: alignbit for 16/24, rotl1 via lshl_add_u64 for 63
__device__ __forceinline__ uint64_t rotr_ab1(uint64_t x, int n) {
  if (n == 63) {
    uint64_t t = (uint64_t)((uint32_t)(x >> 32) >> 31);
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(x), "v"(t));
    return r;
  }
  return rotr_ab(x, n);
}

#define G(R, a, b, c, d, x, y) \
  a = a + b + (x); d = R(d ^ a, 32); c = c + d; b = R(b ^ c, 24); \
  a = a + b + (y); d = R(d ^ a, 16); c = c + d; b = R(b ^ c, 63);
#define ROUND(R, m, s0,s1,s2,s3,s4,s5,s6,s7,s8,s9,s10,s11,s12,s13,s14,s15) \
  G(R, v0, v4, v8, v12, m[s0], m[s1]) G(R, v1, v5, v9, v13, m[s2], m[s3]) \
  G(R, v2, v6, v10, v14, m[s4], m[s5]) G(R, v3, v7, v11, v15, m[s6], m[s7]) \
  G(R, v0, v5, v10, v15, m[s8], m[s9]) G(R, v1, v6, v11, v12, m[s10], m[s11]) \
  G(R, v2, v7, v8, v13, m[s12], m[s13]) G(R, v3, v4, v9, v14, m[s14], m[s15])

#define COMPRESS(R) \
  uint64_t v0 = 0x6a09e667f3bcc908ull ^ 0x01010040ull, v1 = 0xbb67ae8584caa73bull, v2 = 0x3c6ef372fe94f82bull, v3 = 0xa54ff53a5f1d36f1ull; \
  uint64_t v4 = 0x510e527fade682d1ull, v5 = 0x9b05688c2b3e6c1full, v6 = 0x1f83d9abfb41bd6bull, v7 = 0x5be0cd19137e2179ull; \
  uint64_t v8 = 0x6a09e667f3bcc908ull, v9 = 0xbb67ae8584caa73bull, v10 = 0x3c6ef372fe94f82bull, v11 = 0xa54ff53a5f1d36f1ull; \
  uint64_t v12 = 0x510e527fade682d1ull ^ 128, v13 = 0x9b05688c2b3e6c1full, v14 = ~0x1f83d9abfb41bd6bull, v15 = 0x5be0cd19137e2179ull; \
  ROUND(R, m, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15) \
  ROUND(R, m, 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3) \
  ROUND(R, m, 11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4) \
  ROUND(R, m, 7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8) \
  ROUND(R, m, 9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13) \
  ROUND(R, m, 2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9) \
  ROUND(R, m, 12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11) \
  ROUND(R, m, 13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10) \
  ROUND(R, m, 6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5) \
  ROUND(R, m, 10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0) \
  ROUND(R, m, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15) \
  ROUND(R, m, 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3) \
  m[0] ^= v0 ^ v8; m[1] ^= v1 ^ v9; m[2] ^= v2 ^ v10; m[3] ^= v3 ^ v11; \
  m[4] ^= v4 ^ v12; m[5] ^= v5 ^ v13; m[6] ^= v6 ^ v14; m[7] ^= v7 ^ v15;

template <int V>
__global__ __launch_bounds__(256) void k_blake(uint64_t* out, uint64_t seed) {
  uint64_t m[16];
  for (int i = 0; i < 16; ++i) m[i] = seed * (i + 1) + threadIdx.x + blockIdx.x * 977;
  for (int it = 0; it < ITERS; ++it) {
    if (V == 0) { COMPRESS(rotr_c) }
    else if (V == 1) { COMPRESS(rotr_ab) }
    else if (V == 2) { COMPRESS(rotr_pm) }
    else if (V == 4) { COMPRESS(rotr_ab1) }
    else { COMPRESS(rotr_pm2) }
    // rotate message words so the next compression depends on this one
    uint64_t t = m[0]; for (int i = 0; i < 15; ++i) m[i] = m[i + 1]; m[15] = t;
  }
  uint64_t s = 0; for (int i = 0; i < 16; ++i) s ^= m[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// correctness: all variants must agree
template <int V>
int run(const char* name, uint64_t* ref_host) {
  const int threads = 256, blocks = 256 * 8;
  uint64_t* out; CHK(hipMalloc(&out, 8ull * threads * blocks));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_blake<V>, dim3(blocks), dim3(threads), 0, 0, out, 7ull);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_blake<V>, dim3(blocks), dim3(threads), 0, 0, out, 7ull);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double comps = 5.0 * threads * blocks * ITERS;
  uint64_t h[16]; CHK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
  bool same = true; if (ref_host[0] == 0) { for (int i = 0; i < 16; ++i) ref_host[i] = h[i]; } else for (int i = 0; i < 16; ++i) same &= h[i] == ref_host[i];
  printf("%-10s %8.3f ms/launch  %8.3f G compressions/s  %s\n", name, ms / 5, comps / (ms * 1e-3) / 1e9, same ? "ok" : "MISMATCH");
  CHK(hipFree(out));
  return 0;
}
int main() {
  uint64_t ref[16] = {0};
  run<0>("plain-C", ref);
  run<1>("alignbit", ref);
  run<2>("perm", ref);
  run<3>("perm+rotl1", ref);
  run<4>("ab+rotl1", ref);
  run<1>("alignbit", ref);
  run<4>("ab+rotl1", ref);
  return 0;
}
