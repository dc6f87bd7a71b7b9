// Radix-2 butterfly throughput on gfx950 for two implementations of the
// 128-bit Montgomery arithmetic (V0 = fe128.hpp as first written, V1 = the
// carry-chain version).  Each thread chains butterflies on registers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../zk-stark-tutor_amd/csrc/fe128.hpp"
using namespace sg;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define ITERS 256

namespace v1 {
__device__ __forceinline__ void mac3(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& acc2) {
  uint64_t r; uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %5\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
      : "=&v"(r), "=&s"(cc), "+v"(acc2) : "v"(a), "v"(b), "v"(acc));
  acc = r;
}
__device__ __forceinline__ fe mont_mul(const fe& a, const fe& b) {
  uint32_t t[8];
  {
    uint64_t acc = (uint64_t)a.w[0] * b.w[0];
    uint32_t acc2 = 0;
    t[0] = (uint32_t)acc; acc >>= 32;
    acc += (uint64_t)a.w[0] * b.w[1];  // no overflow: < 2^32 + (2^32-1)^2
    mac3(a.w[1], b.w[0], acc, acc2);
    t[1] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)acc2 << 32); acc2 = 0;
    mac3(a.w[0], b.w[2], acc, acc2); mac3(a.w[1], b.w[1], acc, acc2); mac3(a.w[2], b.w[0], acc, acc2);
    t[2] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)acc2 << 32); acc2 = 0;
    mac3(a.w[0], b.w[3], acc, acc2); mac3(a.w[1], b.w[2], acc, acc2); mac3(a.w[2], b.w[1], acc, acc2); mac3(a.w[3], b.w[0], acc, acc2);
    t[3] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)acc2 << 32); acc2 = 0;
    mac3(a.w[1], b.w[3], acc, acc2); mac3(a.w[2], b.w[2], acc, acc2); mac3(a.w[3], b.w[1], acc, acc2);
    t[4] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)acc2 << 32); acc2 = 0;
    mac3(a.w[2], b.w[3], acc, acc2); mac3(a.w[3], b.w[2], acc, acc2);
    t[5] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)acc2 << 32);
    acc += (uint64_t)a.w[3] * b.w[3];  // top column cannot overflow 64 bits (T < 2^256)
    t[6] = (uint32_t)acc; t[7] = (uint32_t)(acc >> 32);
  }
  unsigned c, br;
  // step 1: eliminate (t0, t1)
  uint32_t m0 = __builtin_subc(0u, t[0], 0u, &br);
  uint32_t m1 = __builtin_subc(0u, t[1], br, &br);  // br = (T0 != 0)
  uint64_t q0 = (uint64_t)m0 * P3;
  uint64_t q1 = (uint64_t)m1 * P3 + (q0 >> 32);
  uint32_t u0 = __builtin_addc(t[2], br, 0u, &c);
  uint32_t u1 = __builtin_addc(t[3], (uint32_t)q0, c, &c);
  uint32_t u2 = __builtin_addc(t[4], (uint32_t)q1, c, &c);
  uint32_t u3 = __builtin_addc(t[5], (uint32_t)(q1 >> 32), c, &c);
  uint32_t u4 = __builtin_addc(t[6], 0u, c, &c);
  uint32_t u5 = t[7] + c;
  // step 2: eliminate (u0, u1)
  uint32_t n0 = __builtin_subc(0u, u0, 0u, &br);
  uint32_t n1 = __builtin_subc(0u, u1, br, &br);
  uint64_t s0 = (uint64_t)n0 * P3;
  uint64_t s1 = (uint64_t)n1 * P3 + (s0 >> 32);
  uint32_t r0 = __builtin_addc(u2, br, 0u, &c);
  uint32_t r1 = __builtin_addc(u3, (uint32_t)s0, c, &c);
  uint32_t r2 = __builtin_addc(u4, (uint32_t)s1, c, &c);
  uint32_t r3 = __builtin_addc(u5, (uint32_t)(s1 >> 32), c, &c);
  // r + c*2^128 < 2p: subtract p if c or r >= p  (r + (2^128 - p) carries iff r >= p)
  unsigned g;
  uint32_t d0 = __builtin_addc(r0, 0xFFFFFFFFu, 0u, &g);
  uint32_t d1 = __builtin_addc(r1, 0xFFFFFFFFu, g, &g);
  uint32_t d2 = __builtin_addc(r2, 0xFFFFFFFFu, g, &g);
  uint32_t d3 = __builtin_addc(r3, 0x347FFFFFu, g, &g);
  bool take = (c | g) != 0;
  fe r = {{take ? d0 : r0, take ? d1 : r1, take ? d2 : r2, take ? d3 : r3}};
  return r;
}
__device__ __forceinline__ fe add(const fe& a, const fe& b) {
  unsigned c, g;
  uint32_t s0 = __builtin_addc(a.w[0], b.w[0], 0u, &c);
  uint32_t s1 = __builtin_addc(a.w[1], b.w[1], c, &c);
  uint32_t s2 = __builtin_addc(a.w[2], b.w[2], c, &c);
  uint32_t s3 = __builtin_addc(a.w[3], b.w[3], c, &c);
  uint32_t d0 = __builtin_addc(s0, 0xFFFFFFFFu, 0u, &g);
  uint32_t d1 = __builtin_addc(s1, 0xFFFFFFFFu, g, &g);
  uint32_t d2 = __builtin_addc(s2, 0xFFFFFFFFu, g, &g);
  uint32_t d3 = __builtin_addc(s3, 0x347FFFFFu, g, &g);
  bool take = (c | g) != 0;
  fe r = {{take ? d0 : s0, take ? d1 : s1, take ? d2 : s2, take ? d3 : s3}};
  return r;
}
__device__ __forceinline__ fe sub(const fe& a, const fe& b) {
  unsigned br, c;
  uint32_t d0 = __builtin_subc(a.w[0], b.w[0], 0u, &br);
  uint32_t d1 = __builtin_subc(a.w[1], b.w[1], br, &br);
  uint32_t d2 = __builtin_subc(a.w[2], b.w[2], br, &br);
  uint32_t d3 = __builtin_subc(a.w[3], b.w[3], br, &br);
  uint32_t e0 = __builtin_addc(d0, 1u, 0u, &c);
  uint32_t e1 = __builtin_addc(d1, 0u, c, &c);
  uint32_t e2 = __builtin_addc(d2, 0u, c, &c);
  uint32_t e3 = __builtin_addc(d3, P3, c, &c);
  bool neg = br != 0;
  fe r = {{neg ? e0 : d0, neg ? e1 : d1, neg ? e2 : d2, neg ? e3 : d3}};
  return r;
}
}  // namespace v1

template <int V>
__global__ __launch_bounds__(256) void k_bfly(fe* out, const fe* in, const fe* tw) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fe x[4];
  for (int k = 0; k < 4; ++k) x[k] = in[(i * 4 + k) & 1023];
  fe w0 = tw[threadIdx.x & 63], w1 = tw[(threadIdx.x + 7) & 63];
  for (int it = 0; it < ITERS; ++it) {
    if (V == 0) {
      fe o = mont_mul(x[1], w0); fe e = x[0]; x[0] = fe_add(e, o); x[1] = fe_sub(e, o);
      o = mont_mul(x[3], w1); e = x[2]; x[2] = fe_add(e, o); x[3] = fe_sub(e, o);
      o = mont_mul(x[2], w0); e = x[0]; x[0] = fe_add(e, o); x[2] = fe_sub(e, o);
      o = mont_mul(x[3], w1); e = x[1]; x[1] = fe_add(e, o); x[3] = fe_sub(e, o);
    } else {
      fe o = v1::mont_mul(x[1], w0); fe e = x[0]; x[0] = v1::add(e, o); x[1] = v1::sub(e, o);
      o = v1::mont_mul(x[3], w1); e = x[2]; x[2] = v1::add(e, o); x[3] = v1::sub(e, o);
      o = v1::mont_mul(x[2], w0); e = x[0]; x[0] = v1::add(e, o); x[2] = v1::sub(e, o);
      o = v1::mont_mul(x[3], w1); e = x[1]; x[1] = v1::add(e, o); x[3] = v1::sub(e, o);
    }
  }
  for (int k = 0; k < 4; ++k) out[i * 4 + k] = x[k];
}

int main() {
  const int threads = 256, blocks = 256 * 8, n = threads * blocks * 4;
  // random canonical inputs and twiddles (hi limb < P3 keeps them < p)
  fe* h = (fe*)malloc(sizeof(fe) * 1024);
  uint64_t s = 88172645463325252ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  for (int i = 0; i < 1024; ++i) { h[i] = fe_make(rnd(), rnd() % ((uint64_t)P3 << 32)); }
  fe *in, *tw, *o0, *o1;
  CHK(hipMalloc(&in, sizeof(fe) * 1024)); CHK(hipMalloc(&tw, sizeof(fe) * 64));
  CHK(hipMalloc(&o0, sizeof(fe) * n)); CHK(hipMalloc(&o1, sizeof(fe) * n));
  CHK(hipMemcpy(in, h, sizeof(fe) * 1024, hipMemcpyHostToDevice));
  CHK(hipMemcpy(tw, h + 512, sizeof(fe) * 64, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float ms[2];
  for (int rep = 0; rep < 2; ++rep)
  for (int v = 0; v < 2; ++v) {
    fe* o = v ? o1 : o0;
    if (v == 0) hipLaunchKernelGGL(k_bfly<0>, dim3(blocks), dim3(threads), 0, 0, o, in, tw);
    else hipLaunchKernelGGL(k_bfly<1>, dim3(blocks), dim3(threads), 0, 0, o, in, tw);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) {
      if (v == 0) hipLaunchKernelGGL(k_bfly<0>, dim3(blocks), dim3(threads), 0, 0, o, in, tw);
      else hipLaunchKernelGGL(k_bfly<1>, dim3(blocks), dim3(threads), 0, 0, o, in, tw);
    }
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms[v], e0, e1));
    double bf = 5.0 * threads * blocks * ITERS * 4;
    printf("V%d: %.3f ms/launch  %.1f G butterflies/s\n", v, ms[v] / 5, bf / (ms[v] * 1e-3) / 1e9);
  }
  fe* a = (fe*)malloc(sizeof(fe) * n); fe* b = (fe*)malloc(sizeof(fe) * n);
  CHK(hipMemcpy(a, o0, sizeof(fe) * n, hipMemcpyDeviceToHost)); CHK(hipMemcpy(b, o1, sizeof(fe) * n, hipMemcpyDeviceToHost));
  long bad = 0; for (int i = 0; i < n; ++i) bad += !fe_eq(a[i], b[i]);
  // host check of a few V0 results against the host implementation
  long hbad = 0;
  for (int i = 0; i < 64; ++i) {
    int t = i; fe x[4]; for (int k = 0; k < 4; ++k) x[k] = h[(t * 4 + k) & 1023];
    fe w0 = h[512 + (t & 63)], w1 = h[512 + ((t + 7) & 63)];
    for (int it = 0; it < ITERS; ++it) {
      fe o = mont_mul(x[1], w0); fe e = x[0]; x[0] = fe_add(e, o); x[1] = fe_sub(e, o);
      o = mont_mul(x[3], w1); e = x[2]; x[2] = fe_add(e, o); x[3] = fe_sub(e, o);
      o = mont_mul(x[2], w0); e = x[0]; x[0] = fe_add(e, o); x[2] = fe_sub(e, o);
      o = mont_mul(x[3], w1); e = x[1]; x[1] = fe_add(e, o); x[3] = fe_sub(e, o);
    }
    for (int k = 0; k < 4; ++k) hbad += !fe_eq(x[k], b[t * 4 + k]);
  }
  printf("V0 vs V1 mismatches: %ld / %d ; host vs V1 mismatches: %ld / 256\n", bad, n, hbad);
  return 0;
}
