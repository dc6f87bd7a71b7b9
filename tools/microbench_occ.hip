// Radix-2 butterfly throughput (fe128.hpp: lazy add/sub + Montgomery product) against
// occupancy: dynamic LDS per 256-thread block limits the resident blocks per CU, so the
// same register-only loop runs at 1..8 waves per SIMD.  Tells whether the NTT passes
// (125 VGPRs: 4 waves/SIMD) lose issue rate to VALU latency at that occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../zk-stark-tutor_amd/csrc/fe128.hpp"
using namespace sg;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define ITERS 256

__global__ __launch_bounds__(256) void k_bfly(fe* out, const fe* in, const fe* tw) {
  extern __shared__ char pad[];
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0xFFFFFFFFu) pad[threadIdx.x] = 0;  // keep the allocation
  fe x[8];
  for (int k = 0; k < 8; ++k) x[k] = in[(i * 8 + k) & 1023];
  fe w[4];
  for (int k = 0; k < 4; ++k) w[k] = tw[(threadIdx.x + 7 * k) & 63];
  for (int it = 0; it < ITERS; ++it) {
    // one radix-8 step's worth: 3 sub-stages x 4 independent butterflies
#pragma unroll
    for (int u = 0; u < 3; ++u) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if (m & (1 << u)) continue;
        fe o = mont_mul(x[m + (1 << u)], w[(m >> 1) & 3]);
        fe e = x[m];
        x[m] = fe_add_lazy(e, o);
        x[m + (1 << u)] = fe_sub_lazy(e, o);
      }
    }
  }
  for (int k = 0; k < 8; ++k) out[i * 8 + k] = fe_canon(x[k]);
}

int main() {
  const int threads = 256, blocks = 256 * 16, n = threads * blocks * 8;
  fe* h = (fe*)malloc(sizeof(fe) * 1024);
  uint64_t s = 88172645463325252ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  for (int i = 0; i < 1024; ++i) h[i] = fe_make(rnd(), rnd() % ((uint64_t)P3 << 32));
  fe *in, *tw, *o;
  CHK(hipMalloc(&in, sizeof(fe) * 1024)); CHK(hipMalloc(&tw, sizeof(fe) * 64)); CHK(hipMalloc(&o, sizeof(fe) * n));
  CHK(hipMemcpy(in, h, sizeof(fe) * 1024, hipMemcpyHostToDevice));
  CHK(hipMemcpy(tw, h + 512, sizeof(fe) * 64, hipMemcpyHostToDevice));
  CHK(hipFuncSetAttribute((const void*)k_bfly, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const int wps[] = {1, 2, 3, 4, 5, 6, 8};
  for (int wv : wps) {
    // blocks per CU = waves per SIMD (a 256-thread block is 4 waves, one per SIMD)
    size_t lds = (160 * 1024) / wv - 256;
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_bfly, 256, lds));
    hipLaunchKernelGGL(k_bfly, dim3(blocks), dim3(threads), lds, 0, o, in, tw);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_bfly, dim3(blocks), dim3(threads), lds, 0, o, in, tw);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    double bf = 3.0 * threads * blocks * ITERS * 12;
    printf("waves/SIMD %d (occupancy API %d blocks/CU): %.3f ms/launch  %.1f G butterflies/s\n", wv, occ, ms / 3,
           bf / (ms * 1e-3) / 1e9);
  }
  return 0;
}
