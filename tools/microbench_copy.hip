// HBM copy microbenchmark: variants of a 16-byte-per-lane streaming copy, bytes read + written / s.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_copy.hip -o tools/microbench_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) copy_flat(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
  else d[i] = s[i];
}

template <bool NT, int U>
__global__ void __launch_bounds__(256) copy_stride(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], d + i + u * stride);
      else d[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

// each block copies a contiguous chunk (U per lane per trip)
template <bool NT, int U>
__global__ void __launch_bounds__(256) copy_chunk(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n,
                                                  uint64_t per_block) {
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block, b1 = b0 + per_block < n ? b0 + per_block : n;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < b1) v[u] = NT ? __builtin_nontemporal_load(s + i + u * 256) : s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < b1) {
        if (NT) __builtin_nontemporal_store(v[u], d + i + u * 256);
        else d[i + u * 256] = v[u];
      }
  }
}

template <class F>
double run(F launch, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int it = 0; it < iters; ++it) {
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const uint64_t bytes = 2ull << 30, n = bytes / 16;
  u32x4 *s, *d;
  hipMalloc(&s, bytes);
  hipMalloc(&d, bytes);
  hipMemset(s, 1, bytes);
  hipMemset(d, 0, bytes);
  auto rep = [&](const char* name, double ms) { printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, 2.0 * bytes / (ms * 1e-3) / 1e9); };
  const unsigned flat = (unsigned)((n + 255) / 256);
  rep("flat plain", run([&] { copy_flat<false><<<flat, 256>>>(s, d, n); }, 10));
  rep("flat nt", run([&] { copy_flat<true><<<flat, 256>>>(s, d, n); }, 10));
  for (unsigned g : {1024u, 2048u, 4096u, 8192u, 16384u}) {
    char nm[64];
    snprintf(nm, 64, "stride plain U1 g%u", g);
    rep(nm, run([&] { copy_stride<false, 1><<<g, 256>>>(s, d, n); }, 10));
    snprintf(nm, 64, "stride plain U4 g%u", g);
    rep(nm, run([&] { copy_stride<false, 4><<<g, 256>>>(s, d, n); }, 10));
    snprintf(nm, 64, "stride nt U4 g%u", g);
    rep(nm, run([&] { copy_stride<true, 4><<<g, 256>>>(s, d, n); }, 10));
  }
  for (unsigned g : {2048u, 8192u, 32768u}) {
    char nm[64];
    const uint64_t per = (n + g - 1) / g;
    snprintf(nm, 64, "chunk plain U4 g%u", g);
    rep(nm, run([&] { copy_chunk<false, 4><<<g, 256>>>(s, d, n, per); }, 10));
    snprintf(nm, 64, "chunk nt U4 g%u", g);
    rep(nm, run([&] { copy_chunk<true, 4><<<g, 256>>>(s, d, n, per); }, 10));
  }
  rep("hipMemcpyDtoD", run([&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, 10));
  return 0;
}
