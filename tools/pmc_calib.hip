// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access shapes of the FRI fold-leaf
// kernel (k_merkle_leaf_pairs<512, true>): every kernel here moves a KNOWN number of bytes, so one
// FETCH_SIZE and one WRITE_SIZE pass give the counter-to-bytes factor of each shape
// (MI355X_MICROARCH.md: only the 16-B-per-lane contiguous shape is calibrated, at 1/2 for reads).
//   flat      lane i reads s[i], writes d[i]                         16 B read + 16 B written / lane
//   pairs     lane p reads s[2p], s[2p+1], s[2p+n], s[2p+1+n] and writes d[2p], d[2p+1]:
//             the fold kernel's data movement (x, y of two leaves; the folded pair)  64 B read + 32 B written
//   pairs_tw  pairs + the fold's twiddle gathers Tlo[2p & 4095], Thi[2p >> 12] (64 KiB + 32 KiB tables)
// Build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_flat(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = s[i] + 1u;
}

template <bool TW>
__global__ void __launch_bounds__(512) k_pairs(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t half,
                                               const u32x4* __restrict__ tlo, const u32x4* __restrict__ thi) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * p + 1 >= half) return;
  u32x4 x0 = s[2 * p], x1 = s[2 * p + 1], y0 = s[2 * p + half], y1 = s[2 * p + 1 + half];
  if (TW) {
    x0 ^= tlo[(2 * p) & 4095] ^ thi[(2 * p) >> 12];
    x1 ^= tlo[(2 * p + 1) & 4095] ^ thi[(2 * p + 1) >> 12];
  }
  d[2 * p] = x0 + y0;
  d[2 * p + 1] = x1 + y1;
}

int main() {
  const uint64_t n = 1ull << 26;  // 1 GiB of 16-byte elements: far beyond the 256 MiB MALL
  u32x4 *s, *d, *tlo, *thi;
  hipMalloc(&s, n * 16);
  hipMalloc(&d, n * 16);
  hipMalloc(&tlo, 4096 * 16);
  hipMalloc(&thi, (n / 4096) * 16);
  hipMemset(s, 1, n * 16);
  hipMemset(tlo, 2, 4096 * 16);
  hipMemset(thi, 3, (n / 4096) * 16);
  for (int it = 0; it < 3; ++it) {
    k_flat<<<(unsigned)(n / 256), 256>>>(s, d, n);
    k_pairs<false><<<(unsigned)(n / 2 / 2 / 512), 512>>>(s, d, n / 2, tlo, thi);
    k_pairs<true><<<(unsigned)(n / 2 / 2 / 512), 512>>>(s, d, n / 2, tlo, thi);
  }
  hipDeviceSynchronize();
  printf("lanes: flat %llu (16 B read + 16 B written each); pairs %llu (64 B read + 32 B written each)\n",
         (unsigned long long)n, (unsigned long long)(n / 4));
  return 0;
}
