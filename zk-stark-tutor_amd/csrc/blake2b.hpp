// BLAKE2b-512 (RFC 7693), single-compression forms used by the Merkle tree.
//
// The reference hashes through crate blake2 0.10.6 (crypto/blake2b512.rs:4-14):
// unkeyed, 64-byte digest, so h0 = IV ^ 0x01010040.  Every hash on the hot
// path is ONE compression:
//   * a leaf: the decimal string of a field element, 1..39 bytes
//     (merkle_root.rs:25-30, field_element.rs:46-50) -> t = len, last block;
//   * a node: left digest || right digest = exactly 128 bytes
//     (merkle_root.rs:16-17) -> t = 128, last block.
// Message words are little-endian u64; a digest is the LE serialization of
// h[0..8], so a node's message is literally the two children's h words.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sg {

// 64-bit rotate right.  On the device a 64-bit rotation by n != 32 is two
// v_alignbit_b32 (funnel shifts of the 32-bit halves); by 32 it is a register
// swap.  hipcc's own lowering (64-bit shifts + ORs) measured 23% slower per
// compression on gfx950 (tools/microbench_blake.hip).
__host__ __device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n == 32) return ((uint64_t)lo << 32) | hi;
  if (n > 32) {
    uint32_t t = lo;
    lo = hi;
    hi = t;
    n -= 32;
  }
  uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, n);
  uint32_t nhi = __builtin_amdgcn_alignbit(lo, hi, n);
  return ((uint64_t)nhi << 32) | nlo;
#else
  return (x >> n) | (x << (64 - n));
#endif
}

#define SG_B2B_IV0 0x6a09e667f3bcc908ull
#define SG_B2B_IV1 0xbb67ae8584caa73bull
#define SG_B2B_IV2 0x3c6ef372fe94f82bull
#define SG_B2B_IV3 0xa54ff53a5f1d36f1ull
#define SG_B2B_IV4 0x510e527fade682d1ull
#define SG_B2B_IV5 0x9b05688c2b3e6c1full
#define SG_B2B_IV6 0x1f83d9abfb41bd6bull
#define SG_B2B_IV7 0x5be0cd19137e2179ull

#define SG_B2B_G(a, b, c, d, x, y)   \
  a = a + b + (x);                   \
  d = rotr64(d ^ a, 32);             \
  c = c + d;                         \
  b = rotr64(b ^ c, 24);             \
  a = a + b + (y);                   \
  d = rotr64(d ^ a, 16);             \
  c = c + d;                         \
  b = rotr64(b ^ c, 63);

// sigma rows as compile-time indices (fully unrolled => m[] stays in registers)
#define SG_B2B_ROUND(m, s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  SG_B2B_G(v0, v4, v8, v12, m[s0], m[s1])                                                    \
  SG_B2B_G(v1, v5, v9, v13, m[s2], m[s3])                                                    \
  SG_B2B_G(v2, v6, v10, v14, m[s4], m[s5])                                                   \
  SG_B2B_G(v3, v7, v11, v15, m[s6], m[s7])                                                   \
  SG_B2B_G(v0, v5, v10, v15, m[s8], m[s9])                                                   \
  SG_B2B_G(v1, v6, v11, v12, m[s10], m[s11])                                                 \
  SG_B2B_G(v2, v7, v8, v13, m[s12], m[s13])                                                  \
  SG_B2B_G(v3, v4, v9, v14, m[s14], m[s15])

// Hash of a single final block: h = IV ^ param; t = total length; f0 = ~0.
// m[16] = message words (zero padded).  out[8] = digest words.
__host__ __device__ __forceinline__ void blake2b_single_block(const uint64_t m[16], uint64_t t_len, uint64_t out[8]) {
  const uint64_t h0 = SG_B2B_IV0 ^ 0x01010040ull;  // digest 64, key 0, fanout 1, depth 1
  uint64_t v0 = h0, v1 = SG_B2B_IV1, v2 = SG_B2B_IV2, v3 = SG_B2B_IV3;
  uint64_t v4 = SG_B2B_IV4, v5 = SG_B2B_IV5, v6 = SG_B2B_IV6, v7 = SG_B2B_IV7;
  uint64_t v8 = SG_B2B_IV0, v9 = SG_B2B_IV1, v10 = SG_B2B_IV2, v11 = SG_B2B_IV3;
  uint64_t v12 = SG_B2B_IV4 ^ t_len, v13 = SG_B2B_IV5, v14 = ~SG_B2B_IV6, v15 = SG_B2B_IV7;
  SG_B2B_ROUND(m, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  SG_B2B_ROUND(m, 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  SG_B2B_ROUND(m, 11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  SG_B2B_ROUND(m, 7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  SG_B2B_ROUND(m, 9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  SG_B2B_ROUND(m, 2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  SG_B2B_ROUND(m, 12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  SG_B2B_ROUND(m, 13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  SG_B2B_ROUND(m, 6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  SG_B2B_ROUND(m, 10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  SG_B2B_ROUND(m, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  SG_B2B_ROUND(m, 14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  out[0] = h0 ^ v0 ^ v8;
  out[1] = SG_B2B_IV1 ^ v1 ^ v9;
  out[2] = SG_B2B_IV2 ^ v2 ^ v10;
  out[3] = SG_B2B_IV3 ^ v3 ^ v11;
  out[4] = SG_B2B_IV4 ^ v4 ^ v12;
  out[5] = SG_B2B_IV5 ^ v5 ^ v13;
  out[6] = SG_B2B_IV6 ^ v6 ^ v14;
  out[7] = SG_B2B_IV7 ^ v7 ^ v15;
}

// Node digest: blake2b512(left || right), both 64-byte digests.
__host__ __device__ __forceinline__ void blake2b_node(const uint64_t l[8], const uint64_t r[8], uint64_t out[8]) {
  uint64_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { m[i] = l[i]; m[8 + i] = r[i]; }
  blake2b_single_block(m, 128, out);
}

}  // namespace sg
