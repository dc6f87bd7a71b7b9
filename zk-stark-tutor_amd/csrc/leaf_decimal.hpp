// Merkle leaf message: the decimal ASCII string of a field element.
//
// The reference's leaf bytes are `FieldElement::to_string()` (field_element.rs:46-50):
// decimal, no sign, no leading zeros, "0" for zero; 1..39 bytes for p < 2^128.
// Those bytes become BLAKE2b message words m[0..4] (little-endian), t = len.
//
// Device recipe (all integer VALU, no lookup tables):
//   1. base-10^8 chunks c0..c4 (c0 most significant) by long division of the
//      four 32-bit limbs by 10^8 (each step divides a < 2^59 value by a constant);
//   2. each chunk -> 8 ASCII digits packed into one LE u64, most significant
//      digit in byte 0 => words B0..B4 are the 40-digit zero-padded string;
//   3. shift the 40-byte string left by s = 40 - len bytes (len from the
//      first non-zero chunk), which drops the leading '0's and zero-fills the
//      tail: that is exactly the padded BLAKE2b block.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "fe128.hpp"

namespace sg {

// 4 decimal digits of v (< 10^4) as ASCII, most significant digit in byte 0.
// Two-lane SWAR: t = (v / 100) | (v % 100) << 16, then one multiply splits both
// 2-digit lanes into tens/ones ((x * 103) >> 10 == x / 10 for x < 100).
__host__ __device__ __forceinline__ uint32_t ascii4(uint32_t v) {
  uint32_t a = (v * 5243u) >> 19;  // v / 100 for v < 10^4
  uint32_t t = a | ((v - a * 100u) << 16);
  uint32_t tens = ((t * 103u) >> 10) & 0x000F000Fu;
  uint32_t ones = t - tens * 10u;
  return tens | (ones << 8) | 0x30303030u;
}

// 8 decimal digits of c (< 10^8) as ASCII, most significant digit in byte 0.
__host__ __device__ __forceinline__ uint64_t ascii8(uint32_t c) {
  uint32_t hi4 = c / 10000u;
  return (uint64_t)ascii4(hi4) | ((uint64_t)ascii4(c - hi4 * 10000u) << 32);
}

// number of decimal digits of c (c < 10^8), 1 for c == 0
__host__ __device__ __forceinline__ uint32_t ndigits8(uint32_t c) {
  return 1u + (c >= 10u) + (c >= 100u) + (c >= 1000u) + (c >= 10000u) + (c >= 100000u) +
         (c >= 1000000u) + (c >= 10000000u);
}

// q = floor(x / 10^8), r = x mod 10^8 for x < 10^8 * 2^32
__host__ __device__ __forceinline__ uint32_t div1e8(uint64_t x, uint32_t& r) {
  uint32_t q = (uint32_t)(x / 100000000ull);
  r = (uint32_t)(x - (uint64_t)q * 100000000ull);
  return q;
}

// Fills m[0..4] with the LE message words of decimal(a); returns the length.
__host__ __device__ __forceinline__ uint32_t fe_decimal_words(const fe& a, uint64_t m[5]) {
  uint32_t l0 = a.w[0], l1 = a.w[1], l2 = a.w[2], l3 = a.w[3];
  uint32_t c[5];
  // four long divisions by 10^8; the quotient shrinks so later passes skip top limbs
  {
    uint32_t r = 0;
    l3 = div1e8((uint64_t)l3, r);
    l2 = div1e8(((uint64_t)r << 32) | l2, r);
    l1 = div1e8(((uint64_t)r << 32) | l1, r);
    l0 = div1e8(((uint64_t)r << 32) | l0, r);
    c[4] = r;
  }
  {
    uint32_t r = 0;
    l3 = div1e8((uint64_t)l3, r);
    l2 = div1e8(((uint64_t)r << 32) | l2, r);
    l1 = div1e8(((uint64_t)r << 32) | l1, r);
    l0 = div1e8(((uint64_t)r << 32) | l0, r);
    c[3] = r;
  }
  {
    // value < 2^128 / 10^16 < 2^75: l3 == 0
    uint32_t r = 0;
    l2 = div1e8((uint64_t)l2, r);
    l1 = div1e8(((uint64_t)r << 32) | l1, r);
    l0 = div1e8(((uint64_t)r << 32) | l0, r);
    c[2] = r;
  }
  {
    // value < 2^102 / 10^8... < 2^49: l2 == 0
    uint32_t r = 0;
    l1 = div1e8((uint64_t)l1, r);
    l0 = div1e8(((uint64_t)r << 32) | l0, r);
    c[1] = r;
  }
  c[0] = l0;  // < 2^128 / 10^32 < 3.5e6
  // length: 8 digits per chunk below the first non-zero chunk
  // (select the leading chunk first so ndigits8 is evaluated once)
  uint32_t lead = c[4], base = 0;
  if (c[3]) { lead = c[3]; base = 8; }
  if (c[2]) { lead = c[2]; base = 16; }
  if (c[1]) { lead = c[1]; base = 24; }
  if (c[0]) { lead = c[0]; base = 32; }
  uint32_t len = base + ndigits8(lead);
  // 40-byte zero-padded string as ten LE 32-bit words
  uint32_t w[11];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    uint64_t v = ascii8(c[k]);
    w[2 * k] = (uint32_t)v;
    w[2 * k + 1] = (uint32_t)(v >> 32);
  }
  w[10] = 0;
  // shift left (towards byte 0) by s = 40 - len bytes: word part, then byte part
  uint32_t s = 40u - len;
  uint32_t ws = s >> 2, bs = s & 3u;
#pragma unroll
  for (int bit = 8; bit >= 1; bit >>= 1) {
    bool take = (ws & (uint32_t)bit) != 0;
#pragma unroll
    for (int i = 0; i < 11; ++i) {
      uint32_t src = (i + bit < 11) ? w[i + bit] : 0u;
      w[i] = take ? src : w[i];
    }
  }
  uint32_t o[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // bytes [bs, bs+4) of the pair (w[i], w[i+1]) in little-endian order
    uint64_t pair = (uint64_t)w[i] | ((uint64_t)w[i + 1] << 32);
    o[i] = (uint32_t)(pair >> (8u * bs));
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = (uint64_t)o[2 * i] | ((uint64_t)o[2 * i + 1] << 32);
  return len;
}

}  // namespace sg
