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

// 8 decimal digits of c (< 10^8) as ASCII, most significant digit in byte 0.
__host__ __device__ __forceinline__ uint64_t ascii8(uint32_t c) {
  uint32_t hi4 = c / 10000u;
  uint32_t lo4 = c - hi4 * 10000u;
  uint32_t a = hi4 / 100u, b = hi4 - a * 100u;   // digits 0-1, 2-3
  uint32_t d = lo4 / 100u, e = lo4 - d * 100u;   // digits 4-5, 6-7
  uint32_t a1 = a / 10u, a0 = a - a1 * 10u;
  uint32_t b1 = b / 10u, b0 = b - b1 * 10u;
  uint32_t d1 = d / 10u, d0 = d - d1 * 10u;
  uint32_t e1 = e / 10u, e0 = e - e1 * 10u;
  uint32_t w0 = a1 | (a0 << 8) | (b1 << 16) | (b0 << 24);
  uint32_t w1 = d1 | (d0 << 8) | (e1 << 16) | (e0 << 24);
  return ((uint64_t)(w0 | 0x30303030u)) | ((uint64_t)(w1 | 0x30303030u) << 32);
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
  uint32_t len;
  if (c[0]) len = 32 + ndigits8(c[0]);
  else if (c[1]) len = 24 + ndigits8(c[1]);
  else if (c[2]) len = 16 + ndigits8(c[2]);
  else if (c[3]) len = 8 + ndigits8(c[3]);
  else len = ndigits8(c[4]);
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
