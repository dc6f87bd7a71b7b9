// 128-bit prime-field arithmetic for p = 1 + 407 * 2^119 (field/field.rs:10), CDNA4-first.
//
// Representation: canonical value in [0, p) as four little-endian 32-bit limbs.
// Field data (codewords, coefficients) stays canonical everywhere; only
// constant multiplicands (twiddles, scale factors, alpha terms) are held in
// Montgomery form x*R mod p with R = 2^128, so mont_mul(data, const_mont)
// returns the canonical product without any conversion pass.
//
// p's shape drives the reduction: p = 1 + C * 2^116 with C = 0xCB8, so
// p == 1 (mod 2^64), -p^-1 == -1 (mod 2^64), and m*p = m + (m*C) << 116.
// A 64-bit Montgomery step therefore costs two 32x12-bit multiplies instead
// of a full 64x128 product.  p > 2^127, so a sum of two elements needs a
// 129th bit: add/sub/mul keep an explicit carry and correct once.
//
// The same code compiles for host (used by the library to build constants)
// and device; the device path uses v_mad_u64_u32 with its carry-out.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sg {

struct fe {
  uint32_t w[4];
};

// p limbs: [1, 0, 0, 0xCB800000]
constexpr uint32_t P0 = 1u, P3 = 0xCB800000u;
constexpr uint64_t PC = 0xCB8ull;  // p = 1 + PC * 2^116 = 1 + (P3 << 96)
// R mod p and R^2 mod p (R = 2^128), little-endian 32-bit limbs.
// R mod p   = 2^128 - p           (2^128 < 2p)
// R^2 mod p computed at build time by the host helpers below.

__host__ __device__ __forceinline__ fe fe_zero() { fe r = {{0, 0, 0, 0}}; return r; }
__host__ __device__ __forceinline__ fe fe_make(uint64_t lo, uint64_t hi) {
  fe r = {{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)}};
  return r;
}
__host__ __device__ __forceinline__ uint64_t fe_lo(const fe& a) { return (uint64_t)a.w[0] | ((uint64_t)a.w[1] << 32); }
__host__ __device__ __forceinline__ uint64_t fe_hi(const fe& a) { return (uint64_t)a.w[2] | ((uint64_t)a.w[3] << 32); }
__host__ __device__ __forceinline__ bool fe_eq(const fe& a, const fe& b) {
  return ((a.w[0] ^ b.w[0]) | (a.w[1] ^ b.w[1]) | (a.w[2] ^ b.w[2]) | (a.w[3] ^ b.w[3])) == 0;
}
__host__ __device__ __forceinline__ bool fe_is_canonical(const fe& a) {
  // a < p  <=>  a3 < P3 || (a3 == P3 && a0..a2 == 0)
  return a.w[3] < P3 || (a.w[3] == P3 && (a.w[0] | a.w[1] | a.w[2]) == 0);
}

// All carries are explicit 32-bit add/sub-with-carry chains (__builtin_addc /
// __builtin_subc lower to v_add_co_u32 / v_addc_co_u32 on gfx950), and the
// Montgomery product is 16 v_mad_u64_u32 (product scanning with a 96-bit
// column accumulator) + 4 for the sparse reduction.  tools/microbench_field.hip
// measured 462 G butterflies/s for this form vs 285 G for a 64-bit-word
// formulation on MI355X (bit-identical results).

// "x >= p" as a carry: x + (2^128 - p) overflows iff x >= p (x < 2^128).
// 2^128 - p = 0x347FFFFF_FFFFFFFF_FFFFFFFF_FFFFFFFF.
#define SG_NEG_P3 0x347FFFFFu

// a + b mod p, a,b canonical
__host__ __device__ __forceinline__ fe fe_add(const fe& a, const fe& b) {
  unsigned c, g;
  uint32_t s0 = __builtin_addc(a.w[0], b.w[0], 0u, &c);
  uint32_t s1 = __builtin_addc(a.w[1], b.w[1], c, &c);
  uint32_t s2 = __builtin_addc(a.w[2], b.w[2], c, &c);
  uint32_t s3 = __builtin_addc(a.w[3], b.w[3], c, &c);
  uint32_t d0 = __builtin_addc(s0, 0xFFFFFFFFu, 0u, &g);
  uint32_t d1 = __builtin_addc(s1, 0xFFFFFFFFu, g, &g);
  uint32_t d2 = __builtin_addc(s2, 0xFFFFFFFFu, g, &g);
  uint32_t d3 = __builtin_addc(s3, SG_NEG_P3, g, &g);
  bool take = (c | g) != 0;  // sum >= 2^128, or sum >= p
  fe r = {{take ? d0 : s0, take ? d1 : s1, take ? d2 : s2, take ? d3 : s3}};
  return r;
}

// a - b mod p, a,b canonical
__host__ __device__ __forceinline__ fe fe_sub(const fe& a, const fe& b) {
  unsigned br, c;
  uint32_t d0 = __builtin_subc(a.w[0], b.w[0], 0u, &br);
  uint32_t d1 = __builtin_subc(a.w[1], b.w[1], br, &br);
  uint32_t d2 = __builtin_subc(a.w[2], b.w[2], br, &br);
  uint32_t d3 = __builtin_subc(a.w[3], b.w[3], br, &br);
  uint32_t e0 = __builtin_addc(d0, P0, 0u, &c);
  uint32_t e1 = __builtin_addc(d1, 0u, c, &c);
  uint32_t e2 = __builtin_addc(d2, 0u, c, &c);
  uint32_t e3 = __builtin_addc(d3, P3, c, &c);
  bool neg = br != 0;  // a < b: add p back
  fe r = {{neg ? e0 : d0, neg ? e1 : d1, neg ? e2 : d2, neg ? e3 : d3}};
  return r;
}

__host__ __device__ __forceinline__ fe fe_neg(const fe& a) {
  return fe_sub(fe_zero(), a);
}

// Lazy forms for the NTT butterflies: values anywhere in [0, 2^128) (< 2p), the
// second operand canonical (a Montgomery product).  Only the 129th bit / the
// borrow is corrected, by adding or subtracting p = 1 + (P3 << 96) under one
// mask: 9 instructions instead of the 13 of a full reduction.  The residue is
// the same, so a transform that canonicalizes on its last store is bit-exact.
//   a + b  < 2^128 + p: on carry subtract p  -> [2^128 - p, 2^128)
//   a - b >= -p:        on borrow add p      -> [0, p)
__host__ __device__ __forceinline__ fe fe_add_lazy(const fe& a, const fe& b) {
  unsigned c, g;
  uint32_t s0 = __builtin_addc(a.w[0], b.w[0], 0u, &c);
  uint32_t s1 = __builtin_addc(a.w[1], b.w[1], c, &c);
  uint32_t s2 = __builtin_addc(a.w[2], b.w[2], c, &c);
  uint32_t s3 = __builtin_addc(a.w[3], b.w[3], c, &c);
  // a + b - p = (a + b - 2^128) + (2^128 - p): add 2^128 - p under the carry mask
  const uint32_t m = c ? 0xFFFFFFFFu : 0u;
  const uint32_t m3 = c ? SG_NEG_P3 : 0u;
  fe r;
  r.w[0] = __builtin_addc(s0, m, 0u, &g);
  r.w[1] = __builtin_addc(s1, m, g, &g);
  r.w[2] = __builtin_addc(s2, m, g, &g);
  r.w[3] = __builtin_addc(s3, m3, g, &g);
  return r;
}

__host__ __device__ __forceinline__ fe fe_sub_lazy(const fe& a, const fe& b) {
  unsigned br, c;
  uint32_t d0 = __builtin_subc(a.w[0], b.w[0], 0u, &br);
  uint32_t d1 = __builtin_subc(a.w[1], b.w[1], br, &br);
  uint32_t d2 = __builtin_subc(a.w[2], b.w[2], br, &br);
  uint32_t d3 = __builtin_subc(a.w[3], b.w[3], br, &br);
  const uint32_t m3 = br ? P3 : 0u;
  fe r;
  r.w[0] = __builtin_addc(d0, 0u, br, &c);
  r.w[1] = __builtin_addc(d1, 0u, c, &c);
  r.w[2] = __builtin_addc(d2, 0u, c, &c);
  r.w[3] = __builtin_addc(d3, m3, c, &c);
  return r;
}

// [0, 2^128) -> [0, p): subtract p once if a >= p
__host__ __device__ __forceinline__ fe fe_canon(const fe& a) {
  unsigned g;
  uint32_t d0 = __builtin_addc(a.w[0], 0xFFFFFFFFu, 0u, &g);
  uint32_t d1 = __builtin_addc(a.w[1], 0xFFFFFFFFu, g, &g);
  uint32_t d2 = __builtin_addc(a.w[2], 0xFFFFFFFFu, g, &g);
  uint32_t d3 = __builtin_addc(a.w[3], 0x347FFFFFu, g, &g);
  fe r = {{g ? d0 : a.w[0], g ? d1 : a.w[1], g ? d2 : a.w[2], g ? d3 : a.w[3]}};
  return r;
}

// ---------------------------------------------------------------------------
// 32x32+64 -> 64 multiply-accumulate with carry-out into a 32-bit third word.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void mac3(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& acc2) {
  uint64_t r;
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %5\n\t"
      "v_addc_co_u32 %2, %1, %2, 0, %1"
      : "=v"(r), "=s"(cc), "+v"(acc2)
      : "v"(a), "v"(b), "v"(acc));
  acc = r;
}
// first product of a column: the carry-out initializes the third word
// (one v_cndmask instead of zeroing it and adding the carry)
__device__ __forceinline__ void mac3_first(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& acc2) {
  uint64_t r;
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %5\n\t"
      "v_cndmask_b32_e64 %2, 0, 1, %1"
      : "=v"(r), "=s"(cc), "=v"(acc2)
      : "v"(a), "v"(b), "v"(acc));
  acc = r;
}
#else
__host__ inline void mac3_first(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& acc2) {
  uint64_t p = (uint64_t)a * b;
  uint64_t s = acc + p;
  acc2 = (s < p);
  acc = s;
}
__host__ inline void mac3(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& acc2) {
  uint64_t p = (uint64_t)a * b;
  uint64_t s = acc + p;
  acc2 += (s < p);
  acc = s;
}
#endif

// 128x128 -> 256-bit product, product scanning (Comba) with a 96-bit column accumulator.
__host__ __device__ __forceinline__ void mul_wide(const fe& a, const fe& b, uint32_t t[8]) {
  uint64_t acc = (uint64_t)a.w[0] * b.w[0];
  uint32_t acc2;
#define SG_COL_SHIFT(k)                                   \
  t[k] = (uint32_t)acc;                                   \
  acc = (acc >> 32) | ((uint64_t)acc2 << 32);
  t[0] = (uint32_t)acc;
  acc >>= 32;
  acc += (uint64_t)a.w[0] * b.w[1];  // < 2^32 + (2^32-1)^2: no carry
  mac3_first(a.w[1], b.w[0], acc, acc2);
  SG_COL_SHIFT(1)
  mac3_first(a.w[0], b.w[2], acc, acc2); mac3(a.w[1], b.w[1], acc, acc2); mac3(a.w[2], b.w[0], acc, acc2);
  SG_COL_SHIFT(2)
  mac3_first(a.w[0], b.w[3], acc, acc2); mac3(a.w[1], b.w[2], acc, acc2); mac3(a.w[2], b.w[1], acc, acc2);
  mac3(a.w[3], b.w[0], acc, acc2);
  SG_COL_SHIFT(3)
  mac3_first(a.w[1], b.w[3], acc, acc2); mac3(a.w[2], b.w[2], acc, acc2); mac3(a.w[3], b.w[1], acc, acc2);
  SG_COL_SHIFT(4)
  mac3_first(a.w[2], b.w[3], acc, acc2); mac3(a.w[3], b.w[2], acc, acc2);
  t[5] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)acc2 << 32);
  acc += (uint64_t)a.w[3] * b.w[3];  // the top column cannot overflow: T < 2^256
  t[6] = (uint32_t)acc;
  t[7] = (uint32_t)(acc >> 32);
#undef SG_COL_SHIFT
}

// Montgomery product a*b*R^-1 mod p (R = 2^128) for a < 2^128, b < p; result canonical.
// Two 64-bit reduction steps: m = -x0 mod 2^64 (p == 1 mod 2^64), x0 + m
// carries exactly (x0 != 0), and m*(p-1) = (m * P3) << 96 is a 96-bit term.
__host__ __device__ __forceinline__ fe mont_mul(const fe& a, const fe& b) {
  uint32_t t[8];
  mul_wide(a, b, t);
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
  uint32_t u5 = t[7] + c;  // U < 2^192
  // step 2: eliminate (u0, u1)
  uint32_t n0 = __builtin_subc(0u, u0, 0u, &br);
  uint32_t n1 = __builtin_subc(0u, u1, br, &br);
  uint64_t s0 = (uint64_t)n0 * P3;
  uint64_t s1 = (uint64_t)n1 * P3 + (s0 >> 32);
  uint32_t r0 = __builtin_addc(u2, br, 0u, &c);
  uint32_t r1 = __builtin_addc(u3, (uint32_t)s0, c, &c);
  uint32_t r2 = __builtin_addc(u4, (uint32_t)s1, c, &c);
  uint32_t r3 = __builtin_addc(u5, (uint32_t)(s1 >> 32), c, &c);
  // r + c*2^128 < 2p: subtract p once if c or r >= p
  unsigned g;
  uint32_t d0 = __builtin_addc(r0, 0xFFFFFFFFu, 0u, &g);
  uint32_t d1 = __builtin_addc(r1, 0xFFFFFFFFu, g, &g);
  uint32_t d2 = __builtin_addc(r2, 0xFFFFFFFFu, g, &g);
  uint32_t d3 = __builtin_addc(r3, SG_NEG_P3, g, &g);
  bool take = (c | g) != 0;
  fe r = {{take ? d0 : r0, take ? d1 : r1, take ? d2 : r2, take ? d3 : r3}};
  return r;
}

}  // namespace sg
