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
constexpr uint64_t PC = 0xCB8ull;  // p = 1 + PC * 2^116
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

// r = x - p if (carry || x >= p) else x, for x < 2p given as 128 bits + carry.
__host__ __device__ __forceinline__ fe fe_reduce_once(uint64_t x0, uint64_t x1, uint32_t carry) {
  // d = x - p = x - 1 - (P3 << 96)
  uint64_t d0 = x0 - 1;
  uint64_t b0 = (x0 == 0);
  uint64_t sub1 = ((uint64_t)P3 << 32) + b0;
  uint64_t d1 = x1 - sub1;
  uint32_t borrow = x1 < sub1;
  // take d when carry==1 (x >= 2^128 > p) or no borrow (x >= p)
  bool take = carry | (borrow ^ 1u);
  uint64_t r0 = take ? d0 : x0;
  uint64_t r1 = take ? d1 : x1;
  return fe_make(r0, r1);
}

// a + b mod p, a,b canonical
__host__ __device__ __forceinline__ fe fe_add(const fe& a, const fe& b) {
  uint64_t a0 = fe_lo(a), a1 = fe_hi(a), b0 = fe_lo(b), b1 = fe_hi(b);
  uint64_t s0 = a0 + b0;
  uint64_t c0 = s0 < a0;
  uint64_t t1 = a1 + c0;
  uint32_t c1 = t1 < c0;
  uint64_t s1 = t1 + b1;
  c1 |= s1 < b1;
  return fe_reduce_once(s0, s1, c1);
}

// a - b mod p, a,b canonical
__host__ __device__ __forceinline__ fe fe_sub(const fe& a, const fe& b) {
  uint64_t a0 = fe_lo(a), a1 = fe_hi(a), b0 = fe_lo(b), b1 = fe_hi(b);
  uint64_t d0 = a0 - b0;
  uint64_t br0 = a0 < b0;
  uint64_t t1 = b1 + br0;          // b1 + br0 cannot overflow: b1 <= P3<<32 < 2^64 - 1
  uint64_t d1 = a1 - t1;
  bool neg = a1 < t1;
  // if negative add p = 1 + (P3 << 96)
  uint64_t e0 = d0 + 1;
  uint64_t ec = (e0 == 0);
  uint64_t e1 = d1 + ((uint64_t)P3 << 32) + ec;
  return neg ? fe_make(e0, e1) : fe_make(d0, d1);
}

__host__ __device__ __forceinline__ fe fe_neg(const fe& a) {
  return fe_sub(fe_zero(), a);
}

// ---------------------------------------------------------------------------
// 32x32+64 -> 64 multiply-accumulate with carry-out into a 32-bit third word.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void mac3(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& acc2) {
  uint64_t r;
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %5\n\t"
      "v_addc_co_u32 %2, %1, %2, 0, %1"
      : "=&v"(r), "=&s"(cc), "+v"(acc2)
      : "v"(a), "v"(b), "v"(acc));
  acc = r;
}
#else
__host__ inline void mac3(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& acc2) {
  uint64_t p = (uint64_t)a * b;
  uint64_t s = acc + p;
  acc2 += (s < p);
  acc = s;
}
#endif

// 128x128 -> 256-bit product, product-scanning (Comba) with a 96-bit column accumulator.
__host__ __device__ __forceinline__ void mul_wide(const fe& a, const fe& b, uint32_t t[8]) {
  uint64_t acc = 0;
  uint32_t acc2 = 0;
#define SG_COL_SHIFT(k)                                   \
  t[k] = (uint32_t)acc;                                   \
  acc = (acc >> 32) | ((uint64_t)acc2 << 32);             \
  acc2 = 0;
  mac3(a.w[0], b.w[0], acc, acc2);
  SG_COL_SHIFT(0)
  mac3(a.w[0], b.w[1], acc, acc2); mac3(a.w[1], b.w[0], acc, acc2);
  SG_COL_SHIFT(1)
  mac3(a.w[0], b.w[2], acc, acc2); mac3(a.w[1], b.w[1], acc, acc2); mac3(a.w[2], b.w[0], acc, acc2);
  SG_COL_SHIFT(2)
  mac3(a.w[0], b.w[3], acc, acc2); mac3(a.w[1], b.w[2], acc, acc2); mac3(a.w[2], b.w[1], acc, acc2);
  mac3(a.w[3], b.w[0], acc, acc2);
  SG_COL_SHIFT(3)
  mac3(a.w[1], b.w[3], acc, acc2); mac3(a.w[2], b.w[2], acc, acc2); mac3(a.w[3], b.w[1], acc, acc2);
  SG_COL_SHIFT(4)
  mac3(a.w[2], b.w[3], acc, acc2); mac3(a.w[3], b.w[2], acc, acc2);
  SG_COL_SHIFT(5)
  mac3(a.w[3], b.w[3], acc, acc2);
  t[6] = (uint32_t)acc;
  t[7] = (uint32_t)(acc >> 32);
#undef SG_COL_SHIFT
}

// One 64-bit Montgomery step on a value (x0 is the word being eliminated).
// in:  X = x0 + x1*2^64 + x2*2^128 + x3*2^192 (x3 small)
// out: (X + m*p) / 2^64 with m = -x0 mod 2^64, as y0 + y1*2^64 + y2*2^128.
__host__ __device__ __forceinline__ void mont_step(uint64_t x0, uint64_t x1, uint64_t x2, uint64_t x3,
                                                   uint64_t& y0, uint64_t& y1, uint64_t& y2) {
  uint64_t m = (uint64_t)0 - x0;
  uint64_t k = (x0 != 0);  // x0 + m == 2^64 * k
  // mc = m * PC (76 bits): lo64 / hi (<= 12 bits)
  uint64_t ml = (uint64_t)(uint32_t)m * PC;                // < 2^44
  uint64_t mh = (uint64_t)(uint32_t)(m >> 32) * PC;        // < 2^44
  uint64_t mc_lo = ml + (mh << 32);
  uint64_t mc_hi = (mh >> 32) + (mc_lo < ml);
  // add mc << 52 (relative to x1) : low word (mc_lo << 52), high word (mc >> 12)
  uint64_t add0 = mc_lo << 52;
  uint64_t add1 = (mc_lo >> 12) | (mc_hi << 52);
  uint64_t s0 = x1 + k;
  uint64_t c0 = s0 < k;
  uint64_t s0b = s0 + add0;
  c0 += s0b < add0;
  uint64_t s1 = x2 + add1;
  uint64_t c1 = s1 < add1;
  uint64_t s1b = s1 + c0;
  c1 += s1b < c0;
  y0 = s0b;
  y1 = s1b;
  y2 = x3 + c1;
}

// Montgomery product a*b*R^-1 mod p for canonical a, b (result canonical).
__host__ __device__ __forceinline__ fe mont_mul(const fe& a, const fe& b) {
  uint32_t t[8];
  mul_wide(a, b, t);
  uint64_t T0 = (uint64_t)t[0] | ((uint64_t)t[1] << 32);
  uint64_t T1 = (uint64_t)t[2] | ((uint64_t)t[3] << 32);
  uint64_t T2 = (uint64_t)t[4] | ((uint64_t)t[5] << 32);
  uint64_t T3 = (uint64_t)t[6] | ((uint64_t)t[7] << 32);
  uint64_t u0, u1, u2;
  mont_step(T0, T1, T2, T3, u0, u1, u2);
  uint64_t r0, r1, r2;
  mont_step(u0, u1, u2, 0, r0, r1, r2);
  return fe_reduce_once(r0, r1, (uint32_t)r2);
}

}  // namespace sg
