// Device load/store of packed field elements (one dwordx4 per element).
#pragma once
#include <hip/hip_runtime.h>
#include "fe128.hpp"

namespace sg {

__device__ __forceinline__ fe ld_fe(const fe* p) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  fe r = {{v.x, v.y, v.z, v.w}};
  return r;
}
__device__ __forceinline__ void st_fe(fe* p, const fe& a) {
  *reinterpret_cast<uint4*>(p) = make_uint4(a.w[0], a.w[1], a.w[2], a.w[3]);
}

// streaming (read-once / write-once) element of a transform too large for the 256 MiB MALL:
// the non-temporal hint keeps it from displacing the twiddle tables (nt = false: plain access --
// a transform that fits the MALL is re-read from it by the next pass)
typedef unsigned int sg_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ fe ld_fe_stream(const fe* p, bool nt) {
  if (!nt) return ld_fe(p);
  const sg_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const sg_u32x4*>(p));
  fe r = {{v.x, v.y, v.z, v.w}};
  return r;
}
__device__ __forceinline__ void st_fe_stream(fe* p, const fe& a, bool nt) {
  if (!nt) return st_fe(p, a);
  sg_u32x4 v = {a.w[0], a.w[1], a.w[2], a.w[3]};
  __builtin_nontemporal_store(v, reinterpret_cast<sg_u32x4*>(p));
}

// (a + p) / 2 if a odd else a / 2 -- a * 2^-1 mod p for canonical a
__device__ __forceinline__ fe fe_halve(const fe& a) {
  uint64_t a0 = fe_lo(a), a1 = fe_hi(a);
  uint64_t odd = a0 & 1u;
  // s = a + odd*p (129 bits)
  uint64_t s0 = a0 + odd;             // p0 = 1
  uint64_t c0 = s0 < odd;
  uint64_t add1 = odd ? ((uint64_t)P3 << 32) : 0;
  uint64_t s1 = a1 + add1;
  uint64_t c1 = s1 < add1;
  uint64_t s1b = s1 + c0;
  c1 += s1b < c0;
  uint64_t r0 = (s0 >> 1) | (s1b << 63);
  uint64_t r1 = (s1b >> 1) | (c1 << 63);
  return fe_make(r0, r1);
}

}  // namespace sg
