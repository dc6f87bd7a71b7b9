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

}  // namespace sg
