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

}  // namespace sg
