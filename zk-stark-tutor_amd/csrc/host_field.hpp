// Host-side field helpers built on the same fe128.hpp arithmetic the kernels use.
// Used for per-call constants (twiddle seeds, n^-1, alpha terms, roots), never
// for bulk data.  Semantics follow field/field.rs and field/field_element.rs.
#pragma once
#include <cstdint>
#include "fe128.hpp"

namespace sg {

inline unsigned __int128 fe_to_u128(const fe& a) {
  return ((unsigned __int128)fe_hi(a) << 64) | fe_lo(a);
}
inline fe fe_from_u128(unsigned __int128 v) { return fe_make((uint64_t)v, (uint64_t)(v >> 64)); }

inline const fe& fe_prime() {
  static const fe p = fe_make(1ull, (uint64_t)P3 << 32);
  return p;
}
inline fe fe_one() { return fe_make(1, 0); }

// R^2 mod p, R = 2^128
inline const fe& fe_r2() {
  static const fe r2 = [] {
    unsigned __int128 p = fe_to_u128(fe_prime());
    fe r = fe_from_u128((unsigned __int128)0 - p);  // 2^128 - p == R mod p
    for (int i = 0; i < 128; ++i) r = fe_add(r, r);
    return r;
  }();
  return r2;
}

inline fe to_mont(const fe& a) { return mont_mul(a, fe_r2()); }
inline fe from_mont(const fe& a) { return mont_mul(a, fe_one()); }
// canonical product
inline fe fe_mul(const fe& a, const fe& b) { return mont_mul(mont_mul(a, b), fe_r2()); }

// a^e (field_element.rs:108-143 computes the same unique value); cost ~2 bitlen(e) products
inline fe fe_pow(const fe& a, unsigned __int128 e) {
  fe acc = to_mont(fe_one());
  if (e == 0) return fe_one();
  fe am = to_mont(a);
  int top = 127;
  while (!((e >> top) & 1)) --top;
  for (int i = top; i >= 0; --i) {
    acc = mont_mul(acc, acc);
    if ((e >> i) & 1) acc = mont_mul(acc, am);
  }
  return from_mont(acc);
}

// field.rs:160-169: xgcd inverse; inv(0) == 0.  Fermat gives the same value for a != 0.
inline fe fe_inv(const fe& a) {
  if ((a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0) return fe_zero();
  unsigned __int128 p = fe_to_u128(fe_prime());
  return fe_pow(a, p - 2);
}

inline fe fe_from_u64(uint64_t v) { return fe_make(v, 0); }

// field.rs:41-44
inline fe fe_generator() {
  // 85408008396924667383611388730472331217
  return fe_from_u128(((unsigned __int128)0x4040fbed12ee470full << 64) | 0xb5038f9c18f6f7d1ull);
}

// field.rs:87-99: fold (acc << 8) ^ b over a u128, then mod p
inline fe fe_sample(const uint8_t* bytes, size_t len) {
  unsigned __int128 acc = 0;
  for (size_t i = 0; i < len; ++i) acc = (acc << 8) ^ bytes[i];
  unsigned __int128 p = fe_to_u128(fe_prime());
  return fe_from_u128(acc % p);
}

}  // namespace sg
