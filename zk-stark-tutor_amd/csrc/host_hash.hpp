#pragma once
#include <cstddef>
#include <cstdint>

namespace sg {
void keccak_f1600(uint64_t a[25]);
// SHAKE256 sponge that can absorb whole 136-byte blocks incrementally and
// finish (pad + squeeze) from a copy, so a growing transcript is hashed once.
struct ShakeSponge {
  uint64_t st[25] = {0};
  void absorb_blocks(const uint8_t* in, size_t nblocks);
  void finish(const uint8_t* tail, size_t len, uint8_t* out, size_t outlen) const;
};
void shake256(const uint8_t* in, size_t len, uint8_t* out, size_t outlen);
void blake2b512(const uint8_t* in, size_t len, uint8_t out[64]);
}  // namespace sg
