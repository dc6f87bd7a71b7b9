#pragma once
#include <cstddef>
#include <cstdint>

namespace sg {
void shake256(const uint8_t* in, size_t len, uint8_t* out, size_t outlen);
void blake2b512(const uint8_t* in, size_t len, uint8_t out[64]);
}  // namespace sg
