#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "host_hash.hpp"

namespace sg {

struct StreamObject {
  uint8_t code;
  std::vector<uint8_t> payload;
};

struct Stream {
  std::vector<StreamObject> objects;
  size_t read_index = 0;
  bool signature = false;
  std::vector<uint8_t> prefix;  // blake2b512(document) for SignatureProofStream

  // fiat_shamir_prover cache: the FS input (signature prefix || digest) of all
  // objects is kept serialized, with a sponge holding its absorbed full blocks;
  // valid while objects are only appended and the field header is unchanged.
  std::vector<uint8_t> fs_input;
  size_t fs_objects = 0;      // objects serialized into fs_input
  bool fs_field = false;      // header value inside fs_input
  size_t fs_absorbed = 0;     // bytes of fs_input absorbed into fs_sponge
  ShakeSponge fs_sponge;

  std::vector<uint8_t> digest(size_t count) const;
  std::vector<uint8_t> digest() const { return digest(objects.size()); }
  void fiat_shamir(size_t count, size_t num_bytes, uint8_t* out) const;
  // fiat_shamir(objects.size(), ...) with the incremental cache above
  void fiat_shamir_all(size_t num_bytes, uint8_t* out);
};

std::vector<uint8_t> serialize_objects(const std::vector<StreamObject>& objs, size_t count);
size_t serialized_size(const std::vector<StreamObject>& objs, size_t count);
void serialize_into(const std::vector<StreamObject>& objs, size_t count, uint8_t* out);
bool deserialize_stream(const uint8_t* b, size_t len, Stream& s, std::string& err);

}  // namespace sg
