#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

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

  std::vector<uint8_t> digest(size_t count) const;
  std::vector<uint8_t> digest() const { return digest(objects.size()); }
  void fiat_shamir(size_t count, size_t num_bytes, uint8_t* out) const;
};

std::vector<uint8_t> serialize_objects(const std::vector<StreamObject>& objs, size_t count);
bool deserialize_stream(const uint8_t* b, size_t len, Stream& s, std::string& err);

}  // namespace sg
