// Native proof streams with the reference's byte-exact serialization.
//
//   IndependentProofStream   proof_stream.rs:15-78
//   SignatureProofStream     rescue_prime/proof_stream.rs:9-61
//   digest()                 stark/proof_stream_enum.rs:161-190:
//       16-byte BE field order (p if any object carries a field element:
//       Codeword, Leafs, Value; else 0) || per object [code u8][len u64 BE][payload]
//   deserialize              stark/stark.rs:30-67
#include "transcript.hpp"

#include <cstring>

#include "host_hash.hpp"

namespace sg {

static void put_be64(std::vector<uint8_t>& out, uint64_t v) {
  for (int i = 7; i >= 0; --i) out.push_back((uint8_t)(v >> (8 * i)));
}

static bool carries_field(uint8_t code, size_t len) {
  // Codeword with >= 1 element, Leafs, Value set the field (proof_stream_enum.rs:75-126, 164-174)
  if (code == 1) return len > 0;
  return code == 3 || code == 4;
}

size_t serialized_size(const std::vector<StreamObject>& objs, size_t count) {
  size_t n = 16;
  for (size_t i = 0; i < count; ++i) n += 9 + objs[i].payload.size();
  return n;
}

// one pass over the objects straight into `out` (serialized_size bytes)
void serialize_into(const std::vector<StreamObject>& objs, size_t count, uint8_t* out) {
  uint8_t* q = out + 16;
  bool field = false;
  for (size_t i = 0; i < count; ++i) {
    const StreamObject& o = objs[i];
    const uint64_t len = o.payload.size();
    field = field || carries_field(o.code, len);
    *q++ = o.code;
    for (int k = 7; k >= 0; --k) *q++ = (uint8_t)(len >> (8 * k));
    if (len) memcpy(q, o.payload.data(), len);
    q += len;
  }
  // p = 1 + 407 * 2^119 big-endian: 0x0cb8 << 116 | 1
  static const uint8_t pbe[16] = {0xcb, 0x80, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x01};
  if (field) memcpy(out, pbe, 16);
  else memset(out, 0, 16);
}

std::vector<uint8_t> serialize_objects(const std::vector<StreamObject>& objs, size_t count) {
  std::vector<uint8_t> out(serialized_size(objs, count));
  serialize_into(objs, count, out.data());
  return out;
}

std::vector<uint8_t> Stream::digest(size_t count) const { return serialize_objects(objects, count); }

void Stream::fiat_shamir_all(size_t num_bytes, uint8_t* out) {
  // header state if all objects are included
  bool field = fs_field;
  for (size_t i = fs_objects; i < objects.size(); ++i) field = field || carries_field(objects[i].code, objects[i].payload.size());
  if (fs_objects == 0 || field != fs_field) {
    // (re)build: [len u64 BE || prefix] for a signature stream, then header, then objects
    fs_input.clear();
    if (signature) {
      put_be64(fs_input, (uint64_t)prefix.size());
      fs_input.insert(fs_input.end(), prefix.begin(), prefix.end());
    }
    std::vector<uint8_t> d = serialize_objects(objects, objects.size());
    fs_input.insert(fs_input.end(), d.begin(), d.end());
    fs_objects = objects.size();
    fs_field = field;
    fs_sponge = ShakeSponge();
    fs_absorbed = 0;
  } else {
    for (size_t i = fs_objects; i < objects.size(); ++i) {
      const StreamObject& o = objects[i];
      fs_input.push_back(o.code);
      put_be64(fs_input, (uint64_t)o.payload.size());
      fs_input.insert(fs_input.end(), o.payload.begin(), o.payload.end());
    }
    fs_objects = objects.size();
  }
  const size_t rate = 136;
  size_t full = fs_input.size() / rate;
  size_t done = fs_absorbed / rate;
  if (full > done) {
    fs_sponge.absorb_blocks(fs_input.data() + done * rate, full - done);
    fs_absorbed = full * rate;
  }
  fs_sponge.finish(fs_input.data() + fs_absorbed, fs_input.size() - fs_absorbed, out, num_bytes);
}

void Stream::fiat_shamir(size_t count, size_t num_bytes, uint8_t* out) const {
  std::vector<uint8_t> d = digest(count);
  if (signature) {
    // shake256(len(prefix) u64 BE || prefix || digest)
    std::vector<uint8_t> in;
    put_be64(in, (uint64_t)prefix.size());
    in.insert(in.end(), prefix.begin(), prefix.end());
    in.insert(in.end(), d.begin(), d.end());
    shake256(in.data(), in.size(), out, num_bytes);
  } else {
    shake256(d.data(), d.size(), out, num_bytes);
  }
}

bool deserialize_stream(const uint8_t* b, size_t len, Stream& s, std::string& err) {
  if (len < 16) { err = "stream shorter than the field header"; return false; }
  size_t pos = 16;
  while (pos < len) {
    if (len - pos < 9) { err = "truncated object header"; return false; }
    uint8_t code = b[pos];
    uint64_t sz = 0;
    for (int i = 0; i < 8; ++i) sz = (sz << 8) | b[pos + 1 + i];
    pos += 9;
    if (sz > len - pos) { err = "truncated object payload"; return false; }
    if (code > 4) { err = "Unknown code"; return false; }
    StreamObject o;
    o.code = code;
    o.payload.assign(b + pos, b + pos + sz);
    s.objects.push_back(std::move(o));
    pos += sz;
  }
  return true;
}

}  // namespace sg
