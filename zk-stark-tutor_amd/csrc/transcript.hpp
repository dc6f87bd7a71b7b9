#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "host_hash.hpp"

namespace sg {

// growable byte buffer without value-initialization (a push writes every byte it adds)
struct ByteBuf {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  ByteBuf() = default;
  ByteBuf(const ByteBuf&) = delete;
  ByteBuf& operator=(const ByteBuf&) = delete;
  ~ByteBuf();
  uint8_t* grow(size_t add);  // n += add; returns the old end
  void reserve(size_t c);     // capacity >= c
  const uint8_t* data() const { return p; }
  size_t size() const { return n; }
  void swap(ByteBuf& o);
  // page-locks the whole capacity for device copies (hipHostRegister; kept until the buffer
  // moves or dies, so a cached body registers once); false if the runtime refuses
  bool pin();
  uint8_t* pinned_p = nullptr;
  uint8_t* pinned_dev = nullptr;  // the registered block's device address (nullptr: not mapped)
  int pinned_device = -1;         // the device current when it was registered (pinned_dev is its view)

 private:
  void unpin();
};

// A proof stream held in its serialized form (stark/proof_stream_enum.rs:161-190 without
// the 16-byte field header): objects are appended as [code u8][len u64 BE][payload] to
// one body, so a push is one append, the digest is one copy and the Fiat-Shamir sponge
// absorbs the body in place.  The body's buffer comes from a small process-wide cache, so
// a proof stream per proof does not fault in fresh pages.
struct Stream {
  ByteBuf body;
  std::vector<size_t> offs;     // header offset of each object in body
  bool field = false;           // an object carries a field element (header = p, else 0)
  size_t read_index = 0;
  bool signature = false;
  std::vector<uint8_t> prefix;  // blake2b512(document) for SignatureProofStream

  // fiat_shamir_prover cache: the sponge has absorbed the first fs_absorbed bytes of
  // fs_head || body (fs_head = signature prefix || field header); valid while objects are
  // only appended and the field header is unchanged.
  std::vector<uint8_t> fs_head;
  bool fs_valid = false;
  bool fs_field = false;
  size_t fs_absorbed = 0;
  ShakeSponge fs_sponge;

  Stream();
  ~Stream();
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;

  size_t count() const { return offs.size(); }
  uint8_t code(size_t i) const { return body.data()[offs[i]]; }
  size_t payload_len(size_t i) const;
  const uint8_t* payload(size_t i) const { return body.data() + offs[i] + 9; }
  // appends an object and returns its payload bytes (len of them) for the caller to fill
  uint8_t* push_reserve(uint8_t code, size_t len);
  void push(uint8_t code, const uint8_t* p, size_t len);
  // appends `bytes` of already serialized objects (headers included) whose headers sit at the
  // given offsets of the block, and returns the block for the caller to fill
  uint8_t* append_block(size_t bytes, const std::vector<size_t>& obj_offsets, bool carries_field);

  size_t digest_size(size_t count) const;
  void digest_into(size_t count, uint8_t* out) const;  // header || first `count` objects
  std::vector<uint8_t> digest(size_t count) const;
  std::vector<uint8_t> digest() const { return digest(count()); }
  void fiat_shamir(size_t count, size_t num_bytes, uint8_t* out) const;
  // fiat_shamir(count(), ...) with the incremental cache above
  void fiat_shamir_all(size_t num_bytes, uint8_t* out);

 private:
  size_t fs_absorb_full();
  void fs_gather(size_t off, size_t len, uint8_t* dst) const;
};

bool deserialize_stream(const uint8_t* b, size_t len, Stream& s, std::string& err);

}  // namespace sg
