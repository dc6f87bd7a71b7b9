// Native proof streams with the reference's byte-exact serialization.
//
//   IndependentProofStream   proof_stream.rs:15-78
//   SignatureProofStream     rescue_prime/proof_stream.rs:9-61
//   digest()                 stark/proof_stream_enum.rs:161-190:
//       16-byte BE field order (p if any object carries a field element:
//       Codeword, Leafs, Value; else 0) || per object [code u8][len u64 BE][payload]
//   deserialize              stark/stark.rs:30-67
#include "transcript.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>

#include "host_hash.hpp"

namespace sg {

// ---------------------------------------------------------------- byte buffer

ByteBuf::~ByteBuf() {
  unpin();
  free(p);
}

void ByteBuf::reserve(size_t want) {
  if (want <= cap) return;
  size_t c = cap ? cap : 4096;
  while (c < want) c *= 2;
  unpin();  // the registration belongs to the old block
  void* q = realloc(p, c);
  if (!q) throw std::bad_alloc();
  p = static_cast<uint8_t*>(q);
  cap = c;
}

uint8_t* ByteBuf::grow(size_t add) {
  reserve(n + add);
  uint8_t* at = p + n;
  n += add;
  return at;
}

void ByteBuf::swap(ByteBuf& o) {
  std::swap(p, o.p);
  std::swap(n, o.n);
  std::swap(cap, o.cap);
  std::swap(pinned_p, o.pinned_p);
  std::swap(pinned_dev, o.pinned_dev);
  std::swap(pinned_device, o.pinned_device);
}

bool ByteBuf::pin() {
  // (a context with option stream_pin = 0 does not call this: its callers take their staging
  // fallback, which the tests exercise that way)
  if (!p) return false;
  if (pinned_p == p) return true;
  unpin();
  if (hipHostRegister(p, cap, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  pinned_p = p;
  // the device's address of the registered block (kernels may write the body directly)
  void* d = nullptr;
  pinned_dev = hipHostGetDevicePointer(&d, p, 0) == hipSuccess ? static_cast<uint8_t*>(d) : nullptr;
  if (!pinned_dev || hipGetDevice(&pinned_device) != hipSuccess) {
    (void)hipGetLastError();
    pinned_dev = nullptr;
    pinned_device = -1;
  }
  return true;
}

void ByteBuf::unpin() {
  if (!pinned_p) return;
  (void)hipHostUnregister(pinned_p);
  pinned_p = nullptr;
  pinned_dev = nullptr;
  pinned_device = -1;
}

namespace {

// released bodies keep their (warm) pages for the next stream: one proof stream per proof
// (never destroyed: streams may be released by a host runtime's own teardown after exit)
std::mutex& g_body_mu = *new std::mutex;
constexpr int kBodyCache = 2;
ByteBuf* const g_bodies = new ByteBuf[kBodyCache];
int g_nbodies = 0;
constexpr size_t kBodyMaxCached = (size_t)256 << 20;

void put_be64(std::vector<uint8_t>& out, uint64_t v) {
  for (int i = 7; i >= 0; --i) out.push_back((uint8_t)(v >> (8 * i)));
}

uint64_t get_be64(const uint8_t* b) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | b[i];
  return v;
}

bool carries_field(uint8_t code, size_t len) {
  // Codeword with >= 1 element, Leafs, Value set the field (proof_stream_enum.rs:75-126, 164-174)
  if (code == 1) return len > 0;
  return code == 3 || code == 4;
}

// p = 1 + 407 * 2^119 big-endian: 0x0cb8 << 116 | 1
const uint8_t kPrimeBE[16] = {0xcb, 0x80, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x01};

}  // namespace

// ---------------------------------------------------------------- stream

Stream::Stream() {
  std::lock_guard<std::mutex> lk(g_body_mu);
  if (g_nbodies > 0) body.swap(g_bodies[--g_nbodies]);
  body.n = 0;
}

Stream::~Stream() {
  if (!body.cap || body.cap > kBodyMaxCached) return;
  std::lock_guard<std::mutex> lk(g_body_mu);
  if (g_nbodies < kBodyCache) body.swap(g_bodies[g_nbodies++]);
}

size_t Stream::payload_len(size_t i) const { return (size_t)get_be64(body.data() + offs[i] + 1); }

uint8_t* Stream::push_reserve(uint8_t code, size_t len) {
  offs.push_back(body.n);
  uint8_t* h = body.grow(9 + len);
  h[0] = code;
  for (int i = 0; i < 8; ++i) h[1 + i] = (uint8_t)((uint64_t)len >> (8 * (7 - i)));
  field = field || carries_field(code, len);
  return h + 9;
}

uint8_t* Stream::append_block(size_t bytes, const std::vector<size_t>& obj_offsets, bool carries_field_) {
  const size_t base = body.n;
  uint8_t* at = body.grow(bytes);
  for (size_t o : obj_offsets) offs.push_back(base + o);
  field = field || carries_field_;
  return at;
}

void Stream::push(uint8_t code, const uint8_t* p, size_t len) {
  uint8_t* d = push_reserve(code, len);
  if (len) memcpy(d, p, len);
}

size_t Stream::digest_size(size_t cnt) const { return 16 + (cnt >= count() ? body.n : offs[cnt]); }

void Stream::digest_into(size_t cnt, uint8_t* out) const {
  bool f = field;
  if (cnt < count()) {
    f = false;
    for (size_t i = 0; i < cnt && !f; ++i) f = carries_field(code(i), payload_len(i));
  }
  if (f) memcpy(out, kPrimeBE, 16);
  else memset(out, 0, 16);
  const size_t len = digest_size(cnt) - 16;
  if (len) memcpy(out + 16, body.data(), len);
}

std::vector<uint8_t> Stream::digest(size_t cnt) const {
  std::vector<uint8_t> d(digest_size(cnt));
  digest_into(cnt, d.data());
  return d;
}

void Stream::fiat_shamir(size_t cnt, size_t num_bytes, uint8_t* out) const {
  std::vector<uint8_t> in;
  if (signature) {
    // shake256(len(prefix) u64 BE || prefix || digest)
    put_be64(in, (uint64_t)prefix.size());
    in.insert(in.end(), prefix.begin(), prefix.end());
  }
  const size_t pre = in.size();
  in.resize(pre + digest_size(cnt));
  digest_into(cnt, in.data() + pre);
  shake256(in.data(), in.size(), out, num_bytes);
}

// absorbs every complete block of fs_head || body not yet absorbed; returns the byte total
size_t Stream::fs_absorb_full() {
  const size_t R = 136;  // SHAKE256 rate
  if (!fs_valid || fs_field != field) {
    fs_head.clear();
    if (signature) {
      put_be64(fs_head, (uint64_t)prefix.size());
      fs_head.insert(fs_head.end(), prefix.begin(), prefix.end());
    }
    const uint8_t zero[16] = {0};
    fs_head.insert(fs_head.end(), field ? kPrimeBE : zero, (field ? kPrimeBE : zero) + 16);
    fs_sponge = ShakeSponge();
    fs_absorbed = 0;
    fs_field = field;
    fs_valid = true;
  }
  const size_t H = fs_head.size(), total = H + body.n;
  uint8_t tmp[R];
  size_t b = fs_absorbed / R;
  const size_t full = total / R;
  for (; b < full && b * R < H; ++b) {  // blocks that start in the head
    fs_gather(b * R, R, tmp);
    fs_sponge.absorb_blocks(tmp, 1);
  }
  if (b < full) {  // the rest straight from the body
    fs_sponge.absorb_blocks(body.data() + (b * R - H), full - b);
    b = full;
  }
  fs_absorbed = full * R;
  return total;
}

// bytes [off, off + len) of fs_head || body
void Stream::fs_gather(size_t off, size_t len, uint8_t* dst) const {
  const size_t H = fs_head.size();
  if (off < H) {
    const size_t a = len < H - off ? len : H - off;
    memcpy(dst, fs_head.data() + off, a);
    dst += a;
    off += a;
    len -= a;
  }
  if (len) memcpy(dst, body.data() + (off - H), len);
}

void Stream::fiat_shamir_all(size_t num_bytes, uint8_t* out) {
  const size_t total = fs_absorb_full();
  uint8_t tmp[136];
  const size_t tail = total - fs_absorbed;
  fs_gather(fs_absorbed, tail, tmp);
  fs_sponge.finish(tmp, tail, out, num_bytes);
}

bool deserialize_stream(const uint8_t* b, size_t len, Stream& s, std::string& err) {
  if (len < 16) { err = "stream shorter than the field header"; return false; }
  size_t pos = 16;
  while (pos < len) {
    if (len - pos < 9) { err = "truncated object header"; return false; }
    const uint8_t code = b[pos];
    const uint64_t sz = get_be64(b + pos + 1);
    pos += 9;
    if (sz > len - pos) { err = "truncated object payload"; return false; }
    if (code > 4) { err = "Unknown code"; return false; }
    s.push(code, b + pos, (size_t)sz);
    pos += sz;
  }
  return true;
}

}  // namespace sg
