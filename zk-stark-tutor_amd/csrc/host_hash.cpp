// Host hashes for the transcript and verifier side of the path.
//   shake256: FIPS 202 SHAKE256 (rate 136 B, suffix 0x1F), replacing crate
//             sha3 0.10.8 behind crypto/shake256.rs:7-19.
//   blake2b512: RFC 7693 BLAKE2b, 64-byte digest, unkeyed, any length, replacing
//             crate blake2 0.10.6 behind crypto/blake2b512.rs:4-14 (used on the
//             host by FRI::sample_indices, fri.rs:102, and Merkle verify).
#include "host_hash.hpp"

#include <cstring>

namespace sg {

// ------------------------------------------------------------ Keccak-f[1600]
static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
static const int KECCAK_ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                                   25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static inline uint64_t rotl(uint64_t x, int n) { return n == 0 ? x : (x << n) | (x >> (64 - n)); }

static void keccak_f1600(uint64_t st[25]) {
  for (int round = 0; round < 24; ++round) {
    uint64_t c[5], d[5], b[25];
    for (int x = 0; x < 5; ++x) c[x] = st[x] ^ st[x + 5] ^ st[x + 10] ^ st[x + 15] ^ st[x + 20];
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) st[i] ^= d[i % 5];
    // rho + pi: b[y, 2x+3y] = rotl(a[x, y], r[x, y])
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(st[x + 5 * y], KECCAK_ROT[x + 5 * y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y)
        st[x + 5 * y] = b[x + 5 * y] ^ ((~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]);
    st[0] ^= KECCAK_RC[round];
  }
}

void shake256(const uint8_t* in, size_t len, uint8_t* out, size_t outlen) {
  const size_t rate = 136;
  uint64_t st[25];
  memset(st, 0, sizeof(st));
  uint8_t* sb = reinterpret_cast<uint8_t*>(st);  // little-endian lane bytes (x86/AMD host)
  while (len >= rate) {
    for (size_t i = 0; i < rate; ++i) sb[i] ^= in[i];
    keccak_f1600(st);
    in += rate;
    len -= rate;
  }
  for (size_t i = 0; i < len; ++i) sb[i] ^= in[i];
  sb[len] ^= 0x1F;
  sb[rate - 1] ^= 0x80;
  keccak_f1600(st);
  while (outlen > 0) {
    size_t k = outlen < rate ? outlen : rate;
    memcpy(out, sb, k);
    out += k;
    outlen -= k;
    if (outlen) keccak_f1600(st);
  }
}

// ------------------------------------------------------------ BLAKE2b-512
static const uint64_t B2B_IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                   0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                   0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
static const uint8_t B2B_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void b2b_compress(uint64_t h[8], const uint8_t block[128], uint64_t t, bool last) {
  uint64_t m[16], v[16];
  memcpy(m, block, 128);
  for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = B2B_IV[i]; }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
  auto G = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
    v[a] = v[a] + v[b] + x; v[d] = rotr(v[d] ^ v[a], 32);
    v[c] = v[c] + v[d];     v[b] = rotr(v[b] ^ v[c], 24);
    v[a] = v[a] + v[b] + y; v[d] = rotr(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];     v[b] = rotr(v[b] ^ v[c], 63);
  };
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = B2B_SIGMA[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);   G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);  G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);  G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]); G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

void blake2b512(const uint8_t* in, size_t len, uint8_t out[64]) {
  uint64_t h[8];
  for (int i = 0; i < 8; ++i) h[i] = B2B_IV[i];
  h[0] ^= 0x01010040ull;
  uint8_t block[128];
  uint64_t t = 0;
  // all full blocks except the last one (an empty message is one zero block)
  while (len > 128) {
    t += 128;
    b2b_compress(h, in, t, false);
    in += 128;
    len -= 128;
  }
  memset(block, 0, 128);
  memcpy(block, in, len);
  t += len;
  b2b_compress(h, block, t, true);
  memcpy(out, h, 64);
}

}  // namespace sg
