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

static inline uint64_t rotl(uint64_t x, int n) { return (x << n) | (x >> ((64 - n) & 63)); }

// Unrolled Keccak-f[1600] (lanes a[x + 5y]).
void keccak_f1600(uint64_t a[25]) {
  for (int round = 0; round < 24; ++round) {
    uint64_t c0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20];
    uint64_t c1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];
    uint64_t c2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22];
    uint64_t c3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];
    uint64_t c4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];
    uint64_t d0 = c4 ^ rotl(c1, 1), d1 = c0 ^ rotl(c2, 1), d2 = c1 ^ rotl(c3, 1);
    uint64_t d3 = c2 ^ rotl(c4, 1), d4 = c3 ^ rotl(c0, 1);
    // theta + rho + pi: b[y, 2x+3y] = rotl(a[x,y] ^ d[x], r[x,y])
    uint64_t b00 = a[0] ^ d0;
    uint64_t b10 = rotl(a[6] ^ d1, 44);
    uint64_t b20 = rotl(a[12] ^ d2, 43);
    uint64_t b30 = rotl(a[18] ^ d3, 21);
    uint64_t b40 = rotl(a[24] ^ d4, 14);
    uint64_t b01 = rotl(a[3] ^ d3, 28);
    uint64_t b11 = rotl(a[9] ^ d4, 20);
    uint64_t b21 = rotl(a[10] ^ d0, 3);
    uint64_t b31 = rotl(a[16] ^ d1, 45);
    uint64_t b41 = rotl(a[22] ^ d2, 61);
    uint64_t b02 = rotl(a[1] ^ d1, 1);
    uint64_t b12 = rotl(a[7] ^ d2, 6);
    uint64_t b22 = rotl(a[13] ^ d3, 25);
    uint64_t b32 = rotl(a[19] ^ d4, 8);
    uint64_t b42 = rotl(a[20] ^ d0, 18);
    uint64_t b03 = rotl(a[4] ^ d4, 27);
    uint64_t b13 = rotl(a[5] ^ d0, 36);
    uint64_t b23 = rotl(a[11] ^ d1, 10);
    uint64_t b33 = rotl(a[17] ^ d2, 15);
    uint64_t b43 = rotl(a[23] ^ d3, 56);
    uint64_t b04 = rotl(a[2] ^ d2, 62);
    uint64_t b14 = rotl(a[8] ^ d3, 55);
    uint64_t b24 = rotl(a[14] ^ d4, 39);
    uint64_t b34 = rotl(a[15] ^ d0, 41);
    uint64_t b44 = rotl(a[21] ^ d1, 2);
    // chi (+ iota on lane 0); row y holds b[0..4][y]
    a[0] = b00 ^ (~b10 & b20) ^ KECCAK_RC[round];
    a[1] = b10 ^ (~b20 & b30);
    a[2] = b20 ^ (~b30 & b40);
    a[3] = b30 ^ (~b40 & b00);
    a[4] = b40 ^ (~b00 & b10);
    a[5] = b01 ^ (~b11 & b21);
    a[6] = b11 ^ (~b21 & b31);
    a[7] = b21 ^ (~b31 & b41);
    a[8] = b31 ^ (~b41 & b01);
    a[9] = b41 ^ (~b01 & b11);
    a[10] = b02 ^ (~b12 & b22);
    a[11] = b12 ^ (~b22 & b32);
    a[12] = b22 ^ (~b32 & b42);
    a[13] = b32 ^ (~b42 & b02);
    a[14] = b42 ^ (~b02 & b12);
    a[15] = b03 ^ (~b13 & b23);
    a[16] = b13 ^ (~b23 & b33);
    a[17] = b23 ^ (~b33 & b43);
    a[18] = b33 ^ (~b43 & b03);
    a[19] = b43 ^ (~b03 & b13);
    a[20] = b04 ^ (~b14 & b24);
    a[21] = b14 ^ (~b24 & b34);
    a[22] = b24 ^ (~b34 & b44);
    a[23] = b34 ^ (~b44 & b04);
    a[24] = b44 ^ (~b04 & b14);
  }
}

static const size_t SHAKE_RATE = 136;

void ShakeSponge::absorb_blocks(const uint8_t* in, size_t nblocks) {
  uint8_t* sb = reinterpret_cast<uint8_t*>(st);  // little-endian lanes (x86 host)
  for (size_t b = 0; b < nblocks; ++b) {
    for (size_t i = 0; i < SHAKE_RATE; ++i) sb[i] ^= in[b * SHAKE_RATE + i];
    keccak_f1600(st);
  }
}

void ShakeSponge::finish(const uint8_t* tail, size_t len, uint8_t* out, size_t outlen) const {
  uint64_t s[25];
  memcpy(s, st, sizeof(s));
  uint8_t* sb = reinterpret_cast<uint8_t*>(s);
  for (size_t i = 0; i < len; ++i) sb[i] ^= tail[i];
  sb[len] ^= 0x1F;
  sb[SHAKE_RATE - 1] ^= 0x80;
  keccak_f1600(s);
  while (outlen > 0) {
    size_t k = outlen < SHAKE_RATE ? outlen : SHAKE_RATE;
    memcpy(out, sb, k);
    out += k;
    outlen -= k;
    if (outlen) keccak_f1600(s);
  }
}

void shake256(const uint8_t* in, size_t len, uint8_t* out, size_t outlen) {
  ShakeSponge sp;
  size_t full = len / SHAKE_RATE;
  sp.absorb_blocks(in, full);
  sp.finish(in + full * SHAKE_RATE, len - full * SHAKE_RATE, out, outlen);
}

// ------------------------------------------------------------ BLAKE2b-512
static constexpr uint64_t B2B_IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                   0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                   0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
static constexpr uint8_t B2B_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// one compression, rounds unrolled by macro (locals v0..v15, the schedule's indices literal):
// 369 -> ~120 ns per block here; the FRI query sampler draws ~70 digests per prove
#define SG_B2B_G(a, b, c, d, x, y) \
  a = a + b + (x);                 \
  d = rotr(d ^ a, 32);             \
  c = c + d;                       \
  b = rotr(b ^ c, 24);             \
  a = a + b + (y);                 \
  d = rotr(d ^ a, 16);             \
  c = c + d;                       \
  b = rotr(b ^ c, 63);
#define SG_B2B_ROUND(r)                                                              \
  SG_B2B_G(v0, v4, v8, v12, m[B2B_SIGMA[r][0]], m[B2B_SIGMA[r][1]])                \
  SG_B2B_G(v1, v5, v9, v13, m[B2B_SIGMA[r][2]], m[B2B_SIGMA[r][3]])                \
  SG_B2B_G(v2, v6, v10, v14, m[B2B_SIGMA[r][4]], m[B2B_SIGMA[r][5]])               \
  SG_B2B_G(v3, v7, v11, v15, m[B2B_SIGMA[r][6]], m[B2B_SIGMA[r][7]])               \
  SG_B2B_G(v0, v5, v10, v15, m[B2B_SIGMA[r][8]], m[B2B_SIGMA[r][9]])               \
  SG_B2B_G(v1, v6, v11, v12, m[B2B_SIGMA[r][10]], m[B2B_SIGMA[r][11]])             \
  SG_B2B_G(v2, v7, v8, v13, m[B2B_SIGMA[r][12]], m[B2B_SIGMA[r][13]])              \
  SG_B2B_G(v3, v4, v9, v14, m[B2B_SIGMA[r][14]], m[B2B_SIGMA[r][15]])

static void b2b_compress(uint64_t h[8], const uint8_t block[128], uint64_t t, bool last) {
  uint64_t m[16];
  memcpy(m, block, 128);
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = B2B_IV[0], v9 = B2B_IV[1], v10 = B2B_IV[2], v11 = B2B_IV[3];
  uint64_t v12 = B2B_IV[4] ^ t, v13 = B2B_IV[5], v14 = last ? ~B2B_IV[6] : B2B_IV[6], v15 = B2B_IV[7];
  SG_B2B_ROUND(0) SG_B2B_ROUND(1) SG_B2B_ROUND(2) SG_B2B_ROUND(3) SG_B2B_ROUND(4) SG_B2B_ROUND(5)
  SG_B2B_ROUND(6) SG_B2B_ROUND(7) SG_B2B_ROUND(8) SG_B2B_ROUND(9) SG_B2B_ROUND(10) SG_B2B_ROUND(11)
  h[0] ^= v0 ^ v8;
  h[1] ^= v1 ^ v9;
  h[2] ^= v2 ^ v10;
  h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12;
  h[5] ^= v5 ^ v13;
  h[6] ^= v6 ^ v14;
  h[7] ^= v7 ^ v15;
}
#undef SG_B2B_ROUND
#undef SG_B2B_G

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
