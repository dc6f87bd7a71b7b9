// fast_cpu.cpp -- optimized CPU restatement of the hot path.
//
// TEST INFRASTRUCTURE + CPU BASELINE ONLY: loaded by tests/ (the full-size checker:
// 2^22..2^27 transforms, 2^24/2^25 Merkle trees and FRI proofs, and the barycentric
// pieces the trace-2^20 verifier needs) and by bench.py's all-cores cpu_baseline leg,
// through oracle/fast_cpu.py.  Never linked into libstarkgpu.
//
// Same results as the reference (and as oracle/stark_oracle.py, which it is checked
// against on the reference's known-answer vectors), different arithmetic:
//   * F_p, p = 1 + 407 * 2^119 (field/field.rs:10): Montgomery products with R = 2^128
//     in two 64-bit reduction steps (p == 1 mod 2^64), instead of the bit-serial
//     mul_mod of field.rs:117-131; inverses by Fermat instead of u_xgcd (xgcd.rs:22-48).
//   * ntt (fft/ntt.rs:7-49): the reference's radix-2 DIT graph (bit_reverse_copy, then
//     stage S pairs (j, j + 2^(S-1)) with powtable[k * n / 2^S]), run as cache-sized
//     passes over OpenMP threads; the same butterflies, so identical for ANY root.
//   * intt (ntt.rs:51-68), Polynomial::scale (polynomial.rs:109-121),
//     fast_coset_evaluate (ntt_arithmetics.rs:161-170).
//   * BLAKE2b-512 (RFC 7693; crate blake2 0.10.6, crypto/blake2b512.rs:4-14) over the
//     decimal leaves (field_element.rs:46-50) and 128-byte nodes: MerkleRoot::commit /
//     open (merkle_root.rs:7-66), all levels kept, one thread per leaf range.
//   * SHAKE256 (FIPS 202; crate sha3 0.10.8, crypto/shake256.rs), the serialized proof
//     stream (stark/proof_stream_enum.rs:67-127,161-190, proof_stream.rs:31-48),
//     Field::sample (field.rs:87-99), FRI::commit / sample_indices / query / prove
//     (fri.rs:40-248) with the fold's per-element alpha / (offset omega^i) as a running
//     product of omega^-1.
//   * barycentric evaluation of the interpolant through (q^r, v_r), r < n, and the
//     product prod_{r<n} (x - q^r): what Stark::verify (stark.rs:565-770) evaluates for
//     the Rescue AIR's round-constant polynomials and the transition zerofier at the
//     FRI query points; O(n) per point, so a trace-2^20 proof is checkable.
//
// Element I/O: little-endian (lo, hi) u64 pairs, canonical -- the layout of sg_fe.
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

typedef unsigned __int128 u128;

namespace {

const u128 P = ((u128)0xCB8 << 116) | 1;
const uint64_t PK = 0xCB8ull << 52;  // (p - 1) >> 64: m * p = m + ((m * PK) << 64)

inline u128 ld(const uint64_t* p) { return ((u128)p[1] << 64) | p[0]; }
inline void st(uint64_t* p, u128 v) { p[0] = (uint64_t)v; p[1] = (uint64_t)(v >> 64); }

inline u128 fadd(u128 a, u128 b) {  // a, b < p
  u128 s = a + b;
  if (s < a || s >= P) s -= P;  // wrap-around arithmetic: exact in both cases
  return s;
}
inline u128 fsub(u128 a, u128 b) { return a >= b ? a - b : a - b + P; }

// a * b * 2^-128 mod p for a < 2^128, b < p; canonical result
inline u128 mont(u128 a, u128 b) {
  const uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64), b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  const u128 x00 = (u128)a0 * b0, x01 = (u128)a0 * b1, x10 = (u128)a1 * b0, x11 = (u128)a1 * b1;
  const uint64_t t0 = (uint64_t)x00;
  const u128 s1 = (x00 >> 64) + (uint64_t)x01 + (uint64_t)x10;
  const uint64_t t1 = (uint64_t)s1;
  const u128 s2 = (s1 >> 64) + (x01 >> 64) + (x10 >> 64) + (uint64_t)x11;
  const uint64_t t2 = (uint64_t)s2;
  const uint64_t t3 = (uint64_t)((s2 >> 64) + (x11 >> 64));
  // step 1: m = -t0, (T + m p) / 2^64 = t1 + t2 2^64 + t3 2^128 + (t0 != 0) + m PK
  const uint64_t m = 0 - t0;
  const u128 mk = (u128)m * PK;
  const u128 v0 = (u128)t1 + (t0 != 0) + (uint64_t)mk;
  const u128 v1 = (v0 >> 64) + t2 + (uint64_t)(mk >> 64);
  const uint64_t u0 = (uint64_t)v0, u1 = (uint64_t)v1, u2 = t3 + (uint64_t)(v1 >> 64);
  // step 2
  const uint64_t m2 = 0 - u0;
  const u128 mk2 = (u128)m2 * PK;
  const u128 w0 = (u128)u1 + (u0 != 0) + (uint64_t)mk2;
  const u128 w1 = (w0 >> 64) + u2 + (uint64_t)(mk2 >> 64);  // < 2^65
  u128 r = ((u128)(uint64_t)w1 << 64) | (uint64_t)w0;
  if ((w1 >> 64) || r >= P) r -= P;
  return r;
}

struct Consts {
  u128 R, R2;  // 2^128 mod p, 2^256 mod p
  Consts() {
    u128 r = 1;
    for (int i = 0; i < 128; ++i) r = fadd(r, r);
    R = r;
    for (int i = 0; i < 128; ++i) r = fadd(r, r);
    R2 = r;
  }
};
const Consts& K() {
  static const Consts c;
  return c;
}
inline u128 to_m(u128 a) { return mont(a, K().R2); }
inline u128 from_m(u128 a) { return mont(a, 1); }
inline u128 fmul(u128 a, u128 b) { return mont(mont(a, b), K().R2); }
// Montgomery-domain power
u128 pow_m(u128 am, u128 e) {
  u128 r = K().R;
  while (e) {
    if (e & 1) r = mont(r, am);
    am = mont(am, am);
    e >>= 1;
  }
  return r;
}
u128 fpow(u128 a, u128 e) { return from_m(pow_m(to_m(a), e)); }
u128 finv(u128 a) { return fpow(a, P - 2); }

uint64_t bitrev64(uint64_t x) {
  x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
  x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
  return __builtin_bswap64(x);
}

int log2_exact(uint64_t n) {
  int l = 0;
  while (((uint64_t)1 << l) < n) ++l;
  return l;
}

// pw[k] = Montgomery(w^k), k < cnt, in parallel chunks
void powers_m(u128 w, uint64_t cnt, u128* pw) {
  const u128 wm = to_m(w);
#pragma omp parallel
  {
    const int T = omp_get_num_threads(), id = omp_get_thread_num();
    const uint64_t per = (cnt + T - 1) / T, k0 = std::min(cnt, per * id), k1 = std::min(cnt, k0 + per);
    if (k0 < k1) {
      u128 v = pow_m(wm, k0);
      for (uint64_t k = k0; k < k1; ++k) {
        pw[k] = v;
        v = mont(v, wm);
      }
    }
  }
}

// ------------------------------------------------------------------ NTT (ntt.rs:7-49)

// In-place DIT over a bit-reversed array; pw[k] = Montgomery(root^k), k < n/2.
void dit(u128* a, int logn, const u128* pw) {
  const uint64_t n = (uint64_t)1 << logn;
  // pass 1: stages 1..L1 inside contiguous blocks of 2^L1
  const int L1 = std::min(logn, 12);
  const uint64_t B = (uint64_t)1 << L1;
#pragma omp parallel for schedule(static)
  for (int64_t blk = 0; blk < (int64_t)(n / B); ++blk) {
    u128* x = a + blk * B;
    for (int S = 1; S <= L1; ++S) {
      const uint64_t half = (uint64_t)1 << (S - 1), stride = n >> S;
      for (uint64_t j0 = 0; j0 < B; j0 += 2 * half)
        for (uint64_t k = 0; k < half; ++k) {
          const u128 u = x[j0 + k], v = mont(x[j0 + k + half], pw[k * stride]);
          x[j0 + k] = fadd(u, v);
          x[j0 + k + half] = fsub(u, v);
        }
    }
  }
  // later passes: stages b0+1 .. b0+L on tiles of 2^L rows x C consecutive columns
  int b0 = L1;
  while (b0 < logn) {
    const int L = std::min(logn - b0, 9);
    const int logC = std::min(b0, 4);
    const uint64_t C = (uint64_t)1 << logC, rows = (uint64_t)1 << L;
    const uint64_t ncb = (uint64_t)1 << (b0 - logC), nh = n >> (b0 + L);
#pragma omp parallel
    {
      std::vector<u128> tile(rows * C);
#pragma omp for schedule(static)
      for (int64_t t = 0; t < (int64_t)(nh * ncb); ++t) {
        const uint64_t h = t / ncb, cb = t % ncb;
        const uint64_t base = (h << (b0 + L)) + cb * C;
        for (uint64_t g = 0; g < rows; ++g) memcpy(&tile[g * C], a + base + (g << b0), C * sizeof(u128));
        for (int s = 1; s <= L; ++s) {
          const int S = b0 + s;
          const uint64_t half = (uint64_t)1 << (s - 1), stride = n >> S;
          for (uint64_t g0 = 0; g0 < rows; g0 += 2 * half)
            for (uint64_t gl = 0; gl < half; ++gl) {
              const uint64_t kb = (gl << b0) + cb * C;
              u128* lo = &tile[(g0 + gl) * C];
              u128* hi = &tile[(g0 + gl + half) * C];
              for (uint64_t c = 0; c < C; ++c) {
                const u128 u = lo[c], v = mont(hi[c], pw[(kb + c) * stride]);
                lo[c] = fadd(u, v);
                hi[c] = fsub(u, v);
              }
            }
        }
        for (uint64_t g = 0; g < rows; ++g) memcpy(a + base + (g << b0), &tile[g * C], C * sizeof(u128));
      }
    }
    b0 += L;
  }
}

// out[j] = in[rev(j)] (zero beyond n_in), optionally scaled by Montgomery(offset^rev(j))
void bitrev_load(const uint64_t* in, uint64_t n_in, int logn, u128* out, const u128* scale_pw) {
  const uint64_t n = (uint64_t)1 << logn;
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < (int64_t)n; ++j) {
    const uint64_t i = logn ? (bitrev64((uint64_t)j) >> (64 - logn)) : 0;
    u128 v = 0;
    if (i < n_in) {
      v = ld(in + 2 * i);
      if (scale_pw) v = mont(v, scale_pw[i]);
    }
    out[j] = v;
  }
}

void store_all(const u128* a, uint64_t n, uint64_t* out, u128 post_m, bool post) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) st(out + 2 * i, post ? mont(a[i], post_m) : a[i]);
}

// ------------------------------------------------------------------ hashes

const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                        0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
constexpr uint8_t SG[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// one compression; m = 16 little-endian message words.  Fully unrolled with constant
// sigma indices so the 16-word state stays in registers.
#define FC_G(a, b, c, d, x, y)                   \
  a = a + b + (x); d = rotr(d ^ a, 32);          \
  c = c + d;       b = rotr(b ^ c, 24);          \
  a = a + b + (y); d = rotr(d ^ a, 16);          \
  c = c + d;       b = rotr(b ^ c, 63);
#define FC_ROUND(r)                                                          \
  FC_G(v0, v4, v8, v12, m[SG[r][0]], m[SG[r][1]])                            \
  FC_G(v1, v5, v9, v13, m[SG[r][2]], m[SG[r][3]])                            \
  FC_G(v2, v6, v10, v14, m[SG[r][4]], m[SG[r][5]])                           \
  FC_G(v3, v7, v11, v15, m[SG[r][6]], m[SG[r][7]])                           \
  FC_G(v0, v5, v10, v15, m[SG[r][8]], m[SG[r][9]])                           \
  FC_G(v1, v6, v11, v12, m[SG[r][10]], m[SG[r][11]])                         \
  FC_G(v2, v7, v8, v13, m[SG[r][12]], m[SG[r][13]])                          \
  FC_G(v3, v4, v9, v14, m[SG[r][14]], m[SG[r][15]])
inline void b2b_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = IV[0], v9 = IV[1], v10 = IV[2], v11 = IV[3], v12 = IV[4] ^ t, v13 = IV[5];
  uint64_t v14 = last ? ~IV[6] : IV[6], v15 = IV[7];
  FC_ROUND(0) FC_ROUND(1) FC_ROUND(2) FC_ROUND(3) FC_ROUND(4) FC_ROUND(5)
  FC_ROUND(6) FC_ROUND(7) FC_ROUND(8) FC_ROUND(9) FC_ROUND(0) FC_ROUND(1)
  h[0] ^= v0 ^ v8; h[1] ^= v1 ^ v9; h[2] ^= v2 ^ v10; h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12; h[5] ^= v5 ^ v13; h[6] ^= v6 ^ v14; h[7] ^= v7 ^ v15;
}
#undef FC_ROUND
#undef FC_G

void b2b_init(uint64_t h[8]) {
  for (int i = 0; i < 8; ++i) h[i] = IV[i];
  h[0] ^= 0x01010040ULL;  // digest 64 bytes, no key, fanout 1, depth 1
}

void blake2b512(const uint8_t* in, size_t len, uint8_t out[64]) {
  uint64_t h[8], m[16];
  b2b_init(h);
  uint64_t t = 0;
  while (len > 128) {
    memcpy(m, in, 128);
    t += 128;
    b2b_compress(h, m, t, false);
    in += 128;
    len -= 128;
  }
  memset(m, 0, 128);
  memcpy(m, in, len);
  t += len;
  b2b_compress(h, m, t, true);
  memcpy(out, h, 64);
}

// field_element.rs:46-50: the decimal string of the value (v < 2^128 < 10^39):
// v = hi * 10^19 + lo by one u128 division, hi < 10^20 split once more in 64 bits
int to_decimal(u128 v, char* buf) {
  const uint64_t E19 = 10000000000000000000ull;
  char tmp[48];
  int n = 0;
  uint64_t parts[3];
  int np = 0;
  if (v >> 64) {
    const u128 q = v / E19;
    parts[np++] = (uint64_t)(v - q * E19);
    if (q >> 64 || (uint64_t)q >= E19) {
      const u128 q2 = q / E19;
      parts[np++] = (uint64_t)(q - q2 * E19);
      parts[np++] = (uint64_t)q2;
    } else {
      parts[np++] = (uint64_t)q;
    }
  } else {
    const uint64_t lo = (uint64_t)v;
    if (lo >= E19) {
      parts[np++] = lo % E19;
      parts[np++] = lo / E19;
    } else {
      parts[np++] = lo;
    }
  }
  for (int k = 0; k < np; ++k) {
    uint64_t c = parts[k];
    const bool top = k == np - 1;
    for (int d = 0; d < 19 && (!top || c); ++d) {
      tmp[n++] = (char)('0' + c % 10);
      c /= 10;
    }
  }
  if (n == 0) tmp[n++] = '0';
  for (int i = 0; i < n; ++i) buf[i] = tmp[n - 1 - i];
  return n;
}

void leaf_digest(u128 v, uint64_t d[8]) {
  uint64_t m[16] = {0};
  const int len = to_decimal(v, reinterpret_cast<char*>(m));
  b2b_init(d);
  b2b_compress(d, m, (uint64_t)len, true);
}

void node_digest(const uint64_t l[8], const uint64_t r[8], uint64_t d[8]) {
  uint64_t m[16];
  memcpy(m, l, 64);
  memcpy(m + 8, r, 64);
  b2b_init(d);
  b2b_compress(d, m, 128, true);
}

// Keccak-f[1600] / SHAKE256 (rate 136, domain byte 0x1F)
const uint64_t RC[24] = {0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
                         0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
                         0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
                         0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
                         0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
                         0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
const int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

inline uint64_t rotl(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

void keccakf(uint64_t s[25]) {
  for (int round = 0; round < 24; ++round) {
    uint64_t c[5], b[25];
    for (int x = 0; x < 5; ++x) c[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
    for (int x = 0; x < 5; ++x) {
      const uint64_t d = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
      for (int y = 0; y < 25; y += 5) s[x + y] ^= d;
    }
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(s[x + 5 * y], ROT[x + 5 * y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) s[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    s[0] ^= RC[round];
  }
}

void shake256(const uint8_t* in, size_t len, uint8_t* out, size_t outlen) {
  uint64_t s[25] = {0};
  uint8_t* sb = reinterpret_cast<uint8_t*>(s);
  const size_t rate = 136;
  while (len >= rate) {
    for (size_t i = 0; i < rate; ++i) sb[i] ^= in[i];
    keccakf(s);
    in += rate;
    len -= rate;
  }
  for (size_t i = 0; i < len; ++i) sb[i] ^= in[i];
  sb[len] ^= 0x1F;
  sb[rate - 1] ^= 0x80;
  keccakf(s);
  while (outlen) {
    const size_t k = outlen < rate ? outlen : rate;
    memcpy(out, sb, k);
    out += k;
    outlen -= k;
    if (outlen) keccakf(s);
  }
}

// ------------------------------------------------------------------ Merkle (merkle_root.rs)

// all levels: level k (n >> k digests) at digest offset 2n - 2(n >> k); 8 u64 per digest
struct Tree {
  uint64_t n = 0;
  std::vector<uint64_t> d;
  const uint64_t* level(int k) const { return d.data() + 8 * (2 * n - 2 * (n >> k)); }
  const uint64_t* root() const { return d.data() + 8 * (2 * n - 2); }
};

void build_tree(const u128* leaves, uint64_t n, Tree& t) {
  t.n = n;
  t.d.resize(8 * (2 * n - 1));
  uint64_t* L0 = t.d.data();
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) leaf_digest(leaves[i], L0 + 8 * i);
  const int logn = log2_exact(n);
  for (int k = 1; k <= logn; ++k) {
    const uint64_t* ch = t.d.data() + 8 * (2 * n - 2 * (n >> (k - 1)));
    uint64_t* lv = t.d.data() + 8 * (2 * n - 2 * (n >> k));
    const int64_t cnt = (int64_t)(n >> k);
#pragma omp parallel for schedule(static) if (cnt > 1024)
    for (int64_t i = 0; i < cnt; ++i) node_digest(ch + 16 * i, ch + 16 * i + 8, lv + 8 * i);
  }
}

// ------------------------------------------------------------------ proof stream

struct Stream {
  std::vector<uint8_t> body;  // objects after the 16-byte header
  bool field = false;
  // Fiat-Shamir input prefix: empty for IndependentProofStream (proof_stream.rs:31-48);
  // [len u64 BE][blake2b512(document)] for SignatureProofStream (rescue_prime/proof_stream.rs:22-39)
  std::vector<uint8_t> fs_prefix;
  void push(uint8_t code, const uint8_t* p, size_t len, bool carries_field) {
    body.push_back(code);
    for (int b = 7; b >= 0; --b) body.push_back((uint8_t)((uint64_t)len >> (8 * b)));
    body.insert(body.end(), p, p + len);
    field = field || carries_field;
  }
  std::vector<uint8_t> digest() const {
    std::vector<uint8_t> out(16 + body.size());
    if (field)
      for (int b = 0; b < 16; ++b) out[b] = (uint8_t)(P >> (8 * (15 - b)));
    memcpy(out.data() + 16, body.data(), body.size());
    return out;
  }
  void fiat_shamir(uint8_t out[32]) const {
    std::vector<uint8_t> d = fs_prefix;
    const std::vector<uint8_t> b = digest();
    d.insert(d.end(), b.begin(), b.end());
    shake256(d.data(), d.size(), out, 32);
  }
};

void put_be128(uint8_t* p, u128 v) {
  for (int b = 0; b < 16; ++b) p[b] = (uint8_t)(v >> (8 * (15 - b)));
}

u128 sample_field(const uint8_t* b, size_t len) {  // field.rs:87-99
  u128 acc = 0;
  for (size_t i = 0; i < len; ++i) acc = (acc << 8) ^ b[i];
  return acc % P;
}

uint64_t sample_index(const uint8_t* d, size_t dlen, uint64_t size) {  // fri.rs:60-86
  int lg = 63 - __builtin_clzll(size);
  size_t nb = (size_t)lg / 8 + 1;
  if (nb > dlen) nb = dlen;
  uint64_t acc = 0;
  for (size_t i = dlen - nb; i < dlen; ++i) acc = (acc << 8) ^ d[i];
  return acc % size;
}

// path payload of leaf i (merkle_root.rs:34-53, proof_stream_enum.rs:95-126): per level
// [64 as u64 BE][sibling digest], leaf level first
std::vector<uint8_t> path_payload(const Tree& t, uint64_t i) {
  const int lg = log2_exact(t.n);
  std::vector<uint8_t> pl(72 * (size_t)lg);
  for (int k = 0; k < lg; ++k) {
    uint8_t* q = &pl[72 * (size_t)k];
    memset(q, 0, 8);
    q[7] = 64;
    memcpy(q + 8, t.level(k) + 8 * ((i >> k) ^ 1), 64);
  }
  return pl;
}

thread_local std::string g_err;  // message of the last failed checker call

struct CheckError {
  int code;
  std::string msg;
};
#define FC_REQUIRE(cond, code, msg) \
  do {                              \
    if (!(cond)) throw CheckError{code, msg}; \
  } while (0)

// FRI::prove (fri.rs:210-248): commit (fri.rs:115-172), sample_indices (fri.rs:88-113) over
// len(codewords[1]) reduced by len(codewords[-1]), query per round (fri.rs:174-208).  Returns the
// number of rounds; the c top-level indices land in `top`.
uint64_t fri_prove(Stream& ps, u128 offset, u128 omega, std::vector<u128>&& cw0, uint64_t expansion,
                   uint64_t colinearity, std::vector<uint64_t>& top) {
  const uint64_t n = cw0.size();
  FC_REQUIRE(n && !(n & (n - 1)), -1, "FRI codeword length must be a power of two");
  uint64_t rounds = 0;
  for (uint64_t len = n; len > expansion && len > 4 * colinearity; len /= 2) ++rounds;  // fri.rs:40-50
  FC_REQUIRE(rounds >= 2, -1, "FRI prove needs at least two rounds (reference indexes codewords[1])");
  u128 w = omega, o = offset;
  std::vector<std::vector<u128>> cws(rounds);
  std::vector<Tree> trees(rounds);
  cws[0] = std::move(cw0);
  const u128 inv2m = to_m(finv(2));
  for (uint64_t r = 0; r < rounds; ++r) {
    const uint64_t len = cws[r].size();
    FC_REQUIRE(fpow(w, len - 1) == finv(w), -2, "error in commit: omega does not have the right order!");
    build_tree(cws[r].data(), len, trees[r]);
    ps.push(0, reinterpret_cast<const uint8_t*>(trees[r].root()), 64, false);
    if (r == rounds - 1) break;
    uint8_t ch[32];
    ps.fiat_shamir(ch);
    const u128 alpha = sample_field(ch, 32);
    // c'[i] = 2^-1 ((1 + a/(o w^i)) c[i] + (1 - a/(o w^i)) c[i + h]);  a/(o w^i) = a o^-1 (w^-1)^i
    const uint64_t half = len / 2;
    cws[r + 1].resize(half);
    const u128 am = to_m(fmul(alpha, finv(o))), wim = to_m(finv(w)), Rm = K().R;
    const u128* c = cws[r].data();
    u128* nx = cws[r + 1].data();
#pragma omp parallel
    {
      const int T = omp_get_num_threads(), id = omp_get_thread_num();
      const uint64_t per = (half + T - 1) / T, i0 = std::min(half, per * id), i1 = std::min(half, i0 + per);
      if (i0 < i1) {
        u128 abo = mont(am, pow_m(wim, i0));  // Montgomery(a o^-1 w^-i0)
        for (uint64_t i = i0; i < i1; ++i) {
          const u128 f = mont(c[i], fadd(Rm, abo)), s = mont(c[half + i], fsub(Rm, abo));
          nx[i] = mont(fadd(f, s), inv2m);
          abo = mont(abo, wim);
        }
      }
    }
    w = fmul(w, w);
    o = fmul(o, o);
  }
  {  // last codeword (fri.rs:166)
    const std::vector<u128>& last = cws[rounds - 1];
    std::vector<uint8_t> pl(16 * last.size());
    for (size_t i = 0; i < last.size(); ++i) put_be128(&pl[16 * i], last[i]);
    ps.push(1, pl.data(), pl.size(), !last.empty());
  }
  uint8_t seed[32];
  ps.fiat_shamir(seed);
  const uint64_t size = cws[1].size(), reduced = cws[rounds - 1].size();
  FC_REQUIRE(colinearity <= 2 * reduced, -3, "Not enough entropy in indices with reference to last codeword");
  FC_REQUIRE(colinearity <= reduced, -3, "Cannot sample more indices than available in the last codeword");
  std::vector<uint64_t> idx, red;
  std::vector<uint8_t> msg(seed, seed + 32);
  for (uint64_t counter = 0; idx.size() < colinearity; ++counter) {
    msg.resize(32 + counter, 0);
    uint8_t d[64];
    blake2b512(msg.data(), msg.size(), d);
    const uint64_t index = sample_index(d, 64, size), rr = index % reduced;
    if (std::find(red.begin(), red.end(), rr) == red.end()) {
      idx.push_back(index);
      red.push_back(rr);
    }
  }
  top = idx;
  std::vector<uint64_t> cur = idx;
  for (uint64_t r = 0; r + 1 < rounds; ++r) {
    const uint64_t half = cws[r].size() / 2;
    for (auto& i : cur) i %= half;
    for (uint64_t s = 0; s < colinearity; ++s) {
      uint8_t pl[48];
      put_be128(pl, cws[r][cur[s]]);
      put_be128(pl + 16, cws[r][cur[s] + half]);
      put_be128(pl + 32, cws[r + 1][cur[s]]);
      ps.push(3, pl, 48, true);
    }
    for (uint64_t s = 0; s < colinearity; ++s) {
      std::vector<uint8_t> a = path_payload(trees[r], cur[s]), b = path_payload(trees[r], cur[s] + half),
                           c = path_payload(trees[r + 1], cur[s]);
      ps.push(2, a.data(), a.size(), false);
      ps.push(2, b.data(), b.size(), false);
      ps.push(2, c.data(), c.size(), false);
    }
  }
  return rounds;
}

// ------------------------------------------------------------------ Stark::prove (checker)
//
// stark/stark.rs:276-562 for a Rescue-Prime AIR, restated with fast CPU algorithms that give the
// reference's exact outputs (every polynomial below is the unique one the reference computes, and
// every step whose result depends on the algorithm -- fast_coset_divide, fast_multiply, the
// NTT butterfly graph for roots of smaller order -- is the reference's own step):
//   * trace / round-constant interpolation over q^i, i < n (fast_interpolate_domain,
//     ntt_arithmetics.rs:172-237; the unique interpolant of degree < n, length n): values on the
//     whole group <q> by the barycentric formula with closed-form weights, the sum over the domain
//     as one cyclic convolution, then one INTT;
//   * the transition zerofier prod_{i<n} (x - q^i) (fast_zerofier, ntt_arithmetics.rs:66-113; no
//     wrap-around below the domain order) by doubling: Z_2k(x) = Z_k(x) q^(k^2) Z_k(q^-k x);
//   * evaluate_symbolic of the Rescue-Prime AIR (m_polynomial.rs:124-139 over rescue_prime.rs:
//     246-283): its values on a coset of size L > its length from the factored form, then one
//     INTT (the coefficient vector is exact: degree < length <= L);
//   * fast_coset_divide / fast_multiply / fast_coset_evaluate literally (ntt_arithmetics.rs:5-64,
//     161-170, 239-310), incl. a NTT of a vector longer than the root's order (the reference's
//     ntt pads to the next power of two and runs its butterfly graph with the smaller-order root).
using Vec = std::vector<u128>;

u128 generator_fe() {  // field.rs:41-44: 85408008396924667383611388730472331217
  static const u128 g = [] {
    const char* s = "85408008396924667383611388730472331217";
    u128 v = 0;
    for (const char* c = s; *c; ++c) v = v * 10 + (u128)(*c - '0');
    return v;
  }();
  return g;
}

// field.rs:58-71: square the generator (order 2^119) down to order n
u128 root_of_order(uint64_t n) {
  FC_REQUIRE(n && !(n & (n - 1)) && log2_exact(n) <= 119, -1, "root order must be a power of two <= 2^119");
  u128 r = generator_fe();
  for (int k = 119; k > log2_exact(n); --k) r = fmul(r, r);
  return r;
}

int64_t pdegree(const Vec& a) {  // polynomial.rs:41-58
  for (size_t i = a.size(); i-- > 0;)
    if (a[i]) return (int64_t)i;
  return -1;
}

Vec pneg(const Vec& a) {
  Vec o(a.size());
  for (size_t i = 0; i < a.size(); ++i) o[i] = a[i] ? P - a[i] : 0;
  return o;
}

// polynomial.rs:251-276: a zero operand returns the other one unchanged (its length kept)
Vec padd(const Vec& a, const Vec& b) {
  if (pdegree(a) < 0) return b;
  if (pdegree(b) < 0) return a;
  Vec o(std::max(a.size(), b.size()), 0);
  for (size_t i = 0; i < a.size(); ++i) o[i] = a[i];
  for (size_t i = 0; i < b.size(); ++i) o[i] = fadd(o[i], b[i]);
  return o;
}

Vec psub(const Vec& a, const Vec& b) { return padd(a, pneg(b)); }

// polynomial.rs:109-121: c_i f^i
Vec pscale(const Vec& a, u128 f) {
  Vec pw(a.size()), o(a.size());
  powers_m(f, a.size(), pw.data());
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)a.size(); ++i) o[i] = mont(a[i], pw[i]);
  return o;
}

// in place: a[i] *= c (canonical)
void pmul_const(Vec& a, u128 c) {
  const u128 cm = to_m(c);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)a.size(); ++i) a[i] = mont(a[i], cm);
}

// ntt.rs:7-49 (literal): zero-pad to next_pow2(len), bit-reverse, radix-2 DIT with powtable
// root^k, k < n/2 -- the same butterflies for any root, including roots of smaller order
Vec ref_ntt(u128 root, const Vec& in) {
  FC_REQUIRE(!in.empty(), -1, "ntt of an empty input");
  const int logn = log2_exact(in.size());
  const uint64_t n = (uint64_t)1 << logn;
  Vec a(n), pw(std::max<uint64_t>(n / 2, 1));
  powers_m(root, std::max<uint64_t>(n / 2, 1), pw.data());
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < (int64_t)n; ++j) {
    const uint64_t i = logn ? (bitrev64((uint64_t)j) >> (64 - logn)) : 0;
    a[j] = i < in.size() ? in[i] : 0;
  }
  dit(a.data(), logn, pw.data());
  return a;
}

// ntt.rs:51-68: fewer than 2 elements are returned unchanged
Vec ref_intt(u128 root, const Vec& in) {
  if (in.size() < 2) return in;
  Vec a = ref_ntt(finv(root), in);
  pmul_const(a, finv((u128)a.size()));
  return a;
}

// ntt_arithmetics.rs:161-170: scale by offset^i, pad to root_order (longer: the reference
// panics on the usize underflow), ntt(generator)
Vec coset_eval(u128 gen, uint64_t root_order, u128 offset, const Vec& c) {
  FC_REQUIRE(c.size() <= root_order, -1, "fast_coset_evaluate: polynomial longer than root_order");
  Vec s = pscale(c, offset);
  s.resize(root_order, 0);
  return ref_ntt(gen, s);
}

// pointwise a[i] / b[i] with Montgomery's batch inversion (chunks over the threads); a zero
// divisor is the reference's "divide by zero" panic (field_element.rs:82-90)
Vec batch_div(const Vec& a, const Vec& b) {
  const uint64_t n = std::min(a.size(), b.size());
  Vec out(n);
  bool zero = false;
#pragma omp parallel reduction(|| : zero)
  {
    const int T = omp_get_num_threads(), id = omp_get_thread_num();
    const uint64_t per = (n + T - 1) / T, i0 = std::min(n, per * id), i1 = std::min(n, i0 + per);
    if (i0 < i1) {
      Vec pre(i1 - i0);
      u128 acc = K().R;
      for (uint64_t i = i0; i < i1; ++i) {
        if (!b[i]) zero = true;
        pre[i - i0] = acc;
        acc = mont(acc, to_m(b[i] ? b[i] : 1));
      }
      u128 iv = to_m(finv(from_m(acc)));  // Montgomery(1 / prod)
      for (uint64_t i = i1; i-- > i0;) {
        const u128 bi = to_m(b[i] ? b[i] : 1);
        const u128 inv_b = mont(iv, pre[i - i0]);  // Montgomery(1 / b_i)
        iv = mont(iv, bi);
        out[i] = mont(a[i], inv_b);
      }
    }
  }
  FC_REQUIRE(!zero, -5, "divide by zero");
  return out;
}

Vec hadamard(const Vec& a, const Vec& b) {
  const uint64_t n = std::min(a.size(), b.size());
  Vec o(n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) o[i] = fmul(a[i], b[i]);
  return o;
}

void check_root(u128 root, uint64_t order) {  // ntt_arithmetics.rs:11-24
  FC_REQUIRE(fpow(root, order) == 1, -1, "supplied root does not have supplied root_order");
  FC_REQUIRE(fpow(root, order / 2) != 1, -1, "supplied root is not a primitive of root_order");
}

// ntt_arithmetics.rs:5-64
Vec fast_multiply(u128 root, uint64_t root_order, const Vec& lhs, const Vec& rhs) {
  check_root(root, root_order);
  const int64_t dl = pdegree(lhs), dr = pdegree(rhs);
  if (dl < 0 || dr < 0) return {};
  const uint64_t deg = (uint64_t)(dl + dr), result_len = deg + 1;
  uint64_t order = root_order;
  while (deg < order / 2) {
    root = fmul(root, root);
    order /= 2;
  }
  auto inner = [&](const Vec& p) {
    Vec q = p;
    if (q.size() < order) q.resize(order, 0);
    return ref_ntt(root, q);
  };
  Vec c = ref_intt(root, hadamard(inner(lhs), inner(rhs)));
  if (result_len < c.size()) c.resize(result_len);
  return c;
}

// ntt_arithmetics.rs:239-310
Vec fast_coset_divide(u128 root, uint64_t root_order, u128 offset, const Vec& lhs, const Vec& rhs) {
  check_root(root, root_order);
  FC_REQUIRE(pdegree(rhs) >= 0, -1, "cannot divide by zero polynomial");
  if (pdegree(lhs) < 0) return {};
  const int64_t dl = pdegree(lhs), dr = pdegree(rhs);
  FC_REQUIRE(dl >= dr, -1, "cannot divide by polynomial of larger degree");
  const uint64_t deg = (uint64_t)std::max(dl, dr), result_len = (uint64_t)(dl - dr + 1);
  uint64_t order = root_order;
  while (deg < order / 2) {
    root = fmul(root, root);
    order /= 2;
  }
  auto inner = [&](const Vec& p) {
    Vec q = pscale(p, offset);
    if (q.size() < order) q.resize(order, 0);
    return ref_ntt(root, q);
  };
  Vec c = ref_intt(root, batch_div(inner(lhs), inner(rhs)));
  if (result_len < c.size()) c.resize(result_len);
  return pscale(c, finv(offset));
}

// exact product by NTT (both degrees known; no wrap-around: transform length > deg)
Vec poly_mul_exact(const Vec& a, const Vec& b) {
  if (a.empty() || b.empty()) return {};
  const uint64_t len = a.size() + b.size() - 1, n = (uint64_t)1 << log2_exact(len);
  const u128 w = root_of_order(std::max<uint64_t>(n, 2));
  Vec x = a, y = b;
  x.resize(std::max<uint64_t>(n, 2), 0);
  y.resize(std::max<uint64_t>(n, 2), 0);
  Vec c = ref_intt(w, hadamard(ref_ntt(w, x), ref_ntt(w, y)));
  c.resize(len);
  return c;
}

// inclusive prefix products in the Montgomery domain (chunks over the threads)
Vec prefix_prod_m(const Vec& xm) {
  const uint64_t n = xm.size();
  Vec out(n);
  const int T = omp_get_max_threads();
  Vec tot(T, K().R);
#pragma omp parallel num_threads(T)
  {
    const int nt = omp_get_num_threads(), id = omp_get_thread_num();
    const uint64_t per = (n + nt - 1) / nt, i0 = std::min(n, per * id), i1 = std::min(n, i0 + per);
    u128 acc = K().R;
    for (uint64_t i = i0; i < i1; ++i) {
      acc = mont(acc, xm[i]);
      out[i] = acc;
    }
    tot[id] = acc;
#pragma omp barrier
    u128 base = K().R;
    for (int t = 0; t < id; ++t) base = mont(base, tot[t]);
    for (uint64_t i = i0; i < i1; ++i) out[i] = mont(out[i], base);
  }
  return out;
}

// The unique interpolant of degree < n through (q^i, y_i), i < n, q of order D (a power of two),
// length n: what fast_interpolate_domain (ntt_arithmetics.rs:172-237) returns on this domain.
//   P(q^m) = y_m (m < n);  P(q^m) = q^(m(n-1)) C_m / C_(m-n) S(m)  (n <= m < D)
//   S(m) = sum_i a_i K_(m-i),  a_i = y_i / Z'(q^i),  K_j = 1 / (1 - q^-j),  C_k = prod_{j<=k} (1 - q^-j)
//   Z'(q^i) = (-1)^(n-1-i) q^(E_i) C_i C_(n-1-i),  E_i = i(n-1) + (n-1-i)(n-i)/2
// then INTT over <q>; S is one cyclic convolution of length D.
Vec geo_interpolate(u128 q, uint64_t D, const Vec& y) {
  const uint64_t n = y.size();
  FC_REQUIRE(n <= D, -1, "more points than the domain order");
  if (n == 0) return {};
  if (n == 1) return {y[0]};
  if (n == D) return ref_intt(q, y);
  const u128 qinv = finv(q);
  // u_j = 1 - q^-j (j >= 1; u_0 := 1), K_j = 1 / u_j (K_0 := 0 for the convolution)
  Vec qp(D), um(D);
  powers_m(qinv, D, qp.data());
  const u128 one_m = K().R;
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < (int64_t)D; ++j) um[j] = j ? fsub(one_m, qp[j]) : one_m;  // Montgomery(u_j)
  Vec u(D);
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < (int64_t)D; ++j) u[j] = from_m(um[j]);
  Vec ones(D, 1);
  Vec Kc = batch_div(ones, u);  // canonical 1 / u_j
  Vec Km(D);
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < (int64_t)D; ++j) Km[j] = to_m(Kc[j]);
  const Vec Cm = prefix_prod_m(um), Cim = prefix_prod_m(Km);  // Montgomery C_k, 1 / C_k (index 0 = 1)
  // a_i = y_i (-1)^(n-1-i) q^(-E_i) / (C_i C_(n-1-i)); E_(i+1) = E_i + i, E_0 = n(n-1)/2
  Vec a(D, 0);
  const u128 qim = to_m(qinv);
#pragma omp parallel
  {
    const int T = omp_get_num_threads(), id = omp_get_thread_num();
    const uint64_t per = (n + T - 1) / T, i0 = std::min(n, per * id), i1 = std::min(n, i0 + per);
    if (i0 < i1) {
      const u128 E0 = ((u128)i0 * (n - 1) + (u128)(n - 1 - i0) * (n - i0) / 2) % D;
      u128 qe = pow_m(qim, E0), qi = pow_m(qim, i0);  // q^-E_i, q^-i
      for (uint64_t i = i0; i < i1; ++i) {
        u128 v = mont(mont(mont(to_m(y[i]), qe), Cim[i]), Cim[n - 1 - i]);
        v = from_m(v);
        a[i] = ((n - 1 - i) & 1) && v ? P - v : v;
        qe = mont(qe, qi);
        qi = mont(qi, qim);
      }
    }
  }
  Kc[0] = 0;
  const Vec S = ref_intt(q, hadamard(ref_ntt(q, a), ref_ntt(q, Kc)));
  Vec vals(D);
  const u128 qm = to_m(q);
#pragma omp parallel
  {
    const int T = omp_get_num_threads(), id = omp_get_thread_num();
    const uint64_t per = (D + T - 1) / T, m0 = std::min(D, per * id), m1 = std::min(D, m0 + per);
    if (m0 < m1) {
      u128 qe = pow_m(qm, ((u128)m0 * (n - 1)) % D);
      const u128 step = pow_m(qm, n - 1);
      for (uint64_t m = m0; m < m1; ++m) {
        if (m < n) {
          vals[m] = y[m];
        } else {
          vals[m] = from_m(mont(mont(mont(to_m(S[m]), qe), Cm[m]), Cim[m - n]));
        }
        qe = mont(qe, step);
      }
    }
  }
  Vec c = ref_intt(q, vals);
  c.resize(n);
  return c;
}

// prod_{i < nz} (x - q^i), length nz + 1 (fast_zerofier, ntt_arithmetics.rs:66-113, below the
// domain order): doubling Z_2k(x) = Z_k(x) q^(k^2) Z_k(q^-k x), Z_(k+1) = Z_k(x) (x - q^k)
Vec geo_zerofier(u128 q, uint64_t nz) {
  if (nz == 0) return {};
  Vec Z = {1};
  uint64_t k = 0;
  for (int bit = 63 - __builtin_clzll(nz); bit >= 0; --bit) {
    if (k) {
      Vec R = pscale(Z, fpow(finv(q), k));
      pmul_const(R, fpow(q, (u128)k * k));
      Z = poly_mul_exact(Z, R);
      k *= 2;
    }
    if ((nz >> bit) & 1) {  // Z * (x - q^k)
      const u128 qk = fpow(q, k), qkm = to_m(qk);
      Vec N(Z.size() + 1, 0);
      for (size_t j = 0; j <= Z.size(); ++j) {
        const u128 lo = j ? Z[j - 1] : 0, hi = j < Z.size() ? mont(Z[j], qkm) : 0;
        N[j] = fsub(lo, hi);
      }
      Z.swap(N);
      ++k;
    }
  }
  return Z;
}

// small domains (boundary constraints): fast_zerofier / fast_interpolate_domain restated directly
Vec small_zerofier(const Vec& dom) {
  if (dom.empty()) return {};
  Vec Z = {1};
  for (u128 d : dom) {
    Vec N(Z.size() + 1, 0);
    for (size_t j = 0; j <= Z.size(); ++j) N[j] = fsub(j ? Z[j - 1] : 0, j < Z.size() ? fmul(Z[j], d) : 0);
    Z.swap(N);
  }
  return Z;
}

Vec small_interpolate(const Vec& dom, const Vec& val) {  // Lagrange; length n (n >= 1)
  const size_t n = dom.size();
  if (n == 0) return {};
  if (n == 1) return {val[0]};
  Vec out(n, 0);
  for (size_t i = 0; i < n; ++i) {
    Vec others;
    u128 den = 1;
    for (size_t j = 0; j < n; ++j)
      if (j != i) {
        others.push_back(dom[j]);
        FC_REQUIRE(dom[i] != dom[j], -5, "divide by zero");
        den = fmul(den, fsub(dom[i], dom[j]));
      }
    Vec L = small_zerofier(others);
    const u128 s = fmul(val[i], finv(den));
    for (size_t j = 0; j < L.size(); ++j) out[j] = fadd(out[j], fmul(L[j], s));
  }
  return out;
}

// Rescue-Prime transition polynomials (rescue_prime.rs:246-283) as evaluate_symbolic returns them
// for the point [x, P_s(x), P_s(omicron x)] (stark.rs:388-400): values on the coset g <w_L> of
//   sum_k MDS[i][k] P_k^alpha + first_i - (sum_k MDSinv[i][k] (P_k(omicron x) - second_k))^alpha
// and one INTT.  The vector length is 1 + alpha (T - 1): the longest monomials are prev_k^alpha
// and next_k^alpha over trace polynomials of length T (the round-constant terms have x-degree
// <= alpha (N - 1) < alpha (T - 1)).
std::vector<Vec> rescue_tpolys(const std::vector<Vec>& tp, const std::vector<Vec>& first, const std::vector<Vec>& second,
                               const Vec& mds, const Vec& mds_inv, uint64_t alpha, u128 omicron, u128 g,
                               uint64_t sym_len) {
  const size_t m = tp.size();
  const uint64_t L = (uint64_t)1 << log2_exact(sym_len);
  const u128 wL = root_of_order(std::max<uint64_t>(L, 2));
  std::vector<Vec> P(m), Nx(m), F(m), S(m);
  for (size_t k = 0; k < m; ++k) {
    P[k] = coset_eval(wL, L, g, tp[k]);
    Nx[k] = coset_eval(wL, L, fmul(g, omicron), tp[k]);
    F[k] = coset_eval(wL, L, g, first[k]);
    S[k] = coset_eval(wL, L, g, second[k]);
  }
  std::vector<Vec> out(m);
  const u128 ginv = finv(g);
  for (size_t i = 0; i < m; ++i) {
    Vec vals(L);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < (int64_t)L; ++j) {
      u128 lhs = F[i][j], acc = 0;
      for (size_t k = 0; k < m; ++k) {
        lhs = fadd(lhs, fmul(mds[i * m + k], fpow(P[k][j], alpha)));
        acc = fadd(acc, fmul(mds_inv[i * m + k], fsub(Nx[k][j], S[k][j])));
      }
      vals[j] = fsub(lhs, fpow(acc, alpha));
    }
    Vec c = pscale(ref_intt(wL, vals), ginv);
    for (uint64_t j = sym_len; j < c.size(); ++j)
      FC_REQUIRE(c[j] == 0, -6, "transition polynomial longer than its symbolic length");
    c.resize(sym_len);
    out[i] = std::move(c);
  }
  return out;
}

struct StarkArgs {
  uint64_t m, T_orig, num_randomizers, D, Nf, expansion, colinearity;
  u128 omicron, omega, g;
  uint64_t alpha;
  const Vec* mds;
  const Vec* mds_inv;
  const Vec* rc;   // 2 m N round constants
  uint64_t N;      // Rescue rounds
  const std::vector<uint64_t>* tqdb;  // transition quotient degree bounds (stark.rs:162-176)
  uint64_t tcd;                       // max_degree (stark.rs:178-196)
};

std::vector<uint8_t> stark_prove(const StarkArgs& A, const Vec& trace, uint64_t rows, const Vec& trace_rand,
                                 const Vec& rcoef, const std::vector<uint64_t>& bcyc, const std::vector<uint64_t>& breg,
                                 const Vec& bval, double* phase_s, const std::vector<uint8_t>& fs_prefix) {
  auto clk = [] { return omp_get_wtime(); };
  double t0 = clk();
  int ph = 0;
  auto mark = [&] {
    if (phase_s) phase_s[ph++] = clk() - t0;
  };
  const uint64_t m = A.m, D = A.D, Nf = A.Nf;
  const uint64_t T = rows + A.num_randomizers;  // stark.rs:285-301
  FC_REQUIRE(T <= D, -1, "randomized trace longer than the omicron domain");
  FC_REQUIRE(rcoef.size() == A.tcd + 1, -1, "randomizer polynomial must have max_degree + 1 coefficients");
  Stream ps;
  ps.fs_prefix = fs_prefix;
  // trace polynomials (stark.rs:303-324)
  std::vector<Vec> tp(m);
  for (uint64_t s = 0; s < m; ++s) {
    Vec col(T);
    for (uint64_t r = 0; r < rows; ++r) col[r] = trace[r * m + s];
    for (uint64_t r = 0; r < A.num_randomizers; ++r) col[rows + r] = trace_rand[r * m + s];
    tp[s] = geo_interpolate(A.omicron, D, col);
  }
  mark();
  // boundary quotients (stark.rs:326-362)
  std::vector<Vec> bqs(m), bzs(m);
  for (uint64_t s = 0; s < m; ++s) {
    Vec dom, val;
    for (size_t b = 0; b < bcyc.size(); ++b)
      if (breg[b] == s) {
        dom.push_back(fpow(A.omicron, bcyc[b]));
        val.push_back(bval[b]);
      }
    bzs[s] = small_zerofier(dom);
    bqs[s] = fast_coset_divide(A.omicron, D, A.g, psub(tp[s], small_interpolate(dom, val)), bzs[s]);
  }
  mark();
  // boundary-quotient codewords + commitments (stark.rs:364-386)
  std::vector<Vec> bq_cw(m);
  std::vector<Tree> bq_tree(m);
  for (uint64_t s = 0; s < m; ++s) {
    bq_cw[s] = coset_eval(A.omega, Nf, A.g, bqs[s]);
    build_tree(bq_cw[s].data(), Nf, bq_tree[s]);
    ps.push(0, reinterpret_cast<const uint8_t*>(bq_tree[s].root()), 64, false);
  }
  mark();
  // transition quotients (stark.rs:388-422)
  std::vector<Vec> first(m), second(m);
  for (uint64_t i = 0; i < m; ++i) {
    Vec c1(A.N), c2(A.N);
    for (uint64_t r = 0; r < A.N; ++r) {
      c1[r] = (*A.rc)[2 * r * m + i];
      c2[r] = (*A.rc)[2 * r * m + m + i];
    }
    first[i] = geo_interpolate(A.omicron, D, c1);
    second[i] = geo_interpolate(A.omicron, D, c2);
  }
  for (uint64_t s = 0; s < m; ++s) FC_REQUIRE(tp[s].size() == T, -1, "trace polynomial length");
  const uint64_t sym_len = 1 + A.alpha * (T - 1);
  std::vector<Vec> tpolys = rescue_tpolys(tp, first, second, *A.mds, *A.mds_inv, A.alpha, A.omicron, A.g, sym_len);
  FC_REQUIRE(A.T_orig >= 1, -1, "original trace length");
  const Vec tz = geo_zerofier(A.omicron, A.T_orig - 1);  // stark.rs:198-206
  std::vector<Vec> tqs(m);
  for (uint64_t i = 0; i < m; ++i) tqs[i] = fast_coset_divide(A.omicron, D, A.g, tpolys[i], tz);
  mark();
  // randomizer polynomial + commitment (stark.rs:424-445)
  const Vec r_cw = coset_eval(A.omega, Nf, A.g, rcoef);
  Tree r_tree;
  build_tree(r_cw.data(), Nf, r_tree);
  ps.push(0, reinterpret_cast<const uint8_t*>(r_tree.root()), 64, false);
  mark();
  // weights (stark.rs:447-450), degree check (:451-465)
  uint8_t fs[32];
  ps.fiat_shamir(fs);
  const size_t nw = 1 + 2 * tqs.size() + 2 * bqs.size();
  Vec weights(nw);
  for (size_t i = 0; i < nw; ++i) {
    std::vector<uint8_t> buf(i, 0);
    buf.insert(buf.end(), fs, fs + 32);
    weights[i] = sample_field(buf.data(), buf.size());
  }
  for (uint64_t i = 0; i < m; ++i)
    FC_REQUIRE(pdegree(tqs[i]) >= 0 && (uint64_t)pdegree(tqs[i]) == (*A.tqdb)[i], -7,
               "transition quotient degrees do not match with expectation");
  // terms + combination (stark.rs:467-512)
  std::vector<Vec> terms;
  terms.push_back(rcoef);
  auto xpow = [](uint64_t e) {  // polynomial.rs:328-356: [0,1]^e, length e + 1
    Vec v(e + 1, 0);
    v[e] = 1;
    return v;
  };
  for (uint64_t i = 0; i < m; ++i) {
    terms.push_back(tqs[i]);
    terms.push_back(fast_multiply(A.omicron, D, xpow(A.tcd - (*A.tqdb)[i]), tqs[i]));
  }
  for (uint64_t s = 0; s < m; ++s) {
    const int64_t dz = pdegree(bzs[s]);
    FC_REQUIRE(dz >= 0, -1, "Couldnt get degree of boundary zerofier");
    const uint64_t bqdb = T - 1 - (uint64_t)dz;
    terms.push_back(bqs[s]);
    terms.push_back(fast_multiply(A.omicron, D, xpow(A.tcd - bqdb), bqs[s]));
  }
  Vec comb;
  bool have = false;
  for (size_t t = 0; t < terms.size(); ++t) {
    Vec wt = terms[t];
    if (!wt.empty()) pmul_const(wt, weights[t]);  // p_mul([w], t): length len(t)
    comb = have ? padd(comb, wt) : wt;
    have = true;
  }
  const Vec comb_cw = coset_eval(A.omega, Nf, A.g, comb);
  mark();
  // FRI (stark.rs:514-522)
  std::vector<uint64_t> top;
  fri_prove(ps, A.g, A.omega, Vec(comb_cw), A.expansion, A.colinearity, top);
  mark();
  // openings (stark.rs:524-560)
  std::vector<uint64_t> dup = top;
  for (uint64_t i : top) dup.push_back((i + A.expansion) % Nf);
  std::vector<uint64_t> quad = dup;
  for (uint64_t i : dup) quad.push_back((i + Nf / 2) % Nf);
  std::sort(quad.begin(), quad.end());
  auto open = [&](const Vec& cw, const Tree& t) {
    for (uint64_t i : quad) {
      uint8_t v[16];
      put_be128(v, cw[i]);
      ps.push(4, v, 16, true);
      std::vector<uint8_t> pl = path_payload(t, i);
      ps.push(2, pl.data(), pl.size(), false);
    }
  };
  for (uint64_t s = 0; s < m; ++s) open(bq_cw[s], bq_tree[s]);
  open(r_cw, r_tree);
  mark();
  return ps.digest();
}

}  // namespace

// ======================================================================== C ABI

extern "C" {

int fc_threads(void) { return omp_get_max_threads(); }
void fc_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

void fc_mul(const uint64_t* a, const uint64_t* b, uint64_t* out) { st(out, fmul(ld(a), ld(b))); }
void fc_inv(const uint64_t* a, uint64_t* out) { st(out, finv(ld(a))); }

// ntt.rs:7-49: n = next_pow2(n_in) (zero padding), out has n elements
int fc_ntt(const uint64_t* root, const uint64_t* in, uint64_t n_in, uint64_t* out) {
  if (n_in == 0) return -1;  // ntt.rs:11 asserts a non-empty input
  const int logn = log2_exact(n_in);
  const uint64_t n = (uint64_t)1 << logn;
  std::vector<u128> a(n), pw(std::max<uint64_t>(n / 2, 1));
  powers_m(ld(root), std::max<uint64_t>(n / 2, 1), pw.data());
  bitrev_load(in, n_in, logn, a.data(), nullptr);
  dit(a.data(), logn, pw.data());
  store_all(a.data(), n, out, 0, false);
  return 0;
}

// ntt.rs:51-68: ntt(root^-1) * n^-1; fewer than 2 elements are returned unchanged
int fc_intt(const uint64_t* root, const uint64_t* in, uint64_t n_in, uint64_t* out) {
  if (n_in < 2) {
    memcpy(out, in, 16 * n_in);
    return 0;
  }
  const int logn = log2_exact(n_in);
  const uint64_t n = (uint64_t)1 << logn;
  std::vector<u128> a(n), pw(n / 2);
  powers_m(finv(ld(root)), n / 2, pw.data());
  bitrev_load(in, n_in, logn, a.data(), nullptr);
  dit(a.data(), logn, pw.data());
  store_all(a.data(), n, out, to_m(finv((u128)n)), true);
  return 0;
}

// ntt_arithmetics.rs:161-170: scale by offset^i, zero-pad to root_order, ntt(generator)
int fc_coset_evaluate(const uint64_t* gen, uint64_t root_order, const uint64_t* offset, const uint64_t* coeffs,
                      uint64_t d, uint64_t* out) {
  if (d > root_order || root_order == 0 || (root_order & (root_order - 1))) return -1;
  const int logn = log2_exact(root_order);
  const uint64_t n = root_order;
  std::vector<u128> a(n), pw(std::max<uint64_t>(n / 2, 1)), sc(std::max<uint64_t>(d, 1));
  powers_m(ld(gen), std::max<uint64_t>(n / 2, 1), pw.data());
  powers_m(ld(offset), std::max<uint64_t>(d, 1), sc.data());
  bitrev_load(coeffs, d, logn, a.data(), sc.data());
  dit(a.data(), logn, pw.data());
  store_all(a.data(), n, out, 0, false);
  return 0;
}

void fc_blake2b512(const uint8_t* in, size_t len, uint8_t* out) { blake2b512(in, len, out); }
void fc_shake256(const uint8_t* in, size_t len, uint8_t* out, size_t outlen) { shake256(in, len, out, outlen); }

// merkle_root.rs:21-32
int fc_merkle_commit(const uint64_t* leaves, uint64_t n, uint8_t* root) {
  if (n == 0 || (n & (n - 1))) return -1;
  std::vector<u128> v(n);
  for (uint64_t i = 0; i < n; ++i) v[i] = ld(leaves + 2 * i);
  Tree t;
  build_tree(v.data(), n, t);
  memcpy(root, t.root(), 64);
  return 0;
}

// FRI::prove (fri.rs:210-248) on a proof stream holding `prefix` (a serialized stream:
// 16-byte header + objects).  Writes the serialized stream after the call into a malloc'd
// buffer (*out, *out_len; free with fc_free) and the c top-level indices into top.
// Returns the number of FRI rounds, or < 0 on error.
long fc_fri_prove(const uint64_t* offset, const uint64_t* omega, const uint64_t* codeword, uint64_t n,
                  uint64_t expansion, uint64_t colinearity, const uint8_t* prefix, size_t prefix_len, uint8_t** out,
                  size_t* out_len, uint64_t* top) {
  if (prefix_len < 16 || n == 0 || (n & (n - 1))) return -1;
  Stream ps;
  ps.body.assign(prefix + 16, prefix + prefix_len);
  for (int b = 0; b < 16; ++b) ps.field = ps.field || prefix[b] != 0;
  std::vector<u128> cw(n);
  for (uint64_t i = 0; i < n; ++i) cw[i] = ld(codeword + 2 * i);
  std::vector<uint64_t> tp;
  uint64_t rounds;
  try {
    rounds = fri_prove(ps, ld(offset), ld(omega), std::move(cw), expansion, colinearity, tp);
  } catch (const CheckError& e) {
    g_err = e.msg;
    return e.code;
  }
  for (uint64_t s = 0; s < colinearity; ++s) top[s] = tp[s];
  const std::vector<uint8_t> d = ps.digest();
  *out = static_cast<uint8_t*>(malloc(d.size()));
  if (!*out) return -4;
  memcpy(*out, d.data(), d.size());
  *out_len = d.size();
  return (long)rounds;
}

const char* fc_last_error(void) { return g_err.c_str(); }

// Stark::prove (stark.rs:276-562) with a Rescue-Prime AIR (rescue_prime.rs:246-283) and explicit
// randomness (the two thread_rng draws), every argument as the reference's Stark / RescuePrime
// hold it.  Elements are (lo, hi) u64 pairs; the serialized proof (stark.rs:562) goes to a malloc'd
// buffer (*out, *out_len; free with fc_free).  phase_s (optional, 8 doubles): cumulative wall
// seconds at the end of each phase.  fs_prefix (fs_prefix_len bytes, may be empty): the bytes a
// SignatureProofStream puts before the digest in every Fiat-Shamir draw
// (rescue_prime/proof_stream.rs:22-39).  Returns 0, or < 0 with fc_last_error().
long fc_stark_prove_rescue(uint64_t m, uint64_t original_trace_length, uint64_t num_randomizers, uint64_t D,
                           uint64_t Nf, uint64_t expansion, uint64_t colinearity, const uint64_t* omicron,
                           const uint64_t* omega, const uint64_t* generator, uint64_t alpha, const uint64_t* mds,
                           const uint64_t* mds_inv, const uint64_t* round_constants, uint64_t rounds,
                           const uint64_t* tqdb, uint64_t tcd, const uint64_t* trace, uint64_t trace_rows,
                           const uint64_t* trace_rand, const uint64_t* rcoef, uint64_t nrc, const uint64_t* bcyc,
                           const uint64_t* breg, const uint64_t* bval, uint64_t nb, uint8_t** out, size_t* out_len,
                           double* phase_s, const uint8_t* fs_prefix, size_t fs_prefix_len) {
  try {
    auto vec = [](const uint64_t* p, uint64_t n) {
      Vec v(n);
      for (uint64_t i = 0; i < n; ++i) {
        v[i] = ld(p + 2 * i);
        FC_REQUIRE(v[i] < P, -1, "non-canonical element");
      }
      return v;
    };
    const Vec vmds = vec(mds, m * m), vmdsi = vec(mds_inv, m * m), vrc = vec(round_constants, 2 * m * rounds);
    const std::vector<uint64_t> vtq(tqdb, tqdb + m);
    StarkArgs A{m, original_trace_length, num_randomizers, D, Nf, expansion, colinearity, ld(omicron), ld(omega),
                ld(generator), alpha, &vmds, &vmdsi, &vrc, rounds, &vtq, tcd};
    std::vector<uint64_t> bc(bcyc, bcyc + nb), br(breg, breg + nb);
    const std::vector<uint8_t> d = stark_prove(A, vec(trace, trace_rows * m), trace_rows,
                                               vec(trace_rand, num_randomizers * m), vec(rcoef, nrc), bc, br,
                                               vec(bval, nb), phase_s,
                                               std::vector<uint8_t>(fs_prefix, fs_prefix + fs_prefix_len));
    *out = static_cast<uint8_t*>(malloc(d.size()));
    if (!*out) return -4;
    memcpy(*out, d.data(), d.size());
    *out_len = d.size();
    return 0;
  } catch (const CheckError& e) {
    g_err = e.msg;
    return e.code;
  }
}

// the unique interpolant through (q^i, y_i), i < n, q of order D (checker building block)
long fc_geo_interpolate(const uint64_t* q, uint64_t D, const uint64_t* y, uint64_t n, uint64_t* out) {
  try {
    Vec v(n);
    for (uint64_t i = 0; i < n; ++i) v[i] = ld(y + 2 * i);
    const Vec c = geo_interpolate(ld(q), D, v);
    for (uint64_t i = 0; i < c.size(); ++i) st(out + 2 * i, c[i]);
    return (long)c.size();
  } catch (const CheckError& e) {
    g_err = e.msg;
    return e.code;
  }
}

// prod_{i < n} (x - q^i), n + 1 coefficients (checker building block)
long fc_geo_zerofier(const uint64_t* q, uint64_t n, uint64_t* out) {
  try {
    const Vec c = geo_zerofier(ld(q), n);
    for (uint64_t i = 0; i < c.size(); ++i) st(out + 2 * i, c[i]);
    return (long)c.size();
  } catch (const CheckError& e) {
    g_err = e.msg;
    return e.code;
  }
}

void fc_free(void* p) { free(p); }

// prod_{r < n} (x_j - q^r) for every x_j
void fc_geometric_prod(const uint64_t* q, uint64_t n, const uint64_t* xs, uint64_t nx, uint64_t* out) {
  std::vector<u128> dom(n);
  powers_m(ld(q), n, dom.data());
  for (uint64_t j = 0; j < nx; ++j) {
    const u128 x = ld(xs + 2 * j);
    u128 acc = K().R;  // Montgomery(1)
#pragma omp parallel
    {
      u128 part = K().R;
#pragma omp for schedule(static) nowait
      for (int64_t r = 0; r < (int64_t)n; ++r) part = mont(part, to_m(fsub(x, from_m(dom[r]))));
#pragma omp critical
      acc = mont(acc, part);
    }
    st(out + 2 * j, mont(acc, 1));
  }
}

// prod_{i<n} (x - d_i) on an ARBITRARY domain, coefficients (length n + 1): the exact product
// that fast_zerofier (ntt_arithmetics.rs:66-113) returns while its fast_multiply does not wrap
// (n < root_order).  Schoolbook, one root at a time, each update split over the threads: O(n^2).
void fc_poly_from_roots(const uint64_t* dom, uint64_t n, uint64_t* out) {
  std::vector<u128> c(n + 1, 0), nxt(n + 1, 0);
  c[0] = 1;
  for (uint64_t i = 0; i < n; ++i) {
    const u128 dm = to_m(ld(dom + 2 * i));
    // c * (x - d): nxt[j] = c[j-1] - d c[j], degree i -> i + 1
#pragma omp parallel for schedule(static) if (i > 4096)
    for (int64_t j = 0; j <= (int64_t)i + 1; ++j) {
      const u128 lo = j ? c[j - 1] : 0;
      const u128 hi = j <= (int64_t)i ? mont(c[j], dm) : 0;
      nxt[j] = fsub(lo, hi);
    }
    std::swap(c, nxt);
  }
  for (uint64_t j = 0; j <= n; ++j) st(out + 2 * j, c[j]);
}

// out[k] = sum_j coeffs[j] xs[k]^j (Polynomial::evaluate, polynomial.rs), Horner, points over threads
void fc_eval_points(const uint64_t* coeffs, uint64_t len, const uint64_t* xs, uint64_t m, uint64_t* out) {
  std::vector<u128> c(len);
  for (uint64_t j = 0; j < len; ++j) c[j] = ld(coeffs + 2 * j);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t k = 0; k < (int64_t)m; ++k) {
    const u128 xm = to_m(ld(xs + 2 * k));
    u128 acc = 0;
    for (uint64_t j = len; j-- > 0;) acc = fadd(mont(acc, xm), c[j]);
    st(out + 2 * k, acc);
  }
}

// Interpolant through (q^r, cols[c][r]), r < n (q of order >= n), evaluated at x by the
// barycentric formula P(x) = Z(x) sum_r v_r w_r / (x - q^r), Z(x) = prod_r (x - q^r),
// 1/w_r = prod_{i != r} (q^r - q^i) = q^(e_r) A_r B_(n-1-r), e_r = r(r-1)/2 + r(n-1-r),
// A_k = prod_{i=1..k} (q^i - 1), B_k = prod_{i=1..k} (1 - q^i).  The unique interpolant of
// degree < n, i.e. the polynomial fast_interpolate_domain returns (ntt_arithmetics.rs:172-237).
// fc_bary_create precomputes the nodes and v_r w_r once; fc_bary_eval is O(n) per point.
struct Bary {
  uint64_t n = 0, ncols = 0;
  std::vector<u128> dom;   // Montgomery(q^r)
  std::vector<u128> vw;    // [c][r]: Montgomery(v_r w_r)
  std::vector<u128> vals;  // [c][r]: canonical v_r (a node's value)
};

void* fc_bary_create(const uint64_t* q, uint64_t n, const uint64_t* cols, uint64_t ncols) {
  Bary* b = new Bary();
  b->n = n;
  b->ncols = ncols;
  b->dom.resize(n);
  const u128 qv = ld(q), one_m = K().R;
  powers_m(qv, n, b->dom.data());
  std::vector<u128> A(n), B(n), wgt(n);
  A[0] = one_m;
  B[0] = one_m;
  for (uint64_t k = 1; k < n; ++k) {
    A[k] = mont(A[k - 1], fsub(b->dom[k], one_m));
    B[k] = mont(B[k - 1], fsub(one_m, b->dom[k]));
  }
  // q^(e_r) by chunks: e_(r+1) = e_r + (n - 2 - r), i.e. q^(e_(r+1)) = q^(e_r) q^(n-2) q^-r
  const u128 qm = to_m(qv), qim = to_m(finv(qv)), step0 = n >= 2 ? pow_m(qm, n - 2) : one_m;
#pragma omp parallel
  {
    const int T = omp_get_num_threads(), id = omp_get_thread_num();
    const uint64_t per = (n + T - 1) / T, r0 = std::min(n, per * id), r1 = std::min(n, r0 + per);
    if (r0 < r1) {
      const u128 rr = r0;
      const u128 e = (rr * (rr ? rr - 1 : 0) / 2 + rr * (u128)(n - 1 - r0)) % (P - 1);
      u128 qe = pow_m(qm, e), qir = pow_m(qim, r0);  // q^(e_r0), q^-r0
      for (uint64_t r = r0; r < r1; ++r) {
        wgt[r] = mont(mont(qe, A[r]), B[n - 1 - r]);  // Montgomery(1/w_r)
        qe = mont(mont(qe, step0), qir);
        qir = mont(qir, qim);
      }
    }
  }
  // batch inversion: wgt[r] = Montgomery(w_r)
  {
    std::vector<u128> pre(n);
    u128 acc = one_m;
    for (uint64_t r = 0; r < n; ++r) {
      pre[r] = acc;
      acc = mont(acc, wgt[r]);
    }
    u128 inv = to_m(finv(from_m(acc)));
    for (uint64_t r = n; r-- > 0;) {
      const u128 wr = mont(inv, pre[r]);
      inv = mont(inv, wgt[r]);
      wgt[r] = wr;
    }
  }
  b->vw.resize(n * ncols);
  b->vals.resize(n * ncols);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)(n * ncols); ++i) {
    const u128 v = ld(cols + 2 * i);
    b->vals[i] = v;
    b->vw[i] = mont(v, mont(wgt[i % n], K().R2));  // v * w (canonical) -> Montgomery(v w) via R2
  }
  return b;
}

void fc_bary_eval(const void* h, const uint64_t* xp, uint64_t* out) {
  const Bary* b = static_cast<const Bary*>(h);
  const uint64_t n = b->n, ncols = b->ncols;
  const u128 x = ld(xp), one_m = K().R;
  const int T = omp_get_max_threads();
  std::vector<u128> sums((size_t)T * ncols, 0), zpart(T, one_m);
  std::vector<int64_t> hit(T, -1);
#pragma omp parallel num_threads(T)
  {
    const int id = omp_get_thread_num(), nt = omp_get_num_threads();
    const uint64_t per = (n + nt - 1) / nt, r0 = std::min(n, per * id), r1 = std::min(n, r0 + per);
    std::vector<u128> diff(r1 - r0), pre(r1 - r0);
    u128 acc = one_m;
    for (uint64_t r = r0; r < r1; ++r) {
      const u128 dv = to_m(fsub(x, from_m(b->dom[r])));
      if (dv == 0) hit[id] = (int64_t)r;
      diff[r - r0] = dv;
      pre[r - r0] = acc;
      if (dv) acc = mont(acc, dv);
    }
    zpart[id] = acc;
    u128 inv = to_m(finv(from_m(acc)));
    for (uint64_t r = r1; r-- > r0;) {
      const u128 dv = diff[r - r0];
      if (!dv) continue;
      const u128 iv = mont(inv, pre[r - r0]);  // Montgomery(1/(x - q^r))
      inv = mont(inv, dv);
      for (uint64_t c = 0; c < ncols; ++c)      // canonical v_r w_r / (x - q^r)
        sums[(size_t)id * ncols + c] = fadd(sums[(size_t)id * ncols + c], from_m(mont(b->vw[c * n + r], iv)));
    }
  }
  int64_t hnode = -1;
  for (int t = 0; t < T; ++t)
    if (hit[t] >= 0) hnode = hit[t];
  u128 z = one_m;
  for (int t = 0; t < T; ++t) z = mont(z, zpart[t]);
  for (uint64_t c = 0; c < ncols; ++c) {
    u128 v;
    if (hnode >= 0) {
      v = b->vals[c * n + (uint64_t)hnode];  // x is a node: the interpolant takes its value
    } else {
      u128 s = 0;
      for (int t = 0; t < T; ++t) s = fadd(s, sums[(size_t)t * ncols + c]);
      v = mont(s, z);  // canonical s * Montgomery(Z) -> canonical s Z
    }
    st(out + 2 * c, v);
  }
}

void fc_bary_free(void* h) { delete static_cast<Bary*>(h); }

void fc_geometric_bary(const uint64_t* q, uint64_t n, const uint64_t* cols, uint64_t ncols, const uint64_t* xs,
                       uint64_t nx, uint64_t* out) {
  void* h = fc_bary_create(q, n, cols, ncols);
  for (uint64_t j = 0; j < nx; ++j) fc_bary_eval(h, xs + 2 * j, out + 2 * j * ncols);
  fc_bary_free(h);
}

}  // extern "C"
