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
    const std::vector<uint8_t> d = digest();
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

}  // namespace

// ======================================================================== C ABI

extern "C" {

int fc_threads(void) { return omp_get_max_threads(); }

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
  uint64_t rounds = 0;
  for (uint64_t len = n; len > expansion && len > 4 * colinearity; len /= 2) ++rounds;  // fri.rs:40-50
  if (rounds < 2) return -1;
  Stream ps;
  ps.body.assign(prefix + 16, prefix + prefix_len);
  for (int b = 0; b < 16; ++b) ps.field = ps.field || prefix[b] != 0;
  u128 w = ld(omega), o = ld(offset);
  std::vector<std::vector<u128>> cws(rounds);
  std::vector<Tree> trees(rounds);
  cws[0].resize(n);
  for (uint64_t i = 0; i < n; ++i) cws[0][i] = ld(codeword + 2 * i);
  const u128 inv2m = to_m(finv(2));
  // commit (fri.rs:115-172)
  for (uint64_t r = 0; r < rounds; ++r) {
    const uint64_t len = cws[r].size();
    if (fpow(w, len - 1) != finv(w)) return -2;  // fri.rs:133 omega of order len
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
  // sample_indices (fri.rs:88-113) over len(codewords[1]) reduced by len(codewords[-1])
  uint8_t seed[32];
  ps.fiat_shamir(seed);
  const uint64_t size = cws[1].size(), reduced = cws[rounds - 1].size();
  if (colinearity > 2 * reduced || colinearity > reduced) return -3;
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
  for (uint64_t s = 0; s < colinearity; ++s) top[s] = idx[s];
  // query (fri.rs:174-208) per round
  std::vector<uint64_t> cur = idx;
  auto path = [&](const Tree& t, uint64_t i) {
    const int lg = log2_exact(t.n);
    std::vector<uint8_t> pl(72 * lg);
    for (int k = 0; k < lg; ++k) {
      uint8_t* q = &pl[72 * k];
      memset(q, 0, 8);
      q[7] = 64;
      memcpy(q + 8, t.level(k) + 8 * ((i >> k) ^ 1), 64);
    }
    return pl;
  };
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
      std::vector<uint8_t> a = path(trees[r], cur[s]), b = path(trees[r], cur[s] + half), c = path(trees[r + 1], cur[s]);
      ps.push(2, a.data(), a.size(), false);
      ps.push(2, b.data(), b.size(), false);
      ps.push(2, c.data(), c.size(), false);
    }
  }
  const std::vector<uint8_t> d = ps.digest();
  *out = static_cast<uint8_t*>(malloc(d.size()));
  if (!*out) return -4;
  memcpy(*out, d.data(), d.size());
  *out_len = d.size();
  return (long)rounds;
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
