/*
 * ref_cpu.c -- reference-faithful C restatement of the LDE / NTT / Merkle /
 * FRI-commit path of SpekalsG3/zk-stark-tutor (Rust), used as the CPU
 * baseline ("port") and as a second, independent parity checker.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ and bench.py's cpu_baseline leg
 * through oracle/ref_cpu.py; never linked into libstarkgpu.
 *
 * It keeps the reference's ALGORITHMS, not just its results, so its timing is
 * a fair single-thread stand-in for the Rust code (which cannot be built
 * here: no cargo/rustc, crates not vendored):
 *   field/field.rs:101-131   add/sub via 3-way compare, bit-serial mul_mod
 *   field/field.rs:160-169   inverse through utils/xgcd.rs:22-48 u_xgcd
 *   field/field_element.rs:108-143  pow by square-and-multiply over bitlen(e)
 *   utils/bit_reverse_copy.rs:3-34, fft/ntt.rs:7-68  bit_reverse_copy + powtable + DIT
 *   field/polynomial.rs:109-121  scale with one pow per coefficient
 *   fft/ntt_arithmetics.rs:161-170  fast_coset_evaluate
 *   merkle_root.rs:7-32  decimal leaves, recursive commit_
 *   fri.rs:115-172  commit: root, SHAKE256 transcript, alpha, per-element
 *                   omega^i pow + division in the fold
 *   stark/proof_stream_enum.rs:161-190 + proof_stream.rs:31-41  transcript bytes
 * BLAKE2b (RFC 7693) and Keccak/SHAKE256 (FIPS 202) are written out below.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef __int128 i128;

static const u128 P = ((u128)0xCB8 << 116) | 1; /* 1 + 407 * 2^119 */

/* ---------------------------------------------------------------- field */
static u128 sub_mod(u128 a, u128 b) {
  if (a > b) return a - b;
  if (a == b) return 0;
  return P - b + a;
}
static u128 add_mod(u128 a, u128 b) {
  if (b == 0) return a;
  return sub_mod(a, P - b);
}
static u128 mul_mod(u128 a, u128 b) {
  u128 res = 0;
  while (b > 0) {
    if (b & 1) res = add_mod(res, a);
    a = add_mod(a, a);
    b >>= 1;
  }
  return res;
}
static void u_xgcd(u128 a, u128 b, i128* x, i128* y, u128* g) {
  i128 x1 = 1, y1 = 0, x0 = 0, y0 = 1;
  u128 r0 = a, r1 = b, q = 0;
  while (r1 != 0) {
    i128 x2 = x0 - (i128)q * x1, y2 = y0 - (i128)q * y1;
    x0 = x1; y0 = y1; x1 = x2; y1 = y2;
    q = r0 / r1;
    u128 t = r0 - q * r1;
    r0 = r1; r1 = t;
  }
  *x = x1; *y = y1; *g = r0;
}
static u128 inv_mod(u128 a) {
  i128 x, y; u128 g;
  u_xgcd(a, P, &x, &y, &g);
  if (x > 0) return (u128)x;
  if (x == 0) return 0;
  return sub_mod(P, (u128)(-x));
}
static u128 pow_mod(u128 a, u128 e) {
  u128 acc = 1;
  int top = 0;
  for (int i = 127; i >= 0; --i) if ((e >> i) & 1) { top = i; break; }
  for (int i = top; i >= 0; --i) {
    acc = mul_mod(acc, acc);
    if ((e >> i) & 1) acc = mul_mod(acc, a);
  }
  return acc;
}
static u128 div_mod(u128 a, u128 b) { return mul_mod(a, inv_mod(b)); }

/* ---------------------------------------------------------------- transforms */
static size_t next_pow2(size_t n) { size_t r = 1; while (r < n) r <<= 1; return r; }

/* out has next_pow2(n) entries */
static void bit_reverse_copy(const u128* in, size_t n_in, u128* out) {
  size_t n = next_pow2(n_in);
  if (n_in < 2) { for (size_t i = 0; i < n_in; ++i) out[i] = in[i]; return; }
  int bits = 0; while (((size_t)1 << bits) < n) ++bits;
  for (size_t k = 0; k < n; ++k) {
    size_t r = 0;
    for (int i = 0; i < bits; ++i) r |= ((k >> (bits - 1 - i)) & 1) << i;
    out[r] = k < n_in ? in[k] : 0;
  }
}

void ora_ntt(const uint64_t* root2, const uint64_t* in, size_t n_in, uint64_t* out) {
  u128 root = ((u128)root2[1] << 64) | root2[0];
  size_t n = next_pow2(n_in);
  u128* x = (u128*)malloc(sizeof(u128) * n);
  u128* inp = (u128*)malloc(sizeof(u128) * (n_in ? n_in : 1));
  for (size_t i = 0; i < n_in; ++i) inp[i] = ((u128)in[2 * i + 1] << 64) | in[2 * i];
  bit_reverse_copy(inp, n_in, x);
  size_t half_n = n / 2;
  u128* pw = (u128*)malloc(sizeof(u128) * (half_n ? half_n : 1));
  u128 t = 1;
  for (size_t i = 0; i < half_n; ++i) { pw[i] = t; t = mul_mod(t, root); }
  for (size_t size = 2; size <= n; size <<= 1) {
    size_t half = size / 2, step = n / size;
    for (size_t i = 0; i < n; i += size) {
      size_t k = 0;
      for (size_t j = i; j < i + half; ++j) {
        u128 e = x[j], o = mul_mod(x[j + half], pw[k]);
        x[j] = add_mod(e, o);
        x[j + half] = sub_mod(e, o);
        k += step;
      }
    }
  }
  for (size_t i = 0; i < n; ++i) { out[2 * i] = (uint64_t)x[i]; out[2 * i + 1] = (uint64_t)(x[i] >> 64); }
  free(x); free(inp); free(pw);
}

void ora_intt(const uint64_t* root2, const uint64_t* in, size_t n_in, uint64_t* out) {
  if (n_in < 2) { memcpy(out, in, 16 * n_in); return; }
  u128 root = ((u128)root2[1] << 64) | root2[0];
  u128 rinv = inv_mod(root);
  uint64_t r2[2] = {(uint64_t)rinv, (uint64_t)(rinv >> 64)};
  size_t n = next_pow2(n_in);
  ora_ntt(r2, in, n_in, out);
  u128 ninv = inv_mod((u128)n);
  for (size_t i = 0; i < n; ++i) {
    u128 v = ((u128)out[2 * i + 1] << 64) | out[2 * i];
    v = mul_mod(ninv, v);
    out[2 * i] = (uint64_t)v; out[2 * i + 1] = (uint64_t)(v >> 64);
  }
}

/* out has next_pow2(root_order) entries; returns -1 if d > root_order (the reference panics) */
int ora_coset_evaluate(const uint64_t* gen2, uint64_t root_order, const uint64_t* off2, const uint64_t* coeffs,
                       size_t d, uint64_t* out) {
  if (d > root_order) return -1;
  u128 off = ((u128)off2[1] << 64) | off2[0];
  uint64_t* c = (uint64_t*)calloc(2 * (root_order ? root_order : 1), 8);
  for (size_t i = 0; i < d; ++i) {
    u128 v = ((u128)coeffs[2 * i + 1] << 64) | coeffs[2 * i];
    v = mul_mod(pow_mod(off, i), v); /* polynomial.rs:114-116: pow per coefficient */
    c[2 * i] = (uint64_t)v; c[2 * i + 1] = (uint64_t)(v >> 64);
  }
  ora_ntt(gen2, c, root_order, out);
  free(c);
  return 0;
}

/* ---------------------------------------------------------------- BLAKE2b-512 */
static const uint64_t B2B_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const uint8_t SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
#define ROTR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
static void b2b_compress(uint64_t h[8], const uint8_t* blk, uint64_t t, int last) {
  uint64_t v[16], m[16];
  for (int i = 0; i < 16; ++i) {
    uint64_t w = 0;
    for (int b = 7; b >= 0; --b) w = (w << 8) | blk[8 * i + b];
    m[i] = w;
  }
  for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = B2B_IV[i]; }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = SIGMA[r];
#define G(a, b, c, d, x, y)                                    \
  v[a] = v[a] + v[b] + (x); v[d] = ROTR64(v[d] ^ v[a], 32);    \
  v[c] = v[c] + v[d]; v[b] = ROTR64(v[b] ^ v[c], 24);          \
  v[a] = v[a] + v[b] + (y); v[d] = ROTR64(v[d] ^ v[a], 16);    \
  v[c] = v[c] + v[d]; v[b] = ROTR64(v[b] ^ v[c], 63);
    G(0, 4, 8, 12, m[s[0]], m[s[1]]) G(1, 5, 9, 13, m[s[2]], m[s[3]])
    G(2, 6, 10, 14, m[s[4]], m[s[5]]) G(3, 7, 11, 15, m[s[6]], m[s[7]])
    G(0, 5, 10, 15, m[s[8]], m[s[9]]) G(1, 6, 11, 12, m[s[10]], m[s[11]])
    G(2, 7, 8, 13, m[s[12]], m[s[13]]) G(3, 4, 9, 14, m[s[14]], m[s[15]])
#undef G
  }
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}
void ora_blake2b512(const uint8_t* in, size_t len, uint8_t out[64]) {
  uint64_t h[8];
  uint8_t blk[128];
  uint64_t t = 0;
  for (int i = 0; i < 8; ++i) h[i] = B2B_IV[i];
  h[0] ^= 0x01010040ULL;
  while (len > 128) { t += 128; b2b_compress(h, in, t, 0); in += 128; len -= 128; }
  memset(blk, 0, 128);
  memcpy(blk, in, len);
  t += len;
  b2b_compress(h, blk, t, 1);
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(h[i] >> (8 * b));
}

/* ---------------------------------------------------------------- Merkle */
static int u128_to_dec(u128 v, char* buf) { /* field_element.rs:46-50 (to_string) */
  char tmp[48];
  int n = 0;
  if (v == 0) { buf[0] = '0'; return 1; }
  while (v) { tmp[n++] = (char)('0' + (int)(v % 10)); v /= 10; }
  for (int i = 0; i < n; ++i) buf[i] = tmp[n - 1 - i];
  return n;
}
static void commit_(const uint8_t* leafs, size_t len, uint8_t out[64]) { /* merkle_root.rs:7-19 */
  if (len == 1) { memcpy(out, leafs, 64); return; }
  uint8_t cat[128];
  commit_(leafs, len / 2, cat);
  commit_(leafs + 64 * (len / 2), len / 2, cat + 64);
  ora_blake2b512(cat, 128, out);
}
int ora_merkle_commit(const uint64_t* leaves, size_t n, uint8_t root[64]) {
  if (n == 0 || (n & (n - 1))) return -1;
  uint8_t* d = (uint8_t*)malloc(64 * n);
  char buf[48];
  for (size_t i = 0; i < n; ++i) {
    u128 v = ((u128)leaves[2 * i + 1] << 64) | leaves[2 * i];
    int l = u128_to_dec(v, buf);
    ora_blake2b512((const uint8_t*)buf, (size_t)l, d + 64 * i);
  }
  commit_(d, n, root);
  free(d);
  return 0;
}

/* merkle_root.rs:34-66: open re-hashes every leaf and recomputes each sibling
 * subtree with commit_ on every call (O(n) per opening, as in the reference). */
static void open_(size_t index, const uint8_t* leafs, size_t len, uint8_t* path, size_t* plen) {
  if (len == 2) {
    memcpy(path + 64 * (*plen), leafs + 64 * (1 - index), 64);
    (*plen)++;
  } else if (index < len / 2) {
    open_(index, leafs, len / 2, path, plen);
    commit_(leafs + 64 * (len / 2), len / 2, path + 64 * (*plen));
    (*plen)++;
  } else {
    open_(index - len / 2, leafs + 64 * (len / 2), len / 2, path, plen);
    commit_(leafs, len / 2, path + 64 * (*plen));
    (*plen)++;
  }
}
long ora_merkle_open(size_t index, const uint64_t* leaves, size_t n, uint8_t* path) {
  if (n < 2 || (n & (n - 1)) || index >= n) return -1;
  uint8_t* d = (uint8_t*)malloc(64 * n);
  char buf[48];
  for (size_t i = 0; i < n; ++i) {
    u128 v = ((u128)leaves[2 * i + 1] << 64) | leaves[2 * i];
    int l = u128_to_dec(v, buf);
    ora_blake2b512((const uint8_t*)buf, (size_t)l, d + 64 * i);
  }
  size_t plen = 0;
  open_(index, d, n, path, &plen);
  free(d);
  return (long)plen;
}

/* ---------------------------------------------------------------- SHAKE256 */
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int ROTC[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static uint64_t rotl(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }
static void keccakf(uint64_t a[25]) {
  for (int r = 0; r < 24; ++r) {
    uint64_t c[5], d[5], b[25];
    for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) a[i] ^= d[i % 5];
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(a[x + 5 * y], ROTC[x + 5 * y]);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) a[x + 5 * y] = b[x + 5 * y] ^ ((~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= RC[r];
  }
}
void ora_shake256(const uint8_t* in, size_t len, uint8_t* out, size_t outlen) {
  uint64_t st[25];
  uint8_t* sb = (uint8_t*)st;
  memset(st, 0, sizeof(st));
  while (len >= 136) { for (int i = 0; i < 136; ++i) sb[i] ^= in[i]; keccakf(st); in += 136; len -= 136; }
  for (size_t i = 0; i < len; ++i) sb[i] ^= in[i];
  sb[len] ^= 0x1F;
  sb[135] ^= 0x80;
  keccakf(st);
  while (outlen) { size_t k = outlen < 136 ? outlen : 136; memcpy(out, sb, k); out += k; outlen -= k; if (outlen) keccakf(st); }
}

/* ---------------------------------------------------------------- FRI commit */
/*
 * fri.rs:115-172 with the transcript held as serialized bytes (prefix =
 * stream bytes before the call, e.g. earlier Roots).  Writes the final
 * serialized stream into stream_out (cap bytes) and returns its length, or
 * -1 on error.  roots_out receives num_rounds x 64 bytes.
 */
long ora_fri_commit(const uint64_t* off2, const uint64_t* omega2, const uint64_t* codeword, size_t n,
                    size_t expansion, size_t colinearity, const uint8_t* prefix, size_t prefix_len,
                    uint8_t* stream_out, size_t cap, uint8_t* roots_out, uint64_t* cw_out) {
  size_t rounds = 0, len = n;
  while (len > expansion && len > 4 * colinearity) { len /= 2; ++rounds; }
  if (rounds == 0) return -1;
  if (prefix_len < 16 || prefix_len > cap) return -1;
  u128 omega = ((u128)omega2[1] << 64) | omega2[0];
  u128 offset = ((u128)off2[1] << 64) | off2[0];
  u128 two_inv = inv_mod(2);
  size_t slen = prefix_len;
  memcpy(stream_out, prefix, prefix_len);
  u128* cw = (u128*)malloc(sizeof(u128) * n);
  uint64_t* tmp = (uint64_t*)malloc(16 * n);
  for (size_t i = 0; i < n; ++i) cw[i] = ((u128)codeword[2 * i + 1] << 64) | codeword[2 * i];
  len = n;
  for (size_t r = 0; r < rounds; ++r) {
    if (pow_mod(omega, len - 1) != inv_mod(omega)) { slen = (size_t)-1; break; }
    for (size_t i = 0; i < len; ++i) { tmp[2 * i] = (uint64_t)cw[i]; tmp[2 * i + 1] = (uint64_t)(cw[i] >> 64); }
    if (cw_out) { memcpy(cw_out, tmp, 16 * len); cw_out += 2 * len; } /* codewords[r] (fri.rs:148) */
    uint8_t root[64];
    ora_merkle_commit(tmp, len, root);
    memcpy(roots_out + 64 * r, root, 64);
    if (slen + 73 > cap) { slen = (size_t)-1; break; }
    stream_out[slen] = 0; /* Root */
    for (int b = 0; b < 8; ++b) stream_out[slen + 1 + b] = (uint8_t)(64ULL >> (8 * (7 - b)));
    memcpy(stream_out + slen + 9, root, 64);
    slen += 73;
    if (r == rounds - 1) break;
    uint8_t chal[32];
    ora_shake256(stream_out, slen, chal, 32);
    u128 alpha = 0;
    for (int b = 0; b < 32; ++b) alpha = (alpha << 8) ^ chal[b];
    alpha %= P;
    size_t half = len / 2;
    for (size_t i = 0; i < half; ++i) { /* fri.rs:152-158 */
      u128 abo = div_mod(alpha, mul_mod(offset, pow_mod(omega, i)));
      u128 first = mul_mod(add_mod(1, abo), cw[i]);
      u128 second = mul_mod(sub_mod(1, abo), cw[half + i]);
      cw[i] = mul_mod(two_inv, add_mod(first, second));
    }
    omega = pow_mod(omega, 2);
    offset = pow_mod(offset, 2);
    len = half;
  }
  if (slen != (size_t)-1) {
    /* last codeword: field header becomes p (proof_stream_enum.rs:171-188) */
    if (slen + 9 + 16 * len > cap) { slen = (size_t)-1; }
    else {
      stream_out[slen] = 1;
      uint64_t pl = 16 * len;
      for (int b = 0; b < 8; ++b) stream_out[slen + 1 + b] = (uint8_t)(pl >> (8 * (7 - b)));
      for (size_t i = 0; i < len; ++i)
        for (int b = 0; b < 16; ++b) stream_out[slen + 9 + 16 * i + b] = (uint8_t)(cw[i] >> (8 * (15 - b)));
      slen += 9 + 16 * len;
      if (len > 0)
        for (int b = 0; b < 16; ++b) stream_out[b] = (uint8_t)(P >> (8 * (15 - b)));
    }
  }
  free(cw); free(tmp);
  return slen == (size_t)-1 ? -1 : (long)slen;
}
