// gfx950 kernels for the polynomial algebra around the LDE:
// pointwise products / quotients with batched inversion, prefix products, the
// closed-form zerofier of a geometric domain, the assembly step of
// geometric-domain interpolation, pointwise AIR evaluation and the weighted
// combination of shifted polynomials.  All elementwise work is HBM-bound
// integer VALU: packed 16-byte elements, one dwordx4 per lane, grid-strided.
//
// Conventions: data arrays are canonical; tables of constants (power tables,
// weights) are Montgomery(x) = x R mod p, R = 2^128; `r2` = R^2 mod p turns a
// canonical value into Montgomery form with one product.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "dev_util.hpp"
#include <cstdlib>
#include "fe128.hpp"
#include "poly_kernels.hpp"
#include "profiler.hpp"
#include "knobs.hpp"

namespace sg {

namespace {

constexpr unsigned kBlock = 256;

__device__ __forceinline__ fe fe_one_c() { return fe_make(1, 0); }
__device__ __forceinline__ bool fe_is_zero(const fe& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }

// x^(p-2) * R for x_m = x R (Montgomery in, Montgomery out): Fermat inverse.
// p - 2 = 407 * 2^119 - 1 = (203 << 120) + (0 << 119) + (2^119 - 1): x^203, one
// squaring for the zero bit, then the 119 trailing ones as 17 windows of 7 bits
// (7 squarings and one product by x^127 each): 158 products instead of 252 for
// bitwise square-and-multiply.
__device__ __forceinline__ fe mont_inv(const fe& xm, const fe& one_m) {
  (void)one_m;
  fe x3 = mont_mul(mont_mul(xm, xm), xm);
  fe w = x3;  // x^(2^k - 1), k = 2..7
#pragma unroll
  for (int k = 3; k <= 7; ++k) w = mont_mul(mont_mul(w, w), xm);
  // x^203: 203 = 0b11001011, from x^3 = 0b11
  fe acc = mont_mul(x3, x3);                  // x^6
  acc = mont_mul(acc, acc);                   // x^12
  acc = mont_mul(mont_mul(acc, acc), xm);     // x^25
  acc = mont_mul(acc, acc);                   // x^50
  acc = mont_mul(mont_mul(acc, acc), xm);     // x^101
  acc = mont_mul(mont_mul(acc, acc), xm);     // x^203
  acc = mont_mul(acc, acc);                   // x^406
#pragma unroll 1
  for (int win = 0; win < 17; ++win) {
#pragma unroll
    for (int s = 0; s < 7; ++s) acc = mont_mul(acc, acc);
    acc = mont_mul(acc, w);
  }
  return acc;
}

uint64_t grid_for(uint64_t n, uint64_t per_thread = 1) {
  uint64_t threads = (n + per_thread - 1) / per_thread;
  uint64_t b = (threads + kBlock - 1) / kBlock;
  const uint64_t cap = 256 * 64;  // enough waves for 256 CUs; grid-stride beyond
  return b < 1 ? 1 : (b > cap ? cap : b);
}

}  // namespace

// ---------------------------------------------------------------- elementwise

// out[i] = a[i] * b[i]
__global__ __launch_bounds__(kBlock) void k_ew_mul(fe* __restrict__ out, const fe* __restrict__ a,
                                                   const fe* __restrict__ b, uint64_t n, fe r2) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    st_fe(out + i, mont_mul(mont_mul(ld_fe(a + i), ld_fe(b + i)), r2));
}

// out[i] = in[i] * f^(i + start) with Montgomery(f^e) = sA[e & 4095] * sB[e >> 12]
__global__ __launch_bounds__(kBlock) void k_mul_pow2(fe* __restrict__ out, const fe* __restrict__ in, uint64_t n,
                                                     uint64_t start, const fe* __restrict__ sA,
                                                     const fe* __restrict__ sB) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t e = i + start;
    fe f = mont_mul(ld_fe(sA + (e & 4095)), ld_fe(sB + (e >> 12)));
    st_fe(out + i, mont_mul(ld_fe(in + i), f));
  }
}

// out[i] = 1 - f^(i + start)  (f^e as above)
__global__ __launch_bounds__(kBlock) void k_one_minus_pow(fe* __restrict__ out, uint64_t n, uint64_t start,
                                                          const fe* __restrict__ sA, const fe* __restrict__ sB) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t e = i + start;
    fe fm = mont_mul(ld_fe(sA + (e & 4095)), ld_fe(sB + (e >> 12)));
    st_fe(out + i, fe_sub(fe_one_c(), mont_mul(fm, fe_one_c())));
  }
}

// out[k] = (k + 1) * c[k + 1], k < n  (formal derivative)
__global__ __launch_bounds__(kBlock) void k_deriv(fe* __restrict__ out, const fe* __restrict__ c, uint64_t n, fe r2) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x)
    st_fe(out + k, mont_mul(mont_mul(ld_fe(c + k + 1), fe_make(k + 1, 0)), r2));
}

// ------------------------------------------------------- batched inversion

// out[i] = a[i] / b[i] (a == nullptr: 1 / b[i]).  Each lane owns K elements
// i = t + k S (S = all lanes, coalesced), Montgomery's trick: K - 1 prefix
// products, one Fermat inversion, 2 (K - 1) products back.  A zero divisor sets
// *zero_flag (the reference panics: "divide by zero", field_element.rs:82-90).
template <int K>
__global__ __launch_bounds__(kBlock) void k_batch_div(fe* __restrict__ out, const fe* __restrict__ a,
                                                      const fe* __restrict__ b, uint64_t n, fe r2, fe one_m,
                                                      unsigned* __restrict__ zero_flag) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe pre[K];
  fe acc = one_m;
  bool zero = false;
#pragma clang loop unroll(full)
  for (int k = 0; k < K; ++k) {
    uint64_t i = t + k * S;
    fe bm = one_m;
    if (i < n) {
      fe bv = ld_fe(b + i);
      zero |= fe_is_zero(bv);
      if (!fe_is_zero(bv)) bm = mont_mul(bv, r2);
    }
    pre[k] = acc;  // product of the elements before k
    acc = mont_mul(acc, bm);
  }
  if (zero) __hip_atomic_fetch_or(zero_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  fe inv = mont_inv(acc, one_m);  // (prod b)^-1 R
#pragma clang loop unroll(full)
  for (int k = K - 1; k >= 0; --k) {
    uint64_t i = t + k * S;
    if (i < n) {
      fe bv = ld_fe(b + i);
      fe bm = fe_is_zero(bv) ? one_m : mont_mul(bv, r2);
      fe ik = mont_mul(inv, pre[k]);  // b_k^-1 R
      inv = mont_mul(inv, bm);
      fe av = a ? ld_fe(a + i) : fe_one_c();
      st_fe(out + i, mont_mul(av, ik));  // a b^-1 (canonical)
    }
  }
}

// ------------------------------------------- product tree (arbitrary domains)
//
// fast_zerofier / fast_interpolate_domain on an arbitrary domain of n points
// (ntt_arithmetics.rs:66-113, 172-237) as a bottom-up product tree over the points
// padded to a power of two (padding leaves are the constant 1).  Level l holds one
// row of 2^(l+1) coefficients per node: Z = prod (x - d_i) over the node's points
// and, for interpolation, N = sum_i c_i Z / (x - d_i) (the reference's
// left * Z_right + right * Z_left, unrolled).  The leaf kernel builds level 3
// (8 points per lane, schoolbook); each level above multiplies pairs in the NTT
// domain of size M = 2^(l+1) and fixes the one wrapped coefficient of a full node
// (its monic x^M term lands on x^0).

constexpr int kTreeLeaf = 8;  // points per lane at the bottom level (level 3, rows of 16)

__global__ __launch_bounds__(kBlock) void k_tree_leaves(const fe* __restrict__ dom, uint64_t n, uint64_t nodes,
                                                        fe* __restrict__ Z, const fe* __restrict__ c,
                                                        fe* __restrict__ N, fe r2) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nodes) return;
  const uint64_t base = t * kTreeLeaf;
  fe z[kTreeLeaf + 1];
  z[0] = fe_one_c();
#pragma unroll
  for (int j = 1; j <= kTreeLeaf; ++j) z[j] = fe_make(0, 0);
  // z *= (x - d_i) for the real points (a prefix of the node): z'[j] = z[j-1] - d z[j]
#pragma unroll
  for (int i = 0; i < kTreeLeaf; ++i) {
    if (base + i < n) {
      const fe dm = mont_mul(ld_fe(dom + base + i), r2);
#pragma unroll
      for (int j = i + 1; j >= 1; --j) z[j] = fe_sub(z[j - 1], mont_mul(z[j], dm));
      z[0] = fe_sub(fe_make(0, 0), mont_mul(z[0], dm));
    }
  }
  fe* zr = Z + t * (2 * kTreeLeaf);
#pragma unroll
  for (int j = 0; j < 2 * kTreeLeaf; ++j) st_fe(zr + j, j <= kTreeLeaf ? z[j] : fe_make(0, 0));
  if (!c) return;
  // N = sum_i c_i q_i, q_i = Z / (x - d_i) by synthetic division (exact: d_i is a root)
  fe acc[kTreeLeaf];
#pragma unroll
  for (int j = 0; j < kTreeLeaf; ++j) acc[j] = fe_make(0, 0);
#pragma unroll
  for (int i = 0; i < kTreeLeaf; ++i) {
    if (base + i < n) {
      const fe dm = mont_mul(ld_fe(dom + base + i), r2);
      const fe cm = mont_mul(ld_fe(c + base + i), r2);
      fe q = z[kTreeLeaf];  // q[k-1] = z[k] + d q[k], from the top
#pragma unroll
      for (int k = kTreeLeaf; k >= 1; --k) {
        if (k < kTreeLeaf) q = fe_add(z[k], mont_mul(q, dm));
        acc[k - 1] = fe_add(acc[k - 1], mont_mul(q, cm));
      }
    }
  }
  fe* nr = N + t * (2 * kTreeLeaf);
#pragma unroll
  for (int j = 0; j < 2 * kTreeLeaf; ++j) st_fe(nr + j, j < kTreeLeaf ? acc[j] : fe_make(0, 0));
}

// parents p < P, j < M (NTT domain): Zp = Zl Zr; Np = Nl Zr + Nr Zl (N optional)
__global__ __launch_bounds__(kBlock) void k_tree_combine(const fe* __restrict__ Zh, const fe* __restrict__ Nh,
                                                         uint64_t P, int logM, fe* __restrict__ Zp,
                                                         fe* __restrict__ Np, fe r2) {
  const uint64_t total = P << logM;
  const uint64_t M = (uint64_t)1 << logM;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t p = i >> logM, j = i & (M - 1);
    const uint64_t l = (2 * p) * M + j, r = l + M;
    const fe zl = ld_fe(Zh + l), zr = ld_fe(Zh + r);
    st_fe(Zp + i, mont_mul(mont_mul(zl, zr), r2));
    if (Nh) st_fe(Np + i, mont_mul(fe_add(mont_mul(ld_fe(Nh + l), zr), mont_mul(ld_fe(Nh + r), zl)), r2));
  }
}

// rows of M coefficients (mod x^M - 1) -> rows of 2M; a full node (all M of its leaf
// positions are real points, p < full) is monic of degree M: move its wrapped 1 from x^0 to x^M
__global__ __launch_bounds__(kBlock) void k_tree_fix(const fe* __restrict__ in, uint64_t P, int logM,
                                                     fe* __restrict__ out, uint64_t full) {
  const uint64_t M = (uint64_t)1 << logM;
  const uint64_t total = P << (logM + 1);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t p = i >> (logM + 1), j = i & (2 * M - 1);
    fe v = fe_make(0, 0);
    if (j < M) v = ld_fe(in + p * M + j);
    if (p < full) {
      if (j == 0) v = fe_sub(v, fe_one_c());
      else if (j == M) v = fe_one_c();
    }
    st_fe(out + i, v);
  }
}

// out[i] = prod_{j != i} (d_i - d_j): Z'(d_i) of the domain's zerofier (barycentric weights'
// reciprocals).  Lanes own i, the block streams tiles of d_j through LDS.  Each Montgomery
// product contributes a factor R^-1: starting from rn = R^(n-1) mod p the n - 1 products
// leave exactly prod (d_i - d_j).
__global__ __launch_bounds__(kBlock) void k_bary_prod(const fe* __restrict__ dom, uint64_t n, fe* __restrict__ out,
                                                      fe rn) {
  __shared__ fe tile[kBlock];  // every lane reads the same entry: an LDS broadcast
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const fe di = i < n ? ld_fe(dom + i) : fe_make(0, 0);
  fe acc = rn;
  for (uint64_t j0 = 0; j0 < n; j0 += kBlock) {
    __syncthreads();
    if (j0 + threadIdx.x < n) tile[threadIdx.x] = ld_fe(dom + j0 + threadIdx.x);
    __syncthreads();
    const uint64_t cnt = n - j0 < kBlock ? n - j0 : kBlock;
    for (uint64_t k = 0; k < cnt; ++k) {
      if (j0 + k == i) continue;
      acc = mont_mul(acc, fe_sub(di, tile[k]));
    }
  }
  if (i < n) st_fe(out + i, acc);
}

// --------------------------------------------------------- prefix products

// Inclusive prefix product over 1024-element tiles (256 lanes x 4): each lane
// multiplies its 4 elements, the block scans the 256 lane totals in LDS
// (Hillis-Steele), lanes rescale.  tile_tot[b] = product of tile b.
__global__ __launch_bounds__(kBlock) void k_scan_tile(fe* __restrict__ data, uint64_t n, fe* __restrict__ tile_tot,
                                                      fe r2, fe one_m) {
  __shared__ fe sm[kBlock];
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  fe v[4];
  fe run = one_m;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fe x = base + k < n ? mont_mul(ld_fe(data + base + k), r2) : one_m;
    run = mont_mul(run, x);
    v[k] = run;
  }
  sm[threadIdx.x] = run;
  __syncthreads();
  for (unsigned off = 1; off < kBlock; off <<= 1) {
    fe mine = sm[threadIdx.x];
    fe other = threadIdx.x >= off ? sm[threadIdx.x - off] : one_m;
    __syncthreads();
    sm[threadIdx.x] = mont_mul(mine, other);
    __syncthreads();
  }
  fe prefix = threadIdx.x ? sm[threadIdx.x - 1] : one_m;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + k < n) st_fe(data + base + k, mont_mul(mont_mul(v[k], prefix), fe_one_c()));
  if (threadIdx.x == kBlock - 1 && tile_tot) st_fe(tile_tot + blockIdx.x, mont_mul(sm[kBlock - 1], fe_one_c()));
}

// data[i] *= scanned_tot[tile(i) - 1] for tiles >= 1
__global__ __launch_bounds__(kBlock) void k_scan_fix(fe* __restrict__ data, uint64_t n,
                                                     const fe* __restrict__ scanned_tot, fe r2) {
  for (uint64_t i = 1024 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    fe f = ld_fe(scanned_tot + (i / 1024) - 1);
    st_fe(data + i, mont_mul(mont_mul(ld_fe(data + i), f), r2));
  }
}

// ------------------------------------------- zerofier of a geometric domain

// Z(x) = prod_{i<n} (x - q^i) = sum_j c_j x^j,
// c_j = (-1)^(n-j) q^((n-j)(n-j-1)/2) F_n / (F_j F_(n-j)), F_k = prod_{l=1..k} (1 - q^l)
// (Gauss binomial theorem).  F and invF hold F_0..F_n canonical; q^e from the
// two-level Montgomery table (e reduced mod ord(q) = D, a power of two).
__global__ __launch_bounds__(kBlock) void k_qbinom(fe* __restrict__ c, const fe* __restrict__ F,
                                                   const fe* __restrict__ invF, uint64_t n, uint64_t D,
                                                   const fe* __restrict__ qA, const fe* __restrict__ qB, fe r2) {
  const fe Fn = ld_fe(F + n);
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= n; j += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = n - j;
    unsigned __int128 tri = (unsigned __int128)k * (k ? k - 1 : 0) / 2;
    uint64_t e = (uint64_t)(tri & (unsigned __int128)(D - 1));
    fe qm = mont_mul(ld_fe(qA + (e & 4095)), ld_fe(qB + (e >> 12)));  // Montgomery(q^e)
    fe v = mont_mul(mont_mul(Fn, ld_fe(invF + j)), r2);               // canonical F_n / F_j
    v = mont_mul(mont_mul(v, ld_fe(invF + k)), r2);                    // / F_(n-j)
    v = mont_mul(v, qm);                                               // * q^e
    if (k & 1) v = fe_neg(v);
    st_fe(c + j, v);
  }
}

// V[c M + k] = P_c(q^m) at m = f k (k < M): y_c[m] for m < n, else Zv[k] * q^-m * S[c M + k]
// (q^-m from the two-level table; f = 1, M = D: every point of the group)
__global__ __launch_bounds__(kBlock) void k_interp_assemble(fe* __restrict__ V, const fe* __restrict__ y, uint64_t ys,
                                                            const fe* __restrict__ Zv, const fe* __restrict__ S,
                                                            uint64_t n, uint64_t M, uint32_t logf, uint64_t total,
                                                            const fe* __restrict__ iA, const fe* __restrict__ iB, fe r2) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = t / M, k = t - c * M, m = k << logf;
    fe v;
    if (m < n) {
      v = ld_fe(y + c * ys + m);
    } else {
      fe im = mont_mul(ld_fe(iA + (m & 4095)), ld_fe(iB + (m >> 12)));  // Montgomery(q^-m)
      v = mont_mul(ld_fe(Zv + k), im);                                   // Zv q^-m
      v = mont_mul(mont_mul(v, ld_fe(S + t)), r2);                       // * S
    }
    st_fe(V + t, v);
  }
}

// k_interp_assemble on a column shard [rows][n2] of S (a sharded prove): local element p = r n2 + j
// is subgroup index k = row0 + r + n1 j; every value is also multiplied by M^-1 (minv = M^-1 R,
// minv_r2 = M^-1 R^2 for the Montgomery products), so the forward transform with root qf^-1 that
// follows is the inverse transform
__global__ __launch_bounds__(kBlock) void k_interp_assemble_cols(fe* __restrict__ V, const fe* __restrict__ y,
                                                                 uint64_t ys, const fe* __restrict__ Zv,
                                                                 const fe* __restrict__ S, uint64_t n, uint32_t logf,
                                                                 uint64_t local, uint64_t total, uint64_t n2,
                                                                 uint64_t n1, uint64_t row0, const fe* __restrict__ iA,
                                                                 const fe* __restrict__ iB, fe minv, fe minv_r2) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = t / local, p = t - c * local;
    const uint64_t r = p / n2, j = p - r * n2;
    const uint64_t k = row0 + r + n1 * j, m = k << logf;
    fe v;
    if (m < n) {
      v = mont_mul(ld_fe(y + c * ys + m), minv);
    } else {
      fe im = mont_mul(ld_fe(iA + (m & 4095)), ld_fe(iB + (m >> 12)));  // Montgomery(q^-m)
      v = mont_mul(ld_fe(Zv + k), im);                                   // Zv q^-m
      v = mont_mul(mont_mul(v, ld_fe(S + t)), minv_r2);                  // * S / M
    }
    st_fe(V + t, v);
  }
}

// Decimated interpolation, residue classes of a_i = y_i / Z'(q^i) (i < n <= M = D / f):
// rows[(c f + r) Mf + j] = a_(c, f j + r) for f j + r < n, else 0  (Mf = M / f rows of column c)
__global__ __launch_bounds__(kBlock) void k_geo_rows(fe* __restrict__ rows, const fe* __restrict__ y, uint64_t ys,
                                                     const fe* __restrict__ Zdi, uint64_t n, uint32_t logf,
                                                     uint64_t M, uint64_t total, fe r2) {
  const uint64_t Mf = M >> logf, f = (uint64_t)1 << logf;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = t / M, m = t - c * M;
    const fe v = m < n ? mont_mul(mont_mul(ld_fe(y + c * ys + m), ld_fe(Zdi + m)), r2) : fe_zero();
    st_fe(rows + (c * f + (m & (f - 1))) * Mf + (m >> logf), v);
  }
}

// K rows of the decimated convolution: out[r M + j] = b[(f j - r) mod D], b[j] = 1 / (1 - q^-j), b[0] = 0
__global__ __launch_bounds__(kBlock) void k_geo_krows(fe* __restrict__ out, const fe* __restrict__ b, uint32_t logf,
                                                      uint64_t M, uint64_t D) {
  const uint64_t total = D;  // f rows of M
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = t / M, j = t - r * M;
    st_fe(out + t, ld_fe(b + (((j << logf) + D - r) & (D - 1))));
  }
}

// S_hat[c M + k] = sum_r A_hat[(c f + r) M + k] * K_hat[r M + k]  (one pointwise product per
// residue class, summed: the f convolutions share one inverse transform)
__global__ __launch_bounds__(kBlock) void k_geo_dot(fe* __restrict__ S, const fe* __restrict__ A,
                                                    const fe* __restrict__ K, uint32_t logf, uint64_t M,
                                                    uint64_t total, fe r2) {
  const uint64_t f = (uint64_t)1 << logf;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = t / M, k = t - c * M;
    fe acc = fe_zero();
    for (uint64_t r = 0; r < f; ++r) acc = fe_add(acc, mont_mul(ld_fe(A + (c * f + r) * M + k), ld_fe(K + r * M + k)));
    st_fe(S + t, mont_mul(acc, r2));
  }
}

// --------------------------------------------------------------- degree

// *last = max{i + 1 : a[i] != 0} (0 when all zero): degree() = *last - 1 (polynomial.rs:41-58)
// Top-down: block b scans the b-th chunk from the end (kDegPer elements per lane, all loads
// in flight together) and first reads *last: if a nonzero at or above its chunk's end is
// already recorded, nothing in the chunk can raise the maximum, so it exits without loading.
// Blocks are dispatched in index order, so a polynomial whose leading coefficient sits near
// the end of its buffer (the usual case) is decided by its top chunks.  A stale read only
// costs the early exit, never the result.
constexpr unsigned kDegPer = 16;
// Batched: up to kDegBatch polynomials in one launch (blockIdx.y = polynomial), into slots that
// are never cleared: a slot holds (gen << kDegGenShift) | (index + 1), raised by atomicMax, and a
// value of an older generation (an earlier call) reads as "no nonzero yet" -- no memset launch
// before the scan, one kernel for the whole batch.
__global__ __launch_bounds__(kBlock) void k_last_nonzero_batch(DegBatch b, unsigned long long* __restrict__ slots,
                                                               unsigned long long gen) {
  __shared__ unsigned long long wmax[kBlock / 64];
  __shared__ int skip;
  constexpr uint64_t chunk = (uint64_t)kBlock * kDegPer;
  const unsigned y = blockIdx.y;
  const uint64_t n = b.n[y];
  if ((uint64_t)blockIdx.x * chunk >= n) return;  // uniform: shorter polynomials of the batch
  const fe* __restrict__ a = b.a[y];
  unsigned long long* last = slots + y;
  const unsigned long long tag = gen << kDegGenShift, mask = (1ull << kDegGenShift) - 1;
  const uint64_t hi = n - (uint64_t)blockIdx.x * chunk;
  const uint64_t lo = hi > chunk ? hi - chunk : 0;
  if (threadIdx.x == 0) {
    const unsigned long long v = __hip_atomic_load(last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    skip = (v >> kDegGenShift) == gen && (v & mask) >= hi;
  }
  __syncthreads();
  if (skip) return;
  unsigned long long best = 0;
  fe v[kDegPer];
#pragma unroll
  for (unsigned k = 0; k < kDegPer; ++k) {
    const uint64_t i = lo + (uint64_t)k * kBlock + threadIdx.x;
    v[k] = i < hi ? ld_fe(a + i) : fe_zero();
  }
#pragma unroll
  for (unsigned k = 0; k < kDegPer; ++k)
    if (!fe_is_zero(v[k])) best = lo + (uint64_t)k * kBlock + threadIdx.x + 1;
  for (int off = 32; off > 0; off >>= 1) {
    unsigned long long o = __shfl_xor(best, off);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (unsigned w = 1; w < kBlock / 64; ++w) best = wmax[w] > best ? wmax[w] : best;
    if (best) atomicMax(last, tag | best);
  }
}

// ----------------------------------------------------------- AIR evaluation

// out[y] = sum_g s_g Q_q(g)[y] * prod_j V_j[y]^exps[g][j]  (m_polynomial.rs:124-139 evaluated
// pointwise on a coset: s_g Q_q(g) are the coset values of the x-polynomial of group g; groups
// whose x-polynomials are proportional share one LDE).
// sum_q Q_q(y) * sum_{g in q} scale_g prod_j V_j(y)^e_gj: groups sorted by their
// distinct x-polynomial, so each point loads every value array once (the next Q is
// prefetched while the current group sum is formed) and a group costs one product
// per variable it holds.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_air_eval(AirEvalArgs a) {
  for (uint64_t y = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; y < a.n; y += (uint64_t)gridDim.x * blockDim.x) {
    // V_j, V_j^2, V_j^3 once per point: the Rescue AIR's monomials have per-variable
    // exponents <= alpha = 3
    fe p1[NV], p2[NV], p3[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) p1[j] = ld_fe(a.V[j] + ((y + a.vshift[j]) & (a.n - 1)));
    fe qnext = ld_fe(a.Q[0] + y);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      p1[j] = mont_mul(p1[j], a.r2);
      p2[j] = mont_mul(p1[j], p1[j]);
      p3[j] = mont_mul(p2[j], p1[j]);
    }
    fe acc = fe_zero();
    for (int q = 0; q < a.nq; ++q) {
      const fe qv = qnext;
      if (q + 1 < a.nq) qnext = ld_fe(a.Q[q + 1] + y);
      fe sum = fe_zero();  // Montgomery
      for (uint32_t g = a.qstart[q]; g < a.qstart[q + 1]; ++g) {
        fe term = ld_fe(a.qscale + g);  // Montgomery(scale)
        const uint32_t* e = a.exps + g * NV;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const uint32_t ej = e[j];  // uniform across the wave
          if (!ej) continue;
          fe pw;
          if (ej == 1) {
            pw = p1[j];
          } else if (ej == 2) {
            pw = p2[j];
          } else if (ej == 3) {
            pw = p3[j];
          } else {  // general exponent: square-and-multiply from V_j
            pw = p1[j];
            for (int b = 30 - __builtin_clz(ej); b >= 0; --b) {
              pw = mont_mul(pw, pw);
              if ((ej >> b) & 1u) pw = mont_mul(pw, p1[j]);
            }
          }
          term = mont_mul(term, pw);
        }
        sum = fe_add(sum, term);
      }
      acc = fe_add(acc, mont_mul(qv, sum));  // canonical Q times Montgomery sum: canonical
    }
    st_fe(a.out + y, acc);
  }
}

// Montgomery x^e (x Montgomery, e >= 1): left-to-right square-and-multiply, a uniform loop
__device__ __forceinline__ fe mont_pow_m(const fe& xm, uint32_t e) {
  fe r = xm;
  for (int b = 30 - __builtin_clz(e); b >= 0; --b) {
    r = mont_mul(r, r);
    if ((e >> b) & 1u) r = mont_mul(r, xm);
  }
  return r;
}

// One Rescue-Prime transition row at every coset point (rescue_prime.rs:246-283 factored):
// ~4 products per register and 4 more for the row, against one product chain per expanded
// monomial in k_air_eval.  Exact field arithmetic: the same values as the expanded polynomial.
__global__ __launch_bounds__(kBlock) void k_air_rescue(AirRescueArgs a) {
  const uint64_t mask = a.n - 1;
  const fe one = {{1u, 0u, 0u, 0u}};
  for (uint64_t y = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; y < a.n; y += (uint64_t)gridDim.x * blockDim.x) {
    fe acc = ld_fe(a.first + y);
    fe lin = fe_zero();
#pragma unroll
    for (int k = 0; k < kAirMaxVars / 2; ++k) {
      if (k >= a.m) break;  // uniform
      const fe v = ld_fe(a.V[k] + ((y + a.vshift[k]) & mask));
      const fe pm = mont_pow_m(mont_mul(v, a.r2), a.alpha);          // Montgomery prev_k^alpha
      acc = fe_add(acc, mont_mul(pm, a.mds[k]));                     // canonical MDS * prev_k^alpha
      const fe w = ld_fe(a.V[a.m + k] + ((y + a.vshift[a.m + k]) & mask));
      lin = fe_add(lin, mont_mul(fe_sub(w, ld_fe(a.second[k] + y)), a.mds_inv_m[k]));
    }
    const fe rhs = mont_mul(mont_pow_m(mont_mul(lin, a.r2), a.alpha), one);  // canonical lin^alpha
    st_fe(a.out + y, fe_sub(acc, rhs));
  }
}

// ------------------------------------------------------- linear combination

// out[k] = sum_t w_t * term_t[k - off_t] over off_t <= k < off_t + len_t (w_t Montgomery)
__global__ __launch_bounds__(kBlock) void k_lincomb(LinCombArgs a) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.n; k += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i = k;  // coefficient index
    if (a.cols_row_len) {
      const uint64_t r = k / a.cols_row_len;
      i = a.cols_base + r + a.cols_n1 * (k - r * a.cols_row_len);
    }
    fe acc = fe_zero();
    for (int t = 0; t < a.nterms; ++t) {
      uint64_t off = a.off[t];
      if (i >= off && i - off < a.len[t]) acc = fe_add(acc, mont_mul(ld_fe(a.term[t] + (i - off)), a.w[t]));
    }
    st_fe(a.out + k, acc);
  }
}

// out[i] = in[i * stride]  (one register column of a row-major trace)
__global__ __launch_bounds__(kBlock) void k_gather_stride(fe* __restrict__ out, const fe* __restrict__ in, uint64_t n,
                                                          uint64_t stride) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    st_fe(out + i, ld_fe(in + i * stride));
}

// out[k] = P(offset w^k), k < n, for a polynomial of at most kSmallPolyMax coefficients (Horner):
// the NTT of the zero-padded, offset-scaled coefficient vector, without the transform
__global__ __launch_bounds__(kBlock) void k_eval_small(fe* __restrict__ out, SmallPoly p, uint64_t n,
                                                       const fe* __restrict__ wA, const fe* __restrict__ wB,
                                                       fe off_m) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    fe xm = mont_mul(mont_mul(ld_fe(wA + (k & 4095)), ld_fe(wB + (k >> 12))), off_m);  // Montgomery(offset w^k)
    fe acc = p.c[p.len - 1];
    for (int j = (int)p.len - 2; j >= 0; --j) acc = fe_add(mont_mul(acc, xm), p.c[j]);
    st_fe(out + k, acc);
  }
}

// ================================================================ launchers

// out[i] = in[i] - p[i] for i < max(len, p.len), each side zero past its length: a polynomial minus a
// small host polynomial (a boundary interpolant) without uploading it -- the canonical values of
// lincomb({in, 1}, {p, -1})
__global__ __launch_bounds__(kBlock) void k_sub_small(fe* __restrict__ out, const fe* __restrict__ in, uint64_t len,
                                                      SmallPoly p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const fe a = i < len ? ld_fe(in + i) : fe_zero();
    const fe b = i < (uint64_t)p.len ? p.c[i] : fe_zero();
    st_fe(out + i, fe_sub(a, b));
  }
}

hipError_t launch_sub_small(fe* out, const fe* in, uint64_t len, const SmallPoly& p, hipStream_t s) {
  const uint64_t n = len > (uint64_t)p.len ? len : (uint64_t)p.len;
  if (!n) return hipSuccess;
  ProfScope ps("lincomb", 32 * n, s);
  hipLaunchKernelGGL(k_sub_small, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, out, in, len, p, n);
  return hipGetLastError();
}

hipError_t launch_eval_small(fe* out, const SmallPoly& p, uint64_t n, const fe* wA, const fe* wB, const fe& off_m,
                             hipStream_t s) {
  if (!n) return hipSuccess;
  if (p.len < 1 || p.len > kSmallPolyMax) return hipErrorInvalidValue;
  ProfScope ps("eval_small", 16 * n, s);
  hipLaunchKernelGGL(k_eval_small, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, out, p, n, wA, wB, off_m);
  return hipGetLastError();
}

// the randomized trace's m register columns side by side (column stride Tp = rows + nrand): column s
// is trace[i m + s] for i < rows, then rand[(i - rows) m + s] -- the 2m strided gathers of the
// trace interpolation (stark.rs:285-301) in one launch
__global__ __launch_bounds__(kBlock) void k_gather_trace_cols(fe* __restrict__ out, const fe* __restrict__ trace,
                                                              uint64_t rows, const fe* __restrict__ rnd, uint64_t nrand,
                                                              uint64_t m) {
  const uint64_t Tp = rows + nrand, total = Tp * m;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = t / m, s = t - i * m;  // consecutive lanes read consecutive trace elements
    const fe v = i < rows ? ld_fe(trace + t) : ld_fe(rnd + (i - rows) * m + s);
    st_fe(out + s * Tp + i, v);
  }
}

hipError_t launch_gather_trace_cols(fe* out, const fe* trace, uint64_t rows, const fe* rnd, uint64_t nrand, uint64_t m,
                                    hipStream_t s) {
  const uint64_t total = (rows + nrand) * m;
  if (!total) return hipSuccess;
  ProfScope ps("gather_stride", 32 * total, s);
  hipLaunchKernelGGL(k_gather_trace_cols, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, s, out, trace, rows, rnd,
                     nrand, m);
  return hipGetLastError();
}

hipError_t launch_gather_stride(fe* out, const fe* in, uint64_t n, uint64_t stride, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("gather_stride", 32 * n, s);
  hipLaunchKernelGGL(k_gather_stride, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, out, in, n, stride);
  return hipGetLastError();
}

hipError_t launch_ew_mul(fe* out, const fe* a, const fe* b, uint64_t n, const fe& r2, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("ew_mul", 48 * n, s);
  hipLaunchKernelGGL(k_ew_mul, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, out, a, b, n, r2);
  return hipGetLastError();
}

hipError_t launch_mul_pow2(fe* out, const fe* in, uint64_t n, uint64_t start, const fe* sA, const fe* sB,
                           hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("mul_pow2", 32 * n, s);
  hipLaunchKernelGGL(k_mul_pow2, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, out, in, n, start, sA, sB);
  return hipGetLastError();
}

hipError_t launch_one_minus_pow(fe* out, uint64_t n, uint64_t start, const fe* sA, const fe* sB, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("one_minus_pow", 16 * n, s);
  hipLaunchKernelGGL(k_one_minus_pow, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, out, n, start, sA, sB);
  return hipGetLastError();
}

hipError_t launch_deriv(fe* out, const fe* c, uint64_t n, const fe& r2, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("deriv", 32 * n, s);
  hipLaunchKernelGGL(k_deriv, dim3((unsigned)grid_for(n)), dim3(kBlock), 0, s, out, c, n, r2);
  return hipGetLastError();
}

hipError_t launch_batch_div(fe* out, const fe* a, const fe* b, uint64_t n, const fe& r2, const fe& one_m,
                            unsigned* zero_flag, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("batch_div", (a ? 48 : 32) * n, s);
  // K elements per lane amortize one Fermat inversion (~160 dependent products); below
  // ~2^17 lanes the chip is latency-bound on that chain, so small n trades the
  // amortization for lanes: K = 16 from n = 2^21, 8 from 2^20, else 4
  static const int env_k = SG_KNOB(BATCH_DIV_K, 0);  // A/B builds: 4, 8 or 16 for every n
  const int K = env_k == 4 || env_k == 8 || env_k == 16 ? env_k : n >= ((uint64_t)1 << 21) ? 16 : n >= ((uint64_t)1 << 20) ? 8 : 4;
  uint64_t lanes = (n + K - 1) / K;  // at least one full block
  uint64_t blocks = (lanes + kBlock - 1) / kBlock;
  switch (K) {
    case 4: hipLaunchKernelGGL((k_batch_div<4>), dim3((unsigned)blocks), dim3(kBlock), 0, s, out, a, b, n, r2, one_m, zero_flag); break;
    case 8: hipLaunchKernelGGL((k_batch_div<8>), dim3((unsigned)blocks), dim3(kBlock), 0, s, out, a, b, n, r2, one_m, zero_flag); break;
    default: hipLaunchKernelGGL((k_batch_div<16>), dim3((unsigned)blocks), dim3(kBlock), 0, s, out, a, b, n, r2, one_m, zero_flag); break;
  }
  return hipGetLastError();
}

hipError_t launch_scan_tile(fe* data, uint64_t n, fe* tile_tot, const fe& r2, const fe& one_m, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("scan_tile", 32 * n, s);
  hipLaunchKernelGGL(k_scan_tile, dim3((unsigned)((n + 1023) / 1024)), dim3(kBlock), 0, s, data, n, tile_tot, r2,
                     one_m);
  return hipGetLastError();
}

hipError_t launch_scan_fix(fe* data, uint64_t n, const fe* scanned_tot, const fe& r2, hipStream_t s) {
  if (n <= 1024) return hipSuccess;
  ProfScope ps("scan_fix", 32 * n, s);
  hipLaunchKernelGGL(k_scan_fix, dim3((unsigned)grid_for(n - 1024)), dim3(kBlock), 0, s, data, n, scanned_tot, r2);
  return hipGetLastError();
}

hipError_t launch_qbinom(fe* c, const fe* F, const fe* invF, uint64_t n, uint64_t D, const fe* qA, const fe* qB,
                         const fe& r2, hipStream_t s) {
  ProfScope ps("qbinom", 48 * (n + 1), s);
  hipLaunchKernelGGL(k_qbinom, dim3((unsigned)grid_for(n + 1)), dim3(kBlock), 0, s, c, F, invF, n, D, qA, qB, r2);
  return hipGetLastError();
}

hipError_t launch_interp_assemble(fe* V, const fe* y, uint64_t ys, const fe* Zv, const fe* S, uint64_t n, uint64_t M,
                                  int logf, uint64_t cols, const fe* iA, const fe* iB, const fe& r2, hipStream_t s) {
  const uint64_t total = cols * M;
  ProfScope ps("interp_assemble", 64 * total, s);
  hipLaunchKernelGGL(k_interp_assemble, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, s, V, y, ys, Zv, S, n, M,
                     (uint32_t)logf, total, iA, iB, r2);
  return hipGetLastError();
}

hipError_t launch_interp_assemble_cols(fe* V, const fe* y, uint64_t ys, const fe* Zv, const fe* S, uint64_t n,
                                       int logf, uint64_t cols, uint64_t rows, uint64_t n2, uint64_t n1, uint64_t row0,
                                       const fe* iA, const fe* iB, const fe& minv_m, const fe& minv_r2,
                                       hipStream_t s) {
  const uint64_t local = rows * n2, total = cols * local;
  ProfScope ps("interp_assemble", 64 * total, s);
  hipLaunchKernelGGL(k_interp_assemble_cols, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, s, V, y, ys, Zv, S, n,
                     (uint32_t)logf, local, total, n2, n1, row0, iA, iB, minv_m, minv_r2);
  return hipGetLastError();
}

hipError_t launch_geo_rows(fe* rows, const fe* y, uint64_t ys, const fe* Zdi, uint64_t n, int logf, uint64_t M,
                           uint64_t cols, const fe& r2, hipStream_t s) {
  const uint64_t total = cols * M;
  ProfScope ps("geo_rows", 48 * total, s);
  hipLaunchKernelGGL(k_geo_rows, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, s, rows, y, ys, Zdi, n,
                     (uint32_t)logf, M, total, r2);
  return hipGetLastError();
}

hipError_t launch_geo_krows(fe* out, const fe* b, int logf, uint64_t M, uint64_t D, hipStream_t s) {
  ProfScope ps("geo_krows", 32 * D, s);
  hipLaunchKernelGGL(k_geo_krows, dim3((unsigned)grid_for(D)), dim3(kBlock), 0, s, out, b, (uint32_t)logf, M, D);
  return hipGetLastError();
}

hipError_t launch_geo_dot(fe* S, const fe* A, const fe* K, int logf, uint64_t M, uint64_t cols, const fe& r2,
                          hipStream_t s) {
  const uint64_t total = cols * M;
  ProfScope ps("geo_dot", (32 * ((uint64_t)1 << logf) + 16) * total, s);
  hipLaunchKernelGGL(k_geo_dot, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, s, S, A, K, (uint32_t)logf, M,
                     total, r2);
  return hipGetLastError();
}

// the degree slots to host-coherent memory, then the ready flag (system scope): the host spins on
// the flag instead of a runtime copy and a stream synchronisation
__global__ void k_publish_slots(const unsigned long long* __restrict__ slots, unsigned long long* host, uint64_t n,
                                unsigned long long* flag, unsigned long long seq) {
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x)
    __hip_atomic_store(host + i, __hip_atomic_load(slots + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t launch_publish_slots(const unsigned long long* slots, unsigned long long* host, uint64_t n,
                                unsigned long long* flag, unsigned long long seq, hipStream_t s) {
  hipLaunchKernelGGL(k_publish_slots, dim3(1), dim3(256), 0, s, slots, host, n, flag, seq);
  return hipGetLastError();
}

hipError_t launch_last_nonzero_batch(const DegBatch& b, int count, unsigned long long* slots, unsigned long long gen,
                                     hipStream_t s) {
  if (count < 1 || count > kDegBatch || gen == 0 || gen >= (1ull << (64 - kDegGenShift))) return hipErrorInvalidValue;
  uint64_t nmax = 0;
  for (int i = 0; i < count; ++i) {
    if (b.n[i] >> kDegGenShift) return hipErrorInvalidValue;
    nmax = b.n[i] > nmax ? b.n[i] : nmax;
  }
  if (!nmax) return hipSuccess;
  ProfScope ps("last_nonzero", 16 * nmax * count, s);
  const uint64_t blocks = (nmax + (uint64_t)kBlock * kDegPer - 1) / ((uint64_t)kBlock * kDegPer);
  hipLaunchKernelGGL(k_last_nonzero_batch, dim3((unsigned)blocks, (unsigned)count), dim3(kBlock), 0, s, b, slots, gen);
  return hipGetLastError();
}

hipError_t launch_air_eval(const AirEvalArgs& a, hipStream_t s) {
  if (!a.n) return hipSuccess;
  if (a.nvars > kAirMaxVars || a.nvars < 1 || a.nq < 1 || (a.n & (a.n - 1))) return hipErrorInvalidValue;
  ProfScope ps("air_eval", 16 * a.n * (a.nvars + a.nq + 1), s);
  const dim3 grid((unsigned)grid_for(a.n));
  switch (a.nvars) {
    case 1: hipLaunchKernelGGL(k_air_eval<1>, grid, dim3(kBlock), 0, s, a); break;
    case 2: hipLaunchKernelGGL(k_air_eval<2>, grid, dim3(kBlock), 0, s, a); break;
    case 3: hipLaunchKernelGGL(k_air_eval<3>, grid, dim3(kBlock), 0, s, a); break;
    case 4: hipLaunchKernelGGL(k_air_eval<4>, grid, dim3(kBlock), 0, s, a); break;
    case 5: hipLaunchKernelGGL(k_air_eval<5>, grid, dim3(kBlock), 0, s, a); break;
    case 6: hipLaunchKernelGGL(k_air_eval<6>, grid, dim3(kBlock), 0, s, a); break;
    case 7: hipLaunchKernelGGL(k_air_eval<7>, grid, dim3(kBlock), 0, s, a); break;
    default: hipLaunchKernelGGL(k_air_eval<8>, grid, dim3(kBlock), 0, s, a); break;
  }
  return hipGetLastError();
}

hipError_t launch_air_rescue(const AirRescueArgs& a, hipStream_t s) {
  if (!a.n) return hipSuccess;
  if (a.m < 1 || a.m > kAirMaxVars / 2 || a.alpha < 1 || (a.n & (a.n - 1))) return hipErrorInvalidValue;
  ProfScope ps("air_eval", 16 * a.n * (2 * a.m + a.m + 2), s);
  hipLaunchKernelGGL(k_air_rescue, dim3((unsigned)grid_for(a.n)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_lincomb(const LinCombArgs& a, hipStream_t s) {
  if (!a.n) return hipSuccess;
  if (a.nterms > kLinCombMaxTerms) return hipErrorInvalidValue;
  ProfScope ps("lincomb", 16 * a.n * (a.nterms + 1), s);
  hipLaunchKernelGGL(k_lincomb, dim3((unsigned)grid_for(a.n)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_tree_leaves(const fe* dom, uint64_t n, uint64_t nodes, fe* Z, const fe* c, fe* N, const fe& r2,
                              hipStream_t s) {
  if (!nodes) return hipSuccess;
  ProfScope ps("tree_leaves", 16 * n * (c ? 2 : 1) + 2 * 16 * 16 * nodes, s);
  hipLaunchKernelGGL(k_tree_leaves, dim3((unsigned)((nodes + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, dom, n,
                     nodes, Z, c, N, r2);
  return hipGetLastError();
}

hipError_t launch_tree_combine(const fe* Zh, const fe* Nh, uint64_t P, int logM, fe* Zp, fe* Np, const fe& r2,
                               hipStream_t s) {
  const uint64_t total = P << logM;
  if (!total) return hipSuccess;
  ProfScope ps("tree_combine", (Nh ? 96 : 48) * total, s);
  hipLaunchKernelGGL(k_tree_combine, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, s, Zh, Nh, P, logM, Zp, Np,
                     r2);
  return hipGetLastError();
}

hipError_t launch_tree_fix(const fe* in, uint64_t P, int logM, fe* out, uint64_t full, hipStream_t s) {
  const uint64_t total = P << (logM + 1);
  if (!total) return hipSuccess;
  ProfScope ps("tree_fix", 16 * (total / 2) + 16 * total, s);
  hipLaunchKernelGGL(k_tree_fix, dim3((unsigned)grid_for(total)), dim3(kBlock), 0, s, in, P, logM, out, full);
  return hipGetLastError();
}

hipError_t launch_bary_prod(const fe* dom, uint64_t n, fe* out, const fe& rn, hipStream_t s) {
  if (!n) return hipSuccess;
  ProfScope ps("bary_prod", 32 * n, s);
  hipLaunchKernelGGL(k_bary_prod, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, dom, n, out, rn);
  return hipGetLastError();
}

}  // namespace sg
