// Launchers for the polynomial-algebra kernels (poly_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "fe128.hpp"

namespace sg {

constexpr int kAirMaxVars = 8;        // point variables besides x (2 m registers, m <= 4)
constexpr int kLinCombMaxTerms = 48;  // terms of one weighted combination

struct AirEvalArgs {
  fe* out;
  const fe* const* Q;     // device array [nq] of coset-value arrays (the distinct x-polynomials)
  const uint32_t* qstart; // device [nq + 1]: groups qstart[q] .. qstart[q+1]-1 have x-polynomial
                          // qscale[g] * Q[q] (groups sorted by q)
  const fe* qscale;       // device [ngroups]: Montgomery(scale)
  const fe* const* V;     // device array [nvars] of coset-value arrays (point variables 1..)
  const uint32_t* exps;   // device [ngroups][nvars]
  int ngroups, nvars, nq;
  uint64_t n;             // a power of two
  uint64_t vshift[kAirMaxVars];  // variable j at point y reads V[j][(y + vshift[j]) mod n]
  fe r2, one_m;
};

constexpr int kSmallPolyMax = 16;
struct SmallPoly {
  fe c[kSmallPolyMax];  // canonical coefficients
  int len;
};

struct LinCombArgs {
  fe* out;
  uint64_t n;
  int nterms;
  const fe* term[kLinCombMaxTerms];
  uint64_t off[kLinCombMaxTerms];
  uint64_t len[kLinCombMaxTerms];
  fe w[kLinCombMaxTerms];  // Montgomery
  // cols_row_len != 0: only a column shard of the result (the sharded prove's combination):
  // output k = r * cols_row_len + j is coefficient cols_base + r + cols_n1 * j
  uint64_t cols_row_len, cols_n1, cols_base;
};

hipError_t launch_ew_mul(fe* out, const fe* a, const fe* b, uint64_t n, const fe& r2, hipStream_t s);
hipError_t launch_mul_pow2(fe* out, const fe* in, uint64_t n, uint64_t start, const fe* sA, const fe* sB,
                           hipStream_t s);
hipError_t launch_one_minus_pow(fe* out, uint64_t n, uint64_t start, const fe* sA, const fe* sB, hipStream_t s);
hipError_t launch_deriv(fe* out, const fe* c, uint64_t n, const fe& r2, hipStream_t s);
hipError_t launch_batch_div(fe* out, const fe* a, const fe* b, uint64_t n, const fe& r2, const fe& one_m,
                            unsigned* zero_flag, hipStream_t s);
hipError_t launch_scan_tile(fe* data, uint64_t n, fe* tile_tot, const fe& r2, const fe& one_m, hipStream_t s);
hipError_t launch_scan_fix(fe* data, uint64_t n, const fe* scanned_tot, const fe& r2, hipStream_t s);
hipError_t launch_qbinom(fe* c, const fe* F, const fe* invF, uint64_t n, uint64_t D, const fe* qA, const fe* qB,
                         const fe& r2, hipStream_t s);
// V[c M + k] = P_c(q^(k f)), f = 2^logf (y_c at ys stride; Zv[k] = Z(q^(k f)))
hipError_t launch_interp_assemble(fe* V, const fe* y, uint64_t ys, const fe* Zv, const fe* S, uint64_t n, uint64_t M,
                                  int logf, uint64_t cols, const fe* iA, const fe* iB, const fe& r2, hipStream_t s);
// decimated geometric interpolation (poly.cpp interpolate_geometric_*): residue-class rows of
// y / Z', the K rows, and the summed pointwise products
// the same on a column shard [rows][n2] (subgroup index row0 + r + n1 j), every value times M^-1
// (minv_m = Montgomery(M^-1), minv_r2 = Montgomery(Montgomery(M^-1)))
hipError_t launch_interp_assemble_cols(fe* V, const fe* y, uint64_t ys, const fe* Zv, const fe* S, uint64_t n,
                                       int logf, uint64_t cols, uint64_t rows, uint64_t n2, uint64_t n1, uint64_t row0,
                                       const fe* iA, const fe* iB, const fe& minv_m, const fe& minv_r2,
                                       hipStream_t s);
hipError_t launch_geo_rows(fe* rows, const fe* y, uint64_t ys, const fe* Zdi, uint64_t n, int logf, uint64_t M,
                           uint64_t cols, const fe& r2, hipStream_t s);
hipError_t launch_geo_krows(fe* out, const fe* b, int logf, uint64_t M, uint64_t D, hipStream_t s);
hipError_t launch_geo_dot(fe* S, const fe* A, const fe* K, int logf, uint64_t M, uint64_t cols, const fe& r2,
                          hipStream_t s);
// last nonzero index + 1 of up to kDegBatch polynomials in one launch, into slots[0..count) tagged
// with generation gen (1 .. 2^24 - 1): slot = (gen << kDegGenShift) | (index + 1); a slot of another
// generation means all zero (the slots are never cleared; sg_ctx::deg_slots)
constexpr int kDegBatch = 8;
constexpr int kDegGenShift = 40;  // polynomials up to 2^40 - 1 coefficients
struct DegBatch {
  const fe* a[kDegBatch];
  uint64_t n[kDegBatch];
};
hipError_t launch_last_nonzero_batch(const DegBatch& b, int count, unsigned long long* slots, unsigned long long gen,
                                     hipStream_t s);
// host[i] = slots[i] (i < n, host-coherent memory, device view), then *flag = seq (system scope)
hipError_t launch_publish_slots(const unsigned long long* slots, unsigned long long* host, uint64_t n,
                                unsigned long long* flag, unsigned long long seq, hipStream_t s);
hipError_t launch_air_eval(const AirEvalArgs& a, hipStream_t s);
// the Rescue-Prime AIR row in its factored form (mpoly.hpp RescueAirForm), pointwise on a coset:
// out = first(y) + sum_k mds[k] V_k^alpha - (sum_k mds_inv[k] (V_{m+k} - second_k(y)))^alpha
struct AirRescueArgs {
  fe* out;
  const fe* V[kAirMaxVars];       // prev_0..m-1, next_0..m-1 (variable j reads V[j][(y + vshift[j]) mod n])
  uint64_t vshift[kAirMaxVars];
  const fe* first;                // first_row on the coset
  const fe* second[kAirMaxVars / 2];
  fe mds[kAirMaxVars / 2];        // canonical
  fe mds_inv_m[kAirMaxVars / 2];  // Montgomery
  fe r2;
  uint32_t alpha;                 // >= 1
  int m;                          // 1 .. kAirMaxVars / 2
  uint64_t n;                     // a power of two
};
hipError_t launch_air_rescue(const AirRescueArgs& a, hipStream_t s);
hipError_t launch_lincomb(const LinCombArgs& a, hipStream_t s);
// out[i] = in[i] - p[i], i < max(len, p.len) (zero past each length; canonical)
hipError_t launch_sub_small(fe* out, const fe* in, uint64_t len, const SmallPoly& p, hipStream_t s);
hipError_t launch_eval_small(fe* out, const SmallPoly& p, uint64_t n, const fe* wA, const fe* wB, const fe& off_m,
                             hipStream_t s);
hipError_t launch_gather_stride(fe* out, const fe* in, uint64_t n, uint64_t stride, hipStream_t s);
// out[s Tp + i] = i < rows ? trace[i m + s] : rnd[(i - rows) m + s] for s < m, i < Tp = rows + nrand
hipError_t launch_gather_trace_cols(fe* out, const fe* trace, uint64_t rows, const fe* rnd, uint64_t nrand, uint64_t m,
                                    hipStream_t s);
// product tree over an arbitrary domain (poly.cpp: tree_exact): level-3 leaves (8 points per lane,
// rows of 16: Z and optionally N = sum c_i Z / (x - d_i)), pairwise NTT-domain combine, wrap fix
hipError_t launch_tree_leaves(const fe* dom, uint64_t n, uint64_t nodes, fe* Z, const fe* c, fe* N, const fe& r2,
                              hipStream_t s);
hipError_t launch_tree_combine(const fe* Zh, const fe* Nh, uint64_t P, int logM, fe* Zp, fe* Np, const fe& r2,
                               hipStream_t s);
hipError_t launch_tree_fix(const fe* in, uint64_t P, int logM, fe* out, uint64_t full, hipStream_t s);
// out[i] = prod_{j != i} (d_i - d_j); rn = R^(n-1) mod p (canonical) undoes the n - 1 Montgomery factors
hipError_t launch_bary_prod(const fe* dom, uint64_t n, fe* out, const fe& rn, hipStream_t s);

}  // namespace sg
