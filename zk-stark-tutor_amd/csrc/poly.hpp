// Device polynomial algebra: fft/ntt_arithmetics.rs (fast_multiply, fast_zerofier,
// fast_interpolate_domain, fast_coset_divide) on the gfx950 NTT, plus the small
// host polynomials the STARK needs for boundary constraints.
//
// A polynomial is a coefficient vector that is never trimmed (field/polynomial.rs
// keeps trailing zeros; degree() skips them).
#pragma once
#include <cstdint>
#include <vector>

#include "context.hpp"
#include "fe128.hpp"

struct sg_poly;

namespace sg {

struct DPoly {
  DevBuf buf;
  uint64_t len = 0;
  fe* p() const { return buf.as<fe>(); }
};

DPoly dpoly_alloc(sg_ctx* ctx, uint64_t len);
DPoly dpoly_upload(sg_ctx* ctx, const fe* host, uint64_t len);
std::vector<fe> dpoly_download(sg_ctx* ctx, const fe* d, uint64_t len);
DPoly dpoly_copy(sg_ctx* ctx, const fe* d, uint64_t len);

// polynomial.rs:41-58 degree(): -1 for None (synchronizes)
int64_t dev_degree(sg_ctx* ctx, const fe* d, uint64_t len);
// degrees of several device polynomials with one host round trip
std::vector<int64_t> dev_degrees(sg_ctx* ctx, const std::vector<std::pair<const fe*, uint64_t>>& polys);
// the same in two halves: launch the scans (and their publication), then wait for the published
// degrees -- host work can go between them
struct DegScan {
  unsigned long long gen = 0;
  size_t n = 0;
};
DegScan dev_degrees_begin(sg_ctx* ctx, const std::vector<std::pair<const fe*, uint64_t>>& polys);
std::vector<int64_t> dev_degrees_end(sg_ctx* ctx, const DegScan& sc);

// primitive root of order n (field.rs:58-71)
fe root_of_order(uint64_t n);
// ntt_arithmetics.rs:11-24 assertions
void check_root(const fe& root, uint64_t root_order);
// Montgomery(f^e) = A[e & 4095] * B[e >> 12] for e < count (cached per context)
void pow_tables2(sg_ctx* ctx, const fe& f, uint64_t count, const fe** A, const fe** B);

// size-2^logn transforms of the first n_in entries (zero beyond), optional offset^i input scale
void ntt_sized(sg_ctx* ctx, const fe& root, const fe* in, uint64_t n_in, int logn, fe* out,
               const fe* scale_offset = nullptr);
void intt_sized(sg_ctx* ctx, const fe& root, const fe* in, int logn, fe* out);

void dev_mul(sg_ctx* ctx, fe* out, const fe* a, const fe* b, uint64_t n);
// out = a / b elementwise (a == nullptr: 1 / b); a zero divisor is reported by check_div_zero
void dev_div(sg_ctx* ctx, fe* out, const fe* a, const fe* b, uint64_t n);
// throws "divide by zero" if a division since the last check saw a zero divisor; call only
// after the stream has drained past those divisions (a synchronize or a tree-root wait)
void check_div_zero(sg_ctx* ctx);
// out[i] = in[i] * f^(start + i)
void dev_scale_pow(sg_ctx* ctx, fe* out, const fe* in, uint64_t n, const fe& f, uint64_t start = 0);
// in-place inclusive prefix product
void dev_prefix_product(sg_ctx* ctx, fe* data, uint64_t n);

// exact product (length la + lb - 1, empty if either is empty): polynomial.rs:285-308 semantics
DPoly poly_mul_exact(sg_ctx* ctx, const fe* a, uint64_t la, const fe* b, uint64_t lb);
// ntt_arithmetics.rs:5-64
DPoly fast_multiply_dev(sg_ctx* ctx, fe root, uint64_t root_order, const fe* a, uint64_t la, const fe* b,
                        uint64_t lb);
// fast_coset_divide in pieces (so a caller holding the lhs coset values can reuse them):
// the order / root / result length the reference derives from the degrees, its padded
// (optionally offset-scaled) NTT, and the pointwise quotient -> INTT -> truncate -> unscale
struct DivPlan {
  fe root;
  uint64_t order = 0;
  uint64_t result_len = 0;
  bool zero_lhs = false;
};
DivPlan coset_divide_plan(fe root, uint64_t root_order, int64_t deg_lhs, int64_t deg_rhs);
// host_copy: the polynomial's coefficients on the host, if the caller has them (saves a read-back)
void ref_inner_ntt(sg_ctx* ctx, const fe& root, uint64_t order, const fe* p, uint64_t len, const fe* scale,
                   DevBuf& out, uint64_t& out_len, const fe* host_copy = nullptr);
// rhs_is_inverse: rhs_v holds 1 / (the divisor's coset values), so the division is a product
DPoly coset_divide_finish(sg_ctx* ctx, const DivPlan& pl, const fe& offset, fe* lhs_v, const fe* rhs_v,
                          bool rhs_is_inverse = false);
// 1 / the coset values (order pl.order, offset) of a small divisor known on the host (<= 64
// coefficients), kept in the context's bounded content-keyed tables (with `keep` and
// SG_NO_DOMAIN_CACHE=1: recomputed into a buffer `keep` owns); a zero value throws
const fe* divisor_inverse_values(sg_ctx* ctx, const DivPlan& pl, const fe& offset, const fe* rhs, uint64_t lr,
                                 const fe* rhs_host, std::vector<DevBuf>* keep = nullptr);
// ntt_arithmetics.rs:239-310
// rhs_degree / lhs_degree: the divisor's / dividend's degree when the caller knows it (-1 = zero
// polynomial), -2 = query the device
DPoly fast_coset_divide_dev(sg_ctx* ctx, fe root, uint64_t root_order, const fe& offset, const fe* lhs, uint64_t ll,
                            const fe* rhs, uint64_t lr, int64_t rhs_degree = -2, const fe* rhs_host = nullptr,
                            int64_t lhs_degree = -2);
// fast_coset_divide_dev for several quotients on one coset at once (the boundary quotients): items
// whose plans share one coset size, with equal dividend lengths and small host-known divisors, run
// their dividends' coset transforms and their inverse transforms as batched launches (up to
// kMaxBatch per launch); any other item goes through fast_coset_divide_dev.  Same results.
struct DivItem {
  const fe* lhs;
  uint64_t ll;
  const fe* rhs;
  uint64_t lr;
  int64_t dr;           // divisor degree (>= 0)
  const fe* rhs_host;   // its coefficients on the host
  int64_t dl;           // dividend degree (-1: zero polynomial)
};
std::vector<DPoly> fast_coset_divide_batch_dev(sg_ctx* ctx, fe root, uint64_t root_order, const fe& offset,
                                               const std::vector<DivItem>& items);
// prod_{i<n} (x - q^i) for q of order D (ntt_arithmetics.rs:66-113 on the domain q^0..q^(n-1)), length n + 1;
// n == D reproduces the reference's wrapped result (D zeros)
DPoly zerofier_geometric_dev(sg_ctx* ctx, const fe& q, uint64_t D, uint64_t n);
// tags of the context's domain tables (sg_ctx::domain_tables keys start with one)
enum : uint64_t { kDomainGeoInterp = 1, kDomainTzCoeffs = 2, kDomainTzValues = 3, kDomainTzInverse = 4,
                  kDomainDivisorInverse = 5, kDomainMpolyCoset = 6, kDomainRescueCoset = 7,
                  // run-shard slices of public coset tables for a sharded prove (key carries G, g)
                  kDomainShard = 8 };
// Z(q^m) (m < D) and 1 / Z'(q^i) (i < n) of the domain q^0..q^(n-1), reusable across
// interpolations on one domain
struct GeoInterpCache {
  fe q;
  uint64_t D = 0, n = 0;
  int logf = 0;     // Zv holds Z(q^(f k)), k < D / f (decimated interpolation, f = 2^logf)
  DevBuf Zv, Zdi;
};
// the decimated geometric interpolation's public tables for (q, D, n), 1 < n < D (context-cached):
// f = 2^logf, M = D / f, qf = q^f (order M), Zv[k] = Z(q^(f k)) (k < M), Zdi[i] = 1 / Z'(q^i) (i < n),
// Khat = the f rows (M each) of the transformed convolution kernel (f = 1: NTT_D(b), one row)
struct GeoPlan {
  int logf = 0;
  uint64_t M = 0;
  fe qf;
  const fe* Zv = nullptr;
  const fe* Zdi = nullptr;
  const fe* Khat = nullptr;
};
// use_option = false: ignore the context option geo_decimate (a sharded prove: every rank must take
// the same plan)
GeoPlan geo_plan(sg_ctx* ctx, const fe& q, uint64_t D, uint64_t n, GeoInterpCache* cache, bool use_option = true);
// the interpolant of degree < n through (q^i, y_i), i < n <= D (ntt_arithmetics.rs:172-237), length n
DPoly interpolate_geometric_dev(sg_ctx* ctx, const fe& q, uint64_t D, const fe* y, uint64_t n,
                                GeoInterpCache* cache = nullptr);
// the same for `cols` columns y + c * ys (batched transforms)
std::vector<DPoly> interpolate_geometric_batch_dev(sg_ctx* ctx, const fe& q, uint64_t D, const fe* y, uint64_t ys,
                                                   size_t cols, uint64_t n, GeoInterpCache* cache = nullptr);
// coefficients (length L) of the polynomial of degree < L with P(offset w^k) = values[k], w of order L
void coset_interpolate_dev(sg_ctx* ctx, const fe* values, uint64_t L, const fe& offset, fe* out);
// out (length L, a power of two >= len) = [P(offset w^k)], w of order L
void coset_values_dev(sg_ctx* ctx, const fe* coeffs, uint64_t len, uint64_t L, const fe& offset, fe* out);

// arbitrary (non-geometric) domains: ntt_arithmetics.rs:66-113 / 172-237 on the device
void ntt_rows_dev(sg_ctx* ctx, const fe& root, const fe* in, uint64_t rows, int logn, fe* out, const fe* post_host);
void ntt_rows_inverse(sg_ctx* ctx, const fe& root, const fe* in, uint64_t rows, int logn, fe* out);
void tree_exact(sg_ctx* ctx, const fe* d_dom, uint64_t n, const fe* d_c, DPoly* Zout, DPoly* Nout);
DPoly zerofier_any_dev(sg_ctx* ctx, const fe& root, uint64_t root_order, const fe* d_dom, uint64_t n);
DPoly interpolate_any_dev(sg_ctx* ctx, const fe& root, uint64_t root_order, const fe* d_dom, const fe* d_val,
                          uint64_t n);

// ---- host polynomials (small: boundary interpolants / zerofiers, constants) ----
using HPoly = std::vector<fe>;
int64_t hp_degree(const HPoly& a);
HPoly hp_add(const HPoly& a, const HPoly& b);  // polynomial.rs:251-276 (zero operand -> other)
HPoly hp_neg(const HPoly& a);
HPoly hp_sub(const HPoly& a, const HPoly& b);
HPoly hp_mul(const HPoly& a, const HPoly& b);  // polynomial.rs:285-308
HPoly hp_scale(const HPoly& a, const fe& f);
fe hp_eval(const HPoly& a, const fe& x);
HPoly hp_zerofier(const std::vector<fe>& domain);                                   // length n + 1 (n > 0)
HPoly hp_interpolate(const std::vector<fe>& domain, const std::vector<fe>& values);  // length n
bool is_geometric(const fe* domain, uint64_t n, const fe& root);                    // domain[i] == root^i

}  // namespace sg

struct sg_poly {
  sg::DPoly d;
};
