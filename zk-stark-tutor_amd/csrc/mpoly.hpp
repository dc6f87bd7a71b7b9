// Multivariate polynomials (m_polynomial.rs) grouped for the GPU.
//
// The reference stores {exponent vector: coefficient} and keeps zero
// coefficients (Add/Mul never remove keys); the STARK's degree bounds are taken
// over the KEYS (stark.rs:117-160).  Here a polynomial is grouped by the
// exponents of variables 1.. (the registers) with a dense coefficient vector in
// variable 0 (x) per group: F[x][v_1..v_k].  A group's vector length is its
// largest x-exponent key + 1, which is exactly what the key-based degree bounds
// read, and every reference operation maps onto groups:
//   add  = union of groups, coefficient vectors added (length max)
//   mul  = all pairs of groups, x-vectors multiplied (length la + lb - 1; large
//          products on the GPU NTT)
// Evaluation on a coset is pointwise: sum_g Q_g(y) prod_j V_j(y)^e_gj.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <vector>

#include <array>

#include "context.hpp"
#include "fe128.hpp"
#include "poly.hpp"

namespace sg {

// device-resident copies of the group x-vectors (trimmed at their degree), uploaded on first
// use by the prover: the constraints are an input of every proof, like the trace
struct MPolyDevice {
  int device = -1;
  std::vector<void*> ptr;       // distinct x-polynomials up to a scalar (first non-zero coefficient 1)
  std::vector<uint64_t> len;    // their degree + 1
  std::vector<HPoly> small;     // host copy of those with len <= kSmallPolyMax (else empty)
  std::vector<int32_t> qidx;    // per group (map order): index into ptr, -1 for an all-zero group
  std::vector<fe> scale;        // per group: x-polynomial = scale * ptr[qidx]
  // per distinct x-polynomial: its content digest (BLAKE2b-512 of the coefficients, first 32
  // bytes). The values of x-polynomial q on a coset are public -- the AIR and the domain -- and
  // live in the proving context's domain tables under {kDomainMpolyCoset, len, digest, L, offset}:
  // per context (two contexts never share a table filled on another stream), keyed by content so
  // a constraint rebuilt for every proof (the reference rebuilds them per sign / verify,
  // rpsss.rs:46,57) finds the tables of the last build instead of adding a set per build; and
  // sg_ctx_trim frees them
  std::vector<std::array<uint64_t, 4>> digest;
  ~MPolyDevice();
};

// The x-polynomials of a Rescue-Prime AIR (its round-constant interpolants first_0..m-1,
// second_0..m-1) and their values on the cosets the prover evaluates it on (public, kept like the
// context's domain tables).
struct RescueXPolys {
  // what determines the polynomials: RescuePrime::new's parameters (m, capacity, security, N:
  // the round constants follow from them, rescue_prime.rs:111-128) and the interpolation domain
  // (omicron, D). Their coset values live in the context's domain tables under
  // {kDomainRescueCoset, content..., poly, L, offset}: a rebuilt AIR reuses them.
  std::vector<uint64_t> content;
  std::vector<HPoly> polys;  // first_0 .. first_{m-1}, second_0 .. second_{m-1}
};

// A transition constraint built by the native Rescue-Prime AIR (rescue_prime.rs:246-283) also
// carries its factored form
//   sum_k MDS[i][k] prev_k^alpha + first_i(x) - (sum_k MDSinv[i][k] (next_k - second_k(x)))^alpha,
// the same polynomial as its expanded groups: the prover evaluates it pointwise in ~4 products per
// register instead of one product chain per expanded monomial (SG_AIR_GENERIC=1: the groups).
constexpr int kRescueMaxM = 4;
struct RescueAirForm {
  int m = 0, row = 0;
  uint32_t alpha = 0;
  fe mds[kRescueMaxM];     // MDS[row][k], canonical
  fe mds_inv[kRescueMaxM]; // MDSinv[row][k], canonical
  std::shared_ptr<const RescueXPolys> xp;
};

struct MPoly {
  uint32_t nvars = 0;                          // key length (0: empty dictionary)
  std::map<std::vector<uint32_t>, HPoly> g;    // exponents of variables 1..nvars-1 -> x coefficients
  // lazily built device copies, one per device (polynomials are immutable once built); a caller
  // holds the shared_ptr mp_device returns for as long as its kernels may read the copy
  mutable std::map<int, std::shared_ptr<const MPolyDevice>> dev;
  std::shared_ptr<const RescueAirForm> rescue; // set by the native Rescue-Prime AIR builder only
};

std::shared_ptr<const MPolyDevice> mp_device(sg_ctx* ctx, const MPoly& a);

MPoly mp_constant(const fe& c);
std::vector<MPoly> mp_variables(uint32_t n);
MPoly mp_lift(const HPoly& poly, uint32_t variable_index);
bool mp_is_zero(const MPoly& a);
MPoly mp_neg(const MPoly& a);
MPoly mp_add(const MPoly& a, const MPoly& b);
MPoly mp_sub(const MPoly& a, const MPoly& b);
MPoly mp_mul(sg_ctx* ctx, const MPoly& a, const MPoly& b);
MPoly mp_pow(sg_ctx* ctx, const MPoly& a, unsigned __int128 e);
fe mp_evaluate(const MPoly& a, const std::vector<fe>& point);
// exact product of two x-vectors (GPU NTT when large)
HPoly x_mul(sg_ctx* ctx, const HPoly& a, const HPoly& b);

}  // namespace sg

struct sg_mpoly {
  sg::MPoly m;
};
