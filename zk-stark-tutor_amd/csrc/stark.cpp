// Rescue-Prime (rescue_prime/rescue_prime.rs) and the end-to-end STARK prover
// (stark/stark.rs:71-562) over the device kernels, and their C ABI.
//
// Stark::prove on the GPU (BASELINE config C4):
//   trace columns --(geometric interpolation, poly.cpp)--> trace polynomials
//   boundary quotients: fast_coset_divide (the reference's algorithm, bit-exact)
//   boundary-quotient / randomizer LDEs + retained Merkle trees (kernels.hip)
//   transition polynomials: the AIR (grouped MPolynomial) evaluated pointwise on
//     a coset of size L > degree and interpolated back (the unique polynomial
//     evaluate_symbolic returns), then fast_coset_divide by the transition zerofier
//   combination polynomial (weighted, shifted terms) -> LDE -> FRI::prove
//   openings of the boundary-quotient and randomizer codewords, serialized on the device
//     together with the FRI query phase (TailWriter: one launch, one copy).
// The thread_rng draws (trace randomizers, randomizer polynomial) are explicit inputs.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <map>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "dist.hpp"
#include "host_field.hpp"
#include "host_hash.hpp"
#include "internal.hpp"
#include "mpoly.hpp"
#include "poly.hpp"
#include "poly_kernels.hpp"

namespace sg {

namespace {

unsigned __int128 u128_gcd(unsigned __int128 a, unsigned __int128 b) {
  while (b) {
    unsigned __int128 t = a % b;
    a = b;
    b = t;
  }
  return a;
}

int bitlen_count(unsigned __int128 x) {  // utils/bit_iter.rs BitIter::from(x).count()
  int n = 0;
  while (x) {
    ++n;
    x >>= 1;
  }
  return n ? n : 1;
}

std::string u128_decimal(unsigned __int128 v) {
  if (v == 0) return "0";
  std::string s;
  while (v) {
    s.push_back((char)('0' + (int)(v % 10)));
    v /= 10;
  }
  std::reverse(s.begin(), s.end());
  return s;
}

fe fe_div(const fe& a, const fe& b) {
  SG_REQUIRE(!fe_eq(b, fe_zero()), "divide by zero");
  return fe_mul(a, fe_inv(b));
}

using Mat = std::vector<std::vector<fe>>;

// utils/matrix.rs:5-49
void rref(Mat& m) {
  size_t lead = 0;
  const size_t rows = m.size(), cols = m[0].size();
  for (size_t r = 0; r < rows; ++r) {
    if (cols <= lead) break;
    size_t i = r;
    bool stop = false;
    while (fe_eq(m[i][lead], fe_zero())) {
      ++i;
      if (rows == i) {
        i = r;
        ++lead;
        if (cols == lead) {
          stop = true;
          break;
        }
      }
    }
    if (stop) break;
    std::swap(m[i], m[r]);
    if (!fe_eq(m[r][lead], fe_zero())) {
      fe piv = m[r][lead];
      for (auto& el : m[r]) el = fe_div(el, piv);
    }
    for (size_t ii = 0; ii < rows; ++ii) {
      if (ii == r) continue;
      fe hold = m[ii][lead];
      for (size_t k = 0; k < cols; ++k) m[ii][k] = fe_sub(m[ii][k], fe_mul(hold, m[r][k]));
    }
    ++lead;
  }
}

Mat transpose(const Mat& m) {
  Mat t(m[0].size(), std::vector<fe>(m.size()));
  for (size_t r = 0; r < m.size(); ++r)
    for (size_t c = 0; c < m[0].size(); ++c) t[c][r] = m[r][c];
  return t;
}

// utils/matrix.rs:68-110
Mat inverse(const Mat& m) {
  const size_t n = m.size();
  Mat aug(n);
  for (size_t i = 0; i < n; ++i) {
    SG_REQUIRE(m[i].size() == n, "Inverse exists only for square matrices");
    aug[i] = m[i];
    aug[i].resize(2 * n, fe_zero());
    aug[i][n + i] = fe_one();
  }
  rref(aug);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j)
      SG_REQUIRE(fe_eq(aug[i][j], i == j ? fe_one() : fe_zero()), "Couldnt construct identity matrix to find inverse");
  Mat out(n);
  for (size_t i = 0; i < n; ++i) out[i].assign(aug[i].begin() + n, aug[i].end());
  return out;
}

}  // namespace
}  // namespace sg

using namespace sg;

// ====================================================================== Rescue-Prime

struct sg_rescue {
  size_t m = 0, capacity = 0, security = 0, N = 0;
  unsigned __int128 alpha = 0, alpha_inv = 0;  // exponents (rescue_prime.rs:120-123)
  Mat mds, mds_inv;
  std::vector<fe> rc;  // 2 m N round constants

  // rescue_prime.rs:52-106, one round r
  void round(std::vector<fe>& state, size_t r) const {
    std::vector<fe> s(m), t(m, fe_zero());
    for (size_t i = 0; i < m; ++i) s[i] = fe_pow(state[i], alpha);
    for (size_t i = 0; i < m; ++i)
      for (size_t j = 0; j < m; ++j) t[j] = fe_add(t[j], fe_mul(mds[j][i], s[i]));
    for (size_t j = 0; j < m; ++j) t[j] = fe_pow(fe_add(t[j], rc[2 * r * m + j]), alpha_inv);
    std::vector<fe> u(m, fe_zero());
    for (size_t i = 0; i < m; ++i)
      for (size_t j = 0; j < m; ++j) u[j] = fe_add(u[j], fe_mul(mds[j][i], t[i]));
    for (size_t j = 0; j < m; ++j) state[j] = fe_add(u[j], rc[2 * r * m + m + j]);
  }
};

namespace {

void rescue_init(sg_rescue& rp, size_t m, size_t capacity, size_t security, size_t N) {
  SG_REQUIRE(m >= 1 && capacity <= m, "invalid Rescue-Prime state size");
  rp.m = m;
  rp.capacity = capacity;
  rp.security = security;
  rp.N = N;
  const unsigned __int128 p = fe_to_u128(fe_prime());
  // field.rs:46-56 smallest_generator
  unsigned __int128 k = 3;
  while (u128_gcd(k, p - 1) != 1) ++k;
  const fe g = fe_from_u128(k);
  rp.alpha = k;
  rp.alpha_inv = fe_to_u128(fe_inv(fe_neg(g)));
  // rescue_prime.rs:130-148 get_mds
  Mat mat(m, std::vector<fe>(2 * m));
  for (size_t i = 0; i < m; ++i)
    for (size_t j = 0; j < 2 * m; ++j) mat[i][j] = fe_pow(g, (unsigned __int128)(i * j));
  rref(mat);
  Mat right(m);
  for (size_t i = 0; i < m; ++i) right[i].assign(mat[i].begin() + m, mat[i].end());
  rp.mds = transpose(right);
  rp.mds_inv = inverse(rp.mds);
  // rescue_prime.rs:150-180 get_round_constants: 17-byte chunks of SHAKE256(seed), sum 256^j b_j
  const size_t bytes_per_int = (size_t)(bitlen_count(p) + 7) / 8 + 1;
  const size_t num = 2 * m * N;
  char seed[256];
  snprintf(seed, sizeof(seed), "Rescue-XLIX(%s,%zu,%zu,%zu)", u128_decimal(p).c_str(), m, capacity, security);
  std::vector<uint8_t> raw(bytes_per_int * std::max<size_t>(num, 1));
  shake256(reinterpret_cast<const uint8_t*>(seed), strlen(seed), raw.data(), bytes_per_int * num);
  rp.rc.resize(num);
  SG_REQUIRE(bytes_per_int == 17, "round constants: 17-byte chunks expected for this field");
  // sum_j 256^j b_j = L + b16 2^128 with L the little-endian u128 of bytes 0..15
  const fe two128 = fe_from_u128((unsigned __int128)0 - p);  // 2^128 mod p (2^128 < 2p)
  for (size_t i = 0; i < num; ++i) {
    const uint8_t* c = raw.data() + bytes_per_int * i;
    unsigned __int128 L = 0;
    for (int j = 15; j >= 0; --j) L = (L << 8) | c[j];
    rp.rc[i] = fe_add(fe_from_u128(L % p), fe_mul(fe_from_u64(c[16]), two128));
  }
}

std::vector<fe> rescue_trace(const sg_rescue& rp, const fe& input) {
  std::vector<fe> state(rp.m, fe_zero());
  state[0] = input;
  std::vector<fe> out;
  out.reserve((rp.N + 1) * rp.m);
  out.insert(out.end(), state.begin(), state.end());
  for (size_t r = 0; r < rp.N; ++r) {
    rp.round(state, r);
    out.insert(out.end(), state.begin(), state.end());
  }
  return out;
}

// rescue_prime.rs:206-283
std::vector<MPoly> rescue_transition_constraints(sg_ctx* ctx, const sg_rescue& rp, const fe& omicron, uint64_t D) {
  const size_t m = rp.m, N = rp.N;
  check_root(omicron, D);
  SG_REQUIRE(N <= D, "more rounds than the omicron domain");
  // round-constant interpolants over omicron^r, r < N (geometric domain, on the GPU)
  auto interp = [&](size_t which) {
    std::vector<fe> vals(N);
    for (size_t r = 0; r < N; ++r) vals[r] = rp.rc[2 * r * m + which];
    DPoly y = dpoly_upload(ctx, vals.data(), N);
    DPoly p = N > 1 ? interpolate_geometric_dev(ctx, omicron, D, y.p(), N) : std::move(y);
    return dpoly_download(ctx, p.p(), p.len);
  };
  auto xp = std::make_shared<RescueXPolys>();
  xp->content = {rp.m, rp.capacity, rp.security, rp.N, fe_lo(omicron), fe_hi(omicron), D};
  for (size_t i = 0; i < 2 * m; ++i) xp->polys.push_back(interp(i));  // first_0..m-1, second_0..m-1
  std::vector<MPoly> first(m), second(m);
  for (size_t i = 0; i < m; ++i) first[i] = mp_lift(xp->polys[i], 0);
  for (size_t i = 0; i < m; ++i) second[i] = mp_lift(xp->polys[m + i], 0);
  std::vector<MPoly> vars = mp_variables((uint32_t)(1 + 2 * m));
  std::vector<MPoly> out;
  for (size_t i = 0; i < m; ++i) {
    MPoly lhs;
    for (size_t k = 0; k < m; ++k) {
      MPoly t = mp_mul(ctx, mp_constant(rp.mds[i][k]), mp_pow(ctx, vars[1 + k], rp.alpha));
      lhs = k ? mp_add(lhs, t) : t;
    }
    lhs = mp_add(lhs, first[i]);
    MPoly rhs;
    for (size_t k = 0; k < m; ++k) {
      MPoly t = mp_mul(ctx, mp_constant(rp.mds_inv[i][k]), mp_sub(vars[1 + m + k], second[k]));
      rhs = k ? mp_add(rhs, t) : t;
    }
    rhs = mp_pow(ctx, rhs, rp.alpha);
    out.push_back(mp_sub(lhs, rhs));
    if (m <= (size_t)kRescueMaxM && rp.alpha >= 1 && rp.alpha <= 0xFFFFFFFFu) {
      auto form = std::make_shared<RescueAirForm>();
      form->m = (int)m;
      form->row = (int)i;
      form->alpha = (uint32_t)rp.alpha;
      for (size_t k = 0; k < m; ++k) {
        form->mds[k] = rp.mds[i][k];
        form->mds_inv[k] = rp.mds_inv[i][k];
      }
      form->xp = xp;
      out.back().rescue = form;
    }
  }
  return out;
}

}  // namespace

// ====================================================================== STARK

struct sg_stark {
  size_t expansion = 0, num_colinearity = 0, security = 0, m = 0, original_trace_length = 0, num_randomizers = 0;
  uint64_t D = 0;  // omicron_domain_length
  fe omicron, omega, generator;
  sg_fri fri;
};

namespace {

struct Boundary {
  uint64_t cycle, reg;
  fe value;
};

// stark.rs:117-160 (over the dictionary KEYS, i.e. group lengths here)
std::vector<uint64_t> transition_degree_bounds(const sg_stark& st, const std::vector<const MPoly*>& tcs) {
  std::vector<uint64_t> pd(2 * st.m + 1, (uint64_t)(st.original_trace_length + st.num_randomizers - 1));
  pd[0] = 1;
  std::vector<uint64_t> out;
  for (const MPoly* a : tcs) {
    SG_REQUIRE(!a->g.empty(), "cannot calculate max on empty vec a");
    uint64_t mx = 0;
    for (auto& kv : a->g) {
      // zip(points_degree, key): x exponent, then registers
      uint64_t s = 0;
      if (a->nvars >= 1 && !pd.empty()) s += pd[0] * (uint64_t)(kv.second.size() - 1);
      for (size_t j = 0; j < kv.first.size() && j + 1 < pd.size(); ++j) s += pd[j + 1] * kv.first[j];
      mx = std::max(mx, s);
    }
    out.push_back(mx);
  }
  return out;
}

std::vector<uint64_t> transition_quotient_degree_bounds(const sg_stark& st, const std::vector<const MPoly*>& tcs) {
  std::vector<uint64_t> b = transition_degree_bounds(st, tcs);
  for (auto& d : b) d -= (uint64_t)(st.original_trace_length - 1);
  return b;
}

uint64_t max_degree(const sg_stark& st, const std::vector<const MPoly*>& tcs) {
  SG_REQUIRE(!tcs.empty(), "Cannot calculate max for empty transition_constraints vector");
  std::vector<uint64_t> b = transition_degree_bounds(st, tcs);
  uint64_t md = *std::max_element(b.begin(), b.end());
  return ((uint64_t)1 << bitlen_count(md)) - 1;
}

fe omicron_pow(const sg_stark& st, uint64_t c) { return fe_pow(st.omicron, (unsigned __int128)c); }

std::vector<HPoly> boundary_zerofiers(const sg_stark& st, const std::vector<Boundary>& bnd) {
  std::vector<HPoly> out;
  for (size_t s = 0; s < st.m; ++s) {
    std::vector<fe> dom;
    for (auto& b : bnd)
      if (b.reg == s) dom.push_back(omicron_pow(st, b.cycle));
    out.push_back(hp_zerofier(dom));
  }
  return out;
}

std::vector<HPoly> boundary_interpolants(const sg_stark& st, const std::vector<Boundary>& bnd) {
  std::vector<HPoly> out;
  for (size_t s = 0; s < st.m; ++s) {
    std::vector<fe> dom, val;
    for (auto& b : bnd)
      if (b.reg == s) {
        dom.push_back(omicron_pow(st, b.cycle));
        val.push_back(b.value);
      }
    out.push_back(hp_interpolate(dom, val));
  }
  return out;
}

// x-exponent + (T'-1) * register-exponent sum over groups with a non-zero x vector:
// the length - 1 of the vector evaluate_symbolic builds (m_polynomial.rs:124-139)
uint64_t symbolic_degree_bound(const MPoly& a, uint64_t point_deg) {
  uint64_t mx = 0;
  for (auto& kv : a.g) {
    int64_t dx = hp_degree(kv.second);
    if (dx < 0) continue;
    uint64_t s = (uint64_t)dx;
    for (uint32_t e : kv.first) s += point_deg * e;
    mx = std::max(mx, s);
  }
  return mx;
}

struct DevTerm {
  const fe* p;
  uint64_t off, len;
  fe w;
};

uint64_t lincomb_len(const std::vector<DevTerm>& terms) {
  uint64_t n = 0;
  for (auto& t : terms) n = std::max(n, t.off + t.len);
  return n;
}

LinCombArgs lincomb_args(const std::vector<DevTerm>& terms) {
  SG_REQUIRE(terms.size() <= (size_t)kLinCombMaxTerms, "too many combination terms");
  LinCombArgs a{};
  a.nterms = (int)terms.size();
  for (size_t t = 0; t < terms.size(); ++t) {
    a.term[t] = terms[t].p;
    a.off[t] = terms[t].off;
    a.len[t] = terms[t].p ? terms[t].len : 0;
    a.w[t] = to_mont(terms[t].w);
  }
  return a;
}

// device linear combination sum_t w_t * x^off_t * term_t, output length max(off + len)
DPoly lincomb(sg_ctx* ctx, const std::vector<DevTerm>& terms) {
  const uint64_t n = lincomb_len(terms);
  DPoly out = dpoly_alloc(ctx, n);
  if (!n) return out;
  LinCombArgs a = lincomb_args(terms);
  a.out = out.p();
  a.n = n;
  SG_HIP(launch_lincomb(a, ctx->stream));
  return out;
}

// the same combination, only rows x row_len of its column shard: out[r][j] = coefficient
// base + r + n1 j (zero past its length) -- what the sharded LDE gathers, computed in place of it
void lincomb_cols(sg_ctx* ctx, const std::vector<DevTerm>& terms, uint64_t rows, uint64_t row_len, uint64_t n1,
                  uint64_t base, fe* out) {
  LinCombArgs a = lincomb_args(terms);
  a.out = out;
  a.n = rows * row_len;
  a.cols_row_len = row_len;
  a.cols_n1 = n1;
  a.cols_base = base;
  SG_HIP(launch_lincomb(a, ctx->stream));
}

// point values on the coset offset * <w_L>: P_s(y) and P_s(omicron y) (the point
// [x, P_s(x), P_s(omicron x)] of stark.rs:388-400), shared by every constraint.  When
// omicron lies in <w_L> (its order divides L: omicron = w_L^(L / order)), P_s(omicron y)
// at y = offset w_L^i is P_s at offset w_L^(i + L / order): the same values rotated, read
// with an index shift instead of a second transform.
struct AirCoset {
  uint64_t L = 0;
  std::vector<DPoly> V;         // distinct value arrays
  std::vector<int> var;         // point variable j -> index into V
  std::vector<uint64_t> shift;  // point variable j reads V[var[j]][(i + shift[j]) mod L]
};

AirCoset air_coset(sg_ctx* ctx, const std::vector<DPoly>& trace_polys, uint64_t L, const fe& omicron,
                   const fe& offset, uint64_t omicron_order) {
  AirCoset c;
  c.L = L;
  const fe wL = root_of_order(L);
  const bool rotate = omicron_order <= L && fe_eq(fe_pow(wL, L / omicron_order), omicron);
  const fe off_omicron = fe_mul(offset, omicron);
  for (int pass = 0; pass < 2; ++pass)
    for (size_t s = 0; s < trace_polys.size(); ++s) {
      if (pass && rotate) {
        c.var.push_back((int)s);
        c.shift.push_back(L / omicron_order);
        continue;
      }
      const DPoly& tp = trace_polys[s];
      c.V.push_back(dpoly_alloc(ctx, L));
      const fe* in = tp.p();
      fe* out = c.V.back().p();
      coset_evaluate_batch(ctx, wL, L, pass ? off_omicron : offset, &in, tp.len, &out, 1);
      c.var.push_back((int)c.V.size() - 1);
      c.shift.push_back(0);
    }
  return c;
}


// A Rescue-Prime row in its factored form (mpoly.hpp RescueAirForm) on the coset: the same values
// as the expanded polynomial.  Its round-constant interpolants' coset values are public and kept
// with the AIR (like the x-polynomial values of the generic path).
// values of a Rescue AIR x-polynomial (first_i / second_k) on offset * <w_L>, kept in the
// context's domain tables (content-keyed) unless SG_NO_DOMAIN_CACHE=1 (then owned by `keep`)
const fe* rescue_xvals(sg_ctx* ctx, const RescueAirForm& f, int idx, uint64_t L, const fe& offset,
                       std::vector<DevBuf>& keep) {
  const bool kept = ctx->domain_cache_on();
  std::vector<uint64_t> key = {kDomainRescueCoset};
  key.insert(key.end(), f.xp->content.begin(), f.xp->content.end());
  key.insert(key.end(), {(uint64_t)idx, L, fe_lo(offset), fe_hi(offset)});
  if (kept)
    if (void* t = ctx->domain_table(key)) return static_cast<const fe*>(t);
  const HPoly& hp = f.xp->polys[(size_t)idx];
  const int64_t deg = hp_degree(hp);
  void* t = nullptr;
  fe* out = nullptr;
  if (kept) {
    SG_HIP(hipMalloc(&t, L * sizeof(fe)));
    out = static_cast<fe*>(t);
  } else {
    keep.emplace_back(ctx, L * sizeof(fe));
    out = keep.back().as<fe>();
  }
  try {
    if (deg < 0) {
      SG_HIP(hipMemsetAsync(out, 0, L * sizeof(fe), ctx->stream));
    } else {
      DPoly in = dpoly_upload(ctx, hp.data(), (uint64_t)deg + 1);
      const fe* ip = in.p();
      coset_evaluate_batch(ctx, root_of_order(L), L, offset, &ip, (size_t)deg + 1, &out, 1);
      keep.push_back(std::move(in.buf));
    }
  } catch (...) {
    if (t) (void)hipFree(t);
    throw;
  }
  if (kept) ctx->domain_table_put(key, t);
  return out;
}

// This rank's run shard of a public table of L coset values (`full`, computed by every rank
// locally: no collective, so ranks whose caches differ stay in step), kept under `key` + (G, g).
// `bounded`: the shard of a table the replicated path keeps bounded (domain_table_put_bounded, e.g.
// the content-keyed boundary-divisor inverses) is kept the same way, so a prover that sees varying
// boundary zerofiers keeps a constant number of tables on the sharded path too.
const fe* shard_table(sg_dist* dd, std::vector<uint64_t> key, const fe* full, uint64_t L, std::vector<DevBuf>& keep,
                      bool bounded = false) {
  sg_ctx* ctx = dist_ctx(dd);
  const bool kept = ctx->domain_cache_on();
  key.insert(key.begin(), kDomainShard);
  key.push_back((uint64_t)dist_world(dd));
  key.push_back((uint64_t)dist_rank(dd));
  if (kept)
    if (void* t = ctx->domain_table(key)) return static_cast<const fe*>(t);
  const uint64_t n = L / (uint64_t)dist_world(dd);
  fe* out = nullptr;
  void* t = nullptr;
  if (kept) {
    SG_HIP(hipMalloc(&t, n * sizeof(fe)));
    out = static_cast<fe*>(t);
  } else {
    keep.emplace_back(ctx, n * sizeof(fe));
    out = keep.back().as<fe>();
  }
  try {
    dist_take_runs(dd, full, L, out);
  } catch (...) {
    if (t) {
      (void)hipStreamSynchronize(ctx->stream);  // the queued slice may still write it
      (void)hipFree(t);
    }
    throw;
  }
  if (kept) {
    if (bounded) ctx->domain_table_put_bounded(key, t);
    else ctx->domain_table_put(key, t);
  }
  return out;
}

// A Rescue-Prime row in its factored form (mpoly.hpp RescueAirForm) on the coset: the same values
// as the expanded polynomial.  Its round-constant interpolants' coset values are public and kept
// with the AIR (like the x-polynomial values of the generic path).  With `dd`, co holds this rank's
// run shards (co.L = L / G points, full_L = L) and the x-polynomial values are sliced to them.
DPoly transition_values_rescue(sg_ctx* ctx, const RescueAirForm& f, const AirCoset& co, const fe& offset,
                               std::vector<DevBuf>& keep, sg_dist* dd = nullptr, uint64_t full_L = 0) {
  const uint64_t L = co.L;
  const int m = f.m;
  auto xvals = [&](int idx) -> const fe* {
    if (!dd) return rescue_xvals(ctx, f, idx, L, offset, keep);
    const fe* full = rescue_xvals(ctx, f, idx, full_L, offset, keep);
    std::vector<uint64_t> key = {kDomainRescueCoset};
    key.insert(key.end(), f.xp->content.begin(), f.xp->content.end());
    key.insert(key.end(), {(uint64_t)idx, full_L, fe_lo(offset), fe_hi(offset)});
    return shard_table(dd, key, full, full_L, keep);
  };
  AirRescueArgs a{};
  DPoly vals = dpoly_alloc(ctx, L);
  a.out = vals.p();
  for (int j = 0; j < 2 * m; ++j) {
    a.V[j] = co.V[(size_t)co.var[(size_t)j]].p();
    a.vshift[j] = co.shift[(size_t)j];
  }
  a.first = xvals(f.row);
  for (int k = 0; k < m; ++k) {
    a.second[k] = xvals(m + k);
    a.mds[k] = f.mds[k];
    a.mds_inv_m[k] = to_mont(f.mds_inv[k]);
  }
  a.r2 = fe_r2();
  a.alpha = f.alpha;
  a.m = m;
  a.n = L;
  SG_HIP(launch_air_rescue(a, ctx->stream));
  return vals;
}

// values on the coset of the polynomial evaluate_symbolic returns (m_polynomial.rs:124-139).
// The x-polynomial values and the kernel's pointer tables move into `keep` (the caller's scope):
// they outlive the launch without a host wait.
DPoly transition_values(sg_ctx* ctx, const MPoly& tc, const AirCoset& co, const fe& offset,
                        std::vector<DevBuf>& keep) {
  if (tc.rescue && (int)co.var.size() == 2 * tc.rescue->m && !ctx->opt.air_generic)  // option air_generic: the expanded groups
    return transition_values_rescue(ctx, *tc.rescue, co, offset, keep);
  const uint64_t L = co.L;
  const int nv = (int)co.var.size();
  SG_REQUIRE(tc.nvars <= 1 + (uint32_t)nv, "transition constraint has more variables than the point");
  SG_REQUIRE(nv <= kAirMaxVars, "at most 4 registers are supported by the AIR kernel");
  // distinct group x-polynomials (device-resident, uploaded once per constraint) on the coset
  const std::shared_ptr<const MPolyDevice> xdp = mp_device(ctx, tc);
  const MPolyDevice& xd = *xdp;
  std::vector<DPoly> Q;        // values computed by this call (when not kept)
  std::vector<const fe*> qp;   // per distinct x-polynomial: its values on the coset
  const bool kept = ctx->domain_cache_on();
  for (size_t q = 0; q < xd.ptr.size(); ++q) {
    const auto& dg = xd.digest[q];
    const std::vector<uint64_t> key = {kDomainMpolyCoset, xd.len[q], dg[0], dg[1], dg[2], dg[3], L, fe_lo(offset),
                                       fe_hi(offset)};
    if (kept) {
      if (void* t = ctx->domain_table(key)) {
        qp.push_back(static_cast<const fe*>(t));
        continue;
      }
    }
    Q.push_back(dpoly_alloc(ctx, L));
    fe* out = Q.back().p();
    if (!xd.small[q].empty()) {  // a tiny polynomial (e.g. the constant 1): Horner at offset w_L^k
      SmallPoly sp{};
      sp.len = (int)xd.small[q].size();
      for (int i = 0; i < sp.len; ++i) sp.c[i] = xd.small[q][(size_t)i];
      const fe *A, *B;
      pow_tables2(ctx, root_of_order(L), L, &A, &B);
      SG_HIP(launch_eval_small(out, sp, L, A, B, to_mont(offset), ctx->stream));
    } else {
      const fe* in = reinterpret_cast<const fe*>(xd.ptr[q]);
      coset_evaluate_batch(ctx, root_of_order(L), L, offset, &in, xd.len[q], &out, 1);
    }
    if (kept) {
      void* t = nullptr;
      SG_HIP(hipMalloc(&t, L * sizeof(fe)));
      SG_HIP(hipMemcpyAsync(t, out, L * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
      ctx->domain_table_put(key, t);
      qp.push_back(static_cast<const fe*>(t));
    } else {
      qp.push_back(out);
    }
  }
  // non-zero groups bucketed by their distinct x-polynomial (an all-zero group adds nothing:
  // its products are zero polynomials)
  const size_t nq = xd.ptr.size();
  std::vector<std::vector<size_t>> by_q(nq);
  std::vector<const std::vector<uint32_t>*> keys;
  for (auto it = tc.g.begin(); it != tc.g.end(); ++it) keys.push_back(&it->first);
  for (size_t gi = 0; gi < keys.size(); ++gi)
    if (xd.qidx[gi] >= 0) by_q[(size_t)xd.qidx[gi]].push_back(gi);
  std::vector<uint32_t> exps, qstart{0};
  std::vector<fe> qscale;
  for (size_t q = 0; q < nq; ++q) {
    for (size_t gi : by_q[q]) {
      qscale.push_back(to_mont(xd.scale[gi]));
      for (int j = 0; j < nv; ++j) exps.push_back(j < (int)keys[gi]->size() ? (*keys[gi])[j] : 0u);
    }
    qstart.push_back((uint32_t)qscale.size());
  }
  DPoly vals = dpoly_alloc(ctx, L);
  if (qscale.empty()) {
    SG_HIP(hipMemsetAsync(vals.p(), 0, L * sizeof(fe), ctx->stream));
    return vals;
  }
  // one upload of the tables: [Q pointers][V pointers][qscale][qstart][exps]
  std::vector<uint8_t> tab;
  auto put = [&](const void* p, size_t bytes) {
    size_t o = (tab.size() + 15) & ~(size_t)15;
    tab.resize(o + bytes);
    memcpy(tab.data() + o, p, bytes);
    return o;
  };
  std::vector<const fe*> vp;
  for (int j = 0; j < nv; ++j) vp.push_back(co.V[co.var[j]].p());
  const size_t oq = put(qp.data(), qp.size() * sizeof(void*));
  const size_t ov = put(vp.data(), vp.size() * sizeof(void*));
  const size_t os = put(qscale.data(), qscale.size() * sizeof(fe));
  const size_t ot = put(qstart.data(), qstart.size() * 4);
  const size_t oe = put(exps.data(), exps.size() * 4);
  DevBuf dt(ctx, tab.size());
  SG_HIP(hipMemcpyAsync(dt.get(), tab.data(), tab.size(), hipMemcpyHostToDevice, ctx->stream));
  uint8_t* base = dt.as<uint8_t>();
  AirEvalArgs a{};
  a.out = vals.p();
  a.Q = reinterpret_cast<const fe* const*>(base + oq);
  a.V = reinterpret_cast<const fe* const*>(base + ov);
  a.qscale = reinterpret_cast<const fe*>(base + os);
  a.qstart = reinterpret_cast<const uint32_t*>(base + ot);
  a.exps = reinterpret_cast<const uint32_t*>(base + oe);
  a.ngroups = (int)qscale.size();
  a.nvars = nv;
  a.nq = (int)nq;
  a.n = L;
  a.r2 = fe_r2();
  a.one_m = to_mont(fe_one());
  for (int j = 0; j < nv; ++j) a.vshift[j] = co.shift[j];
  SG_HIP(launch_air_eval(a, ctx->stream));
  keep.push_back(std::move(dt));
  for (auto& q : Q) keep.push_back(std::move(q.buf));
  return vals;
}

std::vector<fe> sample_weights(size_t number, const uint8_t* randomness, size_t len) {
  // stark.rs:268-274: sample(0^i || randomness)
  std::vector<fe> out;
  std::vector<uint8_t> buf;
  for (size_t i = 0; i < number; ++i) {
    buf.assign(i, 0);
    buf.insert(buf.end(), randomness, randomness + len);
    out.push_back(fe_sample(buf.data(), buf.size()));
  }
  return out;
}

// Drains the side stream when the prover's scope ends (normally already joined; on an
// error it keeps the pool from handing out buffers a side-stream kernel still uses).
// Declared after the buffers the side stream touches, so it runs before they are released.
struct SideDrain {
  sg_ctx* ctx;
  ~SideDrain() { (void)hipStreamSynchronize(ctx->side); }
};

// launches of library helpers that use ctx->stream go to `s` inside the scope
struct StreamSwap {
  sg_ctx* ctx;
  hipStream_t prev;
  StreamSwap(sg_ctx* c, hipStream_t s) : ctx(c), prev(c->stream) { c->stream = s; }
  ~StreamSwap() { ctx->stream = prev; }
  StreamSwap(const StreamSwap&) = delete;
  StreamSwap& operator=(const StreamSwap&) = delete;
};

struct AsyncScope {
  sg_ctx* ctx;
  bool prev;
  explicit AsyncScope(sg_ctx* c) : ctx(c), prev(c->async_dev) { c->async_dev = true; }
  ~AsyncScope() { ctx->async_dev = prev; }
};

// The algebra of Stark::prove (stark.rs:285-512) on one context, in phases: the trace polynomials,
// the boundary quotients, the transition quotients with every quotient's degree, and the
// combination polynomial.  The single-GPU prover interleaves its codeword LDEs and side-stream
// trees between these phases; the sharded prover (sg_dist_stark_prove) runs them as they are on
// every rank (the trace-domain work is replicated, the codeword-domain work sharded).
struct ProveAlgebra {
  uint64_t Tp = 0;                     // randomized trace length
  std::vector<DPoly> trace_polys, bqs, tqs;
  std::vector<HPoly> bz;               // boundary zerofiers (host)
  std::vector<int64_t> qdeg;           // transition quotients' degrees, then the boundary quotients'
  std::vector<DPoly> wrapped;          // products that wrap the omicron domain (alive for the combination)
};

// interpolate_geometric_batch_dev (ntt_arithmetics.rs:172-237 on q^0..q^(n-1)) with its transforms
// on run shards: the f residue-class rows of every column (gathered from the replicated values as
// column shards) go through the distributed NTT, the pointwise products with the kernel rows and
// their sum run on the run shards, the inverse transform of the sum lands as column shards, the
// subgroup values are assembled there (scaled by 1/M) and one more distributed transform (root
// qf^-1) gives the coefficients as run shards, all-gathered into every rank's polynomial.  The
// public tables are the replicated path's (every rank builds them locally: no collective); the
// kernel rows are sliced to the rank's run shards.  Returns false (nothing done) where the plan
// does not split over the ranks; the caller then runs the replicated path.
bool interpolate_geometric_batch_dist(sg_dist* dd, const fe& q, uint64_t D, const fe* y, uint64_t ys, size_t cols,
                                      uint64_t n, std::vector<DPoly>& outs, std::vector<DevBuf>& keep) {
  sg_ctx* ctx = dist_ctx(dd);
  const int G = dist_world(dd);
  if (!dist_shard_algebra(dd) || n <= 1 || n >= D) return false;
  GeoInterpCache local;
  const GeoPlan P = geo_plan(ctx, q, D, n, &local, /*use_option=*/false);
  const uint64_t M = P.M, f = (uint64_t)1 << P.logf, Mf = M >> P.logf;
  if (P.logf < 1 || !dist_can_shard(M, G)) return false;
  uint64_t n1, n2;
  dist_plan(M, G, n1, n2);
  const uint64_t rows = n1 / (uint64_t)G, Ml = M / (uint64_t)G, row0 = (uint64_t)dist_rank(dd) * rows;
  const uint64_t row_len = std::max<uint64_t>((Mf + n1 - 1) / n1, 1);
  // residue-class rows of a_i = y_i / Z'(q^i) (replicated: cols * M elements), then their transforms
  DevBuf rowsbuf(ctx, cols * M * sizeof(fe));
  SG_HIP(launch_geo_rows(rowsbuf.as<fe>(), y, ys, P.Zdi, n, P.logf, M, cols, fe_r2(), ctx->stream));
  // all cols * f rows' column shards in one gather, their transforms as one batch (one exchange)
  const uint64_t nt = cols * f;
  DevBuf A(ctx, nt * Ml * sizeof(fe)), colsbuf(ctx, nt * rows * row_len * sizeof(fe));
  SG_HIP(launch_gather_cols(colsbuf.as<fe>(), rowsbuf.as<fe>(), Mf, rows, row_len, n1, row0, ctx->stream, nt, Mf));
  dist_ntt_batch(dd, P.qf, colsbuf.as<fe>(), row_len, M, A.as<fe>(), nt);
  // the kernel rows on this rank's run shards ([r][Ml], kept with the domain tables)
  std::vector<uint64_t> kkey = {kDomainGeoInterp, fe_lo(q), fe_hi(q), D, (uint64_t)P.logf, 0xB0B};
  const fe* K = nullptr;
  {
    std::vector<uint64_t> key = kkey;
    key.insert(key.begin(), kDomainShard);
    key.push_back((uint64_t)G);
    key.push_back((uint64_t)dist_rank(dd));
    const bool kept = ctx->domain_cache_on();
    if (kept) K = static_cast<const fe*>(ctx->domain_table(key));
    if (!K) {
      fe* out = nullptr;
      void* tbl = nullptr;
      if (kept) {
        SG_HIP(hipMalloc(&tbl, f * Ml * sizeof(fe)));
        out = static_cast<fe*>(tbl);
      } else {
        keep.emplace_back(ctx, f * Ml * sizeof(fe));
        out = keep.back().as<fe>();
      }
      try {
        for (uint64_t r = 0; r < f; ++r) dist_take_runs(dd, P.Khat + r * M, M, out + r * Ml);
      } catch (...) {
        if (tbl) (void)hipFree(tbl);
        throw;
      }
      if (kept) ctx->domain_table_put(key, tbl);
      K = out;
    }
  }
  DevBuf Shat(ctx, cols * Ml * sizeof(fe)), Scol(ctx, cols * Ml * sizeof(fe));
  SG_HIP(launch_geo_dot(Shat.as<fe>(), A.as<fe>(), K, P.logf, Ml, cols, fe_r2(), ctx->stream));
  dist_intt_batch(dd, P.qf, Shat.as<fe>(), M, Scol.as<fe>(), cols);
  // P(q^(f k)) / M on the column shards, then the coefficients (run shards) and every rank's copy
  const fe *iA, *iB;
  pow_tables2(ctx, fe_inv(q), D, &iA, &iB);
  const fe minv_m = to_mont(fe_inv(fe_from_u64(M)));
  DevBuf V(ctx, cols * Ml * sizeof(fe)), runs(ctx, cols * Ml * sizeof(fe));
  SG_HIP(launch_interp_assemble_cols(V.as<fe>(), y, ys, P.Zv, Scol.as<fe>(), n, P.logf, cols, rows, n2, n1, row0, iA, iB,
                                     minv_m, to_mont(minv_m), ctx->stream));
  const fe qfi = fe_inv(P.qf);
  dist_ntt_batch(dd, qfi, V.as<fe>(), n2, M, runs.as<fe>(), cols);
  std::vector<fe*> ptrs;
  for (size_t c = 0; c < cols; ++c) {
    DPoly out = dpoly_alloc(ctx, D);
    if (M < D) SG_HIP(hipMemsetAsync(out.p() + M, 0, (D - M) * sizeof(fe), ctx->stream));
    out.len = n;
    ptrs.push_back(out.p());
    outs.push_back(std::move(out));
  }
  dist_gather_runs_batch(dd, runs.as<fe>(), M, ptrs.data(), cols);
  dist_count_sharded_interpolation(dd, cols);
  return true;
}

// randomized trace (stark.rs:285-324): columns gathered on the device, geometric interpolation
// With `dd` (two ranks or more), the interpolation's transforms run on run shards
// (interpolate_geometric_batch_dist) where its plan splits over the ranks.
void prove_trace_polys(sg_ctx* ctx, const sg_stark& st, const fe* d_trace, size_t rows, const fe* d_trace_rand,
                       ProveAlgebra& A, sg_dist* dd = nullptr) {
  const size_t m = st.m;
  const uint64_t D = st.D, Tp = A.Tp;
  // randomized trace (stark.rs:285-301), columns on the device
  std::vector<DPoly>& trace_polys = A.trace_polys;
  {
    // the m columns side by side (column stride Tp), interpolated as one batch
    DPoly cols = dpoly_alloc(ctx, m * Tp);
    SG_HIP(launch_gather_trace_cols(cols.p(), d_trace, rows, d_trace_rand, st.num_randomizers, m, ctx->stream));
    std::vector<DevBuf> keep;
    if (!(dd && interpolate_geometric_batch_dist(dd, st.omicron, D, cols.p(), Tp, m, Tp, trace_polys, keep)))
      trace_polys = interpolate_geometric_batch_dev(ctx, st.omicron, D, cols.p(), Tp, m, Tp);
  }
}

// boundary quotients (stark.rs:326-362).  With `dd` (two ranks or more) a quotient whose division
// plan splits over the ranks runs its coset work on run shards: the numerator's distributed LDE on
// the coset, the product by 1 / the divisor's coset values (public: computed whole by every rank,
// sliced), the distributed coset interpolation and one all-gather -- the reference's truncated
// quotient, the same coefficients as fast_coset_divide_dev.
void prove_boundary_quotients(sg_ctx* ctx, const sg_stark& st, const std::vector<Boundary>& bnd, ProveAlgebra& A,
                              sg_dist* dd = nullptr) {
  const size_t m = st.m;
  const uint64_t D = st.D;
  const fe g = st.generator;
  // boundary quotients (stark.rs:326-362)
  std::vector<HPoly> bi = boundary_interpolants(st, bnd);
  A.bz = boundary_zerofiers(st, bnd);
  const std::vector<HPoly>& bz = A.bz;
  std::vector<DPoly>& bqs = A.bqs;
  const std::vector<DPoly>& trace_polys = A.trace_polys;
  {
    // every register's numerator first, then their degrees in one host round trip
    std::vector<DPoly> Zs, diffs;
    std::vector<std::pair<const fe*, uint64_t>> nums;
    for (size_t s = 0; s < m; ++s) {
      // the interpolant (host, a few coefficients) is subtracted straight from the kernel's
      // arguments; the zerofier goes to the device only if a path can read it there -- a division
      // by a small host divisor of degree >= 1 takes its coset values from the host copy (Horner,
      // ref_inner_ntt): two uploads fewer per register on the prove's critical path
      if (bi[s].size() <= (size_t)kSmallPolyMax) {
        SmallPoly sp{};
        sp.len = (int)bi[s].size();
        for (size_t k = 0; k < bi[s].size(); ++k) sp.c[k] = bi[s][k];
        DPoly d = dpoly_alloc(ctx, std::max<uint64_t>(trace_polys[s].len, bi[s].size()));
        if (d.len) SG_HIP(launch_sub_small(d.p(), trace_polys[s].p(), trace_polys[s].len, sp, ctx->stream));
        diffs.push_back(std::move(d));
      } else {
        DPoly I = dpoly_upload(ctx, bi[s].data(), bi[s].size());
        diffs.push_back(lincomb(ctx, {{trace_polys[s].p(), 0, trace_polys[s].len, fe_one()},
                                      {I.p(), 0, I.len, fe_neg(fe_one())}}));
      }
      const bool z_host_only = bz[s].size() <= (size_t)kSmallPolyMax && hp_degree(bz[s]) >= 1;
      Zs.push_back(z_host_only ? DPoly{} : dpoly_upload(ctx, bz[s].data(), bz[s].size()));
      nums.emplace_back(diffs.back().p(), diffs.back().len);
    }
    const std::vector<int64_t> dnum = dev_degrees(ctx, nums);
    // the sharded quotients of one coset size go through the distributed LDE, interpolation and
    // all-gather as one batch each; the others through the replicated division
    struct Sharded {
      size_t s;
      DivPlan pl;
      const fe* inv_shard;
    };
    std::vector<Sharded> sh;
    std::vector<DevBuf> keep;  // divisor tables (and their shards) until the batches are enqueued
    // the bounded divisor-shard tables sh[i].inv_shard stay allocated until the batches below are
    // enqueued: no eviction while later inserts (more shards, the replicated divisions) happen
    BoundedPin pin(ctx);
    const size_t b0 = bqs.size();
    bqs.resize(b0 + m);
    std::vector<DivItem> rep_items;
    std::vector<size_t> rep_slots;
    for (size_t s = 0; s < m; ++s) {
      const int64_t dz = hp_degree(bz[s]);
      // (the branch depends only on what every rank shares -- never on a per-rank environment)
      if (dd && dist_shard_algebra(dd) && dz >= 0 && dnum[s] >= dz && bz[s].size() <= 64) {
        const DivPlan pl = coset_divide_plan(st.omicron, D, dnum[s], dz);
        if (diffs[s].len <= pl.order && dist_can_shard(pl.order, dist_world(dd))) {
          const fe* inv = divisor_inverse_values(ctx, pl, g, Zs[s].p(), bz[s].size(), bz[s].data(), &keep);
          std::vector<uint64_t> key = {kDomainDivisorInverse, pl.order, fe_lo(pl.root), fe_hi(pl.root), fe_lo(g),
                                       fe_hi(g), bz[s].size()};
          for (const fe& c : bz[s]) {
            key.push_back(fe_lo(c));
            key.push_back(fe_hi(c));
          }
          sh.push_back(Sharded{s, pl, shard_table(dd, key, inv, pl.order, keep, /*bounded=*/true)});
          continue;
        }
      }
      rep_items.push_back(DivItem{diffs[s].p(), diffs[s].len, Zs[s].p(), bz[s].size(), dz, bz[s].data(), dnum[s]});
      rep_slots.push_back(b0 + s);
    }
    // the replicated quotients' coset divisions, their transforms batched (one coset size)
    {
      std::vector<DPoly> q = fast_coset_divide_batch_dev(ctx, st.omicron, D, g, rep_items);
      for (size_t k = 0; k < q.size(); ++k) bqs[rep_slots[k]] = std::move(q[k]);
    }
    for (size_t i0 = 0; i0 < sh.size();) {
      size_t i1 = i0 + 1;
      while (i1 < sh.size() && sh[i1].pl.order == sh[i0].pl.order) ++i1;
      const DivPlan& pl = sh[i0].pl;
      const uint64_t nv = i1 - i0, nl = pl.order / (uint64_t)dist_world(dd);
      std::vector<fe> offs(nv, g);
      std::vector<const fe*> srcs;
      std::vector<uint64_t> lens;
      std::vector<fe*> outs;
      for (size_t i = i0; i < i1; ++i) {
        srcs.push_back(diffs[sh[i].s].p());
        lens.push_back(diffs[sh[i].s].len);
      }
      DevBuf vals(ctx, nv * nl * sizeof(fe)), cols(ctx, nv * nl * sizeof(fe));
      dist_lde_replicated_batch(dd, pl.root, pl.order, offs.data(), srcs.data(), lens.data(), vals.as<fe>(), nv);
      for (size_t i = i0; i < i1; ++i) {
        fe* v = vals.as<fe>() + (i - i0) * nl;
        dev_mul(ctx, v, v, sh[i].inv_shard, nl);
        DPoly full = dpoly_alloc(ctx, pl.order);
        full.len = std::min(sh[i].pl.result_len, pl.order);  // the reference's truncation (coset_divide_finish)
        outs.push_back(full.p());
        bqs[b0 + sh[i].s] = std::move(full);
        dist_count_sharded_quotient(dd);
      }
      dist_coset_interpolate_batch(dd, pl.root, pl.order, g, vals.as<fe>(), cols.as<fe>(), nv);
      dist_gather_columns_batch(dd, cols.as<fe>(), pl.order, outs.data(), nv);
      i0 = i1;
    }
  }
}

// transition quotients (stark.rs:388-422) and every quotient's degree (one host round trip; a zero
// divisor is reported here, before any root is pushed)
//
// With `dd` (the sharded prove) and a native Rescue-Prime AIR, the coset work is
// split over the communicator: each rank evaluates the trace polynomials on its run shard of the
// coset (2m distributed LDEs: current rows at offset g, next rows at g * omicron), the factored AIR
// and the division by the zerofier there, and the quotient's coset interpolation (distributed INTT);
// one all-gather then hands every rank the whole quotient, so the degree checks, the combination
// and the proof bytes are those of the replicated path.  The public tables (x-polynomial and
// zerofier values) are computed whole by every rank with no collective and sliced to its shard.
void prove_transition_quotients(sg_ctx* ctx, const sg_stark& st, const std::vector<const MPoly*>& tcs,
                                ProveAlgebra& A, sg_dist* dd = nullptr, const std::function<void()>& overlap = {}) {
  const uint64_t D = st.D, Tp = A.Tp;
  const fe g = st.generator;
  const std::vector<DPoly>& trace_polys = A.trace_polys;
  const std::vector<DPoly>& bqs = A.bqs;
  // transition quotients (stark.rs:388-422): evaluate_symbolic's polynomial from its values on a
  // coset of size L > its length, then fast_coset_divide by the transition zerofier.  When the
  // division's order equals L its lhs NTT IS those coset values (same offset, same root), so
  // they are reused; the zerofier's NTT is shared by all constraints.
  const uint64_t T = st.original_trace_length;
  SG_REQUIRE(T >= 2, "transition zerofier needs a trace of at least two rows");
  // The transition zerofier prod_{i < T-1} (x - omicron^i), its coset values and their inverses
  // depend on the public domain only (omicron, D, T, the coset offset): the context keeps them
  // like twiddle plans (sg_ctx::domain_tables; SG_NO_DOMAIN_CACHE=1 recomputes them per prove).
  const bool dcache = ctx->domain_cache_on() && T - 1 < D;
  const std::vector<uint64_t> tz_key = {kDomainTzCoeffs, fe_lo(st.omicron), fe_hi(st.omicron), D, T};
  DPoly tz_own;
  const fe* tz_p = dcache ? static_cast<const fe*>(ctx->domain_table(tz_key)) : nullptr;
  uint64_t tz_len = T;  // T - 1 < D: length T (no wrap-around)
  if (!tz_p) {
    tz_own = zerofier_geometric_dev(ctx, st.omicron, D, T - 1);
    tz_p = tz_own.p();
    tz_len = tz_own.len;
    if (dcache) {
      void* t = nullptr;
      SG_HIP(hipMalloc(&t, tz_len * sizeof(fe)));
      SG_HIP(hipMemcpyAsync(t, tz_p, tz_len * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
      ctx->domain_table_put(tz_key, t);
    }
  }
  // prod_{i < T-1} (x - omicron^i) is monic of degree T - 1 (< D: no wrap-around)
  const int64_t dtz = tz_len == T && T - 1 < D ? (int64_t)(T - 1) : dev_degree(ctx, tz_p, tz_len);
  std::vector<DevBuf> air_keep;  // AIR tables and x-polynomial values, alive until the quotients are done
  std::map<uint64_t, AirCoset> cosets;
  std::map<uint64_t, std::pair<DevBuf, uint64_t>> tz_ntt;  // order -> NTT of scale(tz, g)
  std::vector<DPoly>& tqs = A.tqs;
  auto tz_key_at = [&](uint64_t tag, const DivPlan& pl) {
    return std::vector<uint64_t>{tag, fe_lo(st.omicron), fe_hi(st.omicron), D, T, pl.order, fe_lo(pl.root),
                                 fe_hi(pl.root), fe_lo(g), fe_hi(g)};
  };
  auto tz_values = [&](const DivPlan& pl) -> const fe* {
    const std::vector<uint64_t> key = tz_key_at(kDomainTzValues, pl);
    if (dcache)
      if (void* t = ctx->domain_table(key)) return static_cast<const fe*>(t);
    auto zit = tz_ntt.find(pl.order);
    if (zit == tz_ntt.end()) {
      std::pair<DevBuf, uint64_t> z;
      ref_inner_ntt(ctx, pl.root, pl.order, tz_p, tz_len, &g, z.first, z.second);
      zit = tz_ntt.emplace(pl.order, std::move(z)).first;
    }
    if (dcache) {
      void* t = nullptr;
      SG_HIP(hipMalloc(&t, zit->second.second * sizeof(fe)));
      SG_HIP(hipMemcpyAsync(t, zit->second.first.get(), zit->second.second * sizeof(fe), hipMemcpyDeviceToDevice,
                            ctx->stream));
      ctx->domain_table_put(key, t);
      return static_cast<const fe*>(t);
    }
    return zit->second.first.as<fe>();
  };
  // 1 / tz on the coset, for the fast path's division (a product by the cached inverse: the field's
  // a / b is a * b^-1, field_element.rs:82-90, so the quotient is the same).  Built once per
  // domain; the build checks for a zero divisor before the table is kept.
  auto tz_inverse = [&](const DivPlan& pl) -> const fe* {
    const std::vector<uint64_t> key = tz_key_at(kDomainTzInverse, pl);
    if (void* t = ctx->domain_table(key)) return static_cast<const fe*>(t);
    void* t = nullptr;
    SG_HIP(hipMalloc(&t, pl.order * sizeof(fe)));
    dev_div(ctx, static_cast<fe*>(t), nullptr, tz_values(pl), pl.order);
    host_wait(ctx, ctx->stream);
    try {
      check_div_zero(ctx);
    } catch (...) {
      (void)hipFree(t);
      throw;
    }
    ctx->domain_table_put(key, t);
    return static_cast<const fe*>(t);
  };
  // the reference's steps (inexact division or a degree below L/2)
  auto general_quotient = [&](const DPoly& vals, uint64_t len, uint64_t L) -> DPoly {
    DPoly coeffs = dpoly_alloc(ctx, L);
    coset_interpolate_dev(ctx, vals.p(), L, g, coeffs.p());  // coefficients len..L-1 are zero
    const DivPlan pl = coset_divide_plan(st.omicron, D, dev_degree(ctx, coeffs.p(), len), dtz);
    if (pl.zero_lhs) return DPoly{};
    DevBuf lhs_own;
    fe* lhs_v = vals.p();
    if (!(pl.order == L && len <= pl.order)) {
      uint64_t nl;
      ref_inner_ntt(ctx, pl.root, pl.order, coeffs.p(), len, &g, lhs_own, nl);
      lhs_v = lhs_own.as<fe>();
    }
    return coset_divide_finish(ctx, pl, g, lhs_v, tz_values(pl));
  };
  // Fast path: if the division by Z is exact, q = INTT(vals / Z) has degree dl - dr <= len - 1 - dr
  // and then dl = deg(q) + dr exactly (q Z agrees with the transition polynomial on L > its
  // degree points); with dl >= L/2 the reference's order is L, its lhs NTT is `vals` and its
  // truncated quotient is q -- no coefficient transform of the lhs is needed.  Whether it holds
  // depends on deg(q), which is read with every other quotient's degree in one round trip below;
  // a constraint that fails the check (an inexact division: a false witness) is then redone the
  // reference's way.
  struct Pending {
    size_t idx;
    DPoly vals;  // the transition values on the coset (sharded: this rank's run shard)
    uint64_t len, L;
    bool sharded = false;
  };
  std::vector<Pending> pending;
  // the sharded coset work applies when every constraint carries the factored Rescue form, all
  // share one coset size Ls on the fast path (L <= D, deg Z < len), and Ls splits over the ranks;
  // the decision depends only on inputs every rank shares, so all ranks take the same branch
  // (one rank: its "shard" is the whole coset, which the replicated path evaluates with half the
  // transforms -- the next-row values are a rotation there)
  uint64_t Ls = 0;
  bool sharded = dd && dist_shard_algebra(dd) && !tcs.empty();
  for (const MPoly* tc : tcs) {
    if (!sharded) break;
    const uint64_t len = symbolic_degree_bound(*tc, Tp - 1) + 1;
    const uint64_t L = next_pow2(len);
    if (!tc->rescue || (size_t)tc->rescue->m != trace_polys.size() || !(L <= D && (uint64_t)dtz < len) ||
        (Ls && L != Ls))
      sharded = false;
    Ls = L;
  }
  if (sharded) sharded = dist_can_shard(Ls, dist_world(dd));
  AirCoset sco;  // this rank's run shards of the coset values (sharded)
  const fe* tz_shard = nullptr;
  bool tz_shard_inverse = false;
  if (sharded) {
    const int G = dist_world(dd);
    const fe wL = root_of_order(Ls);
    sco.L = Ls / (uint64_t)G;
    // the 2m distributed LDEs as one batch (one exchange), then each run shard into its array
    std::vector<fe> offs;
    std::vector<const fe*> srcs;
    std::vector<uint64_t> lens;
    for (int pass = 0; pass < 2; ++pass)
      for (size_t s = 0; s < trace_polys.size(); ++s) {
        offs.push_back(pass ? fe_mul(g, st.omicron) : g);
        srcs.push_back(trace_polys[s].p());
        lens.push_back(trace_polys[s].len);
      }
    DevBuf lde(ctx, offs.size() * sco.L * sizeof(fe));
    dist_lde_replicated_batch(dd, wL, Ls, offs.data(), srcs.data(), lens.data(), lde.as<fe>(), offs.size());
    for (size_t v = 0; v < offs.size(); ++v) {
      sco.V.push_back(dpoly_alloc(ctx, sco.L));
      SG_HIP(hipMemcpyAsync(sco.V.back().p(), lde.as<fe>() + v * sco.L, sco.L * sizeof(fe), hipMemcpyDeviceToDevice,
                            ctx->stream));
      sco.var.push_back((int)sco.V.size() - 1);
      sco.shift.push_back(0);
    }
    DivPlan pl;
    pl.root = wL;
    pl.order = Ls;
    tz_shard_inverse = dcache;
    tz_shard = dcache ? shard_table(dd, tz_key_at(kDomainTzInverse, pl), tz_inverse(pl), Ls, air_keep)
                      : shard_table(dd, tz_key_at(kDomainTzValues, pl), tz_values(pl), Ls, air_keep);
  }
  if (sharded) {
    // every constraint's quotient values on the rank's run shard, then their coset interpolations
    // and all-gathers as one batch each (one exchange apiece for all constraints)
    const uint64_t nl = sco.L, nq = tcs.size();
    DevBuf qv(ctx, nq * nl * sizeof(fe)), cols(ctx, nq * nl * sizeof(fe));
    std::vector<fe*> outs;
    for (size_t q = 0; q < nq; ++q) {
      const uint64_t len = symbolic_degree_bound(*tcs[q], Tp - 1) + 1;
      DPoly vals = transition_values_rescue(ctx, *tcs[q]->rescue, sco, g, air_keep, dd, Ls);
      if (tz_shard_inverse) dev_mul(ctx, qv.as<fe>() + q * nl, vals.p(), tz_shard, nl);
      else dev_div(ctx, qv.as<fe>() + q * nl, vals.p(), tz_shard, nl);
      DPoly out = dpoly_alloc(ctx, Ls);  // all Ls coefficients, on every rank
      outs.push_back(out.p());
      pending.push_back(Pending{tqs.size(), std::move(vals), len, Ls, true});
      dist_count_sharded_quotient(dd);
      tqs.push_back(std::move(out));
    }
    dist_coset_interpolate_batch(dd, root_of_order(Ls), Ls, g, qv.as<fe>(), cols.as<fe>(), nq);
    dist_gather_columns_batch(dd, cols.as<fe>(), Ls, outs.data(), nq);
  }
  for (const MPoly* tc : tcs) {
    if (sharded) break;
    const uint64_t len = symbolic_degree_bound(*tc, Tp - 1) + 1;
    const uint64_t L = next_pow2(len);
    auto cit = cosets.find(L);
    if (cit == cosets.end()) cit = cosets.emplace(L, air_coset(ctx, trace_polys, L, st.omicron, g, st.D)).first;
    DPoly vals = transition_values(ctx, *tc, cit->second, g, air_keep);
    if (L <= D && (uint64_t)dtz < len) {
      DivPlan pl;
      pl.root = root_of_order(L);
      pl.order = L;
      DevBuf qv(ctx, L * sizeof(fe)), qc(ctx, L * sizeof(fe));
      if (dcache) dev_mul(ctx, qv.as<fe>(), vals.p(), tz_inverse(pl), L);
      else dev_div(ctx, qv.as<fe>(), vals.p(), tz_values(pl), L);
      intt_sized(ctx, pl.root, qv.as<fe>(), ilog2_exact(L), qc.as<fe>());
      DPoly out = dpoly_alloc(ctx, L);  // all L coefficients unscaled: zeros stay zero
      dev_scale_pow(ctx, out.p(), qc.as<fe>(), L, fe_inv(g));
      pending.push_back(Pending{tqs.size(), std::move(vals), len, L});
      tqs.push_back(std::move(out));
      continue;
    }
    tqs.push_back(general_quotient(vals, len, L));
  }
  // every quotient's degree with one host round trip (checked after the weights, as the
  // reference does, and used again by the terms below); it drains the main stream past
  // every division, so a zero divisor is reported before any root is pushed
  auto quotient_degrees = [&]() {
    std::vector<std::pair<const fe*, uint64_t>> qpolys;
    for (const DPoly& q : tqs) qpolys.emplace_back(q.p(), q.len);
    for (const DPoly& q : bqs) qpolys.emplace_back(q.p(), q.len);
    return dev_degrees(ctx, qpolys);
  };
  std::vector<int64_t>& qdeg = A.qdeg;
  {
    // the caller's host work (stark_prove: roots, weights, the speculative combination) runs
    // between the degree scans' launch and the wait for their published results
    std::vector<std::pair<const fe*, uint64_t>> qpolys;
    for (const DPoly& q : tqs) qpolys.emplace_back(q.p(), q.len);
    for (const DPoly& q : bqs) qpolys.emplace_back(q.p(), q.len);
    const DegScan scan = dev_degrees_begin(ctx, qpolys);
    if (overlap) overlap();
    qdeg = dev_degrees_end(ctx, scan);
  }
  check_div_zero(ctx);
  bool redone = false;
  for (Pending& pd : pending) {
    const int64_t dq = qdeg[pd.idx];
    const uint64_t dl = (uint64_t)dq + (uint64_t)dtz;
    if (dq >= 0 && dl <= pd.len - 1 && std::max<uint64_t>(dl, (uint64_t)dtz) >= pd.L / 2) {
      tqs[pd.idx].len = (uint64_t)dq + 1;  // the reference's truncated quotient
    } else {
      if (pd.sharded) {  // the reference's steps on the whole coset: every rank gathers the values
        DPoly full = dpoly_alloc(ctx, pd.L);
        dist_gather_runs(dd, pd.vals.p(), pd.L, full.p());
        pd.vals = std::move(full);
      }
      tqs[pd.idx] = general_quotient(pd.vals, pd.len, pd.L);
      redone = true;
    }
  }
  if (redone) {
    qdeg = quotient_degrees();
    check_div_zero(ctx);
  }
}

// the degree check (stark.rs:451-465) and the combination polynomial's terms (stark.rs:467-512)
std::vector<DevTerm> combination_terms(sg_ctx* ctx, const sg_stark& st, const std::vector<const MPoly*>& tcs, ProveAlgebra& A,
                        const std::vector<fe>& weights, const fe* d_rcoef, size_t nrc, uint64_t tcd) {
  const size_t m = st.m;
  const uint64_t D = st.D, Tp = A.Tp;
  const std::vector<DPoly>& tqs = A.tqs;
  const std::vector<DPoly>& bqs = A.bqs;
  const std::vector<HPoly>& bz = A.bz;
  const std::vector<int64_t>& qdeg = A.qdeg;
  // degree check (stark.rs:451-465)
  std::vector<uint64_t> tqdb = transition_quotient_degree_bounds(st, tcs);
  for (size_t i = 0; i < tqs.size(); ++i) {
    int64_t d = qdeg[i];
    SG_REQUIRE(d >= 0, "Failed to get degree of transition quotient");
    SG_REQUIRE((uint64_t)d == tqdb[i], "transition quotient degrees do not match with expectation");
  }
  // terms + combination (stark.rs:467-512): x^shift * q via fast_multiply is the exact shift
  std::vector<uint64_t> bqdb;
  for (size_t s = 0; s < m; ++s) {
    int64_t dz = hp_degree(bz[s]);
    SG_REQUIRE(dz >= 0, "Couldnt get degree of boundary zerofier");
    bqdb.push_back(Tp - 1 - (uint64_t)dz);
  }
  std::vector<DevTerm> terms;
  std::vector<DPoly>& wrapped = A.wrapped;  // products that wrap the omicron domain (alive for the combination)
  wrapped.reserve(2 * (tqs.size() + bqs.size()));
  size_t wi = 0;
  terms.push_back({d_rcoef, 0, nrc, weights[wi++]});
  auto add_pair = [&](const DPoly& q, uint64_t shift, int64_t d) {
    terms.push_back({q.p(), 0, q.len, weights[wi++]});
    const fe w = weights[wi++];
    if (d < 0) return;  // fast_multiply of a zero polynomial is the empty polynomial
    if (shift + (uint64_t)d < D) {
      // no wrap-around: fast_multiply(x^shift, q) is exactly q shifted, truncated at its degree
      terms.push_back({q.p(), shift, (uint64_t)d + 1, w});
    } else {
      // degree >= omicron order: the reference's NTT product wraps; reproduce it step by step
      std::vector<fe> xs(shift + 1, fe_zero());
      xs[shift] = fe_one();
      DPoly dx = dpoly_upload(ctx, xs.data(), xs.size());
      wrapped.push_back(fast_multiply_dev(ctx, st.omicron, D, dx.p(), dx.len, q.p(), q.len));
      terms.push_back({wrapped.back().p(), 0, wrapped.back().len, w});
    }
  };
  for (size_t i = 0; i < tqs.size(); ++i) add_pair(tqs[i], tcd - tqdb[i], qdeg[i]);
  for (size_t s = 0; s < m; ++s) add_pair(bqs[s], tcd - bqdb[s], qdeg[tqs.size() + s]);
  return terms;
}

// combination_terms as they will be if every quotient has its expected degree (transition: its
// degree bound, truncated to it; boundary: its division's result length), built before the degrees
// are known; empty when the expectation is not well defined (a truncation past the quotient's
// coefficients, a product wrapping the omicron domain).  stark_prove compares it with the real terms.
std::vector<DevTerm> speculative_terms(const sg_stark& st, const std::vector<const MPoly*>& tcs, const ProveAlgebra& A,
                                       const std::vector<fe>& weights, const fe* d_rcoef, size_t nrc, uint64_t tcd) {
  const uint64_t D = st.D, Tp = A.Tp;
  const std::vector<uint64_t> tqdb = transition_quotient_degree_bounds(st, tcs);
  std::vector<DevTerm> terms;
  size_t wi = 0;
  terms.push_back({d_rcoef, 0, nrc, weights[wi++]});
  auto add_pair = [&](const fe* p, uint64_t len, uint64_t shift, int64_t d) -> bool {
    terms.push_back({p, 0, len, weights[wi++]});
    const fe w = weights[wi++];
    if (d < 0) return true;
    if (shift + (uint64_t)d >= D) return false;
    terms.push_back({p, shift, (uint64_t)d + 1, w});
    return true;
  };
  for (size_t i = 0; i < A.tqs.size(); ++i) {
    if (tqdb[i] + 1 > A.tqs[i].len) return {};
    if (!add_pair(A.tqs[i].p(), tqdb[i] + 1, tcd - tqdb[i], (int64_t)tqdb[i])) return {};
  }
  for (size_t s = 0; s < A.bqs.size(); ++s) {
    const int64_t dz = hp_degree(A.bz[s]);
    if (dz < 0) return {};
    const uint64_t bqdb = Tp - 1 - (uint64_t)dz;
    if (!add_pair(A.bqs[s].p(), A.bqs[s].len, tcd - bqdb, (int64_t)A.bqs[s].len - 1)) return {};
  }
  return terms;
}

bool same_terms(const std::vector<DevTerm>& a, const std::vector<DevTerm>& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (a[i].p != b[i].p || a[i].off != b[i].off || a[i].len != b[i].len || !fe_eq(a[i].w, b[i].w)) return false;
  return true;
}


// stark.rs:276-562
// d_trace: rows x m (row-major), d_trace_rand: num_randomizers x m, d_rcoef: nrc -- all on the device
void stark_prove(sg_ctx* ctx, const sg_stark& st, const fe* d_trace, size_t rows,
                 const std::vector<const MPoly*>& tcs, const std::vector<Boundary>& bnd, const fe* d_trace_rand,
                 const fe* d_rcoef, size_t nrc, const sg_proof_stream* ps) {
  SG_REQUIRE(ps && ps->push && ps->fiat_shamir_prover, "proof stream callbacks required");
  const size_t m = st.m;
  const uint64_t D = st.D;
  const fe g = st.generator;
  const uint64_t Nf = st.fri.domain_length;
  AsyncScope async_scope(ctx);
  PhaseMarks mark;
  const uint64_t Tp = rows + st.num_randomizers;
  SG_REQUIRE(Tp <= D, "randomized trace longer than the omicron domain");
  const uint64_t tcd = max_degree(st, tcs);
  SG_REQUIRE(nrc == tcd + 1, "randomizer polynomial must have max_degree(transition_constraints) + 1 coefficients");
  SG_REQUIRE(nrc <= Nf, "fast_coset_evaluate: polynomial longer than root_order");
  // The Merkle trees of the boundary-quotient and randomizer codewords (VALU-bound BLAKE2b)
  // run on the side stream, overlapped with the main stream's transforms and quotients
  // (which mostly wait on memory).  Everything a side-stream kernel touches is allocated
  // here, with the main stream drained: a pool buffer released by queued main-stream work
  // can then never be handed to a side-stream kernel.
  SG_REQUIRE(m <= 4, "at most 4 registers are supported by the AIR kernel");  // root slots 0..m-1, 4
  host_wait(ctx, ctx->stream);
  std::vector<DPoly> bq_cw;
  std::vector<std::unique_ptr<sg_tree>> bq_trees(m);
  for (size_t s = 0; s < m; ++s) bq_cw.push_back(dpoly_alloc(ctx, Nf));
  DPoly r_cw = dpoly_alloc(ctx, Nf);
  // lean trees: the openings rehash a leaf sibling from these codewords, which live to the end
  for (size_t s = 0; s < m; ++s) bq_trees[s] = new_tree(ctx, Nf, bq_cw[s].p(), 3);
  std::unique_ptr<sg_tree> r_tree = new_tree(ctx, Nf, r_cw.p(), 3);
  SideDrain side_drain{ctx};
  // randomizer codeword (stark.rs:424-445) first: it depends on nothing else, so its LDE and
  // its tree run on the side stream while the main stream interpolates the trace.  The tables
  // the LDE reads are created (cached) on the main stream before the fork: the side stream
  // allocates nothing and only launches the transform passes and the tree.
  constexpr int kRandSlot = 4;
  uint64_t r_seq = 0, bq_seq;
  // where the side stream forks off the randomizer LDE + tree: 0 = at the start (beside the trace
  // interpolation), 1 = after the interpolation, 2 = after the boundary quotients
  // (SG_PROVE_R_FORK in A/B builds, scheduling experiments; the bytes are the same)
  const int r_fork = SG_KNOB(PROVE_R_FORK, 0);
  (void)ctx->stage_twiddles(st.omega, ilog2_exact(next_pow2(Nf)));
  (void)ctx->pow_table(g, 4096);
  (void)ctx->pow_table(fe_pow(g, 4096), (std::max<uint64_t>(nrc, 1) + 4095) / 4096);
  auto fork_randomizer = [&]() {
    SG_HIP(hipEventRecord(ctx->ev_fork, ctx->stream));
    SG_HIP(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    const fe* in = d_rcoef;
    fe* out = r_cw.p();
    {
      StreamSwap on_side(ctx, ctx->side);
      coset_evaluate_batch(ctx, st.omega, Nf, g, &in, nrc, &out, 1);
    }
    const fe* leaves = r_cw.p();
    sg_tree* t = r_tree.get();
    r_seq = launch_trees(ctx, &leaves, 1, &t, kRandSlot, ctx->side);
  };
  if (r_fork <= 0) fork_randomizer();
  ProveAlgebra A;
  A.Tp = Tp;
  prove_trace_polys(ctx, st, d_trace, rows, d_trace_rand, A);
  mark("trace_interpolation");
  if (r_fork == 1) fork_randomizer();
  prove_boundary_quotients(ctx, st, bnd, A);
  mark("boundary_quotients");
  if (r_fork >= 2) fork_randomizer();
  const std::vector<DPoly>& bqs = A.bqs;
  // boundary-quotient codewords (stark.rs:367-386); their trees hash on the side stream
  // while the main stream computes the transition quotients
  for (size_t s = 0; s < m; ++s) {
    SG_REQUIRE(bqs[s].len <= Nf, "fast_coset_evaluate: polynomial longer than root_order");
    const fe* in = bqs[s].p();
    fe* out = bq_cw[s].p();
    if (bqs[s].len)
      coset_evaluate_batch(ctx, st.omega, Nf, g, &in, bqs[s].len, &out, 1);
    else
      SG_HIP(hipMemsetAsync(out, 0, Nf * sizeof(fe), ctx->stream));
  }
  {
    SG_HIP(hipEventRecord(ctx->ev_fork, ctx->stream));
    SG_HIP(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    const fe* leaves[4];
    sg_tree* t[4];
    for (size_t s = 0; s < m; ++s) {
      leaves[s] = bq_cw[s].p();
      t[s] = bq_trees[s].get();
    }
    bq_seq = launch_trees(ctx, leaves, (int)m, t, 0, ctx->side);
    SG_HIP(hipEventRecord(ctx->ev_join, ctx->side));
  }
  mark("bq_lde");
  // The roots, the weights and a speculative combination are done while the quotient degrees are
  // scanned (prove_transition_quotients' overlap hook): the weights depend only on the roots, and
  // the combination's terms on the degrees only through the truncations -- taken as the expected
  // ones (transition: the degree bounds, which any other degree turns into an error anyway;
  // boundary: the division's result length).  Once the degrees are known the real terms are built
  // (combination_terms: the reference's degree checks, stark.rs:451-465); when they differ from
  // the speculative ones in any pointer, offset, length or weight the combination is computed
  // again (stream-ordered, overwriting the speculative codeword), so the bytes never depend on it.
  std::vector<fe> weights;
  auto roots_and_weights = [&]() {
    // roots in the reference's order: boundary quotients (stark.rs:373-386), randomizer (:443)
    sg_tree* t[4];
    for (size_t s = 0; s < m; ++s) t[s] = bq_trees[s].get();
    finish_trees(ctx, t, (int)m, bq_seq, 0, ctx->side);
    sg_tree* rt = r_tree.get();
    finish_trees(ctx, &rt, 1, r_seq, kRandSlot, ctx->side);
    // the main stream joins the side stream only where it reads the side stream's output (the
    // openings below): the combination, its LDE and FRI do not, and a cross-stream wait enqueued
    // here held the combination back ~50 us behind the last tree kernel's completion signal
    for (size_t s = 0; s < m; ++s) push_obj(ps, SG_OBJ_ROOT, bq_trees[s]->root, 64);
    push_obj(ps, SG_OBJ_ROOT, r_tree->root, 64);
    // weights (stark.rs:447-450)
    uint8_t fs[32];
    if (ps->fiat_shamir_prover(ps->user, 32, fs) != 0)
      throw Error{SG_ERR_CALLBACK, "proof stream fiat_shamir callback failed"};
    weights = sample_weights(1 + 2 * A.tqs.size() + 2 * bqs.size(), fs, 32);
  };
  DPoly comb_cw, comb;
  auto combination_lde = [&](const std::vector<DevTerm>& terms) {
    if (!comb_cw.len) comb_cw = dpoly_alloc(ctx, Nf);
    comb = lincomb(ctx, terms);
    SG_REQUIRE(comb.len <= Nf, "fast_coset_evaluate: polynomial longer than root_order");
    const fe* in = comb.p();
    fe* out = comb_cw.p();
    coset_evaluate_batch(ctx, st.omega, Nf, g, &in, comb.len, &out, 1);
  };
  std::vector<DevTerm> spec;
  prove_transition_quotients(ctx, st, tcs, A, nullptr, [&]() {
    roots_and_weights();
    spec = speculative_terms(st, tcs, A, weights, d_rcoef, nrc, tcd);
    if (!spec.empty()) combination_lde(spec);
  });
  mark("transition_quotients");
  if (weights.empty()) roots_and_weights();
  mark("trees_joined");
  const std::vector<DevTerm> terms = combination_terms(ctx, st, tcs, A, weights, d_rcoef, nrc, tcd);
  if (!same_terms(terms, spec)) combination_lde(terms);
  mark("combination_lde");
  // FRI (stark.rs:514-522) and the openings (stark.rs:524-560): the openings' indices follow from
  // FRI's top-level indices, so their Value / Path objects join the FRI query phase's single
  // device serialization (TailWriter)
  std::vector<size_t> top(st.fri.num_colinearity_tests);
  std::vector<std::pair<const fe*, const sg_tree*>> cts;
  for (size_t s = 0; s < m; ++s) cts.emplace_back(bq_cw[s].p(), bq_trees[s].get());
  cts.emplace_back(r_cw.p(), r_tree.get());
  // the openings: for every codeword (boundary quotients, randomizer), a Value and a Path at each
  // of the 4c sorted indices {i, i + expansion, and both + Nf/2} (mod Nf) of the top indices i,
  // table entries c .. 5c - 1 (stark.rs:524-560)
  const size_t c = st.fri.num_colinearity_tests;
  TailExtra openings;
  openings.count = 4 * c;
  openings.plan = [&](TailWriter& tw, uint32_t sel0) {
    SG_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));  // the openings read the side-stream trees
    for (auto& ct : cts)
      for (uint32_t j = 0; j < 4 * c; ++j) {
        tw.value(ct.first, Nf, sel0 + j);
        tw.path(ct.second, sel0 + j, ~0ull);
      }
  };
  openings.indices = [&](const size_t* tp, std::vector<uint64_t>& table) {
    std::vector<uint64_t> quad;
    quad.reserve(4 * c);
    for (size_t k = 0; k < c; ++k) quad.push_back(tp[k]);
    for (size_t k = 0; k < c; ++k) quad.push_back((tp[k] + st.expansion) % Nf);
    for (size_t k = 0; k < 2 * c; ++k) quad.push_back((quad[k] + Nf / 2) % Nf);
    std::sort(quad.begin(), quad.end());
    table.insert(table.end(), quad.begin(), quad.end());
  };
  fri_prove_dev(ctx, &st.fri, comb_cw.p(), Nf, ps, top.data(), &openings);
  mark("fri_prove_and_openings");
  host_wait(ctx, ctx->stream);
  check_div_zero(ctx);
  mark("openings");
}

// Stark::prove (stark.rs:276-562) with its codeword-domain work sharded over a communicator
// (the domain can outgrow one GPU): every rank runs the trace-domain algebra
// (interpolation, quotients, the combination polynomial -- size D = N_fri / expansion) on its own
// copy, and the N_fri-sized work on its run shards: the four LDEs (from the replicated
// coefficients), the three commitments (forests + top trees, kept), FRI::prove (sg_dist_fri_prove)
// and the openings, each from the rank that owns the leaf.  Every rank writes the single-GPU bytes.
void stark_prove_dist(sg_dist* dd, const sg_stark& st, const fe* d_trace, size_t rows,
                      const std::vector<const MPoly*>& tcs, const std::vector<Boundary>& bnd, const fe* d_trace_rand,
                      const fe* d_rcoef, size_t nrc, const sg_proof_stream* ps) {
  SG_REQUIRE(ps && ps->push && ps->fiat_shamir_prover, "proof stream callbacks required");
  sg_ctx* ctx = dist_ctx(dd);
  const size_t m = st.m;
  const uint64_t D = st.D;
  const fe g = st.generator;
  const uint64_t Nf = st.fri.domain_length;
  const uint64_t Tp = rows + st.num_randomizers;
  SG_REQUIRE(Tp <= D, "randomized trace longer than the omicron domain");
  const uint64_t tcd = max_degree(st, tcs);
  SG_REQUIRE(nrc == tcd + 1, "randomizer polynomial must have max_degree(transition_constraints) + 1 coefficients");
  SG_REQUIRE(nrc <= Nf, "fast_coset_evaluate: polynomial longer than root_order");
  SG_REQUIRE(m <= 4, "at most 4 registers are supported by the AIR kernel");
  // a FRI domain too small to split over this many ranks (N1 >= G, N2 >= 4 G) is proved whole
  // by every rank: the same bytes, no collective
  const int G = dist_world(dd);
  const uint64_t p1 = dist_split(Nf), p2 = Nf / p1;
  if (p1 % (uint64_t)G != 0 || p2 % (4 * (uint64_t)G) != 0) {
    stark_prove(ctx, st, d_trace, rows, tcs, bnd, d_trace_rand, d_rcoef, nrc, ps);
    return;
  }
  // one rank: its "shard" is the whole domain and every collective an identity, so the single-GPU
  // prove is the plan (same bytes; at the headline the four-step path costs ~6 ms more per proof).
  // The context option world1_sharded forces the four-step path anyway (tests that exercise the
  // sharded machinery over a one-rank RCCL communicator; one rank, so no cross-rank agreement).
  if (G == 1) {
    if (!ctx->opt.world1_sharded) {
      stark_prove(ctx, st, d_trace, rows, tcs, bnd, d_trace_rand, d_rcoef, nrc, ps);
      return;
    }
  }
  uint64_t n1, n2;
  dist_plan(Nf, G, n1, n2);
  const uint64_t R = n2 / G, shard = n1 * R;
  PhaseMarks mark;
  // The forests of the boundary-quotient and randomizer codewords hash on the side stream while
  // the main stream runs the algebra (as in the single-GPU prove); their run-root all-gathers and
  // top trees follow on the main stream, where every collective of the communicator stays.  The
  // buffers side-stream kernels touch are allocated here, with the main stream drained.
  host_wait(ctx, ctx->stream);
  std::vector<DevBuf> runs;
  std::vector<PendingForest> forests(m + 1);
  for (size_t s = 0; s <= m; ++s) {
    runs.emplace_back(ctx, shard * sizeof(fe));
    dist_forest_alloc(dd, n1, R, forests[s]);
  }
  SideDrain side_drain{ctx};
  auto fork_forests = [&](size_t s0, size_t s1) {
    SG_HIP(hipEventRecord(ctx->ev_fork, ctx->stream));
    SG_HIP(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    for (size_t s = s0; s < s1; ++s) dist_forest_launch(dd, runs[s].as<fe>(), forests[s], ctx->side);
  };
  auto lde = [&](const fe* coeffs, uint64_t len, DevBuf& out) {
    SG_REQUIRE(len <= Nf, "fast_coset_evaluate: polynomial longer than root_order");
    if (len) dist_lde_replicated(dd, st.omega, Nf, g, coeffs, len, out.as<fe>());
    else SG_HIP(hipMemsetAsync(out.get(), 0, shard * sizeof(fe), ctx->stream));
  };
  // randomizer codeword (stark.rs:424-445) first: it depends on nothing else, so its forest hashes
  // beside the trace interpolation and the boundary quotients
  lde(d_rcoef, nrc, runs[m]);
  fork_forests(m, m + 1);
  ProveAlgebra A;
  A.Tp = Tp;
  prove_trace_polys(ctx, st, d_trace, rows, d_trace_rand, A, dd);
  prove_boundary_quotients(ctx, st, bnd, A, dd);
  mark("dist_algebra_boundary");
  // boundary-quotient codewords (stark.rs:364-386), their forests on the side stream
  for (size_t s = 0; s < m; ++s) lde(A.bqs[s].p(), A.bqs[s].len, runs[s]);
  fork_forests(0, m);
  mark("dist_bq_lde");
  prove_transition_quotients(ctx, st, tcs, A, dd);
  mark("dist_transition_quotients");
  SG_HIP(hipEventRecord(ctx->ev_join, ctx->side));
  SG_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
  // run roots all-gathered, top trees, roots in the reference's order
  std::vector<ShardedRound> rounds(m + 1);
  std::vector<std::array<uint8_t, 64>> roots(m + 1);
  for (size_t s = 0; s <= m; ++s) {
    dist_forest_finish(dd, forests[s], roots[s].data(), &rounds[s]);
    rounds[s].cw = runs[s].as<fe>();
  }
  mark("dist_commitments");
  for (size_t s = 0; s <= m; ++s) push_obj(ps, SG_OBJ_ROOT, roots[s].data(), 64);
  uint8_t fs[32];
  if (ps->fiat_shamir_prover(ps->user, 32, fs) != 0)
    throw Error{SG_ERR_CALLBACK, "proof stream fiat_shamir callback failed"};
  std::vector<fe> weights = sample_weights(1 + 2 * A.tqs.size() + 2 * A.bqs.size(), fs, 32);
  // the combination (stark.rs:467-512) only as this rank's column shard of its coefficients --
  // 1/G of the replicated elementwise sum, and the LDE's column gather with it
  const std::vector<DevTerm> terms = combination_terms(ctx, st, tcs, A, weights, d_rcoef, nrc, tcd);
  const uint64_t clen = lincomb_len(terms);
  SG_REQUIRE(clen <= Nf, "fast_coset_evaluate: polynomial longer than root_order");
  DevBuf comb_runs(ctx, shard * sizeof(fe));
  {
    const uint64_t rows = n1 / (uint64_t)G, row_len = std::max<uint64_t>((clen + n1 - 1) / n1, 1);
    DevBuf cols(ctx, rows * row_len * sizeof(fe));
    lincomb_cols(ctx, terms, rows, row_len, n1, (uint64_t)dist_rank(dd) * rows, cols.as<fe>());
    dist_coset_evaluate(dd, st.omega, Nf, g, cols.as<fe>(), row_len, comb_runs.as<fe>());
  }
  mark("dist_combination_lde");
  // FRI (stark.rs:514-522), then the openings (stark.rs:524-560) of the boundary-quotient and
  // randomizer codewords at the quadrupled indices, each value + path from the leaf's owner
  std::vector<size_t> top(st.fri.num_colinearity_tests);
  dist_fri_prove(dd, &st.fri, comb_runs.as<fe>(), Nf, ps, top.data(), [&](const size_t* tp) {
    const size_t c = st.fri.num_colinearity_tests;
    std::vector<uint64_t> dup;
    for (size_t k = 0; k < c; ++k) dup.push_back(tp[k]);
    for (size_t k = 0; k < c; ++k) dup.push_back((tp[k] + st.expansion) % Nf);
    std::vector<uint64_t> quad = dup;
    for (uint64_t i : dup) quad.push_back((i + Nf / 2) % Nf);
    std::sort(quad.begin(), quad.end());
    std::vector<OpenReq> reqs(m + 1);
    for (size_t s = 0; s <= m; ++s) {
      reqs[s].sr = &rounds[s];
      reqs[s].I = quad;
    }
    dist_open_batch(dd, R, n2, reqs);  // all m + 1 codewords: one all-gather
    for (size_t s = 0; s <= m; ++s) {
      const int depth = reqs[s].depth;
      std::vector<uint8_t> pl(72 * (size_t)depth);
      for (size_t k = 0; k < quad.size(); ++k) {
        uint8_t v[16];
        put_u128_be_at(v, reqs[s].vals[k]);
        push_obj(ps, SG_OBJ_VALUE, v, 16);
        for (int l = 0; l < depth; ++l) {
          uint8_t* o = pl.data() + 72 * (size_t)l;
          memset(o, 0, 8);
          o[7] = 64;
          memcpy(o + 8, reqs[s].paths.data() + (k * (size_t)depth + (size_t)l) * 64, 64);
        }
        push_obj(ps, SG_OBJ_PATH, pl.data(), pl.size());
      }
    }
  });
  mark("dist_fri_prove_and_openings");
  host_wait(ctx, ctx->stream);
  check_div_zero(ctx);
}

std::vector<const MPoly*> tc_list(const sg_mpoly* const* tcs, size_t n) {
  std::vector<const MPoly*> v;
  for (size_t i = 0; i < n; ++i) {
    SG_REQUIRE(tcs[i], "null transition constraint");
    v.push_back(&tcs[i]->m);
  }
  return v;
}

}  // namespace

// ====================================================================== C ABI: Rescue-Prime

extern "C" int sg_rescue_create(sg_ctx* ctx, size_t m, size_t capacity, size_t security_level, size_t N,
                                sg_rescue** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out, "null argument");
    std::unique_ptr<sg_rescue> rp(new sg_rescue());
    rescue_init(*rp, m, capacity, security_level, N);
    *out = rp.release();
  });
}

extern "C" void sg_rescue_free(sg_rescue* rp) { delete rp; }

extern "C" int sg_rescue_info(const sg_rescue* rp, sg_fe* alpha, sg_fe* alpha_inv, sg_fe* mds, sg_fe* mds_inv,
                              sg_fe* round_constants) {
  if (!rp) return SG_ERR_INVALID;
  if (alpha) *alpha = from_fe(fe_from_u128(rp->alpha));
  if (alpha_inv) *alpha_inv = from_fe(fe_from_u128(rp->alpha_inv));
  for (size_t i = 0; i < rp->m; ++i)
    for (size_t j = 0; j < rp->m; ++j) {
      if (mds) mds[i * rp->m + j] = from_fe(rp->mds[i][j]);
      if (mds_inv) mds_inv[i * rp->m + j] = from_fe(rp->mds_inv[i][j]);
    }
  if (round_constants)
    for (size_t i = 0; i < rp->rc.size(); ++i) round_constants[i] = from_fe(rp->rc[i]);
  return SG_OK;
}

extern "C" int sg_rescue_hash(sg_ctx* ctx, const sg_rescue* rp, sg_fe input, sg_fe* out) {
  return guard(ctx, [&] {
    SG_REQUIRE(rp && out, "null argument");
    SG_REQUIRE(rp->capacity == 1, "Received wrong number of input elements");
    check_canonical(&input, 1, "input");
    std::vector<fe> state(rp->m, fe_zero());
    state[0] = to_fe(input);
    for (size_t r = 0; r < rp->N; ++r) rp->round(state, r);
    *out = from_fe(state[0]);
  });
}

extern "C" int sg_rescue_trace(sg_ctx* ctx, const sg_rescue* rp, sg_fe input, sg_fe* trace) {
  return guard(ctx, [&] {
    SG_REQUIRE(rp && trace, "null argument");
    SG_REQUIRE(rp->capacity == 1, "Received wrong number of input elements");
    check_canonical(&input, 1, "input");
    std::vector<fe> t = rescue_trace(*rp, to_fe(input));
    memcpy(trace, t.data(), t.size() * sizeof(fe));
  });
}

extern "C" int sg_rescue_transition_constraints(sg_ctx* ctx, const sg_rescue* rp, sg_fe omicron,
                                                uint64_t omicron_domain_length, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(ctx && rp && out, "a GPU context is required (interpolation on the device)");
    set_device(ctx);
    std::vector<MPoly> tcs = rescue_transition_constraints(ctx, *rp, to_fe(omicron), omicron_domain_length);
    host_wait(ctx, ctx->stream);
    check_div_zero(ctx);
    for (size_t i = 0; i < tcs.size(); ++i) {
      out[i] = new sg_mpoly();
      out[i]->m = std::move(tcs[i]);
    }
  });
}

extern "C" int sg_rescue_boundary_constraints(const sg_rescue* rp, sg_fe output, sg_boundary* out) {
  if (!rp || !out) return SG_ERR_INVALID;
  // rescue_prime.rs:285-290
  out[0] = sg_boundary{0, 1, sg_fe{0, 0}};
  out[1] = sg_boundary{rp->N, 0, output};
  return SG_OK;
}

// ====================================================================== C ABI: STARK

extern "C" int sg_stark_create(sg_ctx* ctx, size_t expansion_factor, size_t num_colinearity_checks,
                               size_t security_level, size_t num_registers, size_t num_cycles,
                               size_t transition_constraints_degree, sg_stark** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out, "null argument");
    // stark.rs:71-114
    SG_REQUIRE((size_t)bitlen_count(fe_to_u128(fe_prime())) >= security_level, "field order has to be at least security_level bits");
    SG_REQUIRE(expansion_factor && (expansion_factor & (expansion_factor - 1)) == 0,
               "expansion_factor must be a power of 2");
    SG_REQUIRE(expansion_factor >= 4, "expansion_factor must be at least 4");
    SG_REQUIRE(num_colinearity_checks * 2 >= security_level,
               "number of collinearity checks must be at least half of security_level");
    std::unique_ptr<sg_stark> st(new sg_stark());
    st->expansion = expansion_factor;
    st->num_colinearity = num_colinearity_checks;
    st->security = security_level;
    st->m = num_registers;
    st->original_trace_length = num_cycles;
    st->num_randomizers = 4 * num_colinearity_checks;
    const uint64_t randomized = num_cycles + st->num_randomizers;
    const int bl = bitlen_count((unsigned __int128)randomized * transition_constraints_degree);
    SG_REQUIRE(bl <= 40, "omicron domain too large");
    st->D = (uint64_t)1 << bl;
    const uint64_t Nf = st->D * expansion_factor;
    st->generator = fe_generator();
    st->omega = root_of_order(Nf);
    st->omicron = root_of_order(st->D);
    st->fri.offset = from_fe(st->generator);
    st->fri.omega = from_fe(st->omega);
    st->fri.domain_length = Nf;
    st->fri.expansion_factor = expansion_factor;
    st->fri.num_colinearity_tests = num_colinearity_checks;
    *out = st.release();
  });
}

extern "C" void sg_stark_free(sg_stark* st) { delete st; }

extern "C" int sg_stark_params(const sg_stark* st, sg_fe* omicron, uint64_t* omicron_domain_length, sg_fri* fri,
                               size_t* num_randomizers) {
  if (!st) return SG_ERR_INVALID;
  if (omicron) *omicron = from_fe(st->omicron);
  if (omicron_domain_length) *omicron_domain_length = st->D;
  if (fri) *fri = st->fri;
  if (num_randomizers) *num_randomizers = st->num_randomizers;
  return SG_OK;
}

extern "C" int sg_stark_max_degree(sg_ctx* ctx, const sg_stark* st, const sg_mpoly* const* tcs, size_t ntcs,
                                   uint64_t* out) {
  return guard(ctx, [&] {
    SG_REQUIRE(st && out && (tcs || !ntcs), "null argument");
    *out = max_degree(*st, tc_list(tcs, ntcs));
  });
}

extern "C" int sg_stark_degree_bounds(sg_ctx* ctx, const sg_stark* st, const sg_mpoly* const* tcs, size_t ntcs,
                                      uint64_t* transition_bounds) {
  return guard(ctx, [&] {
    SG_REQUIRE(st && transition_bounds && (tcs || !ntcs), "null argument");
    std::vector<uint64_t> b = transition_degree_bounds(*st, tc_list(tcs, ntcs));
    std::copy(b.begin(), b.end(), transition_bounds);
  });
}

extern "C" int sg_stark_prove(sg_ctx* ctx, const sg_stark* st, const sg_fe* trace, size_t rows,
                              const sg_mpoly* const* tcs, size_t ntcs, const sg_boundary* boundary, size_t nb,
                              const sg_fe* trace_randomizers, const sg_fe* randomizer_coeffs, size_t n_rc,
                              const sg_proof_stream* ps) {
  return guard(ctx, [&] {
    SG_REQUIRE(ctx && st && (trace || !rows) && (tcs || !ntcs) && (boundary || !nb), "null argument");
    SG_REQUIRE(trace_randomizers || !st->num_randomizers, "null argument");
    set_device(ctx);
    check_canonical(trace, rows * st->m, "trace");
    check_canonical(trace_randomizers, st->num_randomizers * st->m, "trace randomizers");
    check_canonical(randomizer_coeffs, n_rc, "randomizer coefficients");
    std::vector<Boundary> bnd;
    for (size_t i = 0; i < nb; ++i) {
      check_canonical(&boundary[i].value, 1, "boundary value");
      SG_REQUIRE(boundary[i].reg < st->m, "boundary register out of range");
      bnd.push_back({boundary[i].cycle, boundary[i].reg, to_fe(boundary[i].value)});
    }
    DPoly dt = dpoly_upload(ctx, reinterpret_cast<const fe*>(trace), rows * st->m);
    DPoly dr = dpoly_upload(ctx, reinterpret_cast<const fe*>(trace_randomizers), st->num_randomizers * st->m);
    DPoly dc = dpoly_upload(ctx, reinterpret_cast<const fe*>(randomizer_coeffs), n_rc);
    host_wait(ctx, ctx->stream);
    stark_prove(ctx, *st, dt.p(), rows, tc_list(tcs, ntcs), bnd, dr.p(), dc.p(), n_rc, ps);
  });
}

extern "C" int sg_stark_prove_dev(sg_ctx* ctx, const sg_stark* st, const sg_fe* d_trace, size_t rows,
                                  const sg_mpoly* const* tcs, size_t ntcs, const sg_boundary* boundary, size_t nb,
                                  const sg_fe* d_trace_randomizers, const sg_fe* d_randomizer_coeffs, size_t n_rc,
                                  const sg_proof_stream* ps) {
  return guard(ctx, [&] {
    SG_REQUIRE(ctx && st && (d_trace || !rows) && (tcs || !ntcs) && (boundary || !nb), "null argument");
    SG_REQUIRE(d_trace_randomizers || !st->num_randomizers, "null argument");
    set_device(ctx);
    std::vector<Boundary> bnd;
    for (size_t i = 0; i < nb; ++i) {
      check_canonical(&boundary[i].value, 1, "boundary value");
      SG_REQUIRE(boundary[i].reg < st->m, "boundary register out of range");
      bnd.push_back({boundary[i].cycle, boundary[i].reg, to_fe(boundary[i].value)});
    }
    stark_prove(ctx, *st, reinterpret_cast<const fe*>(d_trace), rows, tc_list(tcs, ntcs), bnd,
                reinterpret_cast<const fe*>(d_trace_randomizers), reinterpret_cast<const fe*>(d_randomizer_coeffs),
                n_rc, ps);
  });
}

// ====================================================================== C ABI: sharded STARK

namespace {
int dist_prove_entry(sg_dist* d, const sg_stark* st, const sg_fe* trace, size_t rows, const sg_mpoly* const* tcs,
                     size_t ntcs, const sg_boundary* boundary, size_t nb, const sg_fe* trace_randomizers,
                     const sg_fe* randomizer_coeffs, size_t n_rc, const sg_proof_stream* ps, bool host) {
  return dist_run(d, [&] {
    sg_ctx* ctx = dist_ctx(d);
    SG_REQUIRE(st && (trace || !rows) && (tcs || !ntcs) && (boundary || !nb), "null argument");
    SG_REQUIRE(trace_randomizers || !st->num_randomizers, "null argument");
    std::vector<Boundary> bnd;
    for (size_t i = 0; i < nb; ++i) {
      check_canonical(&boundary[i].value, 1, "boundary value");
      SG_REQUIRE(boundary[i].reg < st->m, "boundary register out of range");
      bnd.push_back({boundary[i].cycle, boundary[i].reg, to_fe(boundary[i].value)});
    }
    if (!host) {
      stark_prove_dist(d, *st, reinterpret_cast<const fe*>(trace), rows, tc_list(tcs, ntcs), bnd,
                       reinterpret_cast<const fe*>(trace_randomizers), reinterpret_cast<const fe*>(randomizer_coeffs),
                       n_rc, ps);
      return;
    }
    check_canonical(trace, rows * st->m, "trace");
    check_canonical(trace_randomizers, st->num_randomizers * st->m, "trace randomizers");
    check_canonical(randomizer_coeffs, n_rc, "randomizer coefficients");
    DPoly dt = dpoly_upload(ctx, reinterpret_cast<const fe*>(trace), rows * st->m);
    DPoly dr = dpoly_upload(ctx, reinterpret_cast<const fe*>(trace_randomizers), st->num_randomizers * st->m);
    DPoly dc = dpoly_upload(ctx, reinterpret_cast<const fe*>(randomizer_coeffs), n_rc);
    host_wait(ctx, ctx->stream);
    stark_prove_dist(d, *st, dt.p(), rows, tc_list(tcs, ntcs), bnd, dr.p(), dc.p(), n_rc, ps);
  });
}
}  // namespace

extern "C" int sg_dist_stark_prove(sg_dist* d, const sg_stark* st, const sg_fe* trace, size_t rows,
                                   const sg_mpoly* const* tcs, size_t ntcs, const sg_boundary* boundary, size_t nb,
                                   const sg_fe* trace_randomizers, const sg_fe* randomizer_coeffs, size_t n_rc,
                                   const sg_proof_stream* ps) {
  return dist_prove_entry(d, st, trace, rows, tcs, ntcs, boundary, nb, trace_randomizers, randomizer_coeffs, n_rc, ps,
                          true);
}

extern "C" int sg_dist_stark_prove_dev(sg_dist* d, const sg_stark* st, const sg_fe* d_trace, size_t rows,
                                       const sg_mpoly* const* tcs, size_t ntcs, const sg_boundary* boundary, size_t nb,
                                       const sg_fe* d_trace_randomizers, const sg_fe* d_randomizer_coeffs, size_t n_rc,
                                       const sg_proof_stream* ps) {
  return dist_prove_entry(d, st, d_trace, rows, tcs, ntcs, boundary, nb, d_trace_randomizers, d_randomizer_coeffs,
                          n_rc, ps, false);
}
