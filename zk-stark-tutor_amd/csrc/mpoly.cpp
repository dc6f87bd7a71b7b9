// MPolynomial (m_polynomial.rs) in grouped form, and its C ABI.  See mpoly.hpp.
#include <atomic>
#include <mutex>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "host_field.hpp"
#include "host_hash.hpp"
#include "internal.hpp"
#include "mpoly.hpp"
#include "poly_kernels.hpp"

namespace sg {

namespace {
bool is_zero_fe(const fe& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }

// dictionary union on one group: values added, length = the larger key set
void dense_add_into(HPoly& acc, const HPoly& b) {
  if (acc.size() < b.size()) acc.resize(b.size(), fe_zero());
  for (size_t i = 0; i < b.size(); ++i) acc[i] = fe_add(acc[i], b[i]);
}

std::vector<uint32_t> pad(const std::vector<uint32_t>& k, uint32_t len) {
  std::vector<uint32_t> r(k);
  r.resize(len, 0);
  return r;
}
}  // namespace

HPoly x_mul(sg_ctx* ctx, const HPoly& a, const HPoly& b) {
  if (a.empty() || b.empty()) return {};
  if ((uint64_t)a.size() * b.size() <= (1u << 14) || std::min(a.size(), b.size()) <= 4) {
    // schoolbook, keeping every position (zeros included): length la + lb - 1
    HPoly r(a.size() + b.size() - 1, fe_zero());
    for (size_t i = 0; i < a.size(); ++i) {
      if (is_zero_fe(a[i])) continue;
      fe am = to_mont(a[i]);
      for (size_t j = 0; j < b.size(); ++j) r[i + j] = fe_add(r[i + j], mont_mul(b[j], am));
    }
    return r;
  }
  SG_REQUIRE(ctx, "a GPU context is needed for large polynomial products");
  DPoly da = dpoly_upload(ctx, a.data(), a.size()), db = dpoly_upload(ctx, b.data(), b.size());
  DPoly r = poly_mul_exact(ctx, da.p(), da.len, db.p(), db.len);
  return dpoly_download(ctx, r.p(), r.len);
}

MPoly mp_constant(const fe& c) {
  MPoly m;
  m.nvars = 1;
  m.g[{}] = HPoly{c};
  return m;
}

std::vector<MPoly> mp_variables(uint32_t n) {
  std::vector<MPoly> out;
  for (uint32_t i = 0; i < n; ++i) {
    MPoly m;
    m.nvars = n;
    std::vector<uint32_t> k(n - 1, 0);
    if (i == 0) {
      m.g[k] = HPoly{fe_zero(), fe_one()};
    } else {
      k[i - 1] = 1;
      m.g[k] = HPoly{fe_one()};
    }
    out.push_back(std::move(m));
  }
  return out;
}

bool mp_is_zero(const MPoly& a) {
  for (auto& kv : a.g)
    for (auto& c : kv.second)
      if (!is_zero_fe(c)) return false;
  return true;
}

MPoly mp_lift(const HPoly& poly, uint32_t vi) {
  // m_polynomial.rs:66-81: sum_i constant(c_i) * x_vi^i over every coefficient
  MPoly m;
  if (hp_degree(poly) < 0) return m;
  m.nvars = vi + 1;
  if (vi == 0) {
    m.g[{}] = poly;
    return m;
  }
  for (size_t i = 0; i < poly.size(); ++i) {
    std::vector<uint32_t> k(vi, 0);
    k[vi - 1] = (uint32_t)i;
    dense_add_into(m.g[k], HPoly{poly[i]});
  }
  return m;
}

MPoly mp_neg(const MPoly& a) {
  MPoly r = a;
  r.dev.clear();
  r.rescue.reset();  // the factored form describes +a: the negation is evaluated from its groups
  for (auto& kv : r.g)
    for (auto& c : kv.second) c = fe_neg(c);
  return r;
}

MPoly mp_add(const MPoly& a, const MPoly& b) {
  // m_polynomial.rs:183-222
  if (a.g.empty()) return b;
  if (b.g.empty()) return a;
  MPoly r;
  r.nvars = std::max(a.nvars, b.nvars);
  for (auto& kv : a.g) dense_add_into(r.g[pad(kv.first, r.nvars - 1)], kv.second);
  for (auto& kv : b.g) dense_add_into(r.g[pad(kv.first, r.nvars - 1)], kv.second);
  return r;
}

MPoly mp_sub(const MPoly& a, const MPoly& b) { return mp_add(a, mp_neg(b)); }

MPoly mp_mul(sg_ctx* ctx, const MPoly& a, const MPoly& b) {
  // m_polynomial.rs:231-262 (the reference unwraps the longest key: an empty operand panics)
  SG_REQUIRE(!a.g.empty() && !b.g.empty(), "cannot multiply an empty MPolynomial");
  MPoly r;
  r.nvars = std::max(a.nvars, b.nvars);
  for (auto& ka : a.g) {
    std::vector<uint32_t> ea = pad(ka.first, r.nvars - 1);
    for (auto& kb : b.g) {
      std::vector<uint32_t> e = pad(kb.first, r.nvars - 1);
      for (size_t j = 0; j < e.size(); ++j) e[j] += ea[j];
      dense_add_into(r.g[e], x_mul(ctx, ka.second, kb.second));
    }
  }
  return r;
}

MPoly mp_pow(sg_ctx* ctx, const MPoly& a, unsigned __int128 e) {
  // m_polynomial.rs:265-298: acc = {0^nv: 1}; per bit of BitIter(e) (one bit for e == 0)
  if (mp_is_zero(a)) return MPoly{};
  MPoly acc;
  acc.nvars = a.nvars;
  acc.g[std::vector<uint32_t>(a.nvars - 1, 0)] = HPoly{fe_one()};
  int top = 0;
  for (int i = 127; i >= 0; --i)
    if ((e >> i) & 1) {
      top = i;
      break;
    }
  for (int i = top; i >= 0; --i) {
    acc = mp_mul(ctx, acc, acc);
    if ((e >> i) & 1) acc = mp_mul(ctx, acc, a);
  }
  return acc;
}

MPolyDevice::~MPolyDevice() {
  for (void* p : ptr)
    if (p) (void)hipFree(p);
}

std::shared_ptr<const MPolyDevice> mp_device(sg_ctx* ctx, const MPoly& a) {
  // contexts on several host threads may share a constraint: its device copy is made once per
  // device, and a copy for another device never replaces it
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  auto hit = a.dev.find(ctx->device);
  if (hit != a.dev.end()) return hit->second;
  auto d = std::make_shared<MPolyDevice>();
  d->device = ctx->device;
  // normalize every group's x-vector (trimmed at its degree) by its first non-zero
  // coefficient: proportional groups (e.g. the C^j (next)^e terms of a cubed AIR row) share
  // one device copy and one coset LDE per proof
  std::map<std::vector<uint64_t>, std::vector<int32_t>> by_hash;  // (len, a few limbs) -> candidates
  std::vector<HPoly> normed;
  for (auto& kv : a.g) {
    const int64_t deg = hp_degree(kv.second);
    if (deg < 0) {
      d->qidx.push_back(-1);
      d->scale.push_back(fe_zero());
      continue;
    }
    size_t first = 0;
    while (is_zero_fe(kv.second[first])) ++first;
    const fe s = kv.second[first];
    const fe sinv_m = to_mont(fe_inv(s));
    HPoly v((size_t)deg + 1);
    for (size_t i = 0; i < v.size(); ++i) v[i] = mont_mul(kv.second[i], sinv_m);
    std::vector<uint64_t> key = {v.size(), first};
    for (size_t i = v.size() - std::min<size_t>(v.size(), 4); i < v.size(); ++i) {
      key.push_back(fe_lo(v[i]));
      key.push_back(fe_hi(v[i]));
    }
    int32_t found = -1;
    for (int32_t c : by_hash[key])
      if (normed[(size_t)c].size() == v.size() &&
          memcmp(normed[(size_t)c].data(), v.data(), v.size() * sizeof(fe)) == 0) {
        found = c;
        break;
      }
    if (found < 0) {
      found = (int32_t)normed.size();
      by_hash[key].push_back(found);
      normed.push_back(std::move(v));
    }
    d->qidx.push_back(found);
    d->scale.push_back(s);
  }
  for (auto& v : normed) {
    void* p = nullptr;
    SG_HIP(hipMalloc(&p, v.size() * sizeof(fe)));
    d->ptr.push_back(p);
    d->len.push_back(v.size());
    d->small.push_back(v.size() <= (size_t)kSmallPolyMax ? v : HPoly{});
    SG_HIP(hipMemcpyAsync(p, v.data(), v.size() * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    host_wait(ctx, ctx->stream);
    uint8_t h[64];
    blake2b512(reinterpret_cast<const uint8_t*>(v.data()), v.size() * sizeof(fe), h);
    std::array<uint64_t, 4> dg{};
    memcpy(dg.data(), h, sizeof(dg));
    d->digest.push_back(dg);
  }
  a.dev[ctx->device] = d;
  return d;
}

fe mp_evaluate(const MPoly& a, const std::vector<fe>& point) {
  // m_polynomial.rs:95-122
  SG_REQUIRE(a.g.empty() || point.size() >= a.nvars, "point has fewer values than the polynomial has variables");
  fe acc = fe_zero();
  for (auto& kv : a.g) {
    fe v = hp_eval(kv.second, point[0]);
    for (size_t j = 0; j < kv.first.size(); ++j)
      if (kv.first[j]) v = fe_mul(v, fe_pow(point[j + 1], kv.first[j]));
    acc = fe_add(acc, v);
  }
  return acc;
}

}  // namespace sg

// ====================================================================== C ABI

using namespace sg;

namespace {
sg_mpoly* wrapm(MPoly&& m) {
  sg_mpoly* p = new sg_mpoly();
  p->m = std::move(m);
  return p;
}
}  // namespace

extern "C" int sg_mpoly_create(sg_ctx* ctx, size_t nvars, size_t nterms, const uint32_t* exps, const sg_fe* coeffs,
                               sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && ((exps && coeffs) || !nterms), "null argument");
    SG_REQUIRE(nvars >= 1 || nterms == 0, "keys need at least one variable");
    check_canonical(coeffs, nterms, "coefficients");
    MPoly m;
    if (nterms) m.nvars = (uint32_t)nvars;
    for (size_t t = 0; t < nterms; ++t) {
      const uint32_t* e = exps + t * nvars;
      std::vector<uint32_t> k(e + 1, e + nvars);
      HPoly& v = m.g[k];
      if (v.size() < (size_t)e[0] + 1) v.resize((size_t)e[0] + 1, fe_zero());
      v[e[0]] = fe_add(v[e[0]], to_fe(coeffs[t]));
    }
    *out = wrapm(std::move(m));
  });
}

extern "C" int sg_mpoly_constant(sg_ctx* ctx, sg_fe c, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out, "null argument");
    check_canonical(&c, 1, "constant");
    *out = wrapm(mp_constant(to_fe(c)));
  });
}

extern "C" int sg_mpoly_variable(sg_ctx* ctx, size_t num_variables, size_t index, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && index < num_variables, "variable index out of range");
    *out = wrapm(std::move(mp_variables((uint32_t)num_variables)[index]));
  });
}

extern "C" int sg_mpoly_lift(sg_ctx* ctx, const sg_fe* coeffs, size_t len, size_t variable_index, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && (coeffs || !len), "null argument");
    check_canonical(coeffs, len, "coefficients");
    const fe* c = reinterpret_cast<const fe*>(coeffs);
    *out = wrapm(mp_lift(HPoly(c, c + len), (uint32_t)variable_index));
  });
}

extern "C" int sg_mpoly_lift_poly(sg_ctx* ctx, const sg_poly* p, size_t variable_index, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(ctx && out && p, "a GPU context and a polynomial are required");
    *out = wrapm(mp_lift(dpoly_download(ctx, p->d.p(), p->d.len), (uint32_t)variable_index));
  });
}

extern "C" int sg_mpoly_neg(sg_ctx* ctx, const sg_mpoly* a, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(a && out, "null argument");
    *out = wrapm(mp_neg(a->m));
  });
}

extern "C" int sg_mpoly_add(sg_ctx* ctx, const sg_mpoly* a, const sg_mpoly* b, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(a && b && out, "null argument");
    *out = wrapm(mp_add(a->m, b->m));
  });
}

extern "C" int sg_mpoly_sub(sg_ctx* ctx, const sg_mpoly* a, const sg_mpoly* b, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(a && b && out, "null argument");
    *out = wrapm(mp_sub(a->m, b->m));
  });
}

extern "C" int sg_mpoly_mul(sg_ctx* ctx, const sg_mpoly* a, const sg_mpoly* b, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(a && b && out, "null argument");
    if (ctx) SG_HIP(hipSetDevice(ctx->device));  // ctx == NULL: host-only (small products)
    *out = wrapm(mp_mul(ctx, a->m, b->m));
  });
}

extern "C" int sg_mpoly_pow(sg_ctx* ctx, const sg_mpoly* a, sg_fe exponent, sg_mpoly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(a && out, "null argument");
    if (ctx) SG_HIP(hipSetDevice(ctx->device));  // ctx == NULL: host-only (small products)
    *out = wrapm(mp_pow(ctx, a->m, ((unsigned __int128)exponent.hi << 64) | exponent.lo));
  });
}

extern "C" int sg_mpoly_is_zero(const sg_mpoly* a) { return a ? (mp_is_zero(a->m) ? 1 : 0) : SG_ERR_INVALID; }

extern "C" int sg_mpoly_evaluate(sg_ctx* ctx, const sg_mpoly* a, const sg_fe* point, size_t n, sg_fe* out) {
  return guard(ctx, [&] {
    SG_REQUIRE(a && out && (point || !n), "null argument");
    check_canonical(point, n, "point");
    const fe* p = reinterpret_cast<const fe*>(point);
    *out = from_fe(mp_evaluate(a->m, std::vector<fe>(p, p + n)));
  });
}

extern "C" int sg_mpoly_shape(const sg_mpoly* a, size_t* nvars, size_t* ngroups, size_t* ncoeffs) {
  if (!a) return SG_ERR_INVALID;
  size_t total = 0;
  for (auto& kv : a->m.g) total += kv.second.size();
  if (nvars) *nvars = a->m.nvars;
  if (ngroups) *ngroups = a->m.g.size();
  if (ncoeffs) *ncoeffs = total;
  return SG_OK;
}

extern "C" int sg_mpoly_export(const sg_mpoly* a, uint32_t* exps, uint64_t* lens, sg_fe* coeffs) {
  if (!a) return SG_ERR_INVALID;
  size_t gi = 0, ci = 0;
  const size_t nk = a->m.nvars ? a->m.nvars - 1 : 0;
  for (auto& kv : a->m.g) {
    if (exps) memcpy(exps + gi * nk, kv.first.data(), nk * sizeof(uint32_t));
    if (lens) lens[gi] = kv.second.size();
    if (coeffs)
      for (auto& c : kv.second) coeffs[ci++] = from_fe(c);
    ++gi;
  }
  return SG_OK;
}

extern "C" void sg_mpoly_free(sg_mpoly* a) { delete a; }
