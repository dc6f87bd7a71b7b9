// Device polynomial algebra (fft/ntt_arithmetics.rs) over the gfx950 NTT and
// elementwise kernels, its C ABI (sg_poly_*, sg_fast_*), and small host
// polynomials.  See poly.hpp.
//
// Bit-exactness: fast_multiply / fast_coset_divide follow the reference's own
// algorithm step by step (order shrinking, padding, truncation, unscaling), so
// they return its exact output even when a division is not exact.  Zerofiers
// and interpolants are unique polynomials; on geometric domains (the only
// large ones a STARK uses: omicron^0..omicron^(n-1)) they are computed in closed
// form instead of through the reference's product / remainder trees:
//   * prod_{i<n} (x - q^i) = sum_j (-1)^(n-j) q^((n-j)(n-j-1)/2) [n j]_q x^j
//     (Gauss binomial theorem; [n j]_q from prefix products of (1 - q^l));
//   * the interpolant through (q^i, y_i), i < n < D = ord(q), is the INTT_D of
//     its values on the whole group: y_i for i < n and, for m >= n,
//     Z(q^m) sum_i y_i / (Z'(q^i) (q^m - q^i)) -- one cyclic convolution with
//     1 / (1 - q^-j) (3 NTTs), Z = the zerofier above.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <vector>

#include "host_field.hpp"
#include "internal.hpp"
#include "poly.hpp"
#include "poly_kernels.hpp"

namespace sg {

namespace {
inline fe one_m() { return to_mont(fe_one()); }
inline bool fe_is_zero_h(const fe& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }
}  // namespace

// two-level Montgomery power tables of f for exponents < count
void pow_tables2(sg_ctx* ctx, const fe& f, uint64_t count, const fe** A, const fe** B) {
  *A = ctx->pow_table(f, 4096);
  *B = ctx->pow_table(fe_pow(f, 4096), std::max<uint64_t>((count + 4095) / 4096, 1));
}

// ------------------------------------------------------------------ buffers

DPoly dpoly_alloc(sg_ctx* ctx, uint64_t len) {
  DPoly d;
  d.len = len;
  if (len) d.buf = DevBuf(ctx, len * sizeof(fe));
  return d;
}

DPoly dpoly_upload(sg_ctx* ctx, const fe* host, uint64_t len) {
  DPoly d = dpoly_alloc(ctx, len);
  if (len) SG_HIP(hipMemcpyAsync(d.p(), host, len * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  return d;
}

std::vector<fe> dpoly_download(sg_ctx* ctx, const fe* d, uint64_t len) {
  std::vector<fe> out(len);
  if (len) SG_HIP(hipMemcpyAsync(out.data(), d, len * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
  host_wait(ctx, ctx->stream);
  return out;
}

DPoly dpoly_copy(sg_ctx* ctx, const fe* d, uint64_t len) {
  DPoly o = dpoly_alloc(ctx, len);
  if (len) SG_HIP(hipMemcpyAsync(o.p(), d, len * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
  return o;
}

int64_t dev_degree(sg_ctx* ctx, const fe* d, uint64_t len) {
  return dev_degrees(ctx, {{d, len}})[0];
}

// Every polynomial's degree with one host round trip: batches of kDegBatch per launch into the
// context's degree slots, tagged with a fresh generation (no clearing launch), published to
// host-coherent memory with a ready flag (k_publish_slots) that the host spins on.  Split in two so
// a caller can do host work between the launches and the wait (dev_degrees_begin / _end).
DegScan dev_degrees_begin(sg_ctx* ctx, const std::vector<std::pair<const fe*, uint64_t>>& polys) {
  DegScan sc;
  sc.n = polys.size();
  if (polys.empty()) return sc;
  if (ctx->deg_cap < polys.size()) {
    host_wait(ctx, ctx->stream);  // the old slots may still be in use
    if (ctx->deg_slots) (void)hipFree(ctx->deg_slots);
    if (ctx->deg_host) (void)hipHostFree(ctx->deg_host);
    ctx->deg_slots = nullptr;
    ctx->deg_host = ctx->deg_host_dev = nullptr;
    ctx->deg_cap = 0;
    const size_t cap = std::max<size_t>(64, polys.size());
    SG_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->deg_slots), cap * 8));
    SG_HIP(hipMemsetAsync(ctx->deg_slots, 0, cap * 8, ctx->stream));
    void* h = nullptr;
    void* hd = nullptr;
    SG_HIP(hipHostMalloc(&h, (cap + 1) * 8, hipHostMallocMapped | hipHostMallocCoherent));
    ctx->deg_host = static_cast<unsigned long long*>(h);
    memset(h, 0, (cap + 1) * 8);
    SG_HIP(hipHostGetDevicePointer(&hd, h, 0));
    ctx->deg_host_dev = static_cast<unsigned long long*>(hd);
    ctx->deg_cap = cap;
    ctx->deg_gen = 0;
  }
  if (++ctx->deg_gen >= (1ull << (64 - kDegGenShift))) {  // generations exhausted: clear once
    SG_HIP(hipMemsetAsync(ctx->deg_slots, 0, ctx->deg_cap * 8, ctx->stream));
    ctx->deg_gen = 1;
  }
  sc.gen = ctx->deg_gen;
  for (size_t i0 = 0; i0 < polys.size(); i0 += kDegBatch) {
    DegBatch b{};
    const int cnt = (int)std::min<size_t>(kDegBatch, polys.size() - i0);
    for (int k = 0; k < cnt; ++k) {
      b.a[k] = polys[i0 + k].first;
      b.n[k] = polys[i0 + k].second;
    }
    SG_HIP(launch_last_nonzero_batch(b, cnt, ctx->deg_slots + i0, sc.gen, ctx->stream));
  }
  SG_HIP(launch_publish_slots(ctx->deg_slots, ctx->deg_host_dev, polys.size(), ctx->deg_host_dev + ctx->deg_cap,
                              sc.gen, ctx->stream));
  return sc;
}

std::vector<int64_t> dev_degrees_end(sg_ctx* ctx, const DegScan& sc) {
  std::vector<int64_t> out(sc.n, -1);
  if (!sc.n) return out;
  volatile unsigned long long* flag = ctx->deg_host + ctx->deg_cap;
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  while (*flag != sc.gen) {  // as wait_roots: query the stream now and then, so an error surfaces
    if ((++spins & 255) == 0) {
      if (ctx->watch) ctx->watch(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      const hipError_t q = hipStreamQuery(ctx->stream);
      if (q == hipSuccess) {
        if (*flag != sc.gen) throw Error{SG_ERR_HIP, "degree scan was not published"};
        break;
      }
      if (q != hipErrorNotReady) SG_HIP(q);
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  const unsigned long long mask = (1ull << kDegGenShift) - 1;
  for (size_t i = 0; i < sc.n; ++i) {
    const unsigned long long v = ctx->deg_host[i];
    out[i] = (v >> kDegGenShift) == sc.gen ? (int64_t)(v & mask) - 1 : -1;
  }
  return out;
}

std::vector<int64_t> dev_degrees(sg_ctx* ctx, const std::vector<std::pair<const fe*, uint64_t>>& polys) {
  return dev_degrees_end(ctx, dev_degrees_begin(ctx, polys));
}

// ------------------------------------------------------------------ roots

fe root_of_order(uint64_t n) {
  SG_REQUIRE(n && (n & (n - 1)) == 0, "Field does not have any roots where n > 2^119 or not a power of two.");
  fe root = fe_generator();
  unsigned __int128 order = (unsigned __int128)1 << 119;
  while (order != n) {
    root = fe_mul(root, root);
    order >>= 1;
  }
  return root;
}

void check_root(const fe& root, uint64_t root_order) {
  SG_REQUIRE(fe_eq(fe_pow(root, root_order), fe_one()), "supplied root does not have supplied root_order");
  SG_REQUIRE(!fe_eq(fe_pow(root, root_order / 2), fe_one()), "supplied root is not a primitive of root_order");
}

// ------------------------------------------------------------------ transforms

void ntt_sized(sg_ctx* ctx, const fe& root, const fe* in, uint64_t n_in, int logn, fe* out, const fe* scale_offset) {
  const uint64_t n = (uint64_t)1 << logn;
  SG_REQUIRE(n_in <= n, "ntt_sized: input longer than the transform");
  SG_REQUIRE(!ranges_overlap(in, n_in, out, n), "ntt: output must not alias the input");
  const fe* sA = nullptr;
  const fe* sB = nullptr;
  if (scale_offset) pow_tables2(ctx, *scale_offset, std::max<uint64_t>(n_in, 1), &sA, &sB);
  if (n_in == 0) {
    SG_HIP(hipMemsetAsync(out, 0, n * sizeof(fe), ctx->stream));
    return;
  }
  ntt_run(ctx, &out, &in, 1, n_in, logn, root, sA, sB, 0, nullptr);
}

void intt_sized(sg_ctx* ctx, const fe& root, const fe* in, int logn, fe* out) {
  const uint64_t n = (uint64_t)1 << logn;
  if (n < 2) {  // fft/ntt.rs:56-58
    SG_HIP(hipMemcpyAsync(out, in, n * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
    return;
  }
  fe ninv_m = to_mont(fe_inv(fe_from_u64(n)));
  ntt_run(ctx, &out, &in, 1, n, logn, fe_inv(root), nullptr, nullptr, 0, &ninv_m);
}

// ------------------------------------------------------------------ elementwise

void dev_mul(sg_ctx* ctx, fe* out, const fe* a, const fe* b, uint64_t n) {
  SG_HIP(launch_ew_mul(out, a, b, n, fe_r2(), ctx->stream));
}

void dev_div(sg_ctx* ctx, fe* out, const fe* a, const fe* b, uint64_t n) {
  if (!n) return;
  // a zero divisor raises ctx->div_zero_flag; check_div_zero() reports it once the stream
  // has drained (no round trip per division)
  SG_HIP(launch_batch_div(out, a, b, n, fe_r2(), one_m(), ctx->div_zero_flag_dev, ctx->stream));
}

void check_div_zero(sg_ctx* ctx) {
  if (*reinterpret_cast<volatile uint32_t*>(ctx->div_zero_flag)) {
    *reinterpret_cast<volatile uint32_t*>(ctx->div_zero_flag) = 0;
    throw Error{SG_ERR_INVALID, "divide by zero"};  // field_element.rs:82-90
  }
}

void dev_scale_pow(sg_ctx* ctx, fe* out, const fe* in, uint64_t n, const fe& f, uint64_t start) {
  if (!n) return;
  const fe *A, *B;
  pow_tables2(ctx, f, start + n, &A, &B);
  SG_HIP(launch_mul_pow2(out, in, n, start, A, B, ctx->stream));
}

void dev_prefix_product(sg_ctx* ctx, fe* data, uint64_t n) {
  if (!n) return;
  uint64_t tiles = (n + 1023) / 1024;
  if (tiles == 1) {
    SG_HIP(launch_scan_tile(data, n, nullptr, fe_r2(), one_m(), ctx->stream));
    return;
  }
  DevBuf tot(ctx, tiles * sizeof(fe));
  SG_HIP(launch_scan_tile(data, n, tot.as<fe>(), fe_r2(), one_m(), ctx->stream));
  dev_prefix_product(ctx, tot.as<fe>(), tiles);
  SG_HIP(launch_scan_fix(data, n, tot.as<fe>(), fe_r2(), ctx->stream));
}

// ------------------------------------------------------------------ products

DPoly poly_mul_exact(sg_ctx* ctx, const fe* a, uint64_t la, const fe* b, uint64_t lb) {
  if (!la || !lb) return DPoly{};
  const uint64_t lr = la + lb - 1;
  DPoly out = dpoly_alloc(ctx, lr);
  if (la * lb <= 64 || std::min(la, lb) == 1) {
    // tiny: on the host
    std::vector<fe> ha = dpoly_download(ctx, a, la), hb = dpoly_download(ctx, b, lb);
    HPoly r = hp_mul(ha, hb);
    SG_HIP(hipMemcpyAsync(out.p(), r.data(), lr * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    host_wait(ctx, ctx->stream);
    return out;
  }
  const uint64_t n = next_pow2(lr);
  const int logn = ilog2_exact(n);
  const fe w = root_of_order(n);
  DevBuf va(ctx, n * sizeof(fe)), vb(ctx, n * sizeof(fe)), c(ctx, n * sizeof(fe));
  ntt_sized(ctx, w, a, la, logn, va.as<fe>());
  ntt_sized(ctx, w, b, lb, logn, vb.as<fe>());
  dev_mul(ctx, va.as<fe>(), va.as<fe>(), vb.as<fe>(), n);
  intt_sized(ctx, w, va.as<fe>(), logn, c.as<fe>());
  SG_HIP(hipMemcpyAsync(out.p(), c.get(), lr * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
  return out;
}

void ref_inner_ntt(sg_ctx* ctx, const fe& root, uint64_t order, const fe* p, uint64_t len, const fe* scale,
                   DevBuf& out, uint64_t& out_len, const fe* host_copy) {
  // the reference's inner(): pad to `order` only when shorter, optional scale, ntt
  out_len = std::max<uint64_t>(next_pow2(std::max<uint64_t>(len, 1)), order);
  out = DevBuf(ctx, out_len * sizeof(fe));
  if (len >= 1 && len <= (uint64_t)kSmallPolyMax && out_len == order && order >= 2) {
    // a tiny polynomial (a boundary zerofier): its NTT is its values at offset root^k -- Horner
    SmallPoly sp{};
    sp.len = (int)len;
    if (host_copy) {
      memcpy(sp.c, host_copy, len * sizeof(fe));
    } else {
      SG_HIP(hipMemcpyAsync(sp.c, p, len * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
      host_wait(ctx, ctx->stream);
    }
    const fe *A, *B;
    pow_tables2(ctx, root, order, &A, &B);
    SG_HIP(launch_eval_small(out.as<fe>(), sp, order, A, B, to_mont(scale ? *scale : fe_one()), ctx->stream));
    return;
  }
  ntt_sized(ctx, root, p, len, ilog2_exact(out_len), out.as<fe>(), scale);
}

DivPlan coset_divide_plan(fe root, uint64_t root_order, int64_t dl, int64_t dr) {
  SG_REQUIRE(dr >= 0, "cannot divide by zero polynomial");
  DivPlan pl;
  pl.zero_lhs = dl < 0;
  if (pl.zero_lhs) return pl;
  SG_REQUIRE(dl >= dr, "cannot divide by polynomial of larger degree");
  const uint64_t deg = (uint64_t)std::max(dl, dr);
  pl.result_len = (uint64_t)(dl - dr + 1);
  uint64_t order = root_order;
  while (deg < order / 2) {
    root = fe_mul(root, root);
    order /= 2;
  }
  pl.root = root;
  pl.order = order;
  return pl;
}

DPoly coset_divide_finish(sg_ctx* ctx, const DivPlan& pl, const fe& offset, fe* lhs_v, const fe* rhs_v,
                          bool rhs_is_inverse) {
  if (pl.zero_lhs) return DPoly{};
  if (rhs_is_inverse) dev_mul(ctx, lhs_v, lhs_v, rhs_v, pl.order);  // a / b = a * b^-1 (field_element.rs:82-90)
  else dev_div(ctx, lhs_v, lhs_v, rhs_v, pl.order);
  DevBuf c(ctx, pl.order * sizeof(fe));
  intt_sized(ctx, pl.root, lhs_v, ilog2_exact(pl.order), c.as<fe>());
  uint64_t keep = std::min(pl.result_len, pl.order);
  DPoly out = dpoly_alloc(ctx, keep);
  dev_scale_pow(ctx, out.p(), c.as<fe>(), keep, fe_inv(offset));
  return out;
}

DPoly fast_multiply_dev(sg_ctx* ctx, fe root, uint64_t root_order, const fe* a, uint64_t la, const fe* b,
                        uint64_t lb) {
  check_root(root, root_order);
  int64_t da = dev_degree(ctx, a, la), db = dev_degree(ctx, b, lb);
  if (da < 0 || db < 0) return DPoly{};
  const uint64_t deg = (uint64_t)da + (uint64_t)db;
  const uint64_t result_len = deg + 1;
  uint64_t order = root_order;
  while (deg < order / 2) {
    root = fe_mul(root, root);
    order /= 2;
  }
  DevBuf va, vb;
  uint64_t na, nb;
  ref_inner_ntt(ctx, root, order, a, la, nullptr, va, na);
  ref_inner_ntt(ctx, root, order, b, lb, nullptr, vb, nb);
  // Hadamard over the first `order` entries, intt over `order` entries
  dev_mul(ctx, va.as<fe>(), va.as<fe>(), vb.as<fe>(), order);
  // the inverse transform writes the result's own buffer (order >= keep slots): no copy
  DPoly out = dpoly_alloc(ctx, order);
  intt_sized(ctx, root, va.as<fe>(), ilog2_exact(order), out.p());
  out.len = std::min(result_len, order);
  return out;
}

const fe* divisor_inverse_values(sg_ctx* ctx, const DivPlan& pl, const fe& offset, const fe* rhs, uint64_t lr,
                                 const fe* rhs_host, std::vector<DevBuf>* keep) {
  if (keep && !ctx->domain_cache_on()) {  // recomputed per call, owned by the caller's scope
    DevBuf vr;
    uint64_t nr;
    ref_inner_ntt(ctx, pl.root, pl.order, rhs, lr, &offset, vr, nr, rhs_host);
    keep->emplace_back(ctx, pl.order * sizeof(fe));
    dev_div(ctx, keep->back().as<fe>(), nullptr, vr.as<fe>(), pl.order);
    host_wait(ctx, ctx->stream);
    check_div_zero(ctx);
    return keep->back().as<fe>();
  }
  // a small divisor known on the host (a boundary zerofier: public): 1 / its coset values is
  // kept in the context, keyed by its coefficients and the coset, so the division is a product
  std::vector<uint64_t> key = {kDomainDivisorInverse, pl.order, fe_lo(pl.root), fe_hi(pl.root), fe_lo(offset),
                               fe_hi(offset), lr};
  for (uint64_t i = 0; i < lr; ++i) {
    key.push_back(fe_lo(rhs_host[i]));
    key.push_back(fe_hi(rhs_host[i]));
  }
  const fe* inv = static_cast<const fe*>(ctx->domain_table(key));
  if (!inv) {
    DevBuf vr;
    uint64_t nr;
    ref_inner_ntt(ctx, pl.root, pl.order, rhs, lr, &offset, vr, nr, rhs_host);
    void* t = nullptr;
    SG_HIP(hipMalloc(&t, pl.order * sizeof(fe)));
    dev_div(ctx, static_cast<fe*>(t), nullptr, vr.as<fe>(), pl.order);
    host_wait(ctx, ctx->stream);
    try {
      check_div_zero(ctx);  // a zero divisor is reported now and the table is not kept
    } catch (...) {
      (void)hipFree(t);
      throw;
    }
    ctx->domain_table_put_bounded(key, t);
    inv = static_cast<const fe*>(t);
  }
  return inv;
}

DPoly fast_coset_divide_dev(sg_ctx* ctx, fe root, uint64_t root_order, const fe& offset, const fe* lhs, uint64_t ll,
                            const fe* rhs, uint64_t lr, int64_t rhs_degree, const fe* rhs_host, int64_t lhs_degree) {
  check_root(root, root_order);
  int64_t dl, dr;
  if (rhs_degree >= -1) {
    dr = rhs_degree;
    dl = lhs_degree >= -1 ? lhs_degree : dev_degree(ctx, lhs, ll);
  } else {
    std::vector<int64_t> d = dev_degrees(ctx, {{lhs, ll}, {rhs, lr}});
    dl = d[0];
    dr = d[1];
  }
  SG_REQUIRE(dr >= 0, "cannot divide by zero polynomial");
  const DivPlan pl = coset_divide_plan(root, root_order, dl, dr);
  if (pl.zero_lhs) return DPoly{};
  DevBuf vl, vr;
  uint64_t nl, nr;
  ref_inner_ntt(ctx, pl.root, pl.order, lhs, ll, &offset, vl, nl);
  if (rhs_host && lr <= 64 && ctx->domain_cache_on())
    return coset_divide_finish(ctx, pl, offset, vl.as<fe>(), divisor_inverse_values(ctx, pl, offset, rhs, lr, rhs_host),
                               true);
  ref_inner_ntt(ctx, pl.root, pl.order, rhs, lr, &offset, vr, nr, rhs_host);
  return coset_divide_finish(ctx, pl, offset, vl.as<fe>(), vr.as<fe>());
}

constexpr int kNttBatch = 4;  // transforms per pointer-mode launch (the kernels' kMaxBatch)
// batched only while the transforms are latency-bound (C4: 2^16-2^17 points, 0.09 ms per proof);
// at the headline's 2^20-2^21 the per-column launches on the main stream leave the side stream's
// trees more of the chip (batched: +0.1 ms per proof, profiles/r05_ab_bqbatch_*.log)
constexpr uint64_t kNttBatchMaxOrder = (uint64_t)1 << 18;

std::vector<DPoly> fast_coset_divide_batch_dev(sg_ctx* ctx, fe root, uint64_t root_order, const fe& offset,
                                               const std::vector<DivItem>& items) {
  check_root(root, root_order);
  std::vector<DPoly> out(items.size());
  std::vector<DivPlan> plans(items.size());
  std::vector<size_t> batch;  // items taking the batched path (one coset size, equal dividend lengths)
  for (size_t i = 0; i < items.size(); ++i) {
    const DivItem& it = items[i];
    plans[i] = coset_divide_plan(root, root_order, it.dl, it.dr);
    const DivPlan& pl = plans[i];
    const bool ok = !pl.zero_lhs && it.rhs_host && it.lr <= 64 && ctx->domain_cache_on() && pl.order <= kNttBatchMaxOrder &&
                    it.ll > (uint64_t)kSmallPolyMax && it.ll <= pl.order && pl.order >= 2 &&
                    (batch.empty() || (pl.order == plans[batch[0]].order && it.ll == items[batch[0]].ll));
    if (ok) batch.push_back(i);
  }
  if (batch.size() < 2) batch.clear();
  for (size_t i = 0; i < items.size(); ++i) {
    if (std::find(batch.begin(), batch.end(), i) != batch.end()) continue;
    const DivItem& it = items[i];
    out[i] = fast_coset_divide_dev(ctx, root, root_order, offset, it.lhs, it.ll, it.rhs, it.lr, it.dr, it.rhs_host,
                                   it.dl);
  }
  if (batch.empty()) return out;
  // the reference's inner() on the coset (ref_inner_ntt: len <= order, so no padding beyond order),
  // the product with 1 / the divisor's values, the inverse transform and the offset^-i scale
  const DivPlan& pl = plans[batch[0]];
  const uint64_t ll = items[batch[0]].ll;
  const int logo = ilog2_exact(pl.order);
  const fe *sA, *sB;
  pow_tables2(ctx, offset, std::max<uint64_t>(ll, 1), &sA, &sB);
  const fe ninv_m = to_mont(fe_inv(fe_from_u64(pl.order)));
  for (size_t b0 = 0; b0 < batch.size(); b0 += kNttBatch) {
    const int nb = (int)std::min<size_t>(kNttBatch, batch.size() - b0);
    std::vector<DevBuf> vals, coefs;
    fe* vo[kNttBatch] = {};
    const fe* vi[kNttBatch] = {};
    fe* co[kNttBatch] = {};
    const fe* ci[kNttBatch] = {};
    for (int k = 0; k < nb; ++k) {
      vals.emplace_back(ctx, pl.order * sizeof(fe));
      coefs.emplace_back(ctx, pl.order * sizeof(fe));
      vo[k] = vals.back().as<fe>();
      vi[k] = items[batch[b0 + k]].lhs;
      co[k] = coefs.back().as<fe>();
      ci[k] = vo[k];
    }
    ntt_run(ctx, vo, vi, nb, ll, logo, pl.root, sA, sB, 0, nullptr);
    for (int k = 0; k < nb; ++k) {
      const DivItem& it = items[batch[b0 + k]];
      dev_mul(ctx, vo[k], vo[k], divisor_inverse_values(ctx, plans[batch[b0 + k]], offset, it.rhs, it.lr, it.rhs_host),
              pl.order);  // a / b = a * b^-1 (field_element.rs:82-90)
    }
    ntt_run(ctx, co, ci, nb, pl.order, logo, fe_inv(pl.root), nullptr, nullptr, 0, &ninv_m);
    for (int k = 0; k < nb; ++k) {
      const DivPlan& p = plans[batch[b0 + k]];
      const uint64_t keep = std::min(p.result_len, p.order);
      DPoly q = dpoly_alloc(ctx, keep);
      dev_scale_pow(ctx, q.p(), co[k], keep, fe_inv(offset));
      out[batch[b0 + k]] = std::move(q);
    }
  }
  return out;
}

// ------------------------------------------------------------------ geometric domains

DPoly zerofier_geometric_dev(sg_ctx* ctx, const fe& q, uint64_t D, uint64_t n) {
  SG_REQUIRE(n <= D, "zerofier: more points than the order of the root");
  if (n == 0) return DPoly{};
  if (n == D) {
    // the whole group: the reference's last fast_multiply has degree D = order, so its
    // size-D NTT wraps x^D - 1 onto x^0 - 1 = 0 and returns D zeros (not truncated)
    DPoly z = dpoly_alloc(ctx, D);
    SG_HIP(hipMemsetAsync(z.p(), 0, D * sizeof(fe), ctx->stream));
      return z;
  }
  const fe *qA, *qB;
  pow_tables2(ctx, q, D, &qA, &qB);
  DevBuf F(ctx, (n + 1) * sizeof(fe)), invF(ctx, (n + 1) * sizeof(fe));
  const fe one = fe_one();
  SG_HIP(hipMemcpyAsync(F.get(), &one, sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(launch_one_minus_pow(F.as<fe>() + 1, n, 1, qA, qB, ctx->stream));  // 1 - q^l, l = 1..n
  dev_prefix_product(ctx, F.as<fe>(), n + 1);
  dev_div(ctx, invF.as<fe>(), nullptr, F.as<fe>(), n + 1);
  DPoly z = dpoly_alloc(ctx, n + 1);
  SG_HIP(launch_qbinom(z.p(), F.as<fe>(), invF.as<fe>(), n, D, qA, qB, fe_r2(), ctx->stream));
  return z;
}

namespace {
// b[j] = 1 / (1 - q^-j) (j >= 1), b[0] = 0, j < D
DevBuf interp_b(sg_ctx* ctx, const fe& q, uint64_t D) {
  const fe qinv = fe_inv(q);
  const fe *A, *B;
  pow_tables2(ctx, qinv, D, &A, &B);
  DevBuf b(ctx, D * sizeof(fe));
  SG_HIP(hipMemsetAsync(b.get(), 0, sizeof(fe), ctx->stream));
  SG_HIP(launch_one_minus_pow(b.as<fe>() + 1, D - 1, 1, A, B, ctx->stream));
  dev_div(ctx, b.as<fe>() + 1, nullptr, b.as<fe>() + 1, D - 1);
  return b;
}

// logf = 0: NTT_D(b).  logf > 0: the f = 2^logf rows K_r[j] = b[(f j - r) mod D] (j < M = D / f),
// each transformed with q^f (order M).  Cached per (q, D, f), like a twiddle plan.
const fe* interp_kernel(sg_ctx* ctx, const fe& q, uint64_t D, int logf) {
  auto key = std::make_pair(std::make_pair(fe_lo(q), fe_hi(q)), D | ((uint64_t)logf << 58));
  auto it = ctx->interp_tables.find(key);
  if (it != ctx->interp_tables.end()) return reinterpret_cast<const fe*>(it->second);
  DevBuf b = interp_b(ctx, q, D);
  void* t = nullptr;
  SG_HIP(hipMalloc(&t, D * sizeof(fe)));
  try {
    if (logf == 0) {
      ntt_sized(ctx, q, b.as<fe>(), D, ilog2_exact(D), reinterpret_cast<fe*>(t));
    } else {
      const uint64_t M = D >> logf;
      DevBuf rows(ctx, D * sizeof(fe));
      SG_HIP(launch_geo_krows(rows.as<fe>(), b.as<fe>(), logf, M, D, ctx->stream));
      ntt_rows_dev(ctx, fe_pow(q, (uint64_t)1 << logf), rows.as<fe>(), (uint64_t)1 << logf, ilog2_exact(M),
                   reinterpret_cast<fe*>(t), nullptr);
    }
    // the table outlives this call's temporaries: complete before they return to the pool
    host_wait(ctx, ctx->stream);
  } catch (...) {
    (void)hipFree(t);
    throw;
  }
  ctx->interp_tables[key] = t;
  return reinterpret_cast<const fe*>(t);
}

// decimation of the geometric interpolation: the largest f = 2^logf with n <= D / f, so the
// interpolant (degree < n) is recovered from its values on the subgroup of order M = D / f
// (`decimate` false -- the context option geo_decimate = 0 -- the full-group form, f = 1)
int geo_logf(uint64_t n, uint64_t D, bool decimate = true) {
  if (!decimate) return 0;
  // M = D / f >= n, M >= 64, M / f >= 1 (rows of M / f inputs), f <= 16
  const int logD = ilog2_exact(D);
  int logf = 0;
  while (logf < 4 && (D >> (logf + 1)) >= n && logD - (logf + 1) >= 6 && logD >= 2 * (logf + 1)) ++logf;
  return logf;
}
}  // namespace

GeoPlan geo_plan(sg_ctx* ctx, const fe& q, uint64_t D, uint64_t n, GeoInterpCache* cache, bool use_option) {
  SG_REQUIRE(n > 1 && n < D && D && (D & (D - 1)) == 0, "geo_plan: 1 < n < D, D a power of two");
  GeoPlan P;
  const int logD = ilog2_exact(D);
  const int logf = geo_logf(n, D, !use_option || ctx->opt.geo_decimate);
  const uint64_t M = D >> logf, f = (uint64_t)1 << logf;
  const fe qf = fe_pow(q, f);  // order M
  P.logf = logf;
  P.M = M;
  P.qf = qf;
  // Z(q^(f k)) (k < M) and 1 / Z'(q^i) (i < n): they depend on the domain only, so the context keeps
  // them like a twiddle plan (else `cache` shares them between the calls of one prove)
  const std::vector<uint64_t> key = {kDomainGeoInterp, fe_lo(q), fe_hi(q), D, n, (uint64_t)logf};
  const fe* Zv = ctx->domain_cache_on() ? static_cast<const fe*>(ctx->domain_table(key)) : nullptr;
  const fe* Zdi = Zv ? Zv + M : nullptr;
  GeoInterpCache& zc = *cache;
  if (!Zv) {
    if (!(zc.n == n && zc.D == D && zc.logf == logf && fe_eq(zc.q, q))) {
      DPoly Z = zerofier_geometric_dev(ctx, q, D, n);
      DevBuf Zd(ctx, n * sizeof(fe));
      DevBuf Zfull(ctx, D * sizeof(fe));
      ntt_sized(ctx, q, Z.p(), n + 1, logD, Zfull.as<fe>());
      zc.Zv = DevBuf(ctx, M * sizeof(fe));
      SG_HIP(launch_gather_stride(zc.Zv.as<fe>(), Zfull.as<fe>(), M, f, ctx->stream));  // Z(q^(f k))
      zc.Zdi = DevBuf(ctx, n * sizeof(fe));
      SG_HIP(launch_deriv(Zd.as<fe>(), Z.p(), n, fe_r2(), ctx->stream));
      // Z'(q^i) for i < n (the first n values of its size-D transform), inverted once
      ntt_sized(ctx, q, Zd.as<fe>(), n, logD, Zfull.as<fe>());
      dev_div(ctx, zc.Zdi.as<fe>(), nullptr, Zfull.as<fe>(), n);
      zc.q = q;
      zc.D = D;
      zc.n = n;
      zc.logf = logf;
    }
    Zv = zc.Zv.as<fe>();
    Zdi = zc.Zdi.as<fe>();
    if (ctx->domain_cache_on()) {
      // kept only once the inversion is known to have met no zero (the points are distinct, so
      // Z'(q^i) != 0; a table is never cached unchecked)
      host_wait(ctx, ctx->stream);
      check_div_zero(ctx);
      void* t = nullptr;
      SG_HIP(hipMalloc(&t, (M + n) * sizeof(fe)));
      SG_HIP(hipMemcpyAsync(t, Zv, M * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
      SG_HIP(hipMemcpyAsync(static_cast<fe*>(t) + M, Zdi, n * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
      ctx->domain_table_put(key, t);
    }
  }
  P.Zv = Zv;
  P.Zdi = Zdi;
  P.Khat = interp_kernel(ctx, q, D, logf);
  return P;
}

std::vector<DPoly> interpolate_geometric_batch_dev(sg_ctx* ctx, const fe& q, uint64_t D, const fe* y, uint64_t ys,
                                                   size_t cols, uint64_t n, GeoInterpCache* cache) {
  SG_REQUIRE(n <= D, "interpolate: more points than the order of the root");
  SG_REQUIRE(D && (D & (D - 1)) == 0, "interpolate: root order must be a power of two");
  std::vector<DPoly> outs;
  if (n <= 1 || n == D) {
    for (size_t c = 0; c < cols; ++c) {
      if (n == 0) {
        outs.emplace_back();
      } else if (n == 1) {
        outs.push_back(dpoly_copy(ctx, y + c * ys, 1));
      } else {
        DPoly out = dpoly_alloc(ctx, D);
        intt_sized(ctx, q, y + c * ys, ilog2_exact(D), out.p());
        outs.push_back(std::move(out));
      }
    }
    return outs;
  }
  const int logD = ilog2_exact(D);
  GeoInterpCache local;
  const GeoPlan P = geo_plan(ctx, q, D, n, cache ? cache : &local);
  const int logf = P.logf;
  const uint64_t M = P.M, f = (uint64_t)1 << P.logf;
  const int logM = logD - logf;
  const fe qf = P.qf;
  const fe* Zv = P.Zv;
  const fe* Zdi = P.Zdi;
  // a_i = y_i / Z'(q^i); S(m) = sum_i a_i b[m - i] cyclically, b[j] = 1 / (1 - q^-j).  At m = f k the f
  // residue classes i = f j + r each give a cyclic convolution of length M (root q^f) against the
  // row K_r: their transforms are summed pointwise and share one inverse transform.
  const fe* Khat = P.Khat;
  DevBuf va(ctx, cols * D * sizeof(fe)), S(ctx, cols * M * sizeof(fe));
  if (logf == 0) {
    DevBuf a(ctx, n * sizeof(fe));
    for (size_t c = 0; c < cols; ++c) {
      dev_mul(ctx, a.as<fe>(), y + c * ys, Zdi, n);
      ntt_sized(ctx, q, a.as<fe>(), n, logD, va.as<fe>() + c * D);
      dev_mul(ctx, va.as<fe>() + c * D, va.as<fe>() + c * D, Khat, D);
    }
    S = std::move(va);
    va = DevBuf(ctx, cols * M * sizeof(fe));
  } else {
    const uint64_t Mf = M >> logf;  // every residue class has < n / f + 1 <= Mf entries
    DevBuf rows(ctx, cols * M * sizeof(fe));
    SG_HIP(launch_geo_rows(rows.as<fe>(), y, ys, Zdi, n, logf, M, cols, fe_r2(), ctx->stream));
    // cols * f transforms of length M from Mf inputs each (the first logf stages are copies)
    const fe* tw = ctx->stage_twiddles(qf, logM);
    const fe* in0 = rows.as<fe>();
    fe* out0 = va.as<fe>();
    SG_HIP(launch_ntt_fused(&out0, &in0, (int)(cols * f), Mf, logM, tw, nullptr, nullptr, logf, nullptr, ctx->stream,
                            Mf, M));
    SG_HIP(launch_geo_dot(S.as<fe>(), va.as<fe>(), Khat, logf, M, cols, fe_r2(), ctx->stream));
  }
  // S(f k) for every column (one batched inverse transform), then P(q^(f k)), then the coefficients
  ntt_rows_inverse(ctx, qf, S.as<fe>(), cols, logM, va.as<fe>());
  const fe *iA, *iB;
  pow_tables2(ctx, fe_inv(q), D, &iA, &iB);
  SG_HIP(launch_interp_assemble(S.as<fe>(), y, ys, Zv, va.as<fe>(), n, M, logf, cols, iA, iB, fe_r2(),
                                ctx->stream));
  // the coefficients land in each result's own buffer (D >= n slots, zero above M: degree < n <= M),
  // up to kNttBatch columns' inverse transforms per launch
  const fe ninv_m = to_mont(fe_inv(fe_from_u64(M)));
  for (size_t c0 = 0; c0 < cols; c0 += kNttBatch) {
    const int nb = (int)std::min<size_t>(kNttBatch, cols - c0);
    fe* o[kNttBatch] = {};
    const fe* in[kNttBatch] = {};
    for (int k = 0; k < nb; ++k) {
      DPoly out = dpoly_alloc(ctx, D);
      if (M < D) SG_HIP(hipMemsetAsync(out.p() + M, 0, (D - M) * sizeof(fe), ctx->stream));
      out.len = n;
      o[k] = out.p();
      in[k] = S.as<fe>() + (c0 + k) * M;
      outs.push_back(std::move(out));
    }
    if (M < 2 || M > kNttBatchMaxOrder) {
      for (int k = 0; k < nb; ++k) intt_sized(ctx, qf, in[k], logM, o[k]);
    } else {
      ntt_run(ctx, o, in, nb, M, logM, fe_inv(qf), nullptr, nullptr, 0, &ninv_m);
    }
  }
  return outs;
}

DPoly interpolate_geometric_dev(sg_ctx* ctx, const fe& q, uint64_t D, const fe* y, uint64_t n, GeoInterpCache* cache) {
  return std::move(interpolate_geometric_batch_dev(ctx, q, D, y, 0, 1, n, cache)[0]);
}

void coset_interpolate_dev(sg_ctx* ctx, const fe* values, uint64_t L, const fe& offset, fe* out) {
  const fe w = root_of_order(L);
  DevBuf c(ctx, L * sizeof(fe));
  intt_sized(ctx, w, values, ilog2_exact(L), c.as<fe>());
  dev_scale_pow(ctx, out, c.as<fe>(), L, fe_inv(offset));
}

void coset_values_dev(sg_ctx* ctx, const fe* coeffs, uint64_t len, uint64_t L, const fe& offset, fe* out) {
  SG_REQUIRE(len <= L, "coset values: polynomial longer than the domain");
  ntt_sized(ctx, root_of_order(L), coeffs, len, ilog2_exact(L), out, &offset);
}

// ------------------------------------------------------------------ arbitrary domains

// `rows` contiguous transforms of 2^logn (row stride 2^logn in and out); post (host, Montgomery)
// multiplies every output (the INTT's n^-1)
void ntt_rows_dev(sg_ctx* ctx, const fe& root, const fe* in, uint64_t rows, int logn, fe* out, const fe* post_host) {
  const uint64_t n = (uint64_t)1 << logn;
  SG_REQUIRE(!ranges_overlap(in, n * rows, out, n * rows), "ntt rows: output must not alias the input");
  const fe* tw = ctx->stage_twiddles(root, logn);
  DevBuf dpost;
  const fe* post = nullptr;
  if (post_host) {
    dpost = DevBuf(ctx, sizeof(fe));
    SG_HIP(hipMemcpyAsync(dpost.get(), post_host, sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    post = dpost.as<fe>();
  }
  constexpr uint64_t kRows = 65535;  // grid.y limit
  for (uint64_t r0 = 0; r0 < rows; r0 += kRows) {
    const int cnt = (int)std::min<uint64_t>(kRows, rows - r0);
    fe* o = out + r0 * n;
    const fe* i = in + r0 * n;
    SG_HIP(launch_ntt_fused(&o, &i, cnt, n, logn, tw, nullptr, nullptr, 0, post, ctx->stream, n, n));
  }
}

// `rows` contiguous inverse transforms of 2^logn (intt per row, n^-1 folded into the last pass)
void ntt_rows_inverse(sg_ctx* ctx, const fe& root, const fe* in, uint64_t rows, int logn, fe* out) {
  const fe ninv_m = to_mont(fe_inv(fe_from_u64((uint64_t)1 << logn)));
  ntt_rows_dev(ctx, fe_inv(root), in, rows, logn, out, &ninv_m);
}

// Bottom-up product tree over d_dom[0..n) (see poly_kernels.hip): Z = prod (x - d_i), length n + 1,
// and with d_c, N = sum_i c_i prod_{j != i} (x - d_j), length n.  Exact polynomial products (every
// level's NTT is longer than its products), so the result is the reference's whenever its own
// fast_multiply does not wrap (degree < root_order).
void tree_exact(sg_ctx* ctx, const fe* d_dom, uint64_t n, const fe* d_c, DPoly* Zout, DPoly* Nout) {
  SG_REQUIRE(n >= 1, "product tree: empty domain");
  constexpr int kLeafLog = 3;  // kTreeLeaf = 8 points per lane, level-3 rows of 16
  uint64_t N2 = (uint64_t)1 << kLeafLog;
  while (N2 < n) N2 <<= 1;
  const int L = ilog2_exact(N2);
  const fe r2 = fe_r2();
  uint64_t rows = N2 >> kLeafLog;
  DevBuf Z(ctx, rows * 16 * sizeof(fe)), Nb;
  if (d_c) Nb = DevBuf(ctx, rows * 16 * sizeof(fe));
  SG_HIP(launch_tree_leaves(d_dom, n, rows, Z.as<fe>(), d_c, d_c ? Nb.as<fe>() : nullptr, r2, ctx->stream));
  for (int l = kLeafLog; l < L; ++l) {
    const int logM = l + 1;
    const uint64_t M = (uint64_t)1 << logM, P = rows / 2;
    const fe w = root_of_order(M);
    const fe winv = fe_inv(w);
    const fe minv = to_mont(fe_inv(fe_from_u64(M)));
    DevBuf Zh(ctx, rows * M * sizeof(fe)), Nh;
    ntt_rows_dev(ctx, w, Z.as<fe>(), rows, logM, Zh.as<fe>(), nullptr);
    if (d_c) {
      Nh = DevBuf(ctx, rows * M * sizeof(fe));
      ntt_rows_dev(ctx, w, Nb.as<fe>(), rows, logM, Nh.as<fe>(), nullptr);
    }
    DevBuf Zp(ctx, P * M * sizeof(fe)), Np;
    if (d_c) Np = DevBuf(ctx, P * M * sizeof(fe));
    SG_HIP(launch_tree_combine(Zh.as<fe>(), d_c ? Nh.as<fe>() : nullptr, P, logM, Zp.as<fe>(),
                               d_c ? Np.as<fe>() : nullptr, r2, ctx->stream));
    // back to coefficients (mod x^M - 1), into the next level's rows of 2M
    ntt_rows_dev(ctx, winv, Zp.as<fe>(), P, logM, Zh.as<fe>(), &minv);
    DevBuf Z2(ctx, P * 2 * M * sizeof(fe));
    SG_HIP(launch_tree_fix(Zh.as<fe>(), P, logM, Z2.as<fe>(), n >> logM, ctx->stream));
    Z = std::move(Z2);
    if (d_c) {
      ntt_rows_dev(ctx, winv, Np.as<fe>(), P, logM, Nh.as<fe>(), &minv);
      DevBuf N2b(ctx, P * 2 * M * sizeof(fe));
      SG_HIP(launch_tree_fix(Nh.as<fe>(), P, logM, N2b.as<fe>(), 0, ctx->stream));
      Nb = std::move(N2b);
    }
    rows = P;
  }
  if (Zout) *Zout = dpoly_copy(ctx, Z.as<fe>(), n + 1);
  if (Nout && d_c) *Nout = dpoly_copy(ctx, Nb.as<fe>(), n);
}

namespace {
bool is_pow2(uint64_t v) { return v && (v & (v - 1)) == 0; }
}  // namespace

// ntt_arithmetics.rs:66-113 on any domain (device array d_dom).  A node of the reference's
// recursion (half = len / 2) whose product has degree < root_order (a power of two) is an exact
// product: the product tree.  Larger nodes (degree >= root_order: the reference's fast_multiply
// wraps its cyclic convolution) and every node under a non-power-of-two order follow the
// recursion literally through fast_multiply_dev, so the wrapped results are the reference's too.
DPoly zerofier_any_dev(sg_ctx* ctx, const fe& root, uint64_t root_order, const fe* d_dom, uint64_t n) {
  if (n == 0) return DPoly{};
  if (n == 1 || (is_pow2(root_order) && n < root_order)) {
    DPoly z;
    tree_exact(ctx, d_dom, n, nullptr, &z, nullptr);
    return z;
  }
  const uint64_t half = n / 2;
  DPoly l = zerofier_any_dev(ctx, root, root_order, d_dom, half);
  DPoly r = zerofier_any_dev(ctx, root, root_order, d_dom + half, n - half);
  return fast_multiply_dev(ctx, root, root_order, l.p(), l.len, r.p(), r.len);
}

// ntt_arithmetics.rs:172-237 on any domain: the unique interpolant of degree < n, length n (the
// reference's length: left * Z_right + right * Z_left keeps n coefficients), as
// sum_i y_i / Z'(d_i) * Z / (x - d_i): Z'(d_i) = prod_{j != i} (d_i - d_j) by one O(n^2) kernel,
// the quotients in one batched division (a zero -- a repeated point -- is the reference's
// "divide by zero"), the sum by the product tree.  Exact while every zerofier the reference builds
// (at most ceil(n / 2) points) stays below root_order; above that its result is a wrapped
// artefact, which this path rejects.
DPoly interpolate_any_dev(sg_ctx* ctx, const fe& root, uint64_t root_order, const fe* d_dom, const fe* d_val,
                          uint64_t n) {
  (void)root;
  if (n == 0) return DPoly{};
  if (n == 1) return dpoly_copy(ctx, d_val, 1);
  SG_REQUIRE(is_pow2(root_order) && (n + 1) / 2 < root_order,
             "fast_interpolate_domain: the reference's zerofiers wrap for this domain (ceil(n/2) >= root_order "
             "or a non-power-of-two root_order); not supported");
  DevBuf prod(ctx, n * sizeof(fe)), c(ctx, n * sizeof(fe));
  const fe rn = fe_pow(to_mont(fe_one()), n - 1);  // R^(n-1) mod p
  SG_HIP(launch_bary_prod(d_dom, n, prod.as<fe>(), rn, ctx->stream));
  dev_div(ctx, c.as<fe>(), d_val, prod.as<fe>(), n);
  DPoly out;
  tree_exact(ctx, d_dom, n, c.as<fe>(), nullptr, &out);
  return out;
}

// ------------------------------------------------------------------ host polynomials

int64_t hp_degree(const HPoly& a) {
  for (int64_t i = (int64_t)a.size() - 1; i >= 0; --i)
    if (!fe_is_zero_h(a[i])) return i;
  return -1;
}

HPoly hp_add(const HPoly& a, const HPoly& b) {
  if (hp_degree(a) < 0) return b;
  if (hp_degree(b) < 0) return a;
  HPoly r(std::max(a.size(), b.size()), fe_zero());
  for (size_t i = 0; i < a.size(); ++i) r[i] = fe_add(r[i], a[i]);
  for (size_t i = 0; i < b.size(); ++i) r[i] = fe_add(r[i], b[i]);
  return r;
}

HPoly hp_neg(const HPoly& a) {
  HPoly r(a.size());
  for (size_t i = 0; i < a.size(); ++i) r[i] = fe_neg(a[i]);
  return r;
}

HPoly hp_sub(const HPoly& a, const HPoly& b) { return hp_add(a, hp_neg(b)); }

HPoly hp_mul(const HPoly& a, const HPoly& b) {
  if (a.empty() || b.empty()) return {};
  HPoly r(a.size() + b.size() - 1, fe_zero());
  for (size_t i = 0; i < a.size(); ++i) {
    if (fe_is_zero_h(a[i])) continue;
    fe am = to_mont(a[i]);
    for (size_t j = 0; j < b.size(); ++j) r[i + j] = fe_add(r[i + j], mont_mul(b[j], am));
  }
  return r;
}

HPoly hp_scale(const HPoly& a, const fe& f) {
  HPoly r(a.size());
  fe pw = fe_one();
  for (size_t i = 0; i < a.size(); ++i) {
    r[i] = fe_mul(pw, a[i]);
    pw = fe_mul(pw, f);
  }
  return r;
}

fe hp_eval(const HPoly& a, const fe& x) {
  fe acc = fe_zero();
  fe xm = to_mont(x);
  for (size_t i = a.size(); i-- > 0;) acc = fe_add(mont_mul(acc, xm), a[i]);
  return acc;
}

HPoly hp_zerofier(const std::vector<fe>& domain) {
  if (domain.empty()) return {};
  HPoly acc = {fe_neg(domain[0]), fe_one()};
  for (size_t i = 1; i < domain.size(); ++i) acc = hp_mul(acc, HPoly{fe_neg(domain[i]), fe_one()});
  return acc;
}

HPoly hp_interpolate(const std::vector<fe>& domain, const std::vector<fe>& values) {
  SG_REQUIRE(domain.size() == values.size(), "number of elements in domain does not match number of values");
  const size_t n = domain.size();
  if (n == 0) return {};
  HPoly acc(n, fe_zero());
  for (size_t i = 0; i < n; ++i) {
    HPoly num = {fe_one()};
    fe den = fe_one();
    for (size_t j = 0; j < n; ++j) {
      if (j == i) continue;
      num = hp_mul(num, HPoly{fe_neg(domain[j]), fe_one()});
      den = fe_mul(den, fe_sub(domain[i], domain[j]));
    }
    SG_REQUIRE(!fe_is_zero_h(den), "divide by zero");
    fe c = fe_mul(values[i], fe_inv(den));
    for (size_t k = 0; k < n; ++k) acc[k] = fe_add(acc[k], fe_mul(num[k], c));
  }
  return acc;
}

bool is_geometric(const fe* domain, uint64_t n, const fe& root) {
  fe x = fe_one();
  fe rm = to_mont(root);
  for (uint64_t i = 0; i < n; ++i) {
    if (!fe_eq(domain[i], x)) return false;
    x = mont_mul(x, rm);
  }
  return true;
}

}  // namespace sg

// ====================================================================== C ABI

using namespace sg;

namespace {
sg_poly* wrap(DPoly&& d) {
  sg_poly* p = new sg_poly();
  p->d = std::move(d);
  return p;
}
const fe* dptr(const sg_poly* p) { return p ? p->d.p() : nullptr; }
// ABI calls return after their device work: drain the stream, then report a zero divisor
void done(sg_ctx* ctx) {
  host_wait(ctx, ctx->stream);
  check_div_zero(ctx);
}
uint64_t dlen(const sg_poly* p) { return p ? p->d.len : 0; }
}  // namespace

extern "C" int sg_poly_create(sg_ctx* ctx, const sg_fe* coeffs, size_t len, sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && (coeffs || !len), "null argument");
    set_device(ctx);
    check_canonical(coeffs, len, "coefficients");
    DPoly d = dpoly_upload(ctx, reinterpret_cast<const fe*>(coeffs), len);
    host_wait(ctx, ctx->stream);
    *out = wrap(std::move(d));
  });
}

extern "C" int sg_poly_create_dev(sg_ctx* ctx, const sg_fe* d_coeffs, size_t len, sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && (d_coeffs || !len), "null argument");
    set_device(ctx);
    DPoly d = dpoly_copy(ctx, reinterpret_cast<const fe*>(d_coeffs), len);
    host_wait(ctx, ctx->stream);
    *out = wrap(std::move(d));
  });
}

extern "C" size_t sg_poly_len(const sg_poly* p) { return p ? p->d.len : 0; }
extern "C" const sg_fe* sg_poly_data_dev(const sg_poly* p) {
  return p ? reinterpret_cast<const sg_fe*>(p->d.p()) : nullptr;
}

extern "C" int sg_poly_read(sg_ctx* ctx, const sg_poly* p, sg_fe* out) {
  return guard(ctx, [&] {
    SG_REQUIRE(p && (out || !p->d.len), "null argument");
    set_device(ctx);
    if (p->d.len)
      SG_HIP(hipMemcpyAsync(out, p->d.p(), p->d.len * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_poly_degree(sg_ctx* ctx, const sg_poly* p, int64_t* out) {
  return guard(ctx, [&] {
    SG_REQUIRE(p && out, "null argument");
    set_device(ctx);
    *out = dev_degree(ctx, p->d.p(), p->d.len);
  });
}

extern "C" void sg_poly_free(sg_poly* p) { delete p; }

extern "C" int sg_fast_multiply(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_poly* lhs, const sg_poly* rhs,
                                sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(lhs && rhs && out, "null argument");
    set_device(ctx);
    DPoly r = fast_multiply_dev(ctx, to_fe(root), root_order, dptr(lhs), dlen(lhs), dptr(rhs), dlen(rhs));
    done(ctx);
    *out = wrap(std::move(r));
  });
}

extern "C" int sg_fast_coset_divide(sg_ctx* ctx, sg_fe root, uint64_t root_order, sg_fe offset, const sg_poly* lhs,
                                    const sg_poly* rhs, sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(lhs && rhs && out, "null argument");
    set_device(ctx);
    DPoly r = fast_coset_divide_dev(ctx, to_fe(root), root_order, to_fe(offset), dptr(lhs), dlen(lhs), dptr(rhs),
                                    dlen(rhs));
    done(ctx);
    *out = wrap(std::move(r));
  });
}

extern "C" int sg_fast_zerofier(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_fe* domain, size_t n,
                                sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && (domain || !n), "null argument");
    set_device(ctx);
    check_canonical(domain, n, "domain");
    const fe r = to_fe(root);
    check_root(r, root_order);
    const fe* dom = reinterpret_cast<const fe*>(domain);
    if (n > 1 && is_geometric(dom, n, r) && n <= root_order) {
      DPoly z = zerofier_geometric_dev(ctx, r, root_order, n);
      done(ctx);
      *out = wrap(std::move(z));
      return;
    }
    DPoly dd = dpoly_upload(ctx, dom, n);
    DPoly z = zerofier_any_dev(ctx, r, root_order, dd.p(), n);
    done(ctx);
    *out = wrap(std::move(z));
  });
}

extern "C" int sg_fast_interpolate_domain(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_fe* domain,
                                          const sg_fe* values, size_t n, sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && ((domain && values) || !n), "null argument");
    set_device(ctx);
    check_canonical(domain, n, "domain");
    check_canonical(values, n, "values");
    const fe r = to_fe(root);
    check_root(r, root_order);
    const fe* dom = reinterpret_cast<const fe*>(domain);
    const fe* val = reinterpret_cast<const fe*>(values);
    if (n > 1 && n <= root_order && is_geometric(dom, n, r)) {
      DPoly y = dpoly_upload(ctx, val, n);
      DPoly ip = interpolate_geometric_dev(ctx, r, root_order, y.p(), n);
      done(ctx);
      *out = wrap(std::move(ip));
      return;
    }
    DPoly dd = dpoly_upload(ctx, dom, n), dv = dpoly_upload(ctx, val, n);
    DPoly ip = interpolate_any_dev(ctx, r, root_order, dd.p(), dv.p(), n);
    done(ctx);
    *out = wrap(std::move(ip));
  });
}

extern "C" int sg_fast_zerofier_geometric(sg_ctx* ctx, sg_fe root, uint64_t root_order, size_t n, sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out, "null argument");
    set_device(ctx);
    check_root(to_fe(root), root_order);
    DPoly z = zerofier_geometric_dev(ctx, to_fe(root), root_order, n);
    done(ctx);
    *out = wrap(std::move(z));
  });
}

extern "C" int sg_fast_interpolate_geometric_dev(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_fe* d_values,
                                                 size_t n, sg_poly** out) {
  return guard(ctx, [&] {
    SG_REQUIRE(out && (d_values || !n), "null argument");
    set_device(ctx);
    check_root(to_fe(root), root_order);
    DPoly ip = interpolate_geometric_dev(ctx, to_fe(root), root_order, reinterpret_cast<const fe*>(d_values), n);
    done(ctx);
    *out = wrap(std::move(ip));
  });
}
