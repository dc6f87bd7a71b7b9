// C ABI of libstarkgpu (include/stark_gpu.h): context, transforms, Merkle, proof
// streams and FRI drivers.  Host logic here restates the reference's control
// flow (fri.rs, merkle_root.rs, fft/ntt.rs) around the gfx950 kernels.
#include <hip/hip_runtime.h>

#include <chrono>
#include <thread>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <exception>
#include <ctime>
#include <memory>
#include <string>
#include <vector>

#include "../../include/stark_gpu.h"
#include "context.hpp"
#include "fe128.hpp"
#include "host_field.hpp"
#include "host_hash.hpp"
#include "kernels.hpp"
#include "transcript.hpp"
#include "internal.hpp"

using namespace sg;

// ======================================================================== context

void* sg_ctx::alloc(size_t bytes) {
  size_t r = pool_round(bytes);
  // test knob: a working-set cap below the device's (SG_POOL_LIMIT_BYTES at context creation)
  if (pool_limit && live_bytes + r > pool_limit)
    throw Error{SG_ERR_NOMEM, "device buffer pool limit (SG_POOL_LIMIT_BYTES) reached"};
  auto it = free_bufs.find(r);
  if (it != free_bufs.end()) {
    void* p = it->second;
    free_bufs.erase(it);
    pooled_bytes -= r;
    live_bytes += r;
    if (live_bytes > peak_live_bytes) peak_live_bytes = live_bytes;
    return p;
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, r);
  if (e != hipSuccess) {
    // a failed hipMalloc also sets the thread's HIP last error: clear it, so the failure does not
    // surface later in the caller's own HIP calls (torch checks hipGetLastError after its launches)
    (void)hipGetLastError();
    // drop the cache and retry once
    trim();
    e = hipMalloc(&p, r);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      throw Error{SG_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)};
    }
  }
  live_bytes += r;
  if (live_bytes > peak_live_bytes) peak_live_bytes = live_bytes;
  return p;
}

void sg_ctx::release(void* p, size_t bytes) {
  if (!p) return;
  size_t r = pool_round(bytes);
  free_bufs.emplace(r, p);
  pooled_bytes += r;
  live_bytes -= r;
}

void sg_ctx::trim() {
  (void)hipStreamSynchronize(stream);
  for (auto& kv : free_bufs) (void)hipFree(kv.second);
  free_bufs.clear();
  pooled_bytes = 0;
}

namespace sg {
DevBuf::DevBuf(sg_ctx* ctx, size_t bytes) : ctx_(ctx), ptr_(ctx->alloc(bytes)), bytes_(bytes) {}
DevBuf::~DevBuf() {
  if (ptr_) ctx_->release(ptr_, bytes_);
}
DevBuf& DevBuf::operator=(DevBuf&& o) noexcept {
  if (this != &o) {
    if (ptr_) ctx_->release(ptr_, bytes_);
    ctx_ = o.ctx_;
    ptr_ = o.ptr_;
    bytes_ = o.bytes_;
    o.ptr_ = nullptr;
  }
  return *this;
}
}  // namespace sg

// Montgomery(root^e), e < count, on the device; cached per (root, count).
const fe* sg_ctx::pow_table(const fe& root, uint64_t count) {
  auto key = std::make_pair(std::make_pair(fe_lo(root), fe_hi(root)), count);
  auto it = pow_tables.find(key);
  if (it != pow_tables.end()) return reinterpret_cast<const fe*>(it->second.ptr);
  uint64_t na = count < 4096 ? count : 4096;
  std::vector<fe> A(na);
  fe rm = to_mont(root);
  fe acc = to_mont(fe_one());
  for (uint64_t i = 0; i < na; ++i) {
    A[i] = acc;
    acc = mont_mul(acc, rm);
  }
  void* table = nullptr;
  SG_HIP(hipMalloc(&table, std::max<uint64_t>(count, 1) * sizeof(fe)));
  // a wait that throws (a poisoned communicator's watch) must not leak the fresh table while the
  // queued launch may still write it
  try {
    if (count <= 4096) {
      SG_HIP(hipMemcpyAsync(table, A.data(), na * sizeof(fe), hipMemcpyHostToDevice, stream));
    } else {
      uint64_t nb = (count + 4095) / 4096;
      std::vector<fe> B(nb);
      fe step = acc;  // Montgomery(root^4096)
      fe b = to_mont(fe_one());
      for (uint64_t i = 0; i < nb; ++i) {
        B[i] = b;
        b = mont_mul(b, step);
      }
      DevBuf dA(this, na * sizeof(fe)), dB(this, nb * sizeof(fe));
      SG_HIP(hipMemcpyAsync(dA.get(), A.data(), na * sizeof(fe), hipMemcpyHostToDevice, stream));
      SG_HIP(hipMemcpyAsync(dB.get(), B.data(), nb * sizeof(fe), hipMemcpyHostToDevice, stream));
      SG_HIP(launch_pow_table(reinterpret_cast<fe*>(table), dA.as<fe>(), dB.as<fe>(), count, stream));
      host_wait(this, stream);  // A/B return to the pool below
    }
    host_wait(this, stream);
  } catch (...) {
    (void)hipStreamSynchronize(stream);
    (void)hipFree(table);
    throw;
  }
  pow_tables[key] = PowTable{table, count};
  return reinterpret_cast<const fe*>(table);
}

void* sg_ctx::staging(int slot, size_t bytes) {
  if (staging_bytes[slot] < bytes) {
    host_wait(this, stream);  // the old buffer may still be in flight
    if (staging_ptr[slot]) (void)hipHostFree(staging_ptr[slot]);
    staging_ptr[slot] = nullptr;
    staging_bytes[slot] = 0;
    size_t r = pool_round(bytes);
    SG_HIP(hipHostMalloc(&staging_ptr[slot], r, hipHostMallocDefault));
    staging_bytes[slot] = r;
  }
  return staging_ptr[slot];
}

void* sg_ctx::tail_buffer(size_t bytes) {
  if (tail_dev_bytes < bytes) {
    host_wait(this, side);  // the old buffer may still be in flight
    host_wait(this, stream);
    if (tail_dev) (void)hipFree(tail_dev);
    tail_dev = nullptr;
    tail_dev_bytes = 0;
    const size_t r = pool_round(bytes);
    SG_HIP(hipMalloc(&tail_dev, r));
    tail_dev_bytes = r;
  }
  return tail_dev;
}

namespace sg {
int ab_knob(const char* name, int def) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : def;
}
}  // namespace sg

void sg_ctx::domain_table_put_bounded(const std::vector<uint64_t>& key, void* p) {
  domain_table_put(key, p);
  bounded_keys.push_back(key);
  if (bounded_pins == 0) bounded_evict();
}

void sg_ctx::bounded_evict() {
  if (bounded_keys.size() <= kBoundedTables) return;
  host_wait(this, stream);  // queued work may still read the oldest tables
  host_wait(this, side);
  while (bounded_keys.size() > kBoundedTables) {
    auto it = domain_tables.find(bounded_keys.front());
    if (it != domain_tables.end()) {
      (void)hipFree(it->second);
      domain_tables.erase(it);
    }
    bounded_keys.erase(bounded_keys.begin());
  }
}

void* sg_ctx::domain_table(const std::vector<uint64_t>& key) const {
  auto it = domain_tables.find(key);
  return it == domain_tables.end() ? nullptr : it->second;
}

const fe* sg_ctx::stage_twiddles(const fe& root, int logn) {
  auto key = std::make_pair(std::make_pair(fe_lo(root), fe_hi(root)), logn);
  auto it = stage_tables.find(key);
  if (it != stage_tables.end()) return reinterpret_cast<const fe*>(it->second);
  // two-level powers of root: A (4096) and B (root^4096 powers) cover every exponent e < n/2
  const uint64_t nb = logn > 13 ? (uint64_t)1 << (logn - 13) : 1;
  const fe* A = pow_table(root, 4096);
  const fe* B = pow_table(fe_pow(root, 4096), nb);
  void* t = nullptr;
  const uint64_t entries = ntt_tw_entries(logn);
  SG_HIP(hipMalloc(&t, entries * sizeof(fe)));
  try {
    SG_HIP(launch_stage_twiddles(reinterpret_cast<fe*>(t), A, B, logn, stream));
    const int cut = ntt_tw_cut(logn);
    if (cut < logn) {  // stages above the cut multiply A[e & 4095] * B[e >> 12] on the fly
      fe* tail = reinterpret_cast<fe*>(t) + (((uint64_t)1 << cut) - 1);
      SG_HIP(hipMemcpyAsync(tail, A, 4096 * sizeof(fe), hipMemcpyDeviceToDevice, stream));
      SG_HIP(hipMemcpyAsync(tail + 4096, B, nb * sizeof(fe), hipMemcpyDeviceToDevice, stream));
    }
    host_wait(this, stream);
  } catch (...) {  // as pow_table: no leak, and no free while queued work may write it
    (void)hipStreamSynchronize(stream);
    (void)hipFree(t);
    throw;
  }
  stage_tables[key] = t;
  return reinterpret_cast<const fe*>(t);
}

// ======================================================================== helpers

namespace sg {

void check_canonical(const sg_fe* v, size_t n, const char* what) {
  for (size_t i = 0; i < n; ++i)
    if (!fe_is_canonical(to_fe(v[i]))) throw Error{SG_ERR_NONCANONICAL, std::string(what) + ": element >= p"};
}

bool ranges_overlap(const fe* a, uint64_t na, const fe* b, uint64_t nb) {
  return a < b + nb && b < a + na;
}

// bit-reversal gather (fused into the first pass when large enough) + DIT stages
void ntt_run(sg_ctx* ctx, fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn, const fe& root,
             const fe* sA, const fe* sB, int skip, const fe* post_host) {
  const fe* tw = logn > 0 ? ctx->stage_twiddles(root, logn) : nullptr;
  DevBuf dpost;
  const fe* post = nullptr;
  if (post_host) {
    dpost = DevBuf(ctx, sizeof(fe));
    SG_HIP(hipMemcpyAsync(dpost.get(), post_host, sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    post = dpost.as<fe>();
  }
  SG_HIP(launch_ntt_fused(out, in, batch, n_in, logn, tw, sA, sB, skip, post, ctx->stream));
  // async mode (sg_ctx_set_async): stream-ordered, the caller synchronizes
  if (!ctx->async_dev) host_wait(ctx, ctx->stream);
}

// out (device, next_pow2(n_in)) = ntt(root, in) ; in may alias nothing in out
void ntt_dev(sg_ctx* ctx, const fe& root, const fe* d_in, uint64_t n_in, fe* d_out, const fe* post,
             const fe* scale_offset) {
  SG_REQUIRE(n_in > 0, "ntt: empty input (reference indexes inputs[0])");
  uint64_t n = next_pow2(n_in);
  int logn = ilog2_exact(n);
  const fe* sA = nullptr;
  const fe* sB = nullptr;
  if (scale_offset) {
    sA = ctx->pow_table(*scale_offset, 4096);
    fe off4096 = fe_pow(*scale_offset, 4096);
    sB = ctx->pow_table(off4096, (n_in + 4095) / 4096);
  }
  SG_REQUIRE(!ranges_overlap(d_in, n_in, d_out, n), "ntt: output must not alias the input");
  ntt_run(ctx, &d_out, &d_in, 1, n_in, logn, root, sA, sB, 0, post);
}

}  // namespace sg

// ======================================================================== C ABI: context

extern "C" int sg_ctx_create(int device, sg_ctx** out) {
  if (!out) return SG_ERR_INVALID;
  *out = nullptr;
  auto* ctx = new (std::nothrow) sg_ctx();
  if (!ctx) return SG_ERR_NOMEM;
  ctx->device = device;
  // the library's runtime environment, read here once: the pool cap (a test
  // knob) and the domain-table cache
  if (const char* pl = getenv("SG_POOL_LIMIT_BYTES")) ctx->pool_limit = (size_t)strtoull(pl, nullptr, 0);
  if (const char* dc = getenv("SG_NO_DOMAIN_CACHE")) ctx->opt.domain_cache = !(*dc && *dc != '0');
#if SG_AB_KNOBS
  ctx->opt.air_generic = ab_knob("SG_AIR_GENERIC", 0) != 0;
  ctx->opt.geo_decimate = ab_knob("SG_GEO_DECIMATE", 1) != 0;
  ctx->opt.lean_trees = ab_knob("SG_LEAN_TREES", 1) != 0;
  ctx->opt.stream_pin = getenv("SG_STREAM_NO_PIN") == nullptr;
  ctx->opt.world1_sharded = ab_knob("SG_DIST_WORLD1_SHARDED", 0) != 0;
  ctx->opt.lean_drop = std::min(std::max(ab_knob("SG_LEAN_DROP", 3), 0), 3);
  ctx->opt.fri_gate = ab_knob("SG_FRI_GATE", 1) != 0;
#endif
  // the main stream (the prove's critical path) at the highest priority, the side stream (its
  // Merkle trees, which otherwise hold every CU while a small main-stream kernel waits) at the
  // lowest: C4 prove 3.05-3.19 -> 2.98-3.03 ms, headline unchanged (profiles/r03_ab_stream_priority*.log).
  // SG_STREAM_PRIORITY=0 (A/B builds) creates both at the default priority.
  const bool prio = SG_KNOB(STREAM_PRIORITY, 1) != 0;
  int prio_low = 0, prio_high = 0;
  if (hipSetDevice(device) != hipSuccess ||
      (prio && hipDeviceGetStreamPriorityRange(&prio_low, &prio_high) != hipSuccess) ||
      hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio ? prio_high : 0) != hipSuccess) {
    delete ctx;
    return SG_ERR_HIP;
  }
  void* pinned = nullptr;
  void* pinned_dev = nullptr;
  // root slots (64 B) + ready flags (u64) + the division zero flag (u32, padded), host-coherent
  constexpr size_t kSlots = sg_ctx::kRootSlots;
  constexpr size_t kPinned = kSlots * 64 + kSlots * 8 + 64 + 64;  // + the FRI gate block
  if (hipStreamCreateWithPriority(&ctx->side, hipStreamNonBlocking, prio ? prio_low : 0) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_tail, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc(&pinned, kPinned, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(&pinned_dev, pinned, 0) != hipSuccess) {
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->ev_tail) (void)hipEventDestroy(ctx->ev_tail);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return SG_ERR_HIP;
  }
  ctx->pinned_roots = reinterpret_cast<uint64_t*>(pinned);
  ctx->pinned_roots_dev = reinterpret_cast<uint64_t*>(pinned_dev);
  memset(pinned, 0, kPinned);
  ctx->div_zero_flag = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(pinned) + kSlots * 72);
  ctx->div_zero_flag_dev = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(pinned_dev) + kSlots * 72);
  {
    uint8_t* gh = reinterpret_cast<uint8_t*>(pinned) + kSlots * 72 + 64;
    uint8_t* gd = reinterpret_cast<uint8_t*>(pinned_dev) + kSlots * 72 + 64;
    ctx->gate_word = reinterpret_cast<uint64_t*>(gh);
    ctx->gate_timeout = reinterpret_cast<uint32_t*>(gh + 8);
    ctx->gate_k = reinterpret_cast<uint64_t*>(gh + 16);
    ctx->gate_word_dev = reinterpret_cast<uint64_t*>(gd);
    ctx->gate_timeout_dev = reinterpret_cast<uint32_t*>(gd + 8);
    ctx->gate_k_dev = reinterpret_cast<uint64_t*>(gd + 16);
  }
  *out = ctx;
  return SG_OK;
}

extern "C" void sg_ctx_destroy(sg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  ctx->trim();
  for (auto& kv : ctx->pow_tables) (void)hipFree(kv.second.ptr);
  for (auto& kv : ctx->stage_tables) (void)hipFree(kv.second);
  for (auto& kv : ctx->interp_tables) (void)hipFree(kv.second);
  for (auto& kv : ctx->domain_tables) (void)hipFree(kv.second);
  for (void* p : ctx->staging_ptr)
    if (p) (void)hipHostFree(p);
  if (ctx->pinned_roots) (void)hipHostFree(ctx->pinned_roots);
  (void)hipEventDestroy(ctx->ev_fork);
  (void)hipEventDestroy(ctx->ev_join);
  (void)hipEventDestroy(ctx->ev_tail);
  if (ctx->tail_dev) (void)hipFree(ctx->tail_dev);
  if (ctx->deg_slots) (void)hipFree(ctx->deg_slots);
  if (ctx->deg_host) (void)hipHostFree(ctx->deg_host);
  (void)hipStreamDestroy(ctx->side);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

extern "C" int sg_ctx_set_async(sg_ctx* ctx, int enable) {
  if (!ctx) return SG_ERR_INVALID;
  ctx->async_dev = enable != 0;
  return SG_OK;
}

extern "C" int sg_ctx_synchronize(sg_ctx* ctx) {
  return guard(ctx, [&] { host_wait(ctx, ctx->stream); });
}

extern "C" int sg_ctx_profile(sg_ctx* ctx, int enable) {
  return guard(ctx, [&] {
    host_wait(ctx, ctx->stream);
    ctx->prof.drain();
    ctx->prof.totals.clear();
    ctx->profiling = enable != 0;
  });
}

extern "C" int sg_ctx_profile_only(sg_ctx* ctx, const char* kernel) {
  return guard(ctx, [&] { ctx->prof.only = kernel ? kernel : ""; });
}

extern "C" int sg_ctx_profile_report(sg_ctx* ctx, char* buf, size_t cap, size_t* len) {
  return guard(ctx, [&] {
    host_wait(ctx, ctx->stream);
    ctx->prof.drain();
    std::string js = "{";
    bool first = true;
    for (auto& kv : ctx->prof.totals) {
      char tmp[256];
      snprintf(tmp, sizeof(tmp), "%s\"%s\": {\"launches\": %llu, \"ms\": %.6f, \"bytes\": %.0f, \"elems\": %.0f}",
               first ? "" : ", ", kv.first.c_str(), (unsigned long long)kv.second.launches, kv.second.ms,
               kv.second.bytes, kv.second.elems);
      js += tmp;
      first = false;
    }
    js += "}";
    if (len) *len = js.size() + 1;
    if (buf) {
      SG_REQUIRE(cap > js.size(), "profile report buffer too small");
      memcpy(buf, js.c_str(), js.size() + 1);
    }
  });
}

extern "C" const char* sg_last_error(const sg_ctx* ctx) {
  return ctx ? ctx->last_error.c_str() : host_last_error().c_str();
}
extern "C" void* sg_ctx_stream(sg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }
extern "C" int sg_ctx_trim(sg_ctx* ctx) {
  return guard(ctx, [&] {
    SG_REQUIRE(ctx, "null context");
    host_wait(ctx, ctx->stream);  // nothing queued may still read a table freed here
    host_wait(ctx, ctx->side);
    ctx->trim();
    for (auto& kv : ctx->pow_tables) (void)hipFree(kv.second.ptr);
    ctx->pow_tables.clear();
    for (auto& kv : ctx->stage_tables) (void)hipFree(kv.second);
    ctx->stage_tables.clear();
    for (auto& kv : ctx->interp_tables) (void)hipFree(kv.second);
    ctx->interp_tables.clear();
    for (auto& kv : ctx->domain_tables) (void)hipFree(kv.second);
    ctx->domain_tables.clear();
    ctx->bounded_keys.clear();
  });
}

extern "C" int sg_ctx_memory(sg_ctx* ctx, uint64_t* live, uint64_t* peak, uint64_t* pooled, uint64_t* device_used,
                             uint64_t* device_total, int reset_peak) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(live && peak && pooled && device_used && device_total, "null output");
    *live = ctx->live_bytes;
    *peak = ctx->peak_live_bytes;
    *pooled = ctx->pooled_bytes;
    size_t fr = 0, tot = 0;
    SG_HIP(hipMemGetInfo(&fr, &tot));
    *device_used = tot - fr;
    *device_total = tot;
    if (reset_peak) ctx->peak_live_bytes = ctx->live_bytes;
  });
}

extern "C" int sg_ctx_cached_tables(const sg_ctx* ctx, size_t* domain_tables, size_t* twiddle_tables) {
  if (!ctx || !domain_tables || !twiddle_tables) return SG_ERR_INVALID;
  *domain_tables = ctx->domain_tables.size();
  *twiddle_tables = ctx->pow_tables.size() + ctx->stage_tables.size() + ctx->interp_tables.size();
  return SG_OK;
}

extern "C" int sg_ctx_set_option(sg_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return SG_ERR_INVALID;
  const std::string n(name);
  const bool v = value != 0;
  if (n == "domain_cache") ctx->opt.domain_cache = v;
  else if (n == "air_generic") ctx->opt.air_generic = v;
  else if (n == "geo_decimate") ctx->opt.geo_decimate = v;
  else if (n == "lean_trees") ctx->opt.lean_trees = v;
  else if (n == "stream_pin") ctx->opt.stream_pin = v;
  else if (n == "world1_sharded") ctx->opt.world1_sharded = v;
  else if (n == "lean_drop" && value >= 0 && value <= 3) ctx->opt.lean_drop = (int)value;
  else if (n == "fri_gate") ctx->opt.fri_gate = v;
  else if (n == "fri_gate_timeout_ms" && value >= 1) ctx->opt.fri_gate_timeout_ms = value;
  else {
    ctx->last_error = "unknown context option: " + n;
    return SG_ERR_INVALID;
  }
  return SG_OK;
}

// HBM copy probe: the read + write rate of a dwordx4 streaming copy of `bytes` (SURVEY.md 8(d):
// "measure actual HBM with a copy kernel on the box"), best of `iters` launches, HIP events on the
// context's stream.  blocks = 0: one 16-byte element per lane (the fastest form); else a
// grid-stride copy over `blocks` x 256 lanes.
extern "C" int sg_hbm_copy_probe(sg_ctx* ctx, size_t bytes, int iters, unsigned blocks, double* gbs) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(gbs && iters >= 1 && bytes >= 16 && bytes % 16 == 0, "bytes must be a positive multiple of 16");
    void *src = nullptr, *dst = nullptr;
    SG_HIP(hipMalloc(&src, bytes));
    hipError_t e = hipMalloc(&dst, bytes);
    if (e != hipSuccess) {
      (void)hipFree(src);
      SG_HIP(e);
    }
    struct Free {
      void* a;
      void* b;
      ~Free() {
        (void)hipFree(a);
        (void)hipFree(b);
      }
    } fr{src, dst};
    SG_HIP(hipMemsetAsync(src, 1, bytes, ctx->stream));
    SG_HIP(launch_copy16(src, dst, bytes, blocks, ctx->stream));  // warm (page mapping, clocks)
    hipEvent_t e0, e1;
    SG_HIP(hipEventCreate(&e0));
    SG_HIP(hipEventCreate(&e1));
    double best = 0;
    for (int it = 0; it < iters; ++it) {
      SG_HIP(hipEventRecord(e0, ctx->stream));
      SG_HIP(launch_copy16(src, dst, bytes, blocks, ctx->stream));
      SG_HIP(hipEventRecord(e1, ctx->stream));
      SG_HIP(hipEventSynchronize(e1));
      float ms = 0;
      SG_HIP(hipEventElapsedTime(&ms, e0, e1));
      best = std::max(best, 2.0 * (double)bytes / ((double)ms * 1e-3) / 1e9);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *gbs = best;
  });
}

// ======================================================================== C ABI: field

extern "C" sg_fe sg_field_prime(void) { return from_fe(fe_prime()); }
extern "C" sg_fe sg_field_generator(void) { return from_fe(fe_generator()); }
extern "C" int sg_primitive_nth_root(uint64_t n, sg_fe* out) {
  if (!out || n == 0 || (n & (n - 1))) return SG_ERR_INVALID;
  fe root = fe_generator();
  unsigned __int128 order = (unsigned __int128)1 << 119;
  while (order != n) {
    root = fe_mul(root, root);
    order >>= 1;
  }
  *out = from_fe(root);
  return SG_OK;
}
extern "C" sg_fe sg_field_sample(const uint8_t* bytes, size_t len) { return from_fe(fe_sample(bytes, len)); }
extern "C" sg_fe sg_fe_mul(sg_fe a, sg_fe b) { return from_fe(fe_mul(to_fe(a), to_fe(b))); }
extern "C" sg_fe sg_fe_inverse(sg_fe a) { return from_fe(fe_inv(to_fe(a))); }
extern "C" sg_fe sg_fe_pow(sg_fe a, uint64_t e) { return from_fe(fe_pow(to_fe(a), e)); }

// ======================================================================== C ABI: transforms

extern "C" int sg_ntt_dev(sg_ctx* ctx, sg_fe root, const sg_fe* d_in, size_t n_in, sg_fe* d_out) {
  return guard(ctx, [&] {
    set_device(ctx);
    ntt_dev(ctx, to_fe(root), reinterpret_cast<const fe*>(d_in), n_in, reinterpret_cast<fe*>(d_out), nullptr,
            nullptr);
  });
}

extern "C" int sg_intt_dev(sg_ctx* ctx, sg_fe root, const sg_fe* d_in, size_t n_in, sg_fe* d_out) {
  return guard(ctx, [&] {
    set_device(ctx);
    if (n_in < 2) {
      // fft/ntt.rs:56-58: returned unchanged
      if (n_in) SG_HIP(hipMemcpyAsync(d_out, d_in, n_in * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
      host_wait(ctx, ctx->stream);
      return;
    }
    uint64_t n = next_pow2(n_in);
    fe ninv_m = to_mont(fe_inv(fe_from_u64(n)));
    fe rinv = fe_inv(to_fe(root));
    ntt_dev(ctx, rinv, reinterpret_cast<const fe*>(d_in), n_in, reinterpret_cast<fe*>(d_out), &ninv_m, nullptr);
  });
}

namespace sg {
// fft/ntt_arithmetics.rs:161-170 for `batch` polynomials of equal length d (one launch per pass)
void coset_evaluate_batch(sg_ctx* ctx, const fe& generator, uint64_t root_order, const fe& off,
                          const fe* const* in, size_t d, fe* const* out, int batch) {
  SG_REQUIRE(d <= root_order, "fast_coset_evaluate: polynomial longer than root_order");
  SG_REQUIRE(root_order > 0, "fast_coset_evaluate: empty evaluation domain");
  SG_REQUIRE(batch >= 1 && batch <= 4, "batch must be 1..4");
  // the ntt pads to next_pow2(root_order); coefficients beyond d are zero
  uint64_t n = next_pow2(root_order);
  int logn = ilog2_exact(n);
  const fe* sA = ctx->pow_table(off, 4096);
  const fe* sB = ctx->pow_table(fe_pow(off, 4096), (std::max<uint64_t>(d, 1) + 4095) / 4096);
  // coefficients occupy the first d of n slots: the first `skip` DIT stages
  // are exact copies (replicated by the gather / first pass) when d <= n >> skip
  int skip = 0;
  while (skip < logn && ((uint64_t)std::max<uint64_t>(d, 1) << (skip + 1)) <= n) ++skip;
  for (int b = 0; b < batch; ++b)
    SG_REQUIRE(!ranges_overlap(in[b], d, out[b], n), "fast_coset_evaluate: output must not alias the input");
  ntt_run(ctx, out, in, batch, d, logn, generator, sA, sB, skip, nullptr);
}
}  // namespace sg

extern "C" int sg_fast_coset_evaluate_dev(sg_ctx* ctx, sg_fe generator, uint64_t root_order, sg_fe offset,
                                          const sg_fe* d_coeffs, size_t d, sg_fe* d_out) {
  return guard(ctx, [&] {
    set_device(ctx);
    const fe* in = reinterpret_cast<const fe*>(d_coeffs);
    fe* out = reinterpret_cast<fe*>(d_out);
    coset_evaluate_batch(ctx, to_fe(generator), root_order, to_fe(offset), &in, d, &out, 1);
  });
}

extern "C" int sg_fast_coset_evaluate_batch_dev(sg_ctx* ctx, sg_fe generator, uint64_t root_order, sg_fe offset,
                                                const sg_fe* const* d_coeffs, size_t d, sg_fe* const* d_out,
                                                size_t batch) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(d_coeffs && d_out && batch >= 1 && batch <= 4, "batch must be 1..4");
    coset_evaluate_batch(ctx, to_fe(generator), root_order, to_fe(offset),
                         reinterpret_cast<const fe* const*>(d_coeffs), d, reinterpret_cast<fe* const*>(d_out),
                         (int)batch);
  });
}

namespace {
// host wrapper: upload, run, download
template <class F>
void host_roundtrip(sg_ctx* ctx, const sg_fe* in, size_t n_in, sg_fe* out, size_t n_out, F&& dev_fn) {
  DevBuf din(ctx, std::max<size_t>(n_in, 1) * sizeof(fe));
  DevBuf dout(ctx, std::max<size_t>(n_out, 1) * sizeof(fe));
  if (n_in) SG_HIP(hipMemcpyAsync(din.get(), in, n_in * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  dev_fn(din.as<sg_fe>(), dout.as<sg_fe>());
  if (n_out) SG_HIP(hipMemcpyAsync(out, dout.get(), n_out * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
  host_wait(ctx, ctx->stream);
}
void throw_if(int rc, sg_ctx* ctx) {
  if (rc != SG_OK) throw Error{rc, ctx->last_error};
}
}  // namespace

extern "C" int sg_ntt(sg_ctx* ctx, sg_fe root, const sg_fe* in, size_t n_in, sg_fe* out) {
  return guard(ctx, [&] {
    SG_REQUIRE(n_in > 0, "ntt: empty input (reference indexes inputs[0])");
    check_canonical(in, n_in, "ntt input");
    check_canonical(&root, 1, "ntt root");
    host_roundtrip(ctx, in, n_in, out, next_pow2(n_in),
                   [&](sg_fe* di, sg_fe* dout) { throw_if(sg_ntt_dev(ctx, root, di, n_in, dout), ctx); });
  });
}

extern "C" int sg_intt(sg_ctx* ctx, sg_fe root, const sg_fe* in, size_t n_in, sg_fe* out) {
  return guard(ctx, [&] {
    check_canonical(in, n_in, "intt input");
    check_canonical(&root, 1, "intt root");
    size_t n_out = n_in < 2 ? n_in : next_pow2(n_in);
    host_roundtrip(ctx, in, n_in, out, n_out,
                   [&](sg_fe* di, sg_fe* dout) { throw_if(sg_intt_dev(ctx, root, di, n_in, dout), ctx); });
  });
}

extern "C" int sg_fast_coset_evaluate(sg_ctx* ctx, sg_fe generator, uint64_t root_order, sg_fe offset,
                                      const sg_fe* coeffs, size_t d, sg_fe* out) {
  return guard(ctx, [&] {
    SG_REQUIRE(d <= root_order, "fast_coset_evaluate: polynomial longer than root_order");
    check_canonical(coeffs, d, "coefficients");
    check_canonical(&offset, 1, "offset");
    check_canonical(&generator, 1, "generator");
    host_roundtrip(ctx, coeffs, d, out, next_pow2(root_order), [&](sg_fe* di, sg_fe* dout) {
      throw_if(sg_fast_coset_evaluate_dev(ctx, generator, root_order, offset, di, d, dout), ctx);
    });
  });
}

// ======================================================================== C ABI: Merkle

namespace sg {

void host_wait(sg_ctx* ctx, hipStream_t s) {
  if (!ctx->watch) {
    SG_HIP(hipStreamSynchronize(s));
    return;
  }
  // a spin like hipStreamSynchronize's own (a sleep would add its timer slack, tens of us, to every
  // wait of a prove); the watch runs about once per millisecond
  const auto t0 = std::chrono::steady_clock::now();
  auto next = t0;
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) SG_HIP(q);
    const auto now = std::chrono::steady_clock::now();
    if (now >= next) {
      ctx->watch(std::chrono::duration<double>(now - t0).count());
      next = now + std::chrono::milliseconds(1);
    }
    __builtin_ia32_pause();
  }
}

// Spin until the tree kernels have published `batch` roots (flag == seq) in slots
// slot0.. .  `s` (the stream the trees run on) is queried now and then so a
// finished-without-flag stream or a kernel error surfaces instead of spinning forever.
void wait_roots(sg_ctx* ctx, int batch, uint64_t seq, int slot0, hipStream_t s) {
  volatile uint64_t* flags = ctx->pinned_roots + sg_ctx::kFlagIndex + slot0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int b = 0; b < batch; ++b) {
    uint32_t spins = 0;
    while (flags[b] != seq) {
      if ((++spins & 255) == 0) {
        if (ctx->watch) ctx->watch(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) {
          if (flags[b] != seq) throw Error{SG_ERR_HIP, "tree root was not published"};
          break;
        }
        if (q != hipErrorNotReady) SG_HIP(q);
      }
      __builtin_ia32_pause();
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
}

std::unique_ptr<sg_tree> new_tree(sg_ctx* ctx, uint64_t n, const fe* lean_leaves, int drop) {
  SG_REQUIRE(n > 0 && (n & (n - 1)) == 0, "Leafs len must be power of two");
  std::unique_ptr<sg_tree> t(new sg_tree());
  t->n = n;
  t->logn = ilog2_exact(n);
  // option lean_trees = 0: every tree keeps all its levels (sg_ctx_set_option; a test compares the
  // layouts in one process)
  const bool lean_on = ctx->opt.lean_trees;
  // option lean_drop = k: at most k levels dropped; never more than 3: an opening rehashes the
  // 2^drop-leaf block around its leaf, and k_serialize_tail's LDS rehash buffers (msg[8][16],
  // mt[16][8]) hold 8-leaf blocks
  drop = std::min(std::min(drop, ctx->opt.lean_drop), 3);
  t->drop = (lean_on && lean_leaves && n >= 2) ? std::min(std::max(drop, 0), t->logn) : 0;
  t->leaves = t->drop ? lean_leaves : nullptr;
  t->buf = DevBuf(ctx, (2 * (n >> t->drop) - 1) * 64);  // levels drop .. log2 n
  return t;
}

// merkle_root.rs:21-32 for `batch` equal-size trees (buffers already allocated) in one
// launch sequence on stream `s`; the roots land in pinned slots slot0.. .  Returns the
// sequence number finish_trees waits for.
//
// The kernel that computes each root also stores it into pinned host memory and
// then raises a ready flag: the host spins on the flags instead of a blocking
// stream synchronisation, so its next launches (Fiat-Shamir -> fold -> next
// tree) follow the root within microseconds.
uint64_t launch_trees(sg_ctx* ctx, const fe* const* d_leaves, int batch, sg_tree* const* trees, int slot0,
                      hipStream_t s) {
  SG_REQUIRE(batch >= 1 && batch <= 4 && slot0 >= 0 && slot0 + batch <= sg_ctx::kRootSlots, "batch must be 1..4");
  uint64_t* bufs[4] = {nullptr, nullptr, nullptr, nullptr};
  uint64_t* roots_dev[4] = {nullptr, nullptr, nullptr, nullptr};
  uint64_t* flags_dev[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int b = 0; b < batch; ++b) {
    SG_REQUIRE(trees[b]->n == trees[0]->n, "trees of one launch must have equal sizes");
    SG_REQUIRE(trees[b]->drop == trees[0]->drop, "trees of one launch must be alike lean");
    bufs[b] = trees[b]->buf.as<uint64_t>();
    roots_dev[b] = ctx->pinned_roots_dev + 8 * (slot0 + b);
    flags_dev[b] = ctx->pinned_roots_dev + sg_ctx::kFlagIndex + slot0 + b;
  }
  const uint64_t seq = ++ctx->root_seq;
  SG_HIP(launch_merkle_tree(d_leaves, bufs, batch, trees[0]->n, roots_dev, s, 0, 0, 0, flags_dev, seq, nullptr,
                            trees[0]->drop));
  return seq;
}

void finish_trees(sg_ctx* ctx, sg_tree* const* trees, int batch, uint64_t seq, int slot0, hipStream_t s) {
  wait_roots(ctx, batch, seq, slot0, s);
  for (int b = 0; b < batch; ++b) memcpy(trees[b]->root, ctx->pinned_roots + 8 * (slot0 + b), 64);
}

void build_trees(sg_ctx* ctx, const fe* const* d_leaves, int batch, uint64_t n, std::unique_ptr<sg_tree>* out) {
  SG_REQUIRE(batch >= 1 && batch <= 4, "batch must be 1..4");
  sg_tree* t[4];
  for (int b = 0; b < batch; ++b) {
    out[b] = new_tree(ctx, n);
    t[b] = out[b].get();
  }
  const uint64_t seq = launch_trees(ctx, d_leaves, batch, t, 0, ctx->stream);
  finish_trees(ctx, t, batch, seq, 0, ctx->stream);
}

// build into a tree whose buffer is already allocated; with `fold`, the leaves are
// the FRI fold of fold->src, computed by the leaf kernel and stored to d_leaves
void fill_tree(sg_ctx* ctx, const fe* d_leaves, sg_tree* t, const FoldLeaves* fold) {
  fill_tree_finish(ctx, t, fill_tree_launch(ctx, d_leaves, t, fold));
}

// fill_tree in two halves, so work can be queued behind the tree before the host waits for its root
uint64_t fill_tree_launch(sg_ctx* ctx, const fe* d_leaves, sg_tree* t, const FoldLeaves* fold, hipStream_t s) {
  uint64_t* buf = t->buf.as<uint64_t>();
  uint64_t* root_dev = ctx->pinned_roots_dev;
  uint64_t* flag_dev = ctx->pinned_roots_dev + sg_ctx::kFlagIndex;
  const uint64_t seq = ++ctx->root_seq;
  SG_HIP(launch_merkle_tree(&d_leaves, &buf, 1, t->n, &root_dev, s ? s : ctx->stream, 0, 0, 0, &flag_dev, seq, fold,
                            t->drop));
  return seq;
}

void fill_tree_finish(sg_ctx* ctx, sg_tree* t, uint64_t seq, hipStream_t s) {
  wait_roots(ctx, 1, seq, 0, s ? s : ctx->stream);
  memcpy(t->root, ctx->pinned_roots, 64);
}

sg_tree* build_tree(sg_ctx* ctx, const fe* d_leaves, uint64_t n) {
  std::unique_ptr<sg_tree> t;
  build_trees(ctx, &d_leaves, 1, n, &t);
  return t.release();
}

// digest indices of the authentication path of `index` (merkle_root.rs:34-53 order: leaf level first)
void path_indices(const sg_tree* t, uint64_t index, std::vector<uint64_t>& idx) {
  for (int lv = 0; lv < t->logn; ++lv) idx.push_back(level_offset(t->n, lv) + ((index >> lv) ^ 1));
}

// the gather address of digest `i` of tree t (launch_gather_abs): a lean tree's leaf digest is
// tagged (bit 0) as the address of the leaf value to rehash
// absolute address of digest i (levels concatenated from the leaves up) of a tree; a lean tree's
// dropped digest (level lv < drop <= 3) is named by its 2^lv-leaf block's first value | 1 | lv << 1,
// which k_gather_abs rehashes
uint64_t digest_addr(const sg_tree* t, uint64_t i) {
  SG_REQUIRE(t->drop <= 3, "gathers rehash at most three dropped levels");
  const uint64_t dropped = 2 * t->n - 2 * (t->n >> t->drop);
  if (i < dropped) {
    int lv = 0;
    while (i >= 2 * t->n - 2 * (t->n >> (lv + 1))) ++lv;
    const uint64_t p = i - (2 * t->n - 2 * (t->n >> lv));  // position within level lv
    return ((uint64_t)(uintptr_t)(t->leaves + (p << lv))) | 1 | ((uint64_t)lv << 1);
  }
  return (uint64_t)(uintptr_t)t->buf.get() + 64 * (i - dropped);  // levels >= drop
}

void gather_digests(sg_ctx* ctx, const sg_tree* t, const std::vector<uint64_t>& idx, uint8_t* out) {
  if (idx.empty()) return;
  std::vector<uint64_t> addr(idx.size());
  for (size_t k = 0; k < idx.size(); ++k) addr[k] = digest_addr(t, idx[k]);
  DevBuf di(ctx, idx.size() * 8), dout(ctx, idx.size() * 64);
  SG_HIP(hipMemcpyAsync(di.get(), addr.data(), addr.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(launch_gather_abs(di.as<uint64_t>(), dout.get(), (uint32_t)idx.size(), true, ctx->stream));
  SG_HIP(hipMemcpyAsync(out, dout.get(), idx.size() * 64, hipMemcpyDeviceToHost, ctx->stream));
  host_wait(ctx, ctx->stream);
}
}  // namespace sg

extern "C" int sg_merkle_build_dev(sg_ctx* ctx, const sg_fe* d_leaves, size_t n, sg_tree** out) {
  return guard(ctx, [&] {
    set_device(ctx);
    *out = build_tree(ctx, reinterpret_cast<const fe*>(d_leaves), n);
  });
}
extern "C" int sg_merkle_build_batch_dev(sg_ctx* ctx, const sg_fe* const* d_leaves, size_t n, size_t batch,
                                         sg_tree** out) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(d_leaves && out && batch >= 1 && batch <= 4, "batch must be 1..4");
    std::unique_ptr<sg_tree> t[4];
    build_trees(ctx, reinterpret_cast<const fe* const*>(d_leaves), (int)batch, n, t);
    for (size_t b = 0; b < batch; ++b) out[b] = t[b].release();
  });
}

extern "C" int sg_tree_root(const sg_tree* t, uint8_t root[64]) {
  if (!t || !root) return SG_ERR_INVALID;
  memcpy(root, t->root, 64);
  return SG_OK;
}
extern "C" size_t sg_tree_leaves(const sg_tree* t) { return t ? t->n : 0; }
extern "C" int sg_tree_open(sg_ctx* ctx, const sg_tree* t, size_t index, uint8_t* path, size_t* path_len) {
  return guard(ctx, [&] {
    SG_REQUIRE(t && index < t->n, "cannot open invalid index");
    SG_REQUIRE(t->n >= 2, "cannot open a 1-leaf tree");
    std::vector<uint64_t> idx;
    path_indices(t, index, idx);
    gather_digests(ctx, t, idx, path);
    if (path_len) *path_len = idx.size();
  });
}
extern "C" void sg_tree_free(sg_ctx* ctx, sg_tree* t) {
  (void)ctx;
  delete t;
}

extern "C" int sg_merkle_commit(sg_ctx* ctx, const sg_fe* leaves, size_t n, uint8_t root[64]) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(n > 0 && (n & (n - 1)) == 0, "Leafs len must be power of two");
    check_canonical(leaves, n, "leaf");
    DevBuf d(ctx, n * sizeof(fe));
    SG_HIP(hipMemcpyAsync(d.get(), leaves, n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    std::unique_ptr<sg_tree> t(build_tree(ctx, d.as<fe>(), n));
    memcpy(root, t->root, 64);
  });
}

extern "C" int sg_merkle_open(sg_ctx* ctx, size_t index, const sg_fe* leaves, size_t n, uint8_t* path,
                              size_t* path_len) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(n > 0 && (n & (n - 1)) == 0, "length must be power of two");
    SG_REQUIRE(index < n, "cannot open invalid index");
    check_canonical(leaves, n, "leaf");
    DevBuf d(ctx, n * sizeof(fe));
    SG_HIP(hipMemcpyAsync(d.get(), leaves, n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    std::unique_ptr<sg_tree> t(build_tree(ctx, d.as<fe>(), n));
    SG_REQUIRE(n >= 2, "cannot open a 1-leaf tree");
    std::vector<uint64_t> idx;
    path_indices(t.get(), index, idx);
    gather_digests(ctx, t.get(), idx, path);
    if (path_len) *path_len = idx.size();
  });
}

namespace {
// decimal string of a canonical element (field_element.rs:46-50)
std::string fe_decimal(const fe& a) {
  unsigned __int128 v = fe_to_u128(a);
  if (v == 0) return "0";
  std::string s;
  while (v) {
    s.push_back((char)('0' + (int)(v % 10)));
    v /= 10;
  }
  std::reverse(s.begin(), s.end());
  return s;
}
}  // namespace

extern "C" int sg_merkle_verify(const uint8_t root[64], size_t index, const uint8_t* path, size_t path_len,
                                sg_fe leaf) {
  // merkle_root.rs:69-95
  if (!root || (path_len && !path)) return SG_ERR_INVALID;
  if (path_len == 0) return SG_ERR_INVALID;  // reference indexes path[0]
  if (path_len < 64 && index >= ((size_t)1 << path_len)) return SG_ERR_INVALID;
  std::string dec = fe_decimal(to_fe(leaf));
  uint8_t h[64], buf[128];
  blake2b512(reinterpret_cast<const uint8_t*>(dec.data()), dec.size(), h);
  for (size_t i = 0; i < path_len; ++i) {
    if (index % 2 == 0) {
      memcpy(buf, h, 64);
      memcpy(buf + 64, path + 64 * i, 64);
    } else {
      memcpy(buf, path + 64 * i, 64);
      memcpy(buf + 64, h, 64);
    }
    blake2b512(buf, 128, h);
    index >>= 1;
  }
  return memcmp(h, root, 64) == 0 ? 1 : 0;
}

// ======================================================================== C ABI: proof streams

struct sg_stream {
  Stream s;
};

namespace {
int stream_push_cb(void* user, uint8_t code, const uint8_t* payload, size_t len) {
  return sg_stream_push(reinterpret_cast<sg_stream*>(user), code, payload, len);
}
int stream_fs_cb(void* user, size_t num_bytes, uint8_t* out) {
  return sg_stream_fiat_shamir_prover(reinterpret_cast<sg_stream*>(user), num_bytes, out);
}
}  // namespace

extern "C" sg_stream* sg_stream_create(void) { return new (std::nothrow) sg_stream(); }
extern "C" sg_stream* sg_stream_create_signature(const uint8_t* document, size_t doc_len) {
  auto* s = new (std::nothrow) sg_stream();
  if (!s) return nullptr;
  s->s.signature = true;
  s->s.prefix.resize(64);
  blake2b512(document, doc_len, s->s.prefix.data());
  return s;
}
extern "C" void sg_stream_destroy(sg_stream* s) { delete s; }
extern "C" sg_proof_stream sg_stream_callbacks(sg_stream* s) {
  sg_proof_stream ps;
  ps.user = s;
  ps.push = stream_push_cb;
  ps.fiat_shamir_prover = stream_fs_cb;
  return ps;
}
extern "C" int sg_stream_push(sg_stream* s, uint8_t code, const uint8_t* payload, size_t len) {
  if (!s || code > 4 || (len && !payload)) return SG_ERR_INVALID;
  try {
    s->s.push(code, payload, len);
  } catch (const std::bad_alloc&) {
    return SG_ERR_NOMEM;
  }
  return SG_OK;
}
extern "C" size_t sg_stream_count(const sg_stream* s) { return s ? s->s.count() : 0; }
extern "C" int sg_stream_digest(const sg_stream* s, uint8_t* out, size_t cap, size_t* len) {
  if (!s) return SG_ERR_INVALID;
  const size_t n = s->s.digest_size(s->s.count());
  if (len) *len = n;
  if (out) {
    if (cap < n) return SG_ERR_INVALID;
    s->s.digest_into(s->s.count(), out);
  }
  return SG_OK;
}
extern "C" int sg_stream_fiat_shamir_prover(const sg_stream* s, size_t num_bytes, uint8_t* out) {
  if (!s || (num_bytes && !out)) return SG_ERR_INVALID;
  // the incremental sponge cache is not part of the stream's logical state
  const_cast<sg_stream*>(s)->s.fiat_shamir_all(num_bytes, out);
  return SG_OK;
}
extern "C" int sg_stream_fiat_shamir_verifier(const sg_stream* s, size_t num_bytes, uint8_t* out) {
  if (!s || (num_bytes && !out)) return SG_ERR_INVALID;
  s->s.fiat_shamir(s->s.read_index, num_bytes, out);
  return SG_OK;
}
extern "C" int sg_stream_pull(sg_stream* s, uint8_t* code, const uint8_t** payload, size_t* len) {
  if (!s) return SG_ERR_INVALID;
  if (s->s.read_index >= s->s.count()) return SG_ERR_INVALID;  // "Cannot pull, queue is empty"
  const size_t i = s->s.read_index++;
  if (code) *code = s->s.code(i);
  if (payload) *payload = s->s.payload(i);
  if (len) *len = s->s.payload_len(i);
  return SG_OK;
}
extern "C" int sg_stream_deserialize(const uint8_t* bytes, size_t len, sg_stream** out) {
  if (!out || (len && !bytes)) return SG_ERR_INVALID;
  auto* s = new (std::nothrow) sg_stream();
  if (!s) return SG_ERR_NOMEM;
  std::string err;
  if (!deserialize_stream(bytes, len, s->s, err)) {
    delete s;
    return SG_ERR_INVALID;
  }
  *out = s;
  return SG_OK;
}

// ======================================================================== C ABI: FRI

namespace sg {

size_t fri_num_rounds(const sg_fri* f) {
  // fri.rs:40-50
  uint64_t len = f->domain_length;
  size_t r = 0;
  while (len > f->expansion_factor && len > 4 * f->num_colinearity_tests) {
    len /= 2;
    ++r;
  }
  return r;
}

void push_obj(const sg_proof_stream* ps, uint8_t code, const uint8_t* p, size_t len) {
  if (ps->push(ps->user, code, p, len) != 0) throw Error{SG_ERR_CALLBACK, "proof stream push callback failed"};
}

uint8_t* ObjWriter::begin(uint8_t code_, size_t len) {
  code = code_;
  if (ps->push == stream_push_cb) {  // a native stream: write the payload in place
    direct = true;
    return reinterpret_cast<sg_stream*>(ps->user)->s.push_reserve(code, len);
  }
  direct = false;
  scratch.resize(len);
  return scratch.data();
}

void ObjWriter::commit() {
  if (!direct) push_obj(ps, code, scratch.data(), scratch.size());
}

void TailWriter::value(const fe* base, uint64_t len, uint32_t sel, uint64_t mask) {
  TailItem it{};
  it.src[0] = (uint64_t)(uintptr_t)base;
  it.n = len;
  it.dst = bytes;
  it.code = SG_OBJ_VALUE;
  it.count = 1;
  it.sel = sel;
  it.mask = mask;
  items.push_back(it);
  offs.push_back(bytes);
  bytes += 9 + 16;
  field = true;
}

void TailWriter::leafs(const fe* a, const fe* b, const fe* c, uint64_t len, uint32_t sel, uint64_t mask) {
  TailItem it{};
  it.src[0] = (uint64_t)(uintptr_t)a;
  it.src[1] = (uint64_t)(uintptr_t)b;
  it.src[2] = (uint64_t)(uintptr_t)c;
  it.n = len;
  it.dst = bytes;
  it.code = SG_OBJ_LEAFS;
  it.count = 3;
  it.sel = sel;
  it.mask = mask;
  items.push_back(it);
  offs.push_back(bytes);
  bytes += 9 + 48;
  field = true;
}

void TailWriter::path(const sg_tree* t, uint32_t sel, uint64_t mask, uint64_t add) {
  SG_REQUIRE(t->logn <= 64, "tree too deep");
  // k_serialize_tail rehashes a lean tree's 2^drop-leaf block in LDS sized for 8 leaves
  SG_REQUIRE(t->drop <= 3, "lean tree drops more than 3 levels");
  TailItem it{};
  it.src[0] = (uint64_t)(uintptr_t)t->buf.get();
  it.src[1] = (uint64_t)(uintptr_t)t->leaves;  // lean: the low siblings are rehashed from these
  it.src[2] = (uint64_t)t->drop;
  it.dst = bytes;
  it.n = t->n;
  it.index = add;
  it.code = SG_OBJ_PATH;
  it.count = (uint32_t)t->logn;
  it.sel = sel;
  it.mask = mask;
  items.push_back(it);
  offs.push_back(bytes);
  bytes += 9 + 72 * (size_t)t->logn;
}

void TailWriter::upload(sg_ctx* ctx, size_t n) {
  table_n = n;
  const size_t ib = items.size() * sizeof(TailItem);
  stage = static_cast<uint8_t*>(ctx->staging(0, ib + 8 * n));
  dev = static_cast<uint8_t*>(ctx->tail_buffer(ib + 8 * n));
  // on the side stream (idle here), so the copy runs beside the main stream's FRI rounds rather
  // than between two of them
  memcpy(stage, items.data(), ib);
  SG_HIP(hipMemcpyAsync(dev, stage, ib, hipMemcpyHostToDevice, ctx->side));
  SG_HIP(hipEventRecord(ctx->ev_tail, ctx->side));
}

void TailWriter::flush(sg_ctx* ctx, const sg_proof_stream* ps, const uint64_t* table) {
  if (items.empty()) return;
  SG_REQUIRE(stage != nullptr, "tail items were not uploaded");
  const size_t ni = items.size(), ib = ni * sizeof(TailItem);
  uint64_t* dtable = reinterpret_cast<uint64_t*>(dev + ib);
  SG_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_tail, 0));  // the items' upload
  if (table_n) {
    memcpy(stage + ib, table, 8 * table_n);
    SG_HIP(hipMemcpyAsync(dtable, stage + ib, 8 * table_n, hipMemcpyHostToDevice, ctx->stream));
  }
  DevBuf dout;
  auto serialize = [&](uint8_t* out) {
    SG_HIP(launch_serialize_tail(reinterpret_cast<const TailItem*>(dev), dtable, (uint32_t)ni, out, bytes, ctx->stream));
  };
  auto serialize_dev = [&]() {
    dout = DevBuf(ctx, bytes);
    serialize(dout.as<uint8_t>());
  };
  if (ps->push == stream_push_cb) {
    // a native stream: the serializer writes the block straight into the page-locked body (its
    // whole-dword stores cross PCIe while later objects are still being assembled, instead of a
    // separate 3-4 MB device-to-host copy after it); through a device buffer and staging when the
    // runtime refuses to page-lock or map the body
    Stream& st = reinterpret_cast<sg_stream*>(ps->user)->s;
    st.body.reserve(st.body.size() + bytes);  // grow first: the registration covers the block
    const bool pinned = ctx->opt.stream_pin && st.body.pin();
    uint8_t* dst = st.append_block(bytes, offs, field);
    // (a body registered while another device was current -- a cached body shared by contexts on
    // several GPUs -- takes the copy: its device address is that device's view)
    if (pinned && st.body.pinned_dev && st.body.pinned_device == ctx->device && SG_KNOB(TAIL_DIRECT, 1)) {
      serialize(st.body.pinned_dev + (dst - st.body.pinned_p));
      // a stream synchronisation (not a query): the runtime's system-scope release that makes the
      // kernel's host-memory stores visible here (no deadline watch: the serializer waits on no peer)
      SG_HIP(hipStreamSynchronize(ctx->stream));
    } else if (pinned) {
      serialize_dev();
      SG_HIP(hipMemcpyAsync(dst, dout.get(), bytes, hipMemcpyDeviceToHost, ctx->stream));
      host_wait(ctx, ctx->stream);
    } else {
      serialize_dev();
      uint8_t* stg = static_cast<uint8_t*>(ctx->staging(1, bytes));
      SG_HIP(hipMemcpyAsync(stg, dout.get(), bytes, hipMemcpyDeviceToHost, ctx->stream));
      host_wait(ctx, ctx->stream);
      memcpy(dst, stg, bytes);
    }
  } else {
    serialize_dev();
    uint8_t* stg = static_cast<uint8_t*>(ctx->staging(1, bytes));
    SG_HIP(hipMemcpyAsync(stg, dout.get(), bytes, hipMemcpyDeviceToHost, ctx->stream));
    host_wait(ctx, ctx->stream);
    for (const TailItem& it : items)
      push_obj(ps, (uint8_t)it.code, stg + it.dst + 9, (it.code == SG_OBJ_PATH ? 72 : 16) * (size_t)it.count);
  }
  items.clear();
  offs.clear();
  bytes = 0;
  field = false;
  stage = nullptr;
  table_n = 0;
}

void put_u128_be_at(uint8_t* out, const fe& a) {
  uint64_t hi = fe_hi(a), lo = fe_lo(a);
  for (int i = 0; i < 8; ++i) out[i] = (uint8_t)(hi >> (8 * (7 - i)));
  for (int i = 0; i < 8; ++i) out[8 + i] = (uint8_t)(lo >> (8 * (7 - i)));
}

void put_u128_be(std::vector<uint8_t>& out, const fe& a) {
  uint64_t hi = fe_hi(a), lo = fe_lo(a);
  for (int i = 7; i >= 0; --i) out.push_back((uint8_t)(hi >> (8 * i)));
  for (int i = 7; i >= 0; --i) out.push_back((uint8_t)(lo >> (8 * i)));
}

// fri.rs:115-172.  Retains every round's codeword and tree in `st`.
void fri_commit_dev(sg_ctx* ctx, const sg_fri* f, const fe* d_cw, uint64_t n, const sg_proof_stream* ps,
                    sg_fri_state& st, bool borrow_input, int drop, const std::function<void()>& overlap) {
  SG_REQUIRE(ps && ps->push && ps->fiat_shamir_prover, "proof stream callbacks required");
  size_t rounds = fri_num_rounds(f);
  SG_REQUIRE(rounds >= 1, "FRI: zero rounds for this domain");
  SG_REQUIRE(n == f->domain_length, "Length of the domain doesnt match the length of initial codeword");
  fe omega = to_fe(f->omega), offset = to_fe(f->offset);
  SG_REQUIRE(fe_is_canonical(omega) && fe_is_canonical(offset), "FRI omega/offset must be canonical");
  // fold tables for the base omega: w^-e for e < n/2 via (e & 4095, e >> 12)
  fe winv = fe_inv(omega);   // w_r^-1 = (w^-1)^(2^r), carried by squaring
  fe oinv = fe_inv(offset);  // o_r^-1 likewise
  const fe* Tlo = ctx->pow_table(winv, 4096);
  const fe* Thi = ctx->pow_table(fe_pow(winv, 4096), (n / 2 + 4095) / 4096 + 1);
  const fe inv2 = fe_inv(fe_from_u64(2));

  // round 0 codeword: copy into a state-owned buffer
  // round 0 codeword: borrowed when the state dies inside the call (prove), else copied
  if (borrow_input) {
    st.codewords.emplace_back();
    st.cw.push_back(d_cw);
  } else {
    st.codewords.emplace_back(ctx, n * sizeof(fe));
    SG_HIP(hipMemcpyAsync(st.codewords[0].get(), d_cw, n * sizeof(fe), hipMemcpyDeviceToDevice, ctx->stream));
    st.cw.push_back(st.codewords[0].as<fe>());
  }
  st.lengths.push_back(n);

  // Everything that does not depend on a challenge is prepared before round 0
  // (buffers, fold constants, the fri.rs:133 order checks), so between a root
  // reaching the host and the fold starting there is only Fiat-Shamir + K.
  struct RoundPlan {
    uint64_t len;
    fe omega, oinv, winv;
  };
  std::vector<RoundPlan> plan(rounds);
  {
    uint64_t len = n;
    for (size_t r = 0; r < rounds; ++r) {
      plan[r] = {len, omega, oinv, winv};
      omega = fe_mul(omega, omega);
      winv = fe_mul(winv, winv);
      oinv = fe_mul(oinv, oinv);
      len /= 2;
    }
  }
  // lean trees over the round codewords the state keeps (the query phase rehashes a leaf sibling);
  // every round's tree exists from here on (the query items are planned before the last root)
  SG_REQUIRE(st.trees.empty(), "FRI state already committed");
  st.trees.resize(rounds);
  for (size_t r = 0; r < rounds; ++r) {
    if (r + 1 < rounds) {
      st.codewords.emplace_back(ctx, (plan[r].len / 2) * sizeof(fe));
      st.cw.push_back(st.codewords.back().as<fe>());
      st.lengths.push_back(plan[r].len / 2);
    }
    st.trees[r] = new_tree(ctx, plan[r].len, st.cw[r], drop);
  }
  // the fri.rs:133 order check of every round before any launch: omega_r = omega^(2^r), so all
  // rounds pass when round 0 does, and a failing round 0 has pushed nothing -- the same error at
  // the same point of the stream as the reference's per-round check
  for (size_t r = 0; r < rounds; ++r)
    SG_REQUIRE(fe_eq(fe_pow(plan[r].omega, plan[r].len - 1), plan[r].winv),
               "error in commit: omega does not have the right order!");
  // Round r >= 1 hashes the fold of round r-1 in the same launch that computes it
  // (the fold is written out too: later rounds and the query phase read it).
  // (round 3's device-side Fiat-Shamir -- a one-wave Keccak per round instead of the host round
  // trip -- was byte-identical but slower, profiles/r03_ab_devfs*.log, and was removed in round 6)
  //
  // Option fri_gate (default): round r + 1's fold + tree are queued before round r's root is
  // awaited, behind k_fri_gate, which holds the stream until the host has written K and raised the
  // gate word -- the launches leave the host <-> device round trip between two rounds.  On any
  // exception the pending gate is raised (the queued round computes with a stale K and is
  // discarded), so the stream never stays blocked.
  const bool gated = ctx->opt.fri_gate && rounds >= 2;
  // Gated rounds alternate between the main and the side stream. Round r + 1's gate then is
  // dispatched as soon as round r - 1's tree ends on its stream, and spins while round r hashes on
  // the other one, so the challenge opens an already running gate instead of a kernel dispatched
  // after round r's tree. No cross-stream event is needed: the host raises round r + 1's gate only
  // after round r's root, so round r's codeword (written by its leaf kernel) is complete, and the
  // gate's system-scope acquire orders the fold's reads after it.
  const bool alt = gated && SG_KNOB(FRI_TWO_STREAMS, 1) != 0;
  auto round_stream = [&](size_t r) { return alt && (r & 1) ? ctx->side : ctx->stream; };
  DevBuf kdev[2];  // K of the gated rounds, one per stream (declared first: the gate is raised before it is released)
  // On an exception the side stream's queued round is drained before the round state's buffers go
  // back to the pool: a later main-stream allocation of that memory is ordered after the main
  // stream's own stale work, not after the side stream's (declared before the gate: raised first).
  struct SideDrain {
    sg_ctx* c;
    bool on;
    int exceptions = std::uncaught_exceptions();
    ~SideDrain() {
      if (on && std::uncaught_exceptions() > exceptions) (void)hipStreamSynchronize(c->side);
    }
  } side_drain{ctx, alt};
  struct GateRelease {
    sg_ctx* c;
    uint64_t pending = 0;
    ~GateRelease() {
      if (pending) __atomic_store_n(c->gate_word, pending, __ATOMIC_RELEASE);
    }
  } gate{ctx};
  if (gated) {
    kdev[0] = DevBuf(ctx, sizeof(fe));
    kdev[1] = DevBuf(ctx, sizeof(fe));
    __atomic_store_n(ctx->gate_timeout, 0u, __ATOMIC_RELAXED);
  }
  const double gate_seconds = ctx->opt.fri_gate_timeout_ms / 1e3;
  const uint64_t last_len = st.lengths.back();
  // the last codeword on the host (pinned staging, allocated before any gate is pending)
  fe* last = static_cast<fe*>(ctx->staging(1, last_len * sizeof(fe)));
  // The last round's codeword (its leaves, folded by its own leaf kernel) is copied to the host
  // right behind its tree, so the copy lands while the host waits for the root.  A gated last
  // round is copied only once its gate is raised: the runtime may complete a small device-to-host
  // copy on the host, waiting for the stream -- behind a pending gate that wait never ends.
  auto copy_last = [&]() {
    SG_HIP(hipMemcpyAsync(last, st.cw.back(), last_len * sizeof(fe), hipMemcpyDeviceToHost, round_stream(rounds - 1)));
  };
  std::vector<uint64_t> seqs(rounds);
  auto launch_round = [&](size_t r, const fe* K) {
    if (r == 0) {
      seqs[0] = fill_tree_launch(ctx, st.cw[0], st.trees[0].get(), nullptr);
    } else {
      // c'[i] = (c[i] + c[i + n/2]) / 2 + K w_r^-i (c[i] - c[i + n/2]), K = alpha offset_r^-1 2^-1,
      // w_r^-i = w^-(i << r) from the round-0 tables
      FoldLeaves fold{};
      fold.src = st.cw[r - 1];
      fold.dst = const_cast<fe*>(st.cw[r]);
      fold.Tlo = Tlo;
      fold.Thi = Thi;
      fold.shift = (int)(r - 1);
      if (K) {
        fold.K = *K;
      } else {
        const uint64_t want = ++ctx->gate_seq;
        gate.pending = want;
        SG_HIP(launch_fri_gate(ctx->gate_word_dev, want, ctx->gate_k_dev, kdev[r & 1].as<fe>(), ctx->gate_timeout_dev,
                               gate_seconds, round_stream(r)));
        fold.Kp = kdev[r & 1].as<fe>();
      }
      seqs[r] = fill_tree_launch(ctx, st.cw[r], st.trees[r].get(), &fold, round_stream(r));
    }
    if (r + 1 == rounds && !gated) copy_last();
  };
  launch_round(0, nullptr);
  // the caller's host work that needs only the round state's buffers runs while round 0's tree (the
  // longest) hashes; its stream work is queued here, before any gate (a copy the runtime completes
  // on the host could otherwise wait on a pending gate)
  if (overlap) overlap();
  // SG_FRI_TIMING=1 (A/B builds): per round, the host's clock (CLOCK_MONOTONIC / CLOCK_BOOTTIME ns)
  // when it starts waiting for the root, sees it, and raises the gate -- to align with a kernel trace
  const bool timing = SG_KNOB(FRI_TIMING, 0) != 0;
  auto stamp = [](clockid_t id) {
    timespec ts;
    clock_gettime(id, &ts);
    return (long long)ts.tv_sec * 1000000000ll + ts.tv_nsec;
  };
  std::vector<long long> tw(timing ? 4 * rounds : 0, 0);
  for (size_t r = 0; r < rounds; ++r) {
    if (gated && r + 1 < rounds) launch_round(r + 1, nullptr);
    if (timing) tw[4 * r] = stamp(CLOCK_MONOTONIC);
    fill_tree_finish(ctx, st.trees[r].get(), seqs[r], round_stream(r));
    if (timing) {
      tw[4 * r + 1] = stamp(CLOCK_MONOTONIC);
      tw[4 * r + 3] = stamp(CLOCK_BOOTTIME);
    }
    push_obj(ps, SG_OBJ_ROOT, st.trees[r]->root, 64);
    if (r == rounds - 1) break;
    uint8_t chal[32];
    if (ps->fiat_shamir_prover(ps->user, 32, chal) != 0)
      throw Error{SG_ERR_CALLBACK, "proof stream fiat_shamir callback failed"};
    fe alpha = fe_sample(chal, 32);
    const fe K = to_mont(fe_mul(fe_mul(alpha, plan[r].oinv), inv2));
    if (gated) {
      ctx->gate_k[0] = fe_lo(K);
      ctx->gate_k[1] = fe_hi(K);
      __atomic_store_n(ctx->gate_word, gate.pending, __ATOMIC_RELEASE);
      gate.pending = 0;
      if (timing) tw[4 * r + 2] = stamp(CLOCK_MONOTONIC);
      if (r + 2 == rounds) copy_last();
    } else {
      launch_round(r + 1, &K);
    }
  }
  // push last codeword (fri.rs:166)
  host_wait(ctx, ctx->stream);
  if (alt) host_wait(ctx, ctx->side);  // the odd rounds (their trees and codewords are read later)
  for (size_t r = 0; timing && r < rounds; ++r)
    fprintf(stderr, "sg-fri %zu %lld %lld %lld boot %lld\n", r, tw[4 * r], tw[4 * r + 1], tw[4 * r + 2], tw[4 * r + 3]);
  if (gated && __atomic_load_n(ctx->gate_timeout, __ATOMIC_ACQUIRE))
    throw Error{SG_ERR_HIP, "FRI round gate timed out (no challenge within " +
                            std::to_string(ctx->opt.fri_gate_timeout_ms) + " ms)"};
  ObjWriter w{ps};
  uint8_t* payload = w.begin(SG_OBJ_CODEWORD, last_len * 16);
  for (uint64_t i = 0; i < last_len; ++i) put_u128_be_at(payload + 16 * i, last[i]);
  w.commit();
}

// fri.rs:60-86
size_t sample_index(const uint8_t* bytes, size_t len, size_t size) {
  int bit = 63 - __builtin_clzll((unsigned long long)size);
  size_t nbytes = (size_t)bit / 8 + 1;
  size_t start = nbytes > len ? 0 : len - nbytes;
  uint64_t acc = 0;
  for (size_t i = start; i < len; ++i) acc = (acc << 8) ^ bytes[i];
  return (size_t)(acc % size);
}

void sample_indices(const uint8_t* seed, size_t seed_len, size_t size, size_t reduced_size, size_t number,
                    size_t* out) {
  SG_REQUIRE(size != 0 && reduced_size != 0, "modulo zero is impossible");
  SG_REQUIRE(number <= 2 * reduced_size, "Not enough entropy in indices with reference to last codeword");
  SG_REQUIRE(number <= reduced_size, "Cannot sample more indices than available in the last codeword");
  std::vector<size_t> reduced;
  std::vector<uint8_t> buf(seed, seed + seed_len);
  size_t count = 0;
  uint8_t h[64];
  while (count < number) {
    blake2b512(buf.data(), buf.size(), h);
    size_t index = sample_index(h, 64, size);
    size_t r = index % reduced_size;
    buf.push_back(0);  // seed || 0^(counter+1) for the next draw
    if (std::find(reduced.begin(), reduced.end(), r) == reduced.end()) {
      out[count++] = index;
      reduced.push_back(r);
    }
  }
}

void fri_prove_dev(sg_ctx* ctx, const sg_fri* f, const fe* d_cw, uint64_t n, const sg_proof_stream* ps,
                   size_t* top, const TailExtra* extra) {
  PhaseMarks mark;
  sg_fri_state st;
  const size_t c = f->num_colinearity_tests;
  // Every opening of every round follows from the top indices (fri.rs:174-208, 231-245): the
  // Leafs / Path objects of all rounds, in the reference's order, and the caller's `extra` objects
  // are planned as items over an index table (entry s < c: top[s], masked to the round's half
  // length -- top % (len_r / 2), the reference's repeated reduction) and uploaded behind round 0's
  // tree while it hashes; after the last round the seed only yields the table, serialized in one launch.
  TailWriter tw;
  auto plan = [&]() {
    if (st.codewords.size() < 2) return;  // reported after the commit, where the reference panics
    const size_t R = st.codewords.size() - 1;  // query rounds
    tw.items.reserve(R * 4 * c + (extra ? 2 * extra->count * 4 : 0));
    tw.offs.reserve(tw.items.capacity());
    for (size_t r = 0; r < R; ++r) {
      const uint64_t half = st.lengths[r] / 2;
      const uint64_t mask = half - 1;  // round lengths are powers of two (Merkle leaves)
      const fe* cur = st.cw[r];
      const fe* nxt = st.cw[r + 1];
      for (size_t s = 0; s < c; ++s) tw.leafs(cur, cur + half, nxt, half, (uint32_t)s, mask);
      const sg_tree* tc = st.trees[r].get();
      const sg_tree* tn = st.trees[r + 1].get();
      for (size_t s = 0; s < c; ++s) {
        tw.path(tc, (uint32_t)s, mask);
        tw.path(tc, (uint32_t)s, mask, half);
        tw.path(tn, (uint32_t)s, mask);
      }
    }
    if (extra && extra->plan) extra->plan(tw, (uint32_t)c);
    tw.upload(ctx, c + (extra ? extra->count : 0));
  };
  fri_commit_dev(ctx, f, d_cw, n, ps, st, /*borrow_input=*/true, 3, plan);
  mark("fri_commit");
  SG_REQUIRE(tw.stage != nullptr, "FRI prove needs at least two rounds (reference indexes codewords[1])");
  uint8_t seed[32];
  if (ps->fiat_shamir_prover(ps->user, 32, seed) != 0)
    throw Error{SG_ERR_CALLBACK, "proof stream fiat_shamir callback failed"};
  sample_indices(seed, 32, st.lengths[1], st.lengths.back(), c, top);
  mark("fri_sample_indices");
  std::vector<uint64_t> table(top, top + c);
  if (extra && extra->indices) extra->indices(top, table);
  SG_REQUIRE(table.size() == tw.table_n, "tail index table size");
  tw.flush(ctx, ps, table.data());  // the round states stay alive until the serialization has read them
  mark("fri_query_push");
}

}  // namespace sg

extern "C" size_t sg_fri_num_rounds(const sg_fri* fri) { return fri ? fri_num_rounds(fri) : 0; }

extern "C" int sg_fri_commit_dev(sg_ctx* ctx, const sg_fri* fri, const sg_fe* d_cw, size_t n,
                                 const sg_proof_stream* ps, sg_fri_state** keep) {
  return guard(ctx, [&] {
    set_device(ctx);
    std::unique_ptr<sg_fri_state> st(new sg_fri_state());
    fri_commit_dev(ctx, fri, reinterpret_cast<const fe*>(d_cw), n, ps, *st, /*borrow_input=*/keep == nullptr);
    if (keep) *keep = st.release();
  });
}

extern "C" int sg_fri_commit(sg_ctx* ctx, const sg_fri* fri, const sg_fe* cw, size_t n, const sg_proof_stream* ps,
                             sg_fri_state** keep) {
  return guard(ctx, [&] {
    set_device(ctx);
    check_canonical(cw, n, "codeword");
    DevBuf d(ctx, std::max<size_t>(n, 1) * sizeof(fe));
    if (n) SG_HIP(hipMemcpyAsync(d.get(), cw, n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    std::unique_ptr<sg_fri_state> st(new sg_fri_state());
    fri_commit_dev(ctx, fri, d.as<fe>(), n, ps, *st);
    if (keep) *keep = st.release();
  });
}

extern "C" int sg_fri_prove_dev(sg_ctx* ctx, const sg_fri* fri, const sg_fe* d_cw, size_t n, const sg_proof_stream* ps,
                                size_t* top) {
  return guard(ctx, [&] {
    set_device(ctx);
    fri_prove_dev(ctx, fri, reinterpret_cast<const fe*>(d_cw), n, ps, top);
  });
}

extern "C" int sg_fri_prove(sg_ctx* ctx, const sg_fri* fri, const sg_fe* cw, size_t n, const sg_proof_stream* ps,
                            size_t* top) {
  return guard(ctx, [&] {
    set_device(ctx);
    check_canonical(cw, n, "codeword");
    DevBuf d(ctx, std::max<size_t>(n, 1) * sizeof(fe));
    if (n) SG_HIP(hipMemcpyAsync(d.get(), cw, n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    fri_prove_dev(ctx, fri, d.as<fe>(), n, ps, top);
  });
}

extern "C" void sg_fri_state_free(sg_ctx* ctx, sg_fri_state* st) {
  (void)ctx;
  delete st;
}

extern "C" int sg_fri_sample_indices(const uint8_t* seed, size_t seed_len, size_t size, size_t reduced_size,
                                     size_t number, size_t* out) {
  return guard(nullptr, [&] { sample_indices(seed, seed_len, size, reduced_size, number, out); });
}

// ======================================================================== C ABI: row-sharded blocks
//
// Building blocks of the multi-GPU path: the four-step NTT's
// local transforms / twiddles / transposes, Merkle forests over runs with the
// top tree over gathered run roots, and the run-sharded FRI fold.  The
// exchange itself (one all-to-all, one all-gather per tree) is done by the
// caller's communicator (starkgpu/dist.py: torch.distributed over RCCL).

struct sg_forest {
  uint64_t run = 0;   // leaves per tree
  uint64_t runs = 0;  // trees
  int logn = 0;
  DevBuf buf;         // runs x (2 run - 1) digests x 8 u64
};

namespace {
// three 4096-entry Montgomery power tables of `base` (exponents < 2^36)
void pow_tables3(sg_ctx* ctx, const fe& base, const fe** T) {
  T[0] = ctx->pow_table(base, 4096);
  T[1] = ctx->pow_table(fe_pow(base, (uint64_t)1 << 12), 4096);
  T[2] = ctx->pow_table(fe_pow(base, (uint64_t)1 << 24), 4096);
}
constexpr uint64_t kRowsPerLaunch = 65535;  // grid.y limit
}  // namespace

extern "C" int sg_ntt_rows_dev(sg_ctx* ctx, sg_fe root, const sg_fe* d_in, size_t n_in, size_t rows, sg_fe* d_out,
                               size_t n) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(d_in && d_out, "null buffer");
    SG_REQUIRE(n > 0 && (n & (n - 1)) == 0, "ntt rows: n must be a power of two");
    SG_REQUIRE(n_in > 0 && n_in <= n, "ntt rows: need 0 < n_in <= n");
    if (rows == 0) return;
    const fe* in = reinterpret_cast<const fe*>(d_in);
    fe* out = reinterpret_cast<fe*>(d_out);
    SG_REQUIRE(!ranges_overlap(in, n_in * rows, out, n * rows), "ntt rows: output must not alias the input");
    const fe r = to_fe(root);
    SG_REQUIRE(fe_is_canonical(r), "root must be canonical");
    const int logn = ilog2_exact(n);
    // a zero tail of 2^skip per row makes the first `skip` stages exact copies
    int skip = 0;
    while (skip < logn && ((uint64_t)n_in << (skip + 1)) <= n) ++skip;
    const fe* tw = logn > 0 ? ctx->stage_twiddles(r, logn) : nullptr;
    for (uint64_t r0 = 0; r0 < rows; r0 += kRowsPerLaunch) {
      const int cnt = (int)std::min<uint64_t>(kRowsPerLaunch, rows - r0);
      fe* o = out + r0 * n;
      const fe* i = in + r0 * n_in;
      SG_HIP(launch_ntt_fused(&o, &i, cnt, n_in, logn, tw, nullptr, nullptr, skip, nullptr, ctx->stream, n_in, n));
    }
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_scale_dev(sg_ctx* ctx, sg_fe* d_data, size_t n, sg_fe c) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(fe_is_canonical(to_fe(c)), "scale: constant must be canonical");
    if (n == 0) return;
    fe cm = to_mont(to_fe(c));
    DevBuf dc(ctx, sizeof(fe));
    SG_HIP(hipMemcpyAsync(dc.get(), &cm, sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    SG_HIP(launch_scale_const(reinterpret_cast<fe*>(d_data), n, dc.as<fe>(), ctx->stream));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_mul_pow_dev(sg_ctx* ctx, sg_fe base, sg_fe* d_data, size_t rows, size_t cols, uint64_t a0,
                              uint64_t a1, uint64_t b0, uint64_t b1) {
  return guard(ctx, [&] {
    set_device(ctx);
    const fe b = to_fe(base);
    SG_REQUIRE(fe_is_canonical(b), "mul_pow: base must be canonical");
    if (rows == 0 || cols == 0) return;
    // largest exponent (a0 + a1 (rows-1)) (cols-1) + b0 + b1 (rows-1) must stay below 2^36
    unsigned __int128 emax = ((unsigned __int128)a0 + (unsigned __int128)a1 * (rows - 1)) * (cols - 1) + b0 +
                             (unsigned __int128)b1 * (rows - 1);
    SG_REQUIRE(emax < ((unsigned __int128)1 << 36), "mul_pow: exponent range exceeds 2^36");
    const fe* T[3];
    pow_tables3(ctx, b, T);
    SG_HIP(launch_mul_pow(reinterpret_cast<fe*>(d_data), rows, cols, a0, a1, b0, b1, T[0], T[1], T[2], ctx->stream));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_transpose_dev(sg_ctx* ctx, const sg_fe* d_in, sg_fe* d_out, size_t A, size_t B, size_t C) {
  return guard(ctx, [&] {
    set_device(ctx);
    const uint64_t total = (uint64_t)A * B * C;
    if (total == 0) return;
    SG_REQUIRE(!ranges_overlap(reinterpret_cast<const fe*>(d_in), total, reinterpret_cast<const fe*>(d_out), total),
               "transpose: output must not alias the input");
    SG_HIP(launch_swap01(reinterpret_cast<const fe*>(d_in), reinterpret_cast<fe*>(d_out), A, B, C, ctx->stream));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_merkle_forest_dev(sg_ctx* ctx, const sg_fe* d_leaves, size_t run, size_t runs, sg_forest** out) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(out && d_leaves, "null argument");
    SG_REQUIRE(run > 0 && (run & (run - 1)) == 0, "Leafs len must be power of two");
    SG_REQUIRE(runs >= 1, "forest: zero runs");
    std::unique_ptr<sg_forest> f(new sg_forest());
    f->run = run;
    f->runs = runs;
    f->logn = ilog2_exact(run);
    const uint64_t per = merkle_tree_digests(run) * 8;  // u64 per tree
    f->buf = DevBuf(ctx, runs * per * 8);
    const fe* leaves = reinterpret_cast<const fe*>(d_leaves);
    for (uint64_t r0 = 0; r0 < runs; r0 += kRowsPerLaunch) {
      const int cnt = (int)std::min<uint64_t>(kRowsPerLaunch, runs - r0);
      const fe* lv = leaves + r0 * run;
      uint64_t* tr = f->buf.as<uint64_t>() + r0 * per;
      SG_HIP(launch_merkle_tree(&lv, &tr, cnt, run, nullptr, ctx->stream, run, per, 0));
    }
    host_wait(ctx, ctx->stream);
    *out = f.release();
  });
}

extern "C" int sg_forest_roots_dev(sg_ctx* ctx, const sg_forest* f, uint8_t* d_roots) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(f && d_roots, "null argument");
    const uint64_t per = merkle_tree_digests(f->run) * 8;
    const uint64_t root_off = (2 * f->run - 2) * 8;
    SG_HIP(launch_gather_roots(f->buf.as<uint64_t>(), per, root_off, reinterpret_cast<uint64_t*>(d_roots), f->runs,
                               ctx->stream));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_forest_open(sg_ctx* ctx, const sg_forest* f, size_t tree, size_t index, uint8_t* path,
                              size_t* path_len) {
  return guard(ctx, [&] {
    SG_REQUIRE(f && tree < f->runs && index < f->run, "cannot open invalid index");
    std::vector<uint64_t> idx;
    const uint64_t base = (uint64_t)tree * merkle_tree_digests(f->run);
    for (int lv = 0; lv < f->logn; ++lv) idx.push_back(base + level_offset(f->run, lv) + ((index >> lv) ^ 1));
    if (!idx.empty()) {
      DevBuf di(ctx, idx.size() * 8), dout(ctx, idx.size() * 64);
      SG_HIP(hipMemcpyAsync(di.get(), idx.data(), idx.size() * 8, hipMemcpyHostToDevice, ctx->stream));
      SG_HIP(launch_gather_digests(f->buf.as<uint64_t>(), di.as<uint64_t>(), dout.as<uint64_t>(),
                                   (uint32_t)idx.size(), ctx->stream));
      SG_HIP(hipMemcpyAsync(path, dout.get(), idx.size() * 64, hipMemcpyDeviceToHost, ctx->stream));
      host_wait(ctx, ctx->stream);
    }
    if (path_len) *path_len = idx.size();
  });
}

extern "C" void sg_forest_free(sg_ctx* ctx, sg_forest* f) {
  (void)ctx;
  delete f;
}

extern "C" int sg_merkle_top_dev(sg_ctx* ctx, const uint8_t* d_digests, size_t n, sg_tree** out) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(out && d_digests, "null argument");
    SG_REQUIRE(n > 0 && (n & (n - 1)) == 0, "Leafs len must be power of two");
    std::unique_ptr<sg_tree> t(new sg_tree());
    t->n = n;
    t->logn = ilog2_exact(n);
    t->buf = DevBuf(ctx, merkle_tree_digests(n) * 64);
    SG_HIP(hipMemcpyAsync(t->buf.get(), d_digests, n * 64, hipMemcpyDeviceToDevice, ctx->stream));
    uint64_t* tr = t->buf.as<uint64_t>();
    uint64_t* root_dev = ctx->pinned_roots_dev;
    if (n > 1) SG_HIP(launch_merkle_tree(nullptr, &tr, 1, n, &root_dev, ctx->stream, 0, 0, 1));
    host_wait(ctx, ctx->stream);
    if (n > 1)
      memcpy(t->root, ctx->pinned_roots, 64);
    else
      SG_HIP(hipMemcpy(t->root, d_digests, 64, hipMemcpyDeviceToHost));
    *out = t.release();
  });
}

extern "C" int sg_fri_fold_runs_dev(sg_ctx* ctx, sg_fe omega, sg_fe offset, sg_fe alpha, const sg_fe* d_in,
                                    size_t n_local, size_t run, size_t run_stride, size_t run_off, size_t n_global,
                                    sg_fe* d_out) {
  return guard(ctx, [&] {
    set_device(ctx);
    SG_REQUIRE(d_in && d_out, "null buffer");
    SG_REQUIRE(n_global >= 2 && (n_global & (n_global - 1)) == 0, "fold: global length must be a power of two >= 2");
    SG_REQUIRE(n_local >= 2 && n_local % 2 == 0 && run > 0, "fold: bad local shape");
    const uint64_t half = n_local / 2;
    SG_REQUIRE(half % run == 0, "fold: runs must tile each half of the shard");
    SG_REQUIRE((half / run) * run_stride == n_global / 2, "fold: partner i + n/2 must be local l + n_local/2");
    SG_REQUIRE(run_off + run <= run_stride, "fold: run offset outside its stride");
    const fe w = to_fe(omega), o = to_fe(offset), a = to_fe(alpha);
    SG_REQUIRE(fe_is_canonical(w) && fe_is_canonical(o) && fe_is_canonical(a), "fold: scalars must be canonical");
    const fe winv = fe_inv(w);
    // fri.rs:133: omega must have order exactly n_global
    SG_REQUIRE(fe_eq(fe_pow(w, n_global - 1), winv), "error in commit: omega does not have the right order!");
    SG_REQUIRE(n_global / 2 <= ((uint64_t)1 << 36), "fold: codeword too long");
    const fe* T[3];
    pow_tables3(ctx, winv, T);
    const fe K = to_mont(fe_mul(fe_mul(a, fe_inv(o)), fe_inv(fe_from_u64(2))));
    SG_REQUIRE(!ranges_overlap(reinterpret_cast<const fe*>(d_in), n_local, reinterpret_cast<const fe*>(d_out), half),
               "fold: output must not alias the input");
    SG_HIP(launch_fri_fold_runs(reinterpret_cast<fe*>(d_out), reinterpret_cast<const fe*>(d_in), half, run, run_stride,
                                run_off, T[0], T[1], T[2], K, ctx->stream));
    host_wait(ctx, ctx->stream);
  });
}
