// Library-internal helpers shared by the C-ABI translation units (capi.cpp,
// poly.cpp, stark.cpp): error guard, element conversion, NTT/LDE drivers,
// retained Merkle trees and the FRI driver.
#pragma once
#include <chrono>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/stark_gpu.h"
#include "context.hpp"
#include "knobs.hpp"
#include "fe128.hpp"
#include "kernels.hpp"

// retained device tree: all 2n - 1 digests (merkle_root.rs:7-32 levels, leaf level first)
struct sg_tree {
  uint64_t n = 0;
  int logn = 0;
  sg::DevBuf buf;  // (2n - 1) digests x 8 u64; a lean tree: levels 1.. only (n - 1 digests)
  uint8_t root[64];
  // lean trees (the prove's retained commitments): the levels below `drop` are not kept -- an
  // opening rehashes the 2^drop-leaf block around its leaf from these values, which the tree's
  // owner keeps alive -- so the tree holds 128 / 2^drop B per leaf instead of 128 B
  const sg::fe* leaves = nullptr;
  int drop = 0;
};

namespace sg {
// digest offset of level `level` (>= t->drop) in the tree's buffer: a lean tree's buffer starts at
// level `drop`
inline uint64_t tree_level_offset(const sg_tree* t, int level) {
  return (2 * t->n - 2 * (t->n >> level)) - (2 * t->n - 2 * (t->n >> t->drop));
}
}  // namespace sg

struct sg_fri_state {
  std::vector<sg::DevBuf> codewords;  // round r codeword (device); [0] empty when borrowed
  std::vector<const sg::fe*> cw;      // round r codeword pointer (the caller's buffer for a borrowed round 0)
  std::vector<uint64_t> lengths;
  std::vector<std::unique_ptr<sg_tree>> trees;
};

namespace sg {

inline fe to_fe(sg_fe a) { return fe_make(a.lo, a.hi); }
inline sg_fe from_fe(const fe& a) { return sg_fe{fe_lo(a), fe_hi(a)}; }

// error text of calls made without a context (host-only entry points accept ctx == NULL)
inline std::string& host_last_error() {
  static thread_local std::string s;
  return s;
}

// Host wait for everything queued on stream s: hipStreamSynchronize, or -- while a communicator
// call runs on the context (ctx->watch) -- a polling wait that lets the watch abort a collective
// that never completes (a peer failed) instead of blocking forever.
void host_wait(sg_ctx* ctx, hipStream_t s);

// Runs f, mapping library errors to the C-ABI return code (+ ctx->last_error).
template <class F>
int guard(sg_ctx* ctx, F&& f) {
  struct ProfBind {
    KernelProfiler* prev;
    explicit ProfBind(sg_ctx* c) : prev(g_prof) { g_prof = (c && c->profiling) ? &c->prof : nullptr; }
    ~ProfBind() { g_prof = prev; }
  } bind(ctx);
  try {
    f();
    return SG_OK;
  } catch (const Error& e) {
    if (ctx) {
      ctx->last_error = e.msg;
      // a failed call may leave divisions in flight: drain and clear the zero-divisor flag
      (void)hipStreamSynchronize(ctx->stream);
      if (ctx->div_zero_flag) *reinterpret_cast<volatile uint32_t*>(ctx->div_zero_flag) = 0;
      // the error is reported through the return code and sg_last_error: clear the thread's HIP
      // last error (a failed hipMalloc sets it), so it does not surface in the caller's own HIP calls
      (void)hipGetLastError();
    } else {
      host_last_error() = e.msg;
    }
    return e.code;
  } catch (const std::bad_alloc&) {
    (ctx ? ctx->last_error : host_last_error()) = "host allocation failed";
    return SG_ERR_NOMEM;
  } catch (...) {
    (ctx ? ctx->last_error : host_last_error()) = "unknown error";
    return SG_ERR_INVALID;
  }
}

// device entry points: a context is required (host-only ones accept NULL)
inline void set_device(sg_ctx* ctx) {
  if (!ctx) throw Error{SG_ERR_INVALID, "a GPU context is required"};
  SG_HIP(hipSetDevice(ctx->device));
}

inline int ilog2_exact(uint64_t n) {
  int l = 0;
  while (((uint64_t)1 << l) < n) ++l;
  return l;
}
inline uint64_t next_pow2(uint64_t n) { return n <= 1 ? 1 : (uint64_t)1 << ilog2_exact(n); }
inline uint64_t level_offset(uint64_t n, int level) { return 2 * n - 2 * (n >> level); }

void check_canonical(const sg_fe* v, size_t n, const char* what);
bool ranges_overlap(const fe* a, uint64_t na, const fe* b, uint64_t nb);
// bit-reversal gather + DIT stages of a 2^logn transform (optional offset^i scale via sA/sB, skip, post scale)
void ntt_run(sg_ctx* ctx, fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn, const fe& root,
             const fe* sA, const fe* sB, int skip, const fe* post_host);
// out (next_pow2(n_in)) = ntt(root, in) (fft/ntt.rs:7-49); post: Montgomery constant applied to every output
void ntt_dev(sg_ctx* ctx, const fe& root, const fe* d_in, uint64_t n_in, fe* d_out, const fe* post,
             const fe* scale_offset);
// fft/ntt_arithmetics.rs:161-170 for `batch` (1..4) polynomials of length d
void coset_evaluate_batch(sg_ctx* ctx, const fe& generator, uint64_t root_order, const fe& off,
                          const fe* const* in, size_t d, fe* const* out, int batch);

void build_trees(sg_ctx* ctx, const fe* const* d_leaves, int batch, uint64_t n, std::unique_ptr<sg_tree>* out);
// split form for trees built on another stream: allocate, launch (roots into pinned slots
// slot0..slot0+batch-1), then wait for the published roots
// lean_leaves != nullptr (n >= 2): a lean tree over those values (they must outlive the tree) that
// keeps no digests below level min(drop, log2 n)
std::unique_ptr<sg_tree> new_tree(sg_ctx* ctx, uint64_t n, const fe* lean_leaves = nullptr, int drop = 1);
uint64_t launch_trees(sg_ctx* ctx, const fe* const* d_leaves, int batch, sg_tree* const* trees, int slot0,
                      hipStream_t s);
void finish_trees(sg_ctx* ctx, sg_tree* const* trees, int batch, uint64_t seq, int slot0, hipStream_t s);
sg_tree* build_tree(sg_ctx* ctx, const fe* d_leaves, uint64_t n);
void fill_tree(sg_ctx* ctx, const fe* d_leaves, sg_tree* t, const FoldLeaves* fold = nullptr);
// (s: the stream the tree runs on; nullptr = the context's main stream)
uint64_t fill_tree_launch(sg_ctx* ctx, const fe* d_leaves, sg_tree* t, const FoldLeaves* fold = nullptr,
                          hipStream_t s = nullptr);
void fill_tree_finish(sg_ctx* ctx, sg_tree* t, uint64_t seq, hipStream_t s = nullptr);
void path_indices(const sg_tree* t, uint64_t index, std::vector<uint64_t>& idx);
// launch_gather_abs address of digest i of t (a lean tree's leaf digests: the tagged leaf address)
uint64_t digest_addr(const sg_tree* t, uint64_t i);
void gather_digests(sg_ctx* ctx, const sg_tree* t, const std::vector<uint64_t>& idx, uint8_t* out);

size_t fri_num_rounds(const sg_fri* f);
// fri.rs:88-113 (the reduced-index rejection included)
void sample_indices(const uint8_t* seed, size_t seed_len, size_t size, size_t reduced_size, size_t number,
                    size_t* out);
// SG_PROVE_TIMING=1 (A/B builds, knobs.hpp): host-clock phase marks of the prover on stderr
struct PhaseMarks {
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  PhaseMarks() : on(SG_KNOB(PROVE_TIMING, 0) != 0), t0(std::chrono::steady_clock::now()), last(t0) {}
  void operator()(const char* name) {
    if (!on) return;
    auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "sg-phase %-22s %8.3f ms (at %8.3f)\n", name,
            std::chrono::duration<double, std::milli>(now - last).count(),
            std::chrono::duration<double, std::milli>(now - t0).count());
    last = now;
  }
};

void push_obj(const sg_proof_stream* ps, uint8_t code, const uint8_t* p, size_t len);
// one object's payload, written in place into a native stream (sg_stream_callbacks) or staged
// for the push callback of any other stream: p = begin(code, len); fill p[0..len); commit()
struct ObjWriter {
  const sg_proof_stream* ps;
  std::vector<uint8_t> scratch{};
  uint8_t code = 0;
  bool direct = false;
  uint8_t* begin(uint8_t code, size_t len);
  void commit();
};
void put_u128_be_at(uint8_t* out, const fe& a);
void put_u128_be(std::vector<uint8_t>& out, const fe& a);
// drop: the round trees' levels not kept (lean trees; the sharded prove's tail keeps drop <= 1, which
// its absolute-address openings rehash)
// overlap: called once, after round 0's tree is launched (before any gated round and before the host
// waits for the root); every round's codeword and tree buffer exist by then -- the FRI prove plans
// and uploads its query items there
void fri_commit_dev(sg_ctx* ctx, const sg_fri* f, const fe* d_cw, uint64_t n, const sg_proof_stream* ps,
                    sg_fri_state& st, bool borrow_input = false, int drop = 3,
                    const std::function<void()>& overlap = {});
// Objects pushed after a proof's last Fiat-Shamir draw (the FRI query phase, fri.rs:174-208, and
// the Stark openings, stark.rs:524-560): collected as TailItems, serialized by one device launch
// (k_serialize_tail) and appended with one copy -- straight into a native stream's page-locked
// body, else pushed object by object to the callback stream from pinned staging.  Every object's
// index is entry `sel` of an index table (masked by `mask`): the items are planned and uploaded
// before the indices exist, and only the table follows the seed.
struct TailWriter {
  std::vector<TailItem> items;
  std::vector<size_t> offs;  // header offset of each object in the block
  size_t bytes = 0;
  bool field = false;        // a Value / Leafs object (sets the stream's field header)
  uint8_t* dev = nullptr;    // the context's tail buffer: uploaded items, then the table
  uint8_t* stage = nullptr;  // pinned staging (slot 0): items, then the table
  size_t table_n = 0;
  // Value base[idx]; Leafs a[idx], b[idx], c[idx]; the Path of leaf add + idx (idx = table[sel] & mask;
  // len bounds idx: a larger one reads element 0 rather than faulting, see k_serialize_tail)
  void value(const fe* base, uint64_t len, uint32_t sel, uint64_t mask = ~0ull);
  void leafs(const fe* a, const fe* b, const fe* c, uint64_t len, uint32_t sel, uint64_t mask);
  void path(const sg_tree* t, uint32_t sel, uint64_t mask, uint64_t add = 0);
  // the items to the device ahead of the table (of table_n entries)
  void upload(sg_ctx* ctx, size_t table_n);
  // the table (table_n entries), the serialization launch and the append
  void flush(sg_ctx* ctx, const sg_proof_stream* ps, const uint64_t* table);
};
// The objects a caller appends after the query phase's (the Stark openings), sharing its launch:
// `plan` adds them with table entries sel0 .. sel0 + count - 1, `indices` appends those entries
// once the top-level indices are known.
struct TailExtra {
  size_t count = 0;
  std::function<void(TailWriter& tw, uint32_t sel0)> plan;
  std::function<void(const size_t* top, std::vector<uint64_t>& table)> indices;
};
// fri.rs:210-248 (+ the caller's `extra` objects)
void fri_prove_dev(sg_ctx* ctx, const sg_fri* f, const fe* d_cw, uint64_t n, const sg_proof_stream* ps,
                   size_t* top, const TailExtra* extra = nullptr);

}  // namespace sg
