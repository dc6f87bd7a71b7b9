// Library context: device, stream, pooled device buffers, cached twiddle tables.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <string>
#include <utility>
#include <vector>
#include "fe128.hpp"
#include "profiler.hpp"

struct sg_ctx;

namespace sg {

// Error carrying the C-ABI code; thrown inside the library, caught at the boundary.
struct Error {
  int code;
  std::string msg;
};

#define SG_HIP(call)                                                                              \
  do {                                                                                            \
    hipError_t _e = (call);                                                                       \
    if (_e != hipSuccess) /* out of device memory is SG_ERR_NOMEM, anything else SG_ERR_HIP */    \
      throw ::sg::Error{_e == hipErrorOutOfMemory ? -5 : -2, std::string(#call) + ": " + hipGetErrorString(_e)}; \
  } while (0)
#define SG_REQUIRE(cond, msg)                    \
  do {                                           \
    if (!(cond)) throw ::sg::Error{-1, (msg)};   \
  } while (0)

// Device buffer from the context pool (returned to the pool on destruction).
class DevBuf {
 public:
  DevBuf() = default;
  DevBuf(sg_ctx* ctx, size_t bytes);
  ~DevBuf();
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : ctx_(o.ctx_), ptr_(o.ptr_), bytes_(o.bytes_) { o.ptr_ = nullptr; }
  DevBuf& operator=(DevBuf&& o) noexcept;
  void* get() const { return ptr_; }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(ptr_); }
  size_t bytes() const { return bytes_; }

 private:
  sg_ctx* ctx_ = nullptr;
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
};

// Montgomery power table of a root on the device: tw[e] = root^e * R, e < count.
struct PowTable {
  void* ptr = nullptr;
  uint64_t count = 0;
};

}  // namespace sg

struct sg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // second stream: Merkle trees overlapped with the main stream's algebra (stark_prove)
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  std::string last_error;
  // set while a communicator call runs on this context (dist.cpp DistWatch): every host wait
  // (sg::host_wait, the tree-root spin) polls it; it throws -- after aborting the communicator --
  // on an RCCL asynchronous error or when one wait outlasts the communicator's deadline (the
  // argument: seconds this wait has lasted)
  std::function<void(double)> watch;
  // pool: rounded size -> free pointers
  std::multimap<size_t, void*> free_bufs;
  size_t pooled_bytes = 0;
  // bytes of pool buffers handed out and not yet returned (rounded sizes), and their high-water
  // mark since creation / sg_ctx_memory's reset: the working set of the calls (sg_ctx_memory)
  size_t live_bytes = 0, peak_live_bytes = 0;
  // SG_POOL_LIMIT_BYTES (read at creation; 0 = none): alloc fails with SG_ERR_NOMEM past this many
  // live bytes -- the tests drive every allocation point of a prove into the out-of-memory path
  size_t pool_limit = 0;
  // power tables keyed by (root limbs, count)
  std::map<std::pair<std::pair<uint64_t, uint64_t>, uint64_t>, sg::PowTable> pow_tables;
  // host-coherent pinned slots for tree roots (written by the kernel that computes them)
  static constexpr int kRootSlots = 8;   // concurrent trees: stark_prove uses 0..m-1 and 4
  static constexpr int kFlagIndex = 8 * kRootSlots;  // u64 index of the first ready flag
  uint64_t* pinned_roots = nullptr;      // host view, kRootSlots x 64 bytes, then kRootSlots x u64 ready flags
  uint64_t* pinned_roots_dev = nullptr;  // device view of the same memory
  uint64_t root_seq = 0;                 // last sequence number handed to a tree build
  // host-coherent u32 raised (system-scope atomic) by k_batch_div on a zero divisor; read by
  // the host at points where the stream has already drained past the divisions
  uint32_t* div_zero_flag = nullptr;      // host view (inside the pinned_roots allocation)
  uint32_t* div_zero_flag_dev = nullptr;  // device view
  // FRI round gate (k_fri_gate, inside the pinned_roots allocation): the u64 gate word the host
  // raises, the timeout word the kernel raises, the Montgomery K (2 u64) the host writes first
  uint64_t* gate_word = nullptr;  // host views
  uint32_t* gate_timeout = nullptr;
  uint64_t* gate_k = nullptr;
  uint64_t* gate_word_dev = nullptr;  // device views
  uint32_t* gate_timeout_dev = nullptr;
  uint64_t* gate_k_dev = nullptr;
  uint64_t gate_seq = 0;  // last gate value handed out (monotonic over the context's life)
  bool async_dev = false;                // sg_ctx_set_async: _dev transforms return once enqueued
  // per-kernel event timing (sg_ctx_profile)
  bool profiling = false;
  sg::KernelProfiler prof;

  void* alloc(size_t bytes);
  void release(void* p, size_t bytes);
  void trim();
  // device table of Montgomery(root^e) for e < count (cached)
  const sg::fe* pow_table(const sg::fe& root, uint64_t count);
  // stage-major NTT twiddles of `root` for a 2^logn transform (cached)
  const sg::fe* stage_twiddles(const sg::fe& root, int logn);
  std::map<std::pair<std::pair<uint64_t, uint64_t>, int>, void*> stage_tables;
  // geometric interpolation kernels NTT_D(1 / (1 - q^-j)) keyed by (q limbs, D) (poly.cpp)
  std::map<std::pair<std::pair<uint64_t, uint64_t>, uint64_t>, void*> interp_tables;
  // other values that depend only on a proof's public domain (the trace domain's zerofier and its
  // transforms, the transition zerofier's coset values and their inverses), cached like the
  // twiddle plans: key = a tag and the parameters, value = a device buffer owned by the context.
  // SG_NO_DOMAIN_CACHE=1 recomputes them in every call instead.
  std::map<std::vector<uint64_t>, void*> domain_tables;
  // Options of this context (sg_ctx_set_option; every setting writes the same bytes -- tests use
  // them to compare equivalent paths).  The environment sets only domain_cache, at creation
  // (SG_NO_DOMAIN_CACHE=1: public domain / AIR tables recomputed in every call); A/B builds
  // (knobs.hpp) also read SG_AIR_GENERIC, SG_GEO_DECIMATE, SG_LEAN_TREES, SG_STREAM_NO_PIN and
  // SG_DIST_WORLD1_SHARDED here.
  struct Options {
    bool domain_cache = true;    // keep public domain / AIR tables across calls
    bool air_generic = false;    // Rescue AIR through its expanded monomial groups (else factored)
    bool geo_decimate = true;    // decimated geometric interpolation (else the full group)
    bool lean_trees = true;      // retained prove / FRI trees drop their lowest levels
    bool stream_pin = true;      // native proof streams page-lock their buffer for device copies
    bool world1_sharded = false; // a one-rank communicator proves through the four-step path
    int lean_drop = 3;           // the most levels a lean tree drops (0..3)
    bool fri_gate = true;        // FRI rounds queued behind a device gate before their challenge
    int64_t fri_gate_timeout_ms = 60000;  // a gate left this long times out (the call then fails)
  } opt;
  bool domain_cache_on() const { return opt.domain_cache; }
  void* domain_table(const std::vector<uint64_t>& key) const;
  void domain_table_put(const std::vector<uint64_t>& key, void* p) { domain_tables[key] = p; }
  // content-keyed tables (1 / a small divisor's coset values, poly.cpp) are bounded: beyond
  // kBoundedTables the oldest is freed (after both streams drain), so a long-running prover that
  // meets many boundary sets does not grow device memory without limit
  static constexpr size_t kBoundedTables = 64;
  std::vector<std::vector<uint64_t>> bounded_keys;  // insertion order
  void domain_table_put_bounded(const std::vector<uint64_t>& key, void* p);
  // while > 0 (sg::BoundedPin), bounded tables are not evicted: a caller that holds pointers to
  // several of them across further inserts (the sharded boundary quotients keep every divisor
  // shard until their batch is enqueued) pins the cache; the last unpin evicts down to the bound
  int bounded_pins = 0;
  void bounded_evict();
  // pinned host staging buffers (grown on demand): slot 0 uploads gather addresses,
  // slot 1 receives gathered openings -- pageable copies of MBs cost ~10x more
  void* staging_ptr[2] = {nullptr, nullptr};
  size_t staging_bytes[2] = {0, 0};
  void* staging(int slot, size_t bytes);
  // device buffer of a proof's tail items (TailWriter), kept across calls and grown on demand; its
  // upload runs on the side stream (ev_tail), beside the main stream's FRI rounds -- a pool buffer
  // could still be in use by queued main-stream work there
  void* tail_dev = nullptr;
  size_t tail_dev_bytes = 0;
  hipEvent_t ev_tail = nullptr;
  void* tail_buffer(size_t bytes);
  // degree-scan slots (k_last_nonzero_batch): never cleared, each call tagged with a new generation
  unsigned long long* deg_slots = nullptr;
  size_t deg_cap = 0;
  unsigned long long deg_gen = 0;
  // host-coherent copy of the slots (deg_cap entries, then the ready flag), host and device views
  unsigned long long* deg_host = nullptr;
  unsigned long long* deg_host_dev = nullptr;
};

namespace sg {
// RAII pin of the context's bounded table cache (sg_ctx::bounded_pins)
class BoundedPin {
 public:
  explicit BoundedPin(sg_ctx* c) : c_(c) { ++c_->bounded_pins; }
  ~BoundedPin() {
    if (--c_->bounded_pins == 0) {
      try {
        c_->bounded_evict();
      } catch (...) {  // a failed wait leaves the surplus for the next insert
      }
    }
  }
  BoundedPin(const BoundedPin&) = delete;
  BoundedPin& operator=(const BoundedPin&) = delete;

 private:
  sg_ctx* c_;
};

inline size_t pool_round(size_t bytes) {
  size_t r = 256;
  while (r < bytes) r <<= 1;
  return r;
}
}  // namespace sg
