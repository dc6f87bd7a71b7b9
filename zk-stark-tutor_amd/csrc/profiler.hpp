// Per-kernel timing with HIP events on the launching stream.
// Enabled per context (sg_ctx_profile); every launch records a begin/end event
// pair, its kernel name and its algorithmic bytes (the bytes the algorithm must
// move for that launch).  bench.py reads the totals to report the roofline of
// the dominant kernel from live measurements.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace sg {

struct KernelProfiler {
  // empty: every launch; else only launches whose name equals `only`
  std::string only;
  struct Rec {
    const char* name;
    hipEvent_t a, b;
    uint64_t bytes;
    uint64_t elems;  // transform elements (set on the first launch of an NTT), else 0
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> spare;
  hipEvent_t get() {
    if (!spare.empty()) {
      hipEvent_t e = spare.back();
      spare.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  struct Total {
    uint64_t launches = 0;
    double ms = 0;
    double bytes = 0;
    double elems = 0;
  };
  std::map<std::string, Total> totals;
  // resolve recorded events (caller synchronizes the stream first)
  void drain() {
    for (auto& r : recs) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, r.a, r.b);
      Total& t = totals[r.name];
      t.launches += 1;
      t.ms += ms;
      t.bytes += (double)r.bytes;
      t.elems += (double)r.elems;
      spare.push_back(r.a);
      spare.push_back(r.b);
    }
    recs.clear();
  }
  ~KernelProfiler() {
    for (auto& r : recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto e : spare) (void)hipEventDestroy(e);
  }
};

// the profiler of the context currently driving launches on this thread (or null)
extern thread_local KernelProfiler* g_prof;

struct ProfScope {
  KernelProfiler* p;
  KernelProfiler::Rec r;
  hipStream_t s;
  ProfScope(const char* name, uint64_t bytes, hipStream_t stream, uint64_t elems = 0) : p(g_prof), s(stream) {
    if (p && !p->only.empty() && p->only != name) p = nullptr;
    if (p) {
      r.name = name;
      r.bytes = bytes;
      r.elems = elems;
      r.a = p->get();
      r.b = p->get();
      (void)hipEventRecord(r.a, s);
    }
  }
  ~ProfScope() {
    if (p) {
      (void)hipEventRecord(r.b, s);
      p->recs.push_back(r);
    }
  }
};

}  // namespace sg
