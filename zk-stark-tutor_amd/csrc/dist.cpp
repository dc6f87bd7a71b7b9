// Multi-GPU LDE / NTT / Merkle / FRI commit behind the C ABI.
//
// One process per GPU; a sg_dist binds a context to a communicator: RCCL over xGMI
// (sg_dist_create: ncclCommInitRank from a unique id, collectives stream-ordered on the
// context's stream) or a host-staged transport the caller supplies (sg_dist_create_transport:
// all-to-all / all-gather callbacks over host buffers -- how the tests run 2 and 8 ranks on one
// GPU over gloo, since RCCL refuses two ranks on one device).  The reference is single-threaded
// and has no counterpart; the data path is the four-step decomposition:
//
//   n = N1 N2, input index j = j1 + N1 j2, output index k = k2 + N2 k1
//   X[k2 + N2 k1] = sum_j1 w_N1^(j1 k1) w^(j1 k2) sum_j2 w_N2^(j2 k2) x[j1 + N1 j2]
//
// with G ranks, rows = N1 / G, R = N2 / G:
//   column shard [rows][row_len]  row r = x[(g rows + r) + N1 j2], zero beyond row_len
//   run shard    [N1][R]          element [k1][c] = X[k1 N2 + g R + c]
//
// Per rank, HBM passes of a forward transform:
//   1. size-N2 NTTs over the column shard; their LAST pass multiplies by w^(j1 k2) and stores
//      straight into the all-to-all send buffer [h][r][c] (kernels.hip NttEpilogue);
//   2. ONE all-to-all (ncclAllToAll): recv = [j1][c];
//   3. size-N1 NTTs over the R interleaved columns of recv, read in place by the first pass
//      (launch_ntt_fused in_il) -- no transpose before them;
//   4. one transpose [c][k1] -> [k1][c] into the run shard (the only extra pass).
// The inverse reads the run shard as the interleaved column shard of (N2, N1) and writes the
// column shard directly (n^-1 folded into its last pass): no extra pass at all.
// For a root of order exactly n the DFT is unique, so outputs are bit-identical to the
// reference's radix-2 DIT (fft/ntt.rs:7-49); roots of smaller order are rejected.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "dist.hpp"
#include "host_field.hpp"
#include "internal.hpp"

struct sg_dist {
  sg_ctx* ctx = nullptr;
  int G = 1, g = 0;
  ncclComm_t comm = nullptr;
  sg_dist_transport tr{};
  bool staged = false;
  // pinned staging for the host transport (grown on demand)
  void* hsend = nullptr;
  void* hrecv = nullptr;
  size_t hsend_bytes = 0, hrecv_bytes = 0;
  // failure containment: a call that fails on this rank may leave its peers inside (or on their
  // way into) a collective this rank never joins.  The communicator is then poisoned: RCCL's is
  // aborted (ncclCommAbort ends the collectives in flight), a caller transport gets its abort hook,
  // and every later call returns SG_ERR_INVALID.  A host wait that outlasts timeout_s
  // (SG_DIST_TIMEOUT_S, default 30 s) or an RCCL asynchronous error poisons it the same way.
  // RCCL communicators also share an out-of-band abort flag: a node-local file named from the
  // unique id (/dev/shm/sg_dist_abort_<hash>) that a poisoned rank creates and every rank's host
  // waits poll (every ~10 ms), so the peers of a failed rank fail within milliseconds instead of
  // waiting out the deadline (one process per GPU of one node; across nodes the deadline applies).
  bool dead = false;
  std::string dead_reason;
  double timeout_s = 30.0;
  std::string abort_path;  // empty: no flag (host transport: the caller's abort hook does this)
  double abort_polled = -1.0;
  // codeword size (log2 elements) at which a sharded FRI commit hands over to the single-GPU
  // rounds: part of the collective schedule, so it is agreed by all ranks (sg_dist_set_fri_tail)
  int fri_tail_log = 20;
  // sg_dist_stark_prove shards the trace-domain algebra (transition / boundary quotients, trace
  // interpolation) from two ranks up; 0 keeps it replicated (SG_DIST_SHARD_ALGEBRA at creation,
  // agreed by every rank like the FRI hand-over)
  int shard_algebra = 1;
  // counters (sg_dist_counters): collectives issued, transition quotients computed sharded
  uint64_t collectives = 0, sharded_quotients = 0, sharded_interpolations = 0;
  ~sg_dist() {
    if (comm) (void)ncclCommDestroy(comm);
    if (hsend) (void)hipHostFree(hsend);
    if (hrecv) (void)hipHostFree(hrecv);
  }
};

namespace sg {

// the out-of-band abort flag: created by a rank that poisons its communicator (first writer wins)
void raise_abort_flag(sg_dist* d, const std::string& why) {
  if (d->abort_path.empty()) return;
  FILE* f = fopen(d->abort_path.c_str(), "wx");  // exclusive: an existing flag keeps the first reason
  if (!f) return;
  fprintf(f, "rank %d of %d: %s", d->g, d->G, why.c_str());
  fclose(f);
}

// "" when no peer has raised the flag, else its text
std::string read_abort_flag(const sg_dist* d) {
  if (d->abort_path.empty()) return "";
  FILE* f = fopen(d->abort_path.c_str(), "r");
  if (!f) return "";
  char buf[512] = {0};
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  return std::string(buf, n).empty() ? std::string("a peer rank failed") : std::string(buf, n);
}

void dist_poison(sg_dist* d, const std::string& why) {
  if (d->dead) return;
  d->dead = true;
  d->dead_reason = why;
  raise_abort_flag(d, why);
  if (d->comm) {
    (void)ncclCommAbort(d->comm);  // ends the collectives in flight on this rank
    d->comm = nullptr;
  }
  if (d->staged && d->tr.abort) d->tr.abort(d->tr.user);
}

int dist_run(sg_dist* d, const std::function<void()>& body) {
  sg_ctx* ctx = d ? d->ctx : nullptr;
  if (d && ctx && d->dead) {
    ctx->last_error = "communicator poisoned by an earlier failure: " + d->dead_reason;
    return SG_ERR_INVALID;
  }
  struct WatchScope {
    sg_ctx* ctx;
    WatchScope(sg_dist* dd, sg_ctx* c) : ctx(c) {
      if (!c) return;
      c->watch = [dd](double waited_s) {
        if (dd->comm) {
          ncclResult_t e = ncclSuccess;
          if (ncclCommGetAsyncError(dd->comm, &e) == ncclSuccess && e != ncclSuccess && e != ncclInProgress) {
            const std::string m = std::string("RCCL asynchronous error: ") + ncclGetErrorString(e);
            dist_poison(dd, m);
            throw Error{SG_ERR_HIP, m};
          }
        }
        // the out-of-band flag, polled about every 10 ms of a wait (a stat-sized file read)
        if (!dd->abort_path.empty() && (waited_s - dd->abort_polled >= 0.01 || waited_s < dd->abort_polled)) {
          dd->abort_polled = waited_s;
          const std::string peer = read_abort_flag(dd);
          if (!peer.empty()) {
            const std::string m = "a peer rank failed (" + peer + ")";
            dist_poison(dd, m);
            throw Error{SG_ERR_HIP, m};
          }
        }
        if (waited_s > dd->timeout_s) {
          const std::string m = "a wait on this communicator outlasted its deadline (SG_DIST_TIMEOUT_S = " +
                                std::to_string(dd->timeout_s) + " s): a peer failed or stalled";
          dist_poison(dd, m);
          throw Error{SG_ERR_HIP, m};
        }
      };
    }
    ~WatchScope() {
      if (ctx) ctx->watch = nullptr;
    }
  } watch(d, ctx);
  return guard(ctx, [&] {
    if (!d || !ctx) throw Error{SG_ERR_INVALID, "null communicator"};
    set_device(ctx);
    try {
      body();
    } catch (const Error& e) {
      // before guard drains the stream: collectives queued on it may wait for peers forever
      dist_poison(d, e.msg);
      throw;
    } catch (...) {
      dist_poison(d, "a call failed on this rank");
      throw;
    }
  });
}

namespace {

#define SG_NCCL(call)                                                                          \
  do {                                                                                         \
    ncclResult_t _r = (call);                                                                  \
    if (_r != ncclSuccess) throw Error{SG_ERR_HIP, std::string(#call) + ": " + ncclGetErrorString(_r)}; \
  } while (0)

constexpr uint64_t kRows = 65532;  // rows per launch: grid.y limit, a multiple of 4 (interleaved tiles)
constexpr size_t kMaxCollBytes = (size_t)1 << 30;  // largest per-peer block of one RCCL collective call

void grow_pinned(void*& p, size_t& have, size_t need) {
  if (have >= need) return;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  have = 0;
  SG_HIP(hipHostMalloc(&p, need, hipHostMallocDefault));
  have = need;
}

// equal-block all-to-all (a2a) or all-gather of `bytes` per rank, device buffers
void exchange(sg_dist* d, const void* dsend, void* drecv, size_t bytes, bool a2a) {
  sg_ctx* ctx = d->ctx;
  const size_t total = bytes * d->G;
  ++d->collectives;
  if (d->comm) {  // RCCL over xGMI, stream-ordered (a 1-rank communicator runs the same calls)
    // one call only while the whole exchange (per-peer block x G) stays within kMaxCollBytes: the
    // wrong data was seen at world 1, where per-peer and total bytes coincide, so which of the two
    // RCCL mishandles is not pinned -- bound both
    if (total <= kMaxCollBytes) {
      if (a2a)
        SG_NCCL(ncclAllToAll(dsend, drecv, bytes, ncclUint8, d->comm, ctx->stream));
      else
        SG_NCCL(ncclAllGather(dsend, drecv, bytes, ncclUint8, d->comm, ctx->stream));
      return;
    }
    // larger exchanges (a 2 GiB C5 shard on one rank, 2^27 at world 2): the same exchange as
    // grouped point-to-point transfers, each group moving at most kMaxCollBytes in all -- a single
    // call of 2^31 bytes returned wrong data on the box (tools/c5_dist_time.py at 2^27, world 1)
    const uint8_t* s8 = static_cast<const uint8_t*>(dsend);
    uint8_t* r8 = static_cast<uint8_t*>(drecv);
    const size_t chunk = std::max<size_t>((kMaxCollBytes / d->G) & ~(size_t)255, 256);
    for (size_t off = 0; off < bytes; off += chunk) {
      const size_t len = std::min(chunk, bytes - off);
      SG_NCCL(ncclGroupStart());
      for (int h = 0; h < d->G; ++h) {
        SG_NCCL(ncclSend(s8 + (a2a ? (size_t)h * bytes : 0) + off, len, ncclUint8, h, d->comm, ctx->stream));
        SG_NCCL(ncclRecv(r8 + (size_t)h * bytes + off, len, ncclUint8, h, d->comm, ctx->stream));
      }
      SG_NCCL(ncclGroupEnd());
    }
    return;
  }
  if (d->G == 1) {
    SG_HIP(hipMemcpyAsync(drecv, dsend, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return;
  }
  const size_t sbytes = a2a ? total : bytes;
  grow_pinned(d->hsend, d->hsend_bytes, sbytes);
  grow_pinned(d->hrecv, d->hrecv_bytes, total);
  SG_HIP(hipMemcpyAsync(d->hsend, dsend, sbytes, hipMemcpyDeviceToHost, ctx->stream));
  host_wait(ctx, ctx->stream);
  const int rc = a2a ? d->tr.all_to_all(d->tr.user, d->hsend, d->hrecv, bytes)
                     : d->tr.all_gather(d->tr.user, d->hsend, d->hrecv, bytes);
  if (rc != 0) throw Error{SG_ERR_CALLBACK, a2a ? "all_to_all transport callback failed"
                                                : "all_gather transport callback failed"};
  SG_HIP(hipMemcpyAsync(drecv, d->hrecv, total, hipMemcpyHostToDevice, ctx->stream));
}

void plan(uint64_t n, int G, uint64_t& n1, uint64_t& n2) {
  SG_REQUIRE(n >= 2 && (n & (n - 1)) == 0, "distributed transform: n must be a power of two >= 2");
  SG_REQUIRE(G >= 1 && (G & (G - 1)) == 0, "distributed transform: the rank count must be a power of two");
  n1 = dist_split(n);
  n2 = n / n1;
  SG_REQUIRE(n1 % G == 0 && n2 % (4 * (uint64_t)G) == 0,
             "distributed transform: n too small for this many ranks (needs N1 >= G and N2 >= 4 G)");
}

void check_order_n(const fe& root, uint64_t n) {
  SG_REQUIRE(fe_is_canonical(root), "root must be canonical");
  SG_REQUIRE(fe_eq(fe_pow(root, n / 2), fe_neg(fe_one())), "distributed ntt needs a root of order exactly n");
}

void tables3(sg_ctx* ctx, const fe& base, const fe** T) {
  T[0] = ctx->pow_table(base, 4096);
  T[1] = ctx->pow_table(fe_pow(base, (uint64_t)1 << 12), 4096);
  T[2] = ctx->pow_table(fe_pow(base, (uint64_t)1 << 24), 4096);
}

// X = DFT_root over (n1, n2): input rows (row_len entries per row, zero beyond; or, with in_il,
// R' interleaved rows of n2 entries: row r's element j at in[j * in_il + r]); output
// [R][n1] rows (row c = k2 - g R, element k1); post: Montgomery constant on every output
//
// nv > 1: nv vectors at once, row r of vector v being row v rows + r of the input (at
// in + (v rows + r) row_len, or interleaved: in_il >= nv rows) and its output row c at
// out + (v R + c) n1 -- one exchange and one launch per step for all of them (the epilogue packs
// [h][r][v][c], so the received block is nv R interleaved columns)
void four_step(sg_dist* d, const fe& root, const fe* in, uint64_t row_len, uint64_t in_il, uint64_t n1, uint64_t n2,
               fe* out, const fe* post_host, uint64_t nv = 1) {
  sg_ctx* ctx = d->ctx;
  const int G = d->G;
  const uint64_t rows = n1 / G, R = n2 / G;
  SG_REQUIRE(nv >= 1 && (!in_il || in_il >= nv * rows), "distributed transform: bad batched layout");
  SG_REQUIRE(row_len >= 1 && row_len <= n2, "distributed transform: row length must be in [1, N2]");
  SG_REQUIRE((uint64_t)n1 * n2 <= ((uint64_t)1 << 36), "distributed transform: n above 2^36");
  const int log1 = ilog2_exact(n1), log2 = ilog2_exact(n2);
  const fe w2 = fe_pow(root, n1);  // order n2
  const fe w1 = fe_pow(root, n2);  // order n1
  const fe* tw2 = ctx->stage_twiddles(w2, log2);
  const fe* tw1 = ctx->stage_twiddles(w1, log1);
  const fe* T[3];
  tables3(ctx, root, T);
  const uint64_t vrows = nv * rows, C = nv * R;  // rows of all vectors; received columns
  DevBuf z(ctx, vrows * n2 * sizeof(fe)), send(ctx, vrows * n2 * sizeof(fe)), recv(ctx, n1 * C * sizeof(fe));
  // 1. size-N2 NTTs; the last pass applies w^(j1 k2) and packs [h][r][v][c] for the all-to-all
  int skip = 0;
  if (!in_il)
    while (skip < log2 && (row_len << (skip + 1)) <= n2) ++skip;
  for (uint64_t r0 = 0; r0 < vrows; r0 += kRows) {
    const uint64_t cnt = std::min<uint64_t>(kRows, vrows - r0);
    NttEpilogue ep{send.as<fe>(), T[0], T[1], T[2], r0, (uint64_t)d->g * rows, rows, ilog2_exact(R)};
    if (nv > 1) {
      ep.vlog = ilog2_exact(rows);
      ep.k = nv;
    }
    fe* zo = z.as<fe>() + r0 * n2;
    const fe* ii = in_il ? in + r0 : in + r0 * row_len;
    SG_HIP(launch_ntt_fused(&zo, &ii, (int)cnt, row_len, log2, tw2, nullptr, nullptr, skip, nullptr, ctx->stream,
                            in_il ? 1 : row_len, n2, in_il, &ep));
  }
  // 2. the one exchange: rank h receives block h of every rank -> recv = [j1][v][c]
  exchange(d, send.get(), recv.get(), vrows * R * sizeof(fe), /*a2a=*/true);
  // 3. size-N1 NTTs over the R interleaved columns of recv
  DevBuf dpost;
  const fe* post = nullptr;
  if (post_host) {
    dpost = DevBuf(ctx, sizeof(fe));
    SG_HIP(hipMemcpyAsync(dpost.get(), post_host, sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    post = dpost.as<fe>();
  }
  for (uint64_t c0 = 0; c0 < C; c0 += kRows) {
    const uint64_t cnt = std::min<uint64_t>(kRows, C - c0);
    fe* oo = out + c0 * n1;
    const fe* rr = recv.as<fe>() + c0;
    SG_HIP(launch_ntt_fused(&oo, &rr, (int)cnt, n1, log1, tw1, nullptr, nullptr, 0, post, ctx->stream, 1, n1, C,
                            nullptr));
  }
}

}  // namespace

void dist_ntt(sg_dist* d, const fe& root, const fe* cols, uint64_t row_len, uint64_t n, fe* runs) {
  dist_ntt_batch(d, root, cols, row_len, n, runs, 1);
}

void dist_ntt_batch(sg_dist* d, const fe& root, const fe* cols, uint64_t row_len, uint64_t n, fe* runs, uint64_t nv) {
  if (nv == 0) return;
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  check_order_n(root, n);
  const uint64_t R = n2 / d->G;
  DevBuf t(d->ctx, nv * R * n1 * sizeof(fe));
  four_step(d, root, cols, row_len, 0, n1, n2, t.as<fe>(), nullptr, nv);
  SG_HIP(launch_swap01(t.as<fe>(), runs, R, n1, 1, d->ctx->stream, nv));  // [v][c][k1] -> [v][k1][c]
}

void dist_intt(sg_dist* d, const fe& root, const fe* runs, uint64_t n, fe* cols) {
  dist_intt_batch(d, root, runs, n, cols, 1);
}

void dist_intt_batch(sg_dist* d, const fe& root, const fe* runs, uint64_t n, fe* cols, uint64_t nv) {
  if (nv == 0) return;
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  check_order_n(root, n);
  // the run shard [n1][R] is the interleaved column shard of (N1', N2') = (n2, n1): row c of
  // length n1 at runs[k1 R + c]; the inverse four-step's output rows [n1/G][n2] are the column shard.
  // Batched: the run shards [v][n1][R] transposed to [n1][v][R] first, i.e. nv R interleaved rows
  const fe inv = fe_inv(root);
  const fe ninv = to_mont(fe_inv(fe_from_u64(n)));
  SG_REQUIRE(n2 % d->G == 0 && (n1 / d->G) % 4 == 0 && n1 / d->G >= 4,
             "distributed intt: n too small for this many ranks (needs N1 >= 4 G)");
  const uint64_t R = n2 / d->G;
  if (nv == 1) {
    four_step(d, inv, runs, n1, R, n2, n1, cols, &ninv);
    return;
  }
  DevBuf t(d->ctx, nv * n1 * R * sizeof(fe));
  SG_HIP(launch_swap01(runs, t.as<fe>(), nv, n1, R, d->ctx->stream));
  four_step(d, inv, t.as<fe>(), n1, nv * R, n2, n1, cols, &ninv, nv);
}

void dist_coset_evaluate(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* cols, uint64_t row_len,
                         fe* runs) {
  dist_coset_evaluate_batch(d, gen, n, &offset, cols, row_len, runs, 1);
}

void dist_coset_evaluate_batch(sg_dist* d, const fe& gen, uint64_t n, const fe* offsets, const fe* cols,
                               uint64_t row_len, fe* runs, uint64_t nv) {
  if (nv == 0) return;
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  const uint64_t rows = n1 / d->G, one = rows * row_len;
  SG_REQUIRE(row_len >= 1 && row_len <= n2, "distributed LDE: row length must be in [1, N2]");
  // Polynomial::scale (polynomial.rs:109-121): coefficient j = (g rows + r) + N1 c times offset^j,
  // one launch per run of equal offsets
  DevBuf sc(d->ctx, nv * one * sizeof(fe));
  SG_HIP(hipMemcpyAsync(sc.get(), cols, nv * one * sizeof(fe), hipMemcpyDeviceToDevice, d->ctx->stream));
  for (uint64_t v0 = 0; v0 < nv;) {
    uint64_t v1 = v0 + 1;
    while (v1 < nv && fe_eq(offsets[v1], offsets[v0])) ++v1;
    const fe* T[3];
    tables3(d->ctx, offsets[v0], T);
    SG_HIP(launch_mul_pow(sc.as<fe>() + v0 * one, rows, row_len, n1, 0, (uint64_t)d->g * rows, 1, T[0], T[1], T[2],
                          d->ctx->stream, v1 - v0));
    v0 = v1;
  }
  dist_ntt_batch(d, gen, sc.as<fe>(), row_len, n, runs, nv);
}

// root of the natural-order codeword held as runs [k1s][R] on every rank (merkle_root.rs:21-32):
// a forest of k1s subtrees per rank, the run roots all-gathered (64 B each), the top on every rank.
// With `keep`, the forest and the top tree move into it (openings).
//
// Split in two so the hashing can overlap other work: the forest and its run roots on any stream
// (no collective), then the all-gather and the top tree on the context's stream (every collective
// of a communicator stays on one stream, in the same order on every rank).
void dist_forest_alloc(sg_dist* d, uint64_t k1s, uint64_t R, PendingForest& pf) {
  SG_REQUIRE(R >= 1 && (R & (R - 1)) == 0 && k1s >= 1 && (k1s & (k1s - 1)) == 0, "Leafs len must be power of two");
  pf.k1s = k1s;
  pf.R = R;
  // lean subtrees, like the single-GPU prove's trees: the lowest min(3, log2 R) levels are not
  // stored (2R / 8 - 1 digests per subtree instead of 2R - 1: 16 B per codeword element per rank
  // instead of 128), and an opening rehashes each dropped sibling -- a leaf, or the root of its 2- or
  // 4-leaf block -- from the run (k_gather_abs)
  pf.drop = std::min(std::min(ilog2_exact(R), 3), d->ctx->opt.lean_trees ? d->ctx->opt.lean_drop : 0);
  pf.per = (merkle_tree_digests(R) - (2 * R - 2 * (R >> pf.drop))) * 8;  // u64 per subtree
  pf.forest = DevBuf(d->ctx, k1s * pf.per * 8);
  pf.roots = DevBuf(d->ctx, k1s * 64);
}

void dist_forest_launch(sg_dist* d, const fe* runs, PendingForest& pf, hipStream_t s) {
  (void)d;
  for (uint64_t t0 = 0; t0 < pf.k1s; t0 += kRows) {
    const int cnt = (int)std::min<uint64_t>(kRows, pf.k1s - t0);
    const fe* lv = runs + t0 * pf.R;
    uint64_t* tr = pf.forest.as<uint64_t>() + t0 * pf.per;
    SG_HIP(launch_merkle_tree(&lv, &tr, cnt, pf.R, nullptr, s, pf.R, pf.per, 0, nullptr, 0, nullptr, pf.drop));
  }
  // the subtree roots: digest 2R - 2 of a full subtree, less the dropped levels' digests
  const uint64_t root_digest = 2 * pf.R - 2 - (2 * pf.R - 2 * (pf.R >> pf.drop));
  SG_HIP(launch_gather_roots(pf.forest.as<uint64_t>(), pf.per, root_digest * 8, pf.roots.as<uint64_t>(), pf.k1s, s));
}

void dist_forest_finish(sg_dist* d, PendingForest& pf, uint8_t root[64], ShardedRound* keep) {
  sg_ctx* ctx = d->ctx;
  const uint64_t k1s = pf.k1s;
  DevBuf all(ctx, d->G * k1s * 64), ordered(ctx, d->G * k1s * 64);
  exchange(d, pf.roots.get(), all.get(), k1s * 64, /*a2a=*/false);  // [g][k1]
  // [g][k1] -> [k1][g]: global run order (a digest is 4 field-element slots)
  SG_HIP(launch_swap01(all.as<fe>(), ordered.as<fe>(), d->G, k1s, 4, ctx->stream));
  const uint64_t m = d->G * k1s;
  if (keep) {
    keep->k1s = k1s;
    keep->m = m;
    keep->per = pf.per;
    keep->drop = pf.drop;
  }
  if (m == 1) {
    SG_HIP(hipMemcpyAsync(root, ordered.get(), 64, hipMemcpyDeviceToHost, ctx->stream));
    host_wait(ctx, ctx->stream);
    if (keep) keep->forest = std::move(pf.forest);
    return;
  }
  DevBuf top(ctx, merkle_tree_digests(m) * 64);
  SG_HIP(hipMemcpyAsync(top.get(), ordered.get(), m * 64, hipMemcpyDeviceToDevice, ctx->stream));
  uint64_t* tr = top.as<uint64_t>();
  uint64_t* root_dev = ctx->pinned_roots_dev;
  SG_HIP(launch_merkle_tree(nullptr, &tr, 1, m, &root_dev, ctx->stream, 0, 0, 1));
  host_wait(ctx, ctx->stream);
  memcpy(root, ctx->pinned_roots, 64);
  if (keep) {
    keep->forest = std::move(pf.forest);
    keep->top = std::move(top);
  }
}

void dist_merkle_root(sg_dist* d, const fe* runs, uint64_t k1s, uint64_t R, uint8_t root[64],
                      ShardedRound* keep) {
  PendingForest pf;
  dist_forest_alloc(d, k1s, R, pf);
  dist_forest_launch(d, runs, pf, d->ctx->stream);
  dist_forest_finish(d, pf, root, keep);
}

void dist_lde_replicated(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* coeffs, uint64_t len,
                         fe* runs) {
  dist_lde_replicated_batch(d, gen, n, &offset, &coeffs, &len, runs, 1);
}

void dist_lde_replicated_batch(sg_dist* d, const fe& gen, uint64_t n, const fe* offsets, const fe* const* coeffs,
                               const uint64_t* lens, fe* runs, uint64_t nv) {
  if (nv == 0) return;
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  uint64_t len = 0;
  for (uint64_t v = 0; v < nv; ++v) {
    SG_REQUIRE(lens[v] <= n, "fast_coset_evaluate: polynomial longer than root_order");
    len = std::max(len, lens[v]);
  }
  const uint64_t rows = n1 / d->G;
  const uint64_t row_len = std::max<uint64_t>((len + n1 - 1) / n1, 1);  // the longest vector's
  // column shards: row r = coefficients (g rows + r) + N1 j, zero past each vector's length
  DevBuf cols(d->ctx, nv * rows * row_len * sizeof(fe));
  for (uint64_t v = 0; v < nv; ++v)
    SG_HIP(launch_gather_cols(cols.as<fe>() + v * rows * row_len, coeffs[v], lens[v], rows, row_len, n1,
                              (uint64_t)d->g * rows, d->ctx->stream));
  dist_coset_evaluate_batch(d, gen, n, offsets, cols.as<fe>(), row_len, runs, nv);
}

// Coset interpolation of a run-sharded codeword (the values of a polynomial of degree < n on
// offset * <gen>, ntt_arithmetics.rs:172-181): its coefficients as this rank's column shard
// [N1/G][N2] -- the distributed INTT, then coefficient i = (g rows + r) + N1 j times offset^-i.
void dist_coset_interpolate(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* runs, fe* cols) {
  dist_coset_interpolate_batch(d, gen, n, offset, runs, cols, 1);
}

void dist_coset_interpolate_batch(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* runs, fe* cols,
                                  uint64_t nv) {
  if (nv == 0) return;
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  dist_intt_batch(d, gen, runs, n, cols, nv);
  const uint64_t rows = n1 / d->G;
  const fe* T[3];
  tables3(d->ctx, fe_inv(offset), T);
  SG_HIP(launch_mul_pow(cols, rows, n2, n1, 0, (uint64_t)d->g * rows, 1, T[0], T[1], T[2], d->ctx->stream, nv));
}

// every rank's column shard [N1/G][N2] -> the whole vector in natural order on every rank: one
// all-gather ([g][r][j] = [j1][j]) and one transpose to [j][j1] (index j1 + N1 j)
void dist_gather_columns(sg_dist* d, const fe* cols, uint64_t n, fe* out) {
  dist_gather_columns_batch(d, cols, n, &out, 1);
}

// (nv column shards [v][N1/G][N2] at once: one all-gather, [g][v] -> [v][g], then per vector)
void dist_gather_columns_batch(sg_dist* d, const fe* cols, uint64_t n, fe* const* outs, uint64_t nv) {
  if (nv == 0) return;
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  const uint64_t one = (n1 / d->G) * n2;
  DevBuf all(d->ctx, nv * n * sizeof(fe));
  exchange(d, cols, all.get(), nv * one * sizeof(fe), /*a2a=*/false);  // [g][v][r][j]
  const fe* src = all.as<fe>();
  DevBuf byv;
  if (nv > 1) {
    byv = DevBuf(d->ctx, nv * n * sizeof(fe));
    SG_HIP(launch_swap01(all.as<fe>(), byv.as<fe>(), d->G, nv, one, d->ctx->stream));  // [v][g][r][j]
    src = byv.as<fe>();
  }
  for (uint64_t v = 0; v < nv; ++v) SG_HIP(launch_swap01(src + v * n, outs[v], n1, n2, 1, d->ctx->stream));
}

// every rank's run shard [N1][N2/G] -> the whole codeword in natural order on every rank
void dist_gather_runs(sg_dist* d, const fe* runs, uint64_t n, fe* out) {
  dist_gather_runs_batch(d, runs, n, &out, 1);
}

// (nv run shards [v][N1][R] at once: one all-gather, [g][v] -> [v][g], then per vector)
void dist_gather_runs_batch(sg_dist* d, const fe* runs, uint64_t n, fe* const* outs, uint64_t nv) {
  if (nv == 0) return;
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  const uint64_t R = n2 / d->G, one = n1 * R;
  DevBuf all(d->ctx, nv * n * sizeof(fe));
  exchange(d, runs, all.get(), nv * one * sizeof(fe), /*a2a=*/false);  // [g][v][k1][c]
  const fe* src = all.as<fe>();
  DevBuf byv;
  if (nv > 1) {
    byv = DevBuf(d->ctx, nv * n * sizeof(fe));
    SG_HIP(launch_swap01(all.as<fe>(), byv.as<fe>(), d->G, nv, one, d->ctx->stream));  // [v][g][k1][c]
    src = byv.as<fe>();
  }
  for (uint64_t v = 0; v < nv; ++v)
    SG_HIP(launch_swap01(src + v * n, outs[v], d->G, n1, R, d->ctx->stream));  // [k1][g][c]
}

// this rank's run shard of a natural-order vector every rank holds (no exchange)
void dist_take_runs(sg_dist* d, const fe* full, uint64_t n, fe* runs) {
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  const uint64_t R = n2 / d->G;
  SG_HIP(hipMemcpy2DAsync(runs, R * sizeof(fe), full + (uint64_t)d->g * R, n2 * sizeof(fe), R * sizeof(fe), n1,
                          hipMemcpyDeviceToDevice, d->ctx->stream));
}

// fri.rs:115-172 on a run-sharded codeword.  The fold partner of i is i + n/2: same k2,
// k1 + N1/2, i.e. on the same rank, so folds stay local while more than one run per rank is
// left; every rank pushes the same roots, so the Fiat-Shamir challenges agree without a
// broadcast.  With one run per rank left, the N2-element codeword is all-gathered and the
// remaining rounds run through the single-GPU commit.  With `keep`, every round's codeword
// and trees stay for the query phase.
void dist_fri_commit(sg_dist* d, const sg_fri* f, const fe* runs, uint64_t n, const sg_proof_stream* ps,
                     DistFriState* keep = nullptr) {
  sg_ctx* ctx = d->ctx;
  SG_REQUIRE(ps && ps->push && ps->fiat_shamir_prover, "proof stream callbacks required");
  SG_REQUIRE(n == f->domain_length, "Length of the domain doesnt match the length of initial codeword");
  const size_t rounds = fri_num_rounds(f);
  SG_REQUIRE(rounds >= 1, "FRI: zero rounds for this domain");
  uint64_t n1, n2;
  plan(n, d->G, n1, n2);
  const uint64_t R = n2 / d->G;
  if (keep) {
    keep->n2 = n2;
    keep->R = R;
  }
  fe omega = to_fe(f->omega), offset = to_fe(f->offset);
  SG_REQUIRE(fe_is_canonical(omega) && fe_is_canonical(offset), "FRI omega/offset must be canonical");
  const fe inv2 = fe_inv(fe_from_u64(2));
  const fe* cur = runs;
  DevBuf owned;
  uint64_t k1s = n1, length = n;
  size_t r = 0;
  // once the whole codeword is small (<= 2^SG_DIST_FRI_TAIL elements, default 2^20 = 16 MiB) the
  // remaining rounds are latency-bound: every rank gathers it and continues with the single-GPU
  // commit instead of paying a forest, a collective and a host round trip per sharded round
  const int tail_log = d->fri_tail_log;
  const uint64_t tail_below = tail_log <= 0 ? 0 : (uint64_t)1 << std::min(tail_log, 62);
  bool all_sharded = false;
  while (k1s > 1 && r < rounds) {
    if (length <= tail_below) break;
    const fe winv = fe_inv(omega);
    SG_REQUIRE(fe_eq(fe_pow(omega, length - 1), winv), "error in commit: omega does not have the right order!");
    uint8_t root[64];
    ShardedRound* sr = nullptr;
    if (keep) {
      keep->sharded.emplace_back();
      sr = &keep->sharded.back();
      sr->cw = cur;
      if (owned.get()) sr->cw_own = std::move(owned);  // the previous fold's output, kept
      keep->lengths.push_back(length);
    }
    dist_merkle_root(d, cur, k1s, R, root, sr);
    push_obj(ps, SG_OBJ_ROOT, root, 64);
    if (r == rounds - 1) {
      all_sharded = true;
      break;
    }
    uint8_t chal[32];
    if (ps->fiat_shamir_prover(ps->user, 32, chal) != 0)
      throw Error{SG_ERR_CALLBACK, "proof stream fiat_shamir callback failed"};
    const fe alpha = fe_sample(chal, 32);
    // fri.rs:151-159 on the local runs: local l is global (l / R) n2 + g R + l % R
    const uint64_t half = k1s * R / 2;
    DevBuf nxt(ctx, half * sizeof(fe));
    const fe* T[3];
    tables3(ctx, winv, T);
    const fe K = to_mont(fe_mul(fe_mul(alpha, fe_inv(offset)), inv2));
    SG_HIP(launch_fri_fold_runs(nxt.as<fe>(), cur, half, R, n2, (uint64_t)d->g * R, T[0], T[1], T[2], K,
                                ctx->stream));
    owned = std::move(nxt);
    cur = owned.as<fe>();
    k1s /= 2;
    length /= 2;
    omega = fe_mul(omega, omega);
    offset = fe_mul(offset, offset);
    ++r;
  }
  if (all_sharded && k1s > 1) {
    // every round done while still sharded: gather the last codeword (fri.rs:166) in natural order
    DevBuf all(ctx, d->G * k1s * R * sizeof(fe)), nat(ctx, d->G * k1s * R * sizeof(fe));
    exchange(d, cur, all.get(), k1s * R * sizeof(fe), /*a2a=*/false);          // [g][k1][c]
    SG_HIP(launch_swap01(all.as<fe>(), nat.as<fe>(), d->G, k1s, R, ctx->stream));  // [k1][g][c]
    const uint64_t len = d->G * k1s * R;
    std::vector<fe> last(len);
    SG_HIP(hipMemcpyAsync(last.data(), nat.get(), len * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
    host_wait(ctx, ctx->stream);
    std::vector<uint8_t> payload;
    payload.reserve(len * 16);
    for (auto& v : last) put_u128_be(payload, v);
    push_obj(ps, SG_OBJ_CODEWORD, payload.data(), payload.size());
    return;
  }
  // the rest on the gathered codeword: [g][k1][c] -> [k1][g][c] is its natural order (with one
  // run per rank left, [g][c] already is)
  DevBuf full(ctx, d->G * k1s * R * sizeof(fe));
  if (k1s == 1) {
    exchange(d, cur, full.get(), R * sizeof(fe), /*a2a=*/false);
  } else {
    DevBuf all(ctx, d->G * k1s * R * sizeof(fe));
    exchange(d, cur, all.get(), k1s * R * sizeof(fe), /*a2a=*/false);
    SG_HIP(launch_swap01(all.as<fe>(), full.as<fe>(), d->G, k1s, R, ctx->stream));
  }
  sg_fri sub = *f;
  sub.offset = from_fe(offset);
  sub.omega = from_fe(omega);
  sub.domain_length = length;
  SG_REQUIRE(fri_num_rounds(&sub) == rounds - r, "FRI tail round count mismatch");
  if (keep) {
    fri_commit_dev(ctx, &sub, full.as<fe>(), length, ps, keep->tail, /*borrow_input=*/false, /*drop=*/3);
    for (uint64_t l : keep->tail.lengths) keep->lengths.push_back(l);
    return;
  }
  sg_fri_state st;
  fri_commit_dev(ctx, &sub, full.as<fe>(), length, ps, st, /*borrow_input=*/true);
}

// Openings at global indices I of many rounds at once: values and authentication paths (leaf level
// first), identical on every rank.  A sharded round's value and subtree part come from the rank
// that owns the run (i = k1 n2 + g R + c: rank g, run k1, leaf c); its top part (run index i / R in
// the top tree) is on every rank; a round of the single-GPU tail is local.  Every request's device
// gathers are issued together (one host round trip), and the owned slots of all sharded requests
// travel in ONE all-gather: two round trips for the whole query phase instead of two per round.
void dist_open_batch(sg_dist* d, uint64_t R, uint64_t n2, std::vector<OpenReq>& reqs) {
  sg_ctx* ctx = d->ctx;
  const int lr = ilog2_exact(R);
  const size_t slot = 16 + 64 * (size_t)lr;
  struct Job {
    const void* src;
    bool digest;         // 64-byte digests (else 16-byte elements)
    size_t idx0, count;  // index range in `idx`
    size_t out0;         // output offset in values (elements) or digests (64-byte units)
    const sg_tree* tree = nullptr;  // digests of a local tree (a lean one rehashes its leaf level)
    bool abs = false;    // `idx` holds absolute addresses (bit 0 set: a leaf value to rehash)
  };
  std::vector<uint64_t> idx;
  std::vector<Job> jobs;
  size_t nvals = 0, ndig = 0;
  auto add_job = [&](const void* src, bool digest, const std::vector<uint64_t>& ix,
                     const sg_tree* tree = nullptr, bool abs = false) -> size_t {
    const size_t out0 = digest ? ndig : nvals;
    if (ix.empty()) return out0;
    jobs.push_back({src, digest, idx.size(), ix.size(), out0, tree, abs});
    idx.insert(idx.end(), ix.begin(), ix.end());
    (digest ? ndig : nvals) += ix.size();
    return out0;
  };
  struct Plan {
    size_t own_vals = 0, own_dig = 0, top_dig = 0, path_dig = 0, vals_at = 0;
    std::vector<size_t> own;  // positions in I this rank owns (sharded)
    int lm = 0;
  };
  std::vector<Plan> plans(reqs.size());
  size_t qtot = 0;  // slots of all sharded requests
  for (size_t j = 0; j < reqs.size(); ++j) {
    OpenReq& q = reqs[j];
    Plan& pl = plans[j];
    if (!q.sr) {  // a local round
      std::vector<uint64_t> pidx;
      for (uint64_t i : q.I) path_indices(q.tree, i, pidx);
      q.depth = q.tree->logn;
      pl.vals_at = add_job(q.cw, false, q.I);
      pl.path_dig = add_job(nullptr, true, pidx, q.tree);
      continue;
    }
    const ShardedRound& sr = *q.sr;
    pl.lm = ilog2_exact(sr.m);
    q.depth = lr + pl.lm;
    std::vector<uint64_t> eidx, didx, tidx;
    for (size_t k = 0; k < q.I.size(); ++k) {
      const uint64_t i = q.I[k];
      for (int lv = 0; lv < pl.lm; ++lv) tidx.push_back(level_offset(sr.m, lv) + (((i / R) >> lv) ^ 1));
      if ((i % n2) / R != (uint64_t)d->g) continue;
      const uint64_t k1 = i / n2, c = i % R;
      pl.own.push_back(k);
      eidx.push_back(k1 * R + c);
      // absolute addresses of the subtree path: a dropped sibling (level lv < drop) is named by the
      // first value of its 2^lv-leaf block in the run, | 1 | lv << 1 (k_gather_abs rehashes it); the
      // stored levels sit level_offset(R, drop) digests earlier in the lean subtree
      const uint64_t fbase = reinterpret_cast<uint64_t>(sr.forest.get()) + 64 * k1 * (sr.per / 8);
      const uint64_t dropped = level_offset(R, sr.drop);
      for (int lv = 0; lv < lr; ++lv) {
        const uint64_t sib = (c >> lv) ^ 1;
        if (lv < sr.drop)
          didx.push_back(reinterpret_cast<uint64_t>(sr.cw + k1 * R + (sib << lv)) | 1 | ((uint64_t)lv << 1));
        else
          didx.push_back(fbase + 64 * (level_offset(R, lv) - dropped + sib));
      }
    }
    pl.own_vals = add_job(sr.cw, false, eidx);
    pl.own_dig = add_job(nullptr, true, didx, nullptr, /*abs=*/true);
    if (pl.lm) pl.top_dig = add_job(sr.top.get(), true, tidx);
    qtot += q.I.size();
  }
  // every gather at once, one round trip: the absolute address of every entry (values first, then
  // digests, each in output order), two launches whatever the number of rounds and buffers
  std::vector<fe> vals(nvals);
  std::vector<uint8_t> dig(ndig * 64);
  if (!jobs.empty()) {
    std::vector<uint64_t> addr(nvals + ndig);
    for (const Job& jb : jobs) {
      const uint64_t base = reinterpret_cast<uint64_t>(jb.src);
      uint64_t* a = addr.data() + (jb.digest ? nvals : 0) + jb.out0;
      for (size_t k = 0; k < jb.count; ++k)
        a[k] = jb.abs    ? idx[jb.idx0 + k]
               : jb.tree ? digest_addr(jb.tree, idx[jb.idx0 + k])
                         : base + (jb.digest ? 64 : sizeof(fe)) * idx[jb.idx0 + k];
    }
    DevBuf dA(ctx, addr.size() * 8), dV(ctx, std::max<size_t>(nvals, 1) * sizeof(fe)), dD(ctx, std::max<size_t>(ndig, 1) * 64);
    SG_HIP(hipMemcpyAsync(dA.get(), addr.data(), addr.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    SG_HIP(launch_gather_abs(dA.as<uint64_t>(), dV.get(), (uint32_t)nvals, false, ctx->stream));
    SG_HIP(launch_gather_abs(dA.as<uint64_t>() + nvals, dD.get(), (uint32_t)ndig, true, ctx->stream));
    if (nvals) SG_HIP(hipMemcpyAsync(vals.data(), dV.get(), nvals * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
    if (ndig) SG_HIP(hipMemcpyAsync(dig.data(), dD.get(), ndig * 64, hipMemcpyDeviceToHost, ctx->stream));
    host_wait(ctx, ctx->stream);
  }
  // the owned slots of every sharded request, one all-gather
  std::vector<uint8_t> all;
  if (qtot) {
    std::vector<uint8_t> mine(qtot * slot, 0);
    size_t base = 0;
    for (size_t j = 0; j < reqs.size(); ++j) {
      if (!reqs[j].sr) continue;
      const Plan& pl = plans[j];
      for (size_t o = 0; o < pl.own.size(); ++o) {
        uint8_t* p = mine.data() + (base + pl.own[o]) * slot;
        memcpy(p, &vals[pl.own_vals + o], 16);
        memcpy(p + 16, dig.data() + (pl.own_dig + o * (size_t)lr) * 64, 64 * (size_t)lr);
      }
      base += reqs[j].I.size();
    }
    DevBuf dsend(ctx, qtot * slot), drecv(ctx, d->G * qtot * slot);
    SG_HIP(hipMemcpyAsync(dsend.get(), mine.data(), qtot * slot, hipMemcpyHostToDevice, ctx->stream));
    exchange(d, dsend.get(), drecv.get(), qtot * slot, /*a2a=*/false);
    all.resize((size_t)d->G * qtot * slot);
    SG_HIP(hipMemcpyAsync(all.data(), drecv.get(), all.size(), hipMemcpyDeviceToHost, ctx->stream));
    host_wait(ctx, ctx->stream);
  }
  size_t base = 0;
  for (size_t j = 0; j < reqs.size(); ++j) {
    OpenReq& q = reqs[j];
    const Plan& pl = plans[j];
    const size_t nq = q.I.size(), depth = (size_t)q.depth;
    q.vals.assign(nq, fe_zero());
    q.paths.assign(nq * depth * 64, 0);
    if (!q.sr) {
      for (size_t k = 0; k < nq; ++k) q.vals[k] = vals[pl.vals_at + k];
      if (depth) memcpy(q.paths.data(), dig.data() + pl.path_dig * 64, nq * depth * 64);
      continue;
    }
    for (size_t k = 0; k < nq; ++k) {
      const uint64_t owner = (q.I[k] % n2) / R;
      const uint8_t* p = all.data() + (owner * qtot + base + k) * slot;
      memcpy(&q.vals[k], p, 16);
      uint8_t* out = q.paths.data() + k * depth * 64;
      memcpy(out, p + 16, 64 * (size_t)lr);
      if (pl.lm) memcpy(out + 64 * (size_t)lr, dig.data() + (pl.top_dig + k * (size_t)pl.lm) * 64, 64 * (size_t)pl.lm);
    }
    base += nq;
  }
}

void dist_open_round(sg_dist* d, const ShardedRound& sr, uint64_t R, uint64_t n2, const std::vector<uint64_t>& I,
                     std::vector<fe>& vals, std::vector<uint8_t>& paths, int& depth) {
  std::vector<OpenReq> reqs(1);
  reqs[0].sr = &sr;
  reqs[0].I = I;
  dist_open_batch(d, R, n2, reqs);
  vals = std::move(reqs[0].vals);
  paths = std::move(reqs[0].paths);
  depth = reqs[0].depth;
}

// round r of a sharded FRI commit as an opening request
OpenReq fri_open_req(const DistFriState& s, size_t r, std::vector<uint64_t> I) {
  OpenReq q;
  if (r >= s.sharded.size()) {
    const size_t t = r - s.sharded.size();
    q.cw = s.tail.cw[t];
    q.tree = s.tail.trees[t].get();
  } else {
    q.sr = &s.sharded[r];
  }
  q.I = std::move(I);
  return q;
}

// FRI::prove (fri.rs:210-248) on a run-sharded codeword: the sharded commit with every round kept,
// sample_indices over len(codewords[1]) reduced by len(codewords[-1]) (fri.rs:88-113), then per
// round the c Leafs objects and 3c Path objects (fri.rs:174-208) -- every rank writes the same bytes.
void dist_fri_prove(sg_dist* d, const sg_fri* f, const fe* runs, uint64_t n, const sg_proof_stream* ps,
                    size_t* top, const std::function<void(const size_t* top)>& extra) {
  DistFriState s;
  dist_fri_commit(d, f, runs, n, ps, &s);
  SG_REQUIRE(s.lengths.size() >= 2, "FRI prove needs at least two rounds (reference indexes codewords[1])");
  uint8_t seed[32];
  if (ps->fiat_shamir_prover(ps->user, 32, seed) != 0)
    throw Error{SG_ERR_CALLBACK, "proof stream fiat_shamir callback failed"};
  const size_t c = f->num_colinearity_tests;
  sample_indices(seed, 32, s.lengths[1], s.lengths.back(), c, top);
  std::vector<uint64_t> idx(top, top + c);
  auto put_path = [&](const uint8_t* p, int depth) {
    std::vector<uint8_t> pl(72 * (size_t)depth);
    for (int k = 0; k < depth; ++k) {
      uint8_t* o = pl.data() + 72 * (size_t)k;
      memset(o, 0, 8);
      o[7] = 64;
      memcpy(o + 8, p + 64 * (size_t)k, 64);
    }
    push_obj(ps, SG_OBJ_PATH, pl.data(), pl.size());
  };
  // every round's indices first (fri.rs:182-186: i mod half, then i + half), all openings in one batch
  const size_t nr = s.lengths.size() - 1;
  std::vector<OpenReq> reqs;
  reqs.reserve(2 * nr);
  for (size_t r = 0; r < nr; ++r) {
    const uint64_t half = s.lengths[r] / 2;
    for (auto& i : idx) i %= half;
    std::vector<uint64_t> ab(idx);
    for (uint64_t i : idx) ab.push_back(i + half);
    reqs.push_back(fri_open_req(s, r, std::move(ab)));
    reqs.push_back(fri_open_req(s, r + 1, idx));
  }
  dist_open_batch(d, s.R, s.n2, reqs);
  for (size_t r = 0; r < nr; ++r) {
    const OpenReq& qab = reqs[2 * r];
    const OpenReq& qc = reqs[2 * r + 1];
    const int dab = qab.depth, dc = qc.depth;
    for (size_t k = 0; k < c; ++k) {
      uint8_t pl[48];
      put_u128_be_at(pl, qab.vals[k]);
      put_u128_be_at(pl + 16, qab.vals[c + k]);
      put_u128_be_at(pl + 32, qc.vals[k]);
      push_obj(ps, SG_OBJ_LEAFS, pl, 48);
    }
    for (size_t k = 0; k < c; ++k) {
      put_path(qab.paths.data() + k * (size_t)dab * 64, dab);
      put_path(qab.paths.data() + (c + k) * (size_t)dab * 64, dab);
      put_path(qc.paths.data() + k * (size_t)dc * 64, dc);
    }
  }
  if (extra) extra(top);
}

sg_ctx* dist_ctx(sg_dist* d) { return d->ctx; }
int dist_world(const sg_dist* d) { return d->G; }
int dist_rank(const sg_dist* d) { return d->g; }
bool dist_shard_algebra(const sg_dist* d) { return d->G > 1 && d->shard_algebra; }
void dist_count_sharded_quotient(sg_dist* d) { ++d->sharded_quotients; }
void dist_count_sharded_interpolation(sg_dist* d, uint64_t columns) { d->sharded_interpolations += columns; }
uint64_t dist_split(uint64_t n) {
  // N1 = 2^floor(log2 n / 2).  (Round 4 measured capping N1 at 2^11, so the size-N1 transforms run
  // whole in one launch, against this split: 2^25 four-step 2.33 vs 2.27 ms, 2^27 9.25 vs 8.87 ms
  // on one rank -- the longer size-N2 transforms cost more than the pass it saves)
  return (uint64_t)1 << (ilog2_exact(n) / 2);
}
bool dist_can_shard(uint64_t n, int G) {
  if (n < 2 || (n & (n - 1)) || G < 1 || (G & (G - 1))) return false;
  const uint64_t n1 = dist_split(n), n2 = n / n1;
  // sg_dist_plan (ntt) and the inverse's interleaved first pass (intt)
  return n1 % (uint64_t)G == 0 && n2 % (4 * (uint64_t)G) == 0 && n2 % (uint64_t)G == 0 && n1 / G >= 4 &&
         (n1 / G) % 4 == 0;
}
void dist_plan(uint64_t n, int G, uint64_t& n1, uint64_t& n2) { plan(n, G, n1, n2); }

}  // namespace sg

using namespace sg;

extern "C" int sg_dist_unique_id(uint8_t* id) {
  return guard(nullptr, [&] {
    SG_REQUIRE(id, "null argument");
    ncclUniqueId u;
    SG_NCCL(ncclGetUniqueId(&u));
    memcpy(id, u.internal, SG_DIST_ID_BYTES);
  });
}

namespace {

// settings every rank must share, read from the environment at creation
void dist_defaults(sg_dist* d) {
  if (const char* t = getenv("SG_DIST_TIMEOUT_S")) {
    const double v = atof(t);
    if (v > 0) d->timeout_s = v;
  }
  if (const char* te = getenv("SG_DIST_FRI_TAIL")) d->fri_tail_log = atoi(te);
  if (const char* sa = getenv("SG_DIST_SHARD_ALGEBRA")) d->shard_algebra = atoi(sa) != 0;
}

// all-gathers v over the communicator; every rank throws the same error when the values differ
void agree(sg_dist* d, int64_t v, const char* what) {
  sg_ctx* ctx = d->ctx;
  DevBuf one(ctx, sizeof(int64_t)), all(ctx, sizeof(int64_t) * (size_t)d->G);
  std::vector<int64_t> h((size_t)d->G);
  SG_HIP(hipMemcpyAsync(one.get(), &v, sizeof(v), hipMemcpyHostToDevice, ctx->stream));
  exchange(d, one.get(), all.get(), sizeof(int64_t), /*a2a=*/false);
  SG_HIP(hipMemcpyAsync(h.data(), all.get(), h.size() * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  host_wait(ctx, ctx->stream);
  for (int64_t x : h)
    if (x != h[0]) throw Error{SG_ERR_INVALID, std::string(what) + " differs between ranks"};
}

}  // namespace

extern "C" int sg_dist_create(sg_ctx* ctx, const uint8_t* id, int nranks, int rank, sg_dist** out) {
  std::unique_ptr<sg_dist> d;
  int rc = guard(ctx, [&] {
    SG_REQUIRE(out && id, "null argument");
    SG_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / rank count");
    set_device(ctx);
    d.reset(new sg_dist());
    d->ctx = ctx;
    d->G = nranks;
    d->g = rank;
    dist_defaults(d.get());
    ncclUniqueId u;
    memcpy(u.internal, id, SG_DIST_ID_BYTES);
    // the abort flag's name: FNV-1a of the unique id (the same on every rank of this communicator)
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < SG_DIST_ID_BYTES; ++i) h = (h ^ id[i]) * 1099511628211ull;
    char path[64];
    snprintf(path, sizeof(path), "/dev/shm/sg_dist_abort_%016llx", (unsigned long long)h);
    d->abort_path = path;
    SG_NCCL(ncclCommInitRank(&d->comm, nranks, u, rank));
  });
  if (rc != SG_OK) return rc;
  rc = dist_run(d.get(), [&] {
    agree(d.get(), d->fri_tail_log, "SG_DIST_FRI_TAIL");
    agree(d.get(), d->shard_algebra, "SG_DIST_SHARD_ALGEBRA");
  });
  if (rc != SG_OK) return rc;
  *out = d.release();
  return SG_OK;
}

extern "C" int sg_dist_create_transport(sg_ctx* ctx, int nranks, int rank, const sg_dist_transport* t,
                                        sg_dist** out) {
  std::unique_ptr<sg_dist> d;
  int rc = guard(ctx, [&] {
    SG_REQUIRE(out && t && t->all_to_all && t->all_gather, "transport callbacks required");
    SG_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / rank count");
    set_device(ctx);
    d.reset(new sg_dist());
    d->ctx = ctx;
    d->G = nranks;
    d->g = rank;
    d->tr = *t;
    d->staged = true;
    dist_defaults(d.get());
  });
  if (rc != SG_OK) return rc;
  rc = dist_run(d.get(), [&] {
    agree(d.get(), d->fri_tail_log, "SG_DIST_FRI_TAIL");
    agree(d.get(), d->shard_algebra, "SG_DIST_SHARD_ALGEBRA");
  });
  if (rc != SG_OK) return rc;
  *out = d.release();
  return SG_OK;
}

extern "C" void sg_dist_destroy(sg_dist* d) {
  // a communicator that ended cleanly removes its (never raised) flag name; a raised flag stays
  // for peers that have not yet polled it (a few bytes in /dev/shm per failed communicator)
  if (d && !d->dead && !d->abort_path.empty()) (void)remove(d->abort_path.c_str());
  delete d;
}

extern "C" int sg_dist_set_fri_tail(sg_dist* d, int log2_elements) {
  return dist_run(d, [&] {
    agree(d, log2_elements, "the FRI hand-over size");
    d->fri_tail_log = log2_elements;
  });
}

extern "C" int sg_dist_set_timeout(sg_dist* d, double seconds) {
  if (!d || !d->ctx || !(seconds > 0)) return SG_ERR_INVALID;
  d->timeout_s = seconds;
  return SG_OK;
}

extern "C" int sg_dist_poisoned(const sg_dist* d) { return d && d->dead ? 1 : 0; }

extern "C" int sg_dist_counters(const sg_dist* d, uint64_t* collectives, uint64_t* sharded_quotients,
                                uint64_t* sharded_interpolations) {
  if (!d || !collectives || !sharded_quotients || !sharded_interpolations) return SG_ERR_INVALID;
  *collectives = d->collectives;
  *sharded_quotients = d->sharded_quotients;
  *sharded_interpolations = d->sharded_interpolations;
  return SG_OK;
}

extern "C" int sg_dist_plan(size_t n, int nranks, size_t* n1, size_t* n2) {
  return guard(nullptr, [&] {
    SG_REQUIRE(n1 && n2, "null argument");
    uint64_t a, b;
    plan(n, nranks, a, b);
    *n1 = a;
    *n2 = b;
  });
}

extern "C" int sg_dist_ntt(sg_dist* d, sg_fe root, const sg_fe* d_cols, size_t row_len, size_t n, sg_fe* d_runs) {
  return dist_run(d, [&] {
    sg_ctx* ctx = d->ctx;
    SG_REQUIRE(d_cols && d_runs, "null buffer");
    dist_ntt(d, to_fe(root), reinterpret_cast<const fe*>(d_cols), row_len, n, reinterpret_cast<fe*>(d_runs));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_dist_intt(sg_dist* d, sg_fe root, const sg_fe* d_runs, size_t n, sg_fe* d_cols) {
  return dist_run(d, [&] {
    sg_ctx* ctx = d->ctx;
    SG_REQUIRE(d_cols && d_runs, "null buffer");
    dist_intt(d, to_fe(root), reinterpret_cast<const fe*>(d_runs), n, reinterpret_cast<fe*>(d_cols));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_dist_coset_evaluate(sg_dist* d, sg_fe generator, size_t root_order, sg_fe offset,
                                      const sg_fe* d_cols, size_t row_len, sg_fe* d_runs) {
  return dist_run(d, [&] {
    sg_ctx* ctx = d->ctx;
    SG_REQUIRE(d_cols && d_runs, "null buffer");
    const fe off = to_fe(offset);
    SG_REQUIRE(fe_is_canonical(off), "offset must be canonical");
    dist_coset_evaluate(d, to_fe(generator), root_order, off, reinterpret_cast<const fe*>(d_cols), row_len,
                        reinterpret_cast<fe*>(d_runs));
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_dist_merkle_root(sg_dist* d, const sg_fe* d_runs, size_t n, uint8_t* root) {
  return dist_run(d, [&] {
    SG_REQUIRE(d_runs && root, "null argument");
    uint64_t n1, n2;
    plan(n, d->G, n1, n2);
    dist_merkle_root(d, reinterpret_cast<const fe*>(d_runs), n1, n2 / d->G, root);
  });
}

extern "C" int sg_dist_fri_prove(sg_dist* d, const sg_fri* fri, const sg_fe* d_runs, size_t n,
                                 const sg_proof_stream* ps, size_t* top) {
  return dist_run(d, [&] {
    sg_ctx* ctx = d->ctx;
    SG_REQUIRE(fri && d_runs && top, "null argument");
    dist_fri_prove(d, fri, reinterpret_cast<const fe*>(d_runs), n, ps, top);
    host_wait(ctx, ctx->stream);
  });
}

extern "C" int sg_dist_fri_commit(sg_dist* d, const sg_fri* fri, const sg_fe* d_runs, size_t n,
                                  const sg_proof_stream* ps) {
  return dist_run(d, [&] {
    sg_ctx* ctx = d->ctx;
    SG_REQUIRE(fri && d_runs, "null argument");
    dist_fri_commit(d, fri, reinterpret_cast<const fe*>(d_runs), n, ps);
    host_wait(ctx, ctx->stream);
  });
}
