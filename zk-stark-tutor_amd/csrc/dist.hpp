// Library-internal multi-GPU pieces shared by dist.cpp and the sharded Stark::prove (stark.cpp).
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "internal.hpp"

namespace sg {

// A sharded FRI round kept for the query phase: the rank's runs, its forest (one subtree of R
// leaves per run) and the top tree over the G k1s run roots in global run order (every rank).
struct ShardedRound {
  uint64_t k1s = 0, m = 0, per = 0;  // runs per rank, run roots overall, u64 per subtree
  int drop = 0;                      // 1: the subtrees are lean (leaf digests not stored; rehashed)
  const fe* cw = nullptr;            // [k1s][R]
  DevBuf cw_own;
  DevBuf forest;
  DevBuf top;                        // m leaves' tree (absent for m == 1)
};

// What FRI::prove's query phase (fri.rs:174-248) reads after a sharded commit: the sharded rounds
// (runs, forests, top trees) and, when the commit finished on the gathered codeword, the
// single-GPU state of the remaining rounds (identical on every rank).
struct DistFriState {
  uint64_t n2 = 0, R = 0;
  std::vector<ShardedRound> sharded;
  sg_fri_state tail;
  std::vector<uint64_t> lengths;  // every round's codeword length
};

sg_ctx* dist_ctx(sg_dist* d);
// runs a communicator call: a poisoned communicator fails at once (SG_ERR_INVALID); while the body
// runs, the context's host waits watch the communicator (RCCL async errors, SG_DIST_TIMEOUT_S);
// any failure poisons the communicator before the error is returned (dist.cpp sg_dist::dead)
int dist_run(sg_dist* d, const std::function<void()>& body);
void dist_poison(sg_dist* d, const std::string& why);
int dist_world(const sg_dist* d);
int dist_rank(const sg_dist* d);
// sg_dist_stark_prove shards its trace-domain algebra (two ranks or more, SG_DIST_SHARD_ALGEBRA != 0)
bool dist_shard_algebra(const sg_dist* d);
void dist_count_sharded_quotient(sg_dist* d);
void dist_count_sharded_interpolation(sg_dist* d, uint64_t columns);
// n splits over G ranks for both the forward transform (sg_dist_plan) and the inverse
uint64_t dist_split(uint64_t n);
bool dist_can_shard(uint64_t n, int G);
// sg_dist_plan: n = N1 N2, N1 = dist_split(n) = 2^floor(log2 n / 2); run shards hold N1 runs of N2 / G
// elements
void dist_plan(uint64_t n, int G, uint64_t& n1, uint64_t& n2);
// fft/ntt_arithmetics.rs:161-170 of a coefficient vector every rank holds (device, len <= n) into
// this rank's run shard [N1][N2 / G] (its column shard gathered first)
void dist_lde_replicated(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* coeffs, uint64_t len,
                         fe* runs);
// nv polynomials at once (offsets[v], coeffs[v] of lens[v]) into run shards runs + v n / G
void dist_lde_replicated_batch(sg_dist* d, const fe& gen, uint64_t n, const fe* offsets, const fe* const* coeffs,
                               const uint64_t* lens, fe* runs, uint64_t nv);
// fft/ntt.rs:7-68 over the ranks (a root of order exactly n): column shard [N1/G][row_len] in, run
// shard [N1][N2/G] out; the inverse from a run shard into the column shard [N1/G][N2]
void dist_ntt(sg_dist* d, const fe& root, const fe* cols, uint64_t row_len, uint64_t n, fe* runs);
// nv transforms at once (one exchange, one launch per step): column shard v at cols + v N1/G row_len,
// run shard v at runs + v n / G
void dist_ntt_batch(sg_dist* d, const fe& root, const fe* cols, uint64_t row_len, uint64_t n, fe* runs, uint64_t nv);
// fast_coset_evaluate of a coefficient column shard [N1/G][row_len] into the run shard
void dist_coset_evaluate(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* cols, uint64_t row_len,
                         fe* runs);
// nv column shards at once (v at cols + v N1/G row_len, offsets[v]) into runs + v n / G
void dist_coset_evaluate_batch(sg_dist* d, const fe& gen, uint64_t n, const fe* offsets, const fe* cols,
                               uint64_t row_len, fe* runs, uint64_t nv);
void dist_intt(sg_dist* d, const fe& root, const fe* runs, uint64_t n, fe* cols);
// nv inverses at once: run shard v at runs + v n / G, column shard v at cols + v n / G
void dist_intt_batch(sg_dist* d, const fe& root, const fe* runs, uint64_t n, fe* cols, uint64_t nv);
// coset interpolation of a run-sharded codeword of n points on offset * <gen> into the column shard
// [N1/G][N2] of its coefficients (distributed INTT + offset^-i)
void dist_coset_interpolate(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* runs, fe* cols);
// nv codewords at once (run shard v at runs + v n / G, column shard v at cols + v n / G)
void dist_coset_interpolate_batch(sg_dist* d, const fe& gen, uint64_t n, const fe& offset, const fe* runs, fe* cols,
                                  uint64_t nv);
// all-gathers: column shards / run shards of an n-vector -> the whole vector, natural order, every rank
void dist_gather_columns(sg_dist* d, const fe* cols, uint64_t n, fe* out);
// nv column shards (v at cols + v n / G) into outs[v], one all-gather
void dist_gather_columns_batch(sg_dist* d, const fe* cols, uint64_t n, fe* const* outs, uint64_t nv);
void dist_gather_runs(sg_dist* d, const fe* runs, uint64_t n, fe* out);
// nv run shards (v at runs + v n / G) into outs[v], one all-gather
void dist_gather_runs_batch(sg_dist* d, const fe* runs, uint64_t n, fe* const* outs, uint64_t nv);
// this rank's run shard [N1][N2/G] of a natural-order n-vector (a strided copy, no exchange)
void dist_take_runs(sg_dist* d, const fe* full, uint64_t n, fe* runs);
// merkle_root.rs:21-32 of a run-sharded codeword; with `keep`, the forest and top tree are retained
void dist_merkle_root(sg_dist* d, const fe* runs, uint64_t k1s, uint64_t R, uint8_t root[64],
                      ShardedRound* keep = nullptr);
// the same in two parts: the forest + run roots on any stream (no collective; buffers allocated
// beforehand), then the all-gather of the run roots and the top tree on the context's stream
struct PendingForest {
  uint64_t k1s = 0, R = 0, per = 0;
  int drop = 0;  // lean subtrees: the leaf level is not stored (an opening rehashes the sibling leaf)
  DevBuf forest, roots;
};
void dist_forest_alloc(sg_dist* d, uint64_t k1s, uint64_t R, PendingForest& pf);
void dist_forest_launch(sg_dist* d, const fe* runs, PendingForest& pf, hipStream_t s);
void dist_forest_finish(sg_dist* d, PendingForest& pf, uint8_t root[64], ShardedRound* keep);
// values and authentication paths (leaf level first) of global indices I of a sharded codeword,
// identical on every rank: one all-gather of the owners' slots plus the local top tree
void dist_open_round(sg_dist* d, const ShardedRound& sr, uint64_t R, uint64_t n2, const std::vector<uint64_t>& I,
                     std::vector<fe>& vals, std::vector<uint8_t>& paths, int& depth);
// one opening request: a sharded round (sr) or a local round (cw + tree), indices I; filled with the
// values and the paths (I.size() x depth digests, leaf level first)
struct OpenReq {
  const ShardedRound* sr = nullptr;
  const fe* cw = nullptr;
  const sg_tree* tree = nullptr;
  std::vector<uint64_t> I;
  std::vector<fe> vals;
  std::vector<uint8_t> paths;
  int depth = 0;
};
// many requests with one host round trip for all device gathers and ONE all-gather for every
// sharded request's owned slots (R, n2: the run length and N2 of the sharded rounds)
void dist_open_batch(sg_dist* d, uint64_t R, uint64_t n2, std::vector<OpenReq>& reqs);
// fri.rs:210-248 on a run-sharded codeword; `extra` (optional) pushes further objects after the
// query phase, given the top-level indices
void dist_fri_prove(sg_dist* d, const sg_fri* f, const fe* runs, uint64_t n, const sg_proof_stream* ps, size_t* top,
                    const std::function<void(const size_t* top)>& extra = {});

}  // namespace sg
