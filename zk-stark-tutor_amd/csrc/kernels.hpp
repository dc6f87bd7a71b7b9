// Host-side launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "fe128.hpp"

namespace sg {

// NTT twiddle plan (see k_stage_twiddles): stage-major entries up to ntt_tw_cut(logn), then
// the two power tables A (4096) and B (n / 2^13) the higher stages multiply on the fly.
int ntt_tw_cut(int logn);
uint64_t ntt_tw_entries(int logn);
hipError_t launch_stage_twiddles(fe* out, const fe* A, const fe* B, int logn, hipStream_t s);
hipError_t launch_pow_table(fe* tw, const fe* A, const fe* B, uint64_t count, hipStream_t s);
// Batched over up to 4 independent transforms / trees (one pointer each, blockIdx.y),
// or, with a non-zero row stride (`ys`), over up to 65535 strided rows from
// pointer [0] (row y at ptr[0] + y * stride).
hipError_t launch_bitrev_gather(fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn,
                                const fe* sA, const fe* sB, int skip, hipStream_t s, uint64_t in_ys = 0,
                                uint64_t out_ys = 0, uint64_t in_es = 1);
hipError_t launch_scale_const(fe* data, uint64_t n, const fe* cst, hipStream_t s);
// Four-step epilogue of the last pass (multi-GPU NTT, dist.cpp): output k of row r (= row0 + the
// launch's row) times w^((j0 + r) k), w^e = T0[e & 4095] T1[(e >> 12) & 4095] T2[e >> 24]
// (Montgomery tables, e < 2^36), stored to out[k >> logR][r][k & (2^logR - 1)] (rows = rows of
// the whole shard): the twiddle multiply and the all-to-all pack without their own HBM passes.
struct NttEpilogue {
  fe* out;
  const fe* T0;
  const fe* T1;
  const fe* T2;
  uint64_t row0, j0, rows;
  int logR;
  // batched: k vectors of 2^vlog rows each (row r of the launch = row r mod 2^vlog of vector
  // r >> vlog), send buffer [peer][row][vector][R]
  int vlog = 63;
  uint64_t k = 1;
};
// big_tl (12 / 13): the stages after first_b0 run as ONE pass on 2^big_tl-element tiles when they fit
// (the plan launch_ntt_fused picks for mid-size transforms); 0: passes on 2048-element tiles
hipError_t launch_ntt_dit(fe* const* data, int batch, const fe* tw, int logn, const fe* post, int first_b0,
                          hipStream_t s, uint64_t ys = 0, const NttEpilogue* ep = nullptr, int big_tl = 0);
// first-pass tile of a 2^logn transform (log2 elements): 11, or 12 / 13 where a two-pass plan on
// bigger tiles measured faster (SG_NTT_TILES=0 keeps 11 everywhere)
int ntt_first_tile(int logn);
// bit-reversal (+ LDE scale, + `skip` trivial stages) fused into the first pass; out must not alias in.
// in_il != 0: `batch` interleaved input rows (row y's element i at in[0] + i * in_il + y; batch a
// multiple of 4, strided output rows) -- a transpose folded into the first pass's gather.
hipError_t launch_ntt_fused(fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn, const fe* tw,
                            const fe* sA, const fe* sB, int skip, const fe* post, hipStream_t s, uint64_t in_ys = 0,
                            uint64_t out_ys = 0, uint64_t in_il = 0, const NttEpilogue* ep = nullptr);
// a batch of 2^logn-point transforms (2^6 .. 2^11) in strided rows runs whole in one first-pass
// launch (2^(11 - logn) rows per tile; SG_NTT_SMALL_WHOLE=0 turns it off)
bool ntt_small_whole(int logn, int batch, int skip, bool strided);
uint64_t merkle_tree_digests(uint64_t n);
// root_host (optional, per tree; pointer mode only): host-coherent 64-byte slots that receive the root.
// start_level 1: level 0 of `tree` already holds n digests (a tree over given digests).
// FRI fold fused into the leaf level: leaves = fold(src) (fri.rs:151-159), also stored to dst
struct FoldLeaves {
  const fe* src;
  fe* dst;
  const fe* Tlo;
  const fe* Thi;
  int shift;
  fe K;
  const fe* Kp = nullptr;  // non-null: K is read from this device word (written by k_fri_gate)
};
// FRI round gate: holds stream s until *gate >= want (host-coherent memory, device views), then
// stores the Montgomery K at Kh (2 u64, pinned) to Kd; after `seconds` it raises *timeout instead
hipError_t launch_fri_gate(const uint64_t* gate, uint64_t want, const uint64_t* Kh, fe* Kd, uint32_t* timeout,
                           double seconds, hipStream_t s);
// root_flag (optional, with root_host): set to root_seq after the root is visible to the host.
// drop: a lean tree (n >= 2) -- the levels below `drop` are not stored: `tree` holds levels drop ..
// log2 n, level l at digest offset (2n - 2(n >> l)) - (2n - 2(n >> drop)).
hipError_t launch_merkle_tree(const fe* const* leaves, uint64_t* const* tree, int batch, uint64_t n,
                              uint64_t* const* root_host, hipStream_t s, uint64_t leaves_ys = 0,
                              uint64_t tree_ys = 0, int start_level = 0, uint64_t* const* root_flag = nullptr,
                              uint64_t root_seq = 0, const FoldLeaves* fold = nullptr, int drop = 0);
hipError_t launch_gather_digests(const uint64_t* tree, const uint64_t* idx, uint64_t* out, uint32_t count,
                                 hipStream_t s);
// HBM probe: dst[0, bytes) = src (16-byte units, bytes % 16 == 0); blocks = 0: one element per
// lane, else `blocks` x 256 lanes grid-stride
hipError_t launch_copy16(const void* src, void* dst, uint64_t bytes, unsigned blocks, hipStream_t s);
hipError_t launch_gather_fe(const fe* src, const uint64_t* idx, fe* out, uint32_t count, hipStream_t s);
// gathers from absolute device addresses (one launch for openings spread over many buffers):
// out[i] = the 64-byte digest (digest = true) or 16-byte element at addr[i]
hipError_t launch_gather_abs(const uint64_t* addr, void* out, uint32_t count, bool digest, hipStream_t s);
// out[r][j] = in[base + r + n1 j] for r < rows, j < row_len (0 past len): a column shard; nb such
// gathers at once, vector v from in + v in_stride into out + v rows row_len
hipError_t launch_gather_cols(fe* out, const fe* in, uint64_t len, uint64_t rows, uint64_t row_len, uint64_t n1,
                              uint64_t base, hipStream_t s, uint64_t nb = 1, uint64_t in_stride = 0);

// Proof-stream objects serialized on the device (the tail of a proof: FRI query phase and the
// Stark openings): [code u8][len u64 BE][payload] at byte offset `dst` of the output, with
// Value / Leafs payloads as `count` big-endian u128 elements read from src[0..count) and a Path
// payload as `count` = log2(n) entries [64 u64 BE][digest] of leaf `index` in the tree whose
// digests start at src[0] (merkle_root.rs:34-53 order, proof_stream_enum.rs:95-126); for a lean
// tree src[2] = K > 0 levels are not stored (the digests at src[0] start at level K) and its first
// K siblings are rehashed from the leaf values at src[1].
// An item with sel != kTailLiteral is resolved on the device from an index table: idx =
// table[sel] & mask, then a Value / Leafs item reads src[k] + 16 idx and a Path item opens leaf
// index + idx -- the items exist before the indices do (the query phase's are planned while the
// last FRI round runs and uploaded then; only the table follows the Fiat-Shamir seed).
constexpr uint32_t kTailLiteral = 0xFFFFFFFFu;
struct TailItem {
  uint64_t src[3];
  uint64_t dst;
  uint64_t n;
  uint64_t index;
  uint32_t code;
  uint32_t count;
  uint32_t sel;
  uint32_t pad;
  uint64_t mask;
};
hipError_t launch_serialize_tail(const TailItem* items, const uint64_t* table, uint32_t count, uint8_t* out,
                                 uint64_t bytes, hipStream_t s);

// row-sharded helpers (four-step NTT, sharded Merkle / FRI)
// (nb: that many rows x cols arrays back to back, each scaled alike)
hipError_t launch_mul_pow(fe* data, uint64_t rows, uint64_t cols, uint64_t a0, uint64_t a1, uint64_t b0,
                          uint64_t b1, const fe* T0, const fe* T1, const fe* T2, hipStream_t s, uint64_t nb = 1);
// out[b][a][c] = in[a][b][c] for nb A x B x C arrays back to back
hipError_t launch_swap01(const fe* in, fe* out, uint64_t A, uint64_t B, uint64_t C, hipStream_t s, uint64_t nb = 1);
hipError_t launch_fri_fold_runs(fe* out, const fe* in, uint64_t half, uint64_t run, uint64_t run_stride,
                                uint64_t run_off, const fe* T0, const fe* T1, const fe* T2, const fe& K,
                                hipStream_t s);
hipError_t launch_gather_roots(const uint64_t* tree, uint64_t tree_ys, uint64_t root_off, uint64_t* out,
                               uint64_t count, hipStream_t s);

}  // namespace sg
