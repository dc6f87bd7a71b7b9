// Merkle tree device helpers shared by the lane-per-hash kernels (merkle_kernels.hip, built with
// the max-ILP scheduler) and the quad-lane kernels (kernels.hip): launch arguments, digest
// loads/stores, root publication, the leaf value (plain or FRI-folded) and its digest.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "fe128.hpp"
#include "dev_util.hpp"
#include "blake2b.hpp"
#include "leaf_decimal.hpp"

namespace sg {

constexpr int kMaxBatch = 4;  // transforms / trees per launch (blockIdx.y)

struct Digest {
  uint64_t h[8];
};

__device__ __forceinline__ void st_digest(uint64_t* p, const uint64_t d[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    q[i] = make_uint4((uint32_t)d[2 * i], (uint32_t)(d[2 * i] >> 32), (uint32_t)d[2 * i + 1], (uint32_t)(d[2 * i + 1] >> 32));
}
__device__ __forceinline__ void ld_digest(const uint64_t* p, uint64_t d[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint4 v = q[i];
    d[2 * i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    d[2 * i + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
}

// Hash the first level of a group (leaves when `leaves` != nullptr, else nodes
// from the children at `child_level`), then `fuse - 1` further levels in LDS.
// Level k of the tree starts at digest offset level_off[k] in `tree`.
constexpr int kMaxFuse = 11;  // 1024 threads: up to 11 levels (1024 -> 1) in one launch

struct MerkleArgs {
  const fe* leaves[kMaxBatch];  // level 0 input (field elements) per tree (blockIdx.y)
  uint64_t* tree[kMaxBatch];    // retained trees: 8 u64 per digest
  uint64_t first_level;     // level hashed first by this launch
  uint64_t first_count;     // digests at first_level
  int fuse;                 // levels computed by this launch
  uint64_t off[kMaxFuse + 1];  // digest offsets of levels first_level-1 .. first_level+fuse-1 (off[0] = child level)
  uint64_t* root_host[kMaxBatch];  // optional host-coherent copy of the root (written by the launch reaching it)
  uint64_t root_level;             // log2(n): the level whose single digest is the root
  uint64_t leaves_ys, tree_ys;     // != 0: strided rows of trees (leaves[0] + y * leaves_ys, tree[0] + y * tree_ys)
  uint64_t* root_flag[kMaxBatch];  // with root_host: set to root_seq (system scope) once the root is visible
  uint64_t root_seq;
  // lean trees (the prove's retained trees): the levels below `drop` are not stored -- the
  // openings rehash the 2^drop-leaf block around a leaf from the codeword -- so a tree keeps
  // 2 n / 2^drop - 1 digests, not 2n - 1
  uint32_t drop;
  // FRI: the leaves are the fold of the previous round's codeword (fri.rs:151-159),
  // computed here and also stored (dst) -- one launch instead of fold + leaf hash
  struct {
    const fe* src;   // previous codeword (2 * first_count elements)
    fe* dst;         // this round's codeword
    const fe* Tlo;   // Montgomery(w^-e) tables of the round-0 omega: e & 4095, e >> 12
    const fe* Thi;
    int shift;       // previous round r: exponent = i << r
    fe K;            // Montgomery(alpha * offset_r^-1 * 2^-1)
    const fe* Kp;    // non-null: K is this device word instead (a gated round, k_fri_gate)
  } fold;
};

__device__ __forceinline__ fe fold_k(const MerkleArgs& a) { return a.fold.Kp ? ld_fe(a.fold.Kp) : a.fold.K; }

__device__ __forceinline__ uint64_t* merkle_tree_ptr(const MerkleArgs& a) {
  return a.tree_ys ? a.tree[0] + (uint64_t)blockIdx.y * a.tree_ys : a.tree[blockIdx.y];
}
__device__ __forceinline__ const fe* merkle_leaves_ptr(const MerkleArgs& a) {
  return a.leaves_ys ? a.leaves[0] + (uint64_t)blockIdx.y * a.leaves_ys : a.leaves[blockIdx.y];
}
__device__ __forceinline__ uint64_t* merkle_root_slot(const MerkleArgs& a) {
  return a.tree_ys ? nullptr : a.root_host[blockIdx.y];
}
// publish: every lane's root stores reach system scope before the ready flag
__device__ __forceinline__ void merkle_root_publish(const MerkleArgs& a, bool writer) {
  __threadfence_system();
  if (writer && a.root_flag[blockIdx.y]) *(volatile uint64_t*)a.root_flag[blockIdx.y] = a.root_seq;
}

// Leaf value `idx` of the launch (merkle_root.rs:25-30); FOLD: the FRI fold of the previous
// codeword (fri.rs:151-159), also stored to fold.dst.
template <bool FOLD>
__device__ __forceinline__ fe leaf_value(const MerkleArgs& a, uint64_t idx) {
  if constexpr (FOLD) {
    const fe x = ld_fe(a.fold.src + idx);
    const fe y = ld_fe(a.fold.src + idx + a.first_count);
    const uint64_t e = idx << a.fold.shift;
    const fe K = fold_k(a);
    fe t = mont_mul(K, ld_fe(a.fold.Tlo + (e & 4095)));
    t = mont_mul(t, ld_fe(a.fold.Thi + (e >> 12)));
    const fe v = fe_add(fe_halve(fe_add(x, y)), mont_mul(fe_sub(x, y), t));
    st_fe(a.fold.dst + idx, v);
    return v;
  } else {
    return ld_fe(merkle_leaves_ptr(a) + idx);
  }
}

// Leaf values idx and idx + 1 of the launch (a lane's pair).  FOLD: all four inputs (x, y of both
// leaves) are read before any arithmetic and both folded values are stored together at the end, so
// each lane's 32-byte runs of src and dst move as whole lines: with the second leaf's loads and
// store issued ~450 instructions after the first's (the scheduler's order for two leaf_value
// calls) the PMC pass measured 1.22x the algorithmic bytes for this kernel.
template <bool FOLD>
__device__ __forceinline__ void leaf_value_pair(const MerkleArgs& a, uint64_t idx, fe& v0, fe& v1) {
  if constexpr (FOLD) {
    const fe x0 = ld_fe(a.fold.src + idx), x1 = ld_fe(a.fold.src + idx + 1);
    const fe y0 = ld_fe(a.fold.src + idx + a.first_count), y1 = ld_fe(a.fold.src + idx + 1 + a.first_count);
    const uint64_t e0 = idx << a.fold.shift, e1 = (idx + 1) << a.fold.shift;
    const fe K = fold_k(a);
    const fe t0l = ld_fe(a.fold.Tlo + (e0 & 4095)), t0h = ld_fe(a.fold.Thi + (e0 >> 12));
    const fe t1l = ld_fe(a.fold.Tlo + (e1 & 4095)), t1h = ld_fe(a.fold.Thi + (e1 >> 12));
    const fe t0 = mont_mul(mont_mul(K, t0l), t0h), t1 = mont_mul(mont_mul(K, t1l), t1h);
    v0 = fe_add(fe_halve(fe_add(x0, y0)), mont_mul(fe_sub(x0, y0), t0));
    v1 = fe_add(fe_halve(fe_add(x1, y1)), mont_mul(fe_sub(x1, y1), t1));
    // both stores after both values exist (the scheduler would otherwise sink the second)
    asm("" : "+v"(v0.w[0]), "+v"(v0.w[1]), "+v"(v0.w[2]), "+v"(v0.w[3])
        : "v"(v1.w[0]), "v"(v1.w[1]), "v"(v1.w[2]), "v"(v1.w[3]));
    st_fe(a.fold.dst + idx, v0);
    st_fe(a.fold.dst + idx + 1, v1);
  } else {
    v0 = leaf_value<false>(a, idx);
    v1 = leaf_value<false>(a, idx + 1);
  }
}

// leaf digest: BLAKE2b-512 of the decimal string (field_element.rs:46-50 bytes)
__device__ __forceinline__ void leaf_hash(const fe& v, uint64_t d[8]) {
  uint64_t m[16];
  uint32_t len = fe_decimal_words(v, m);
#pragma unroll
  for (int i = 5; i < 16; ++i) m[i] = 0;
  blake2b_single_block(m, len, d);
}

// Launches one of the Merkle kernels (merkle_kernels.hip): kind 0/1/4 leaf levels with 256/1024/512
// lanes, 2/6 node levels with 256/512 lanes, 8 leaf pairs with 512 lanes, 9 pipelined nodes, 10 node
// pairs; quad-lane kinds 3/5 node levels with 64/256 nodes, 7 leaves with 256 leaves per block.
hipError_t launch_merkle_lanes(int kind, bool fold, dim3 grid, unsigned bs, hipStream_t s, const MerkleArgs& a);

}  // namespace sg
