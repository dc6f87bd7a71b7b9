// Merkle lane-per-hash kernels: one leaf or node compression per lane (two leaves in
// k_merkle_leaf_pairs), the levels above fused through LDS (merkle_root.rs:7-32).
//
// This translation unit is compiled with LLVM's max-ILP machine scheduler (Makefile): it
// interleaves the four independent G functions of each BLAKE2b half-round, trading VGPRs
// (74 -> 104 for the leaf-pair kernel, 6 -> 4 waves per SIMD) for per-wave instruction-level
// parallelism: 2^25 tree 2.5 % faster (profiles/r03_ab_merkle_max_ilp.log).  The quad-lane kernels
// (latency-bound tree tops) live here too since round 4: under max-ILP the 2^14 / 2^16 trees, all
// quad kernels, built 4-6 % faster on the same box (profiles/r04_ab_qilp_14.log, _16.log), although
// the 1024-lane quad blocks (128-VGPR cap) keep 12 bytes per lane in scratch.  The NTT kernels stay
// in kernels.hip on the default scheduler (max-ILP spills them).
#include <cstdlib>

#include "kernels.hpp"
#include "merkle_dev.hpp"
#include "profiler.hpp"

namespace sg {

template <bool LEAF, int MAXB, bool FOLD = false>
__global__ __launch_bounds__(MAXB) void k_merkle_levels(MerkleArgs a) {
  // fused levels hand digests over through LDS word-major (sm[word][lane]): a lane
  // writes word i at an 8-byte lane stride and reads its two children's word i as one
  // 16-byte pair, both conflict-free (a 64-byte digest per lane put every lane of a
  // ds_read at a 128-byte stride, i.e. on the same banks)
  __shared__ uint64_t sm[8][MAXB];
  const uint32_t tid = threadIdx.x;
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + tid;
  uint64_t* __restrict__ tree = merkle_tree_ptr(a);
  uint64_t* const root_slot = merkle_root_slot(a);
  uint64_t d[8];
  if (idx < a.first_count) {
    if (LEAF) {
      uint64_t m[16];
      fe v;
      if constexpr (FOLD) {
        const fe x = ld_fe(a.fold.src + idx);
        const fe y = ld_fe(a.fold.src + idx + a.first_count);
        const uint64_t e = idx << a.fold.shift;
        const fe K = fold_k(a);
        fe t = mont_mul(K, ld_fe(a.fold.Tlo + (e & 4095)));
        t = mont_mul(t, ld_fe(a.fold.Thi + (e >> 12)));
        v = fe_add(fe_halve(fe_add(x, y)), mont_mul(fe_sub(x, y), t));
        st_fe(a.fold.dst + idx, v);
      } else {
        v = ld_fe(merkle_leaves_ptr(a) + idx);
      }
      uint32_t len = fe_decimal_words(v, m);
#pragma unroll
      for (int i = 5; i < 16; ++i) m[i] = 0;
      blake2b_single_block(m, len, d);
    } else {
      uint64_t l[8], r[8];
      const uint64_t* child = tree + a.off[0] * 8;
      ld_digest(child + (2 * idx) * 8, l);
      ld_digest(child + (2 * idx + 1) * 8, r);
      blake2b_node(l, r, d);
    }
    if (a.first_level >= a.drop) st_digest(tree + (a.off[1] + idx) * 8, d);  // lean: dropped levels unstored
    if (a.first_level == a.root_level && root_slot) {
      for (int i = 0; i < 8; ++i) root_slot[i] = d[i];
      merkle_root_publish(a, true);
    }
  }
  uint32_t count = blockDim.x;  // digests of this block at the current level
  for (int lev = 1; lev < a.fuse; ++lev) {
#pragma unroll
    for (int i = 0; i < 8; ++i) sm[i][tid] = d[i];
    __syncthreads();
    count >>= 1;
    if (tid < count) {
      uint64_t l[8], r[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const ulonglong2 lr = *reinterpret_cast<const ulonglong2*>(&sm[i][2 * tid]);
        l[i] = lr.x;
        r[i] = lr.y;
      }
      blake2b_node(l, r, d);
      uint64_t gidx = (uint64_t)blockIdx.x * count + tid;
      if (a.first_level + lev >= a.drop) st_digest(tree + (a.off[lev + 1] + gidx) * 8, d);
      if (a.first_level + lev == a.root_level && root_slot) {
        for (int i = 0; i < 8; ++i) root_slot[i] = d[i];
        merkle_root_publish(a, true);
      }
    }
    __syncthreads();
  }
}

// Leaf level with two leaves per lane: lane p hashes leaves 2p and 2p+1 and their parent (level 1)
// itself, so the first two levels keep every wave of the block busy and need no LDS hand-over;
// levels 2 .. fuse-1 follow through LDS as in k_merkle_levels.  first_count (leaves) is a multiple
// of 2 * blockDim.x (host-checked).  With one leaf per lane, a 512-lane block's fused levels leave
// 4, 2, 1 of its 8 waves busy (74 VGPRs: 6 waves per SIMD), so the SIMDs run short of ready waves;
// here the first two levels keep all 8 busy.
template <int MAXB, bool FOLD>
__global__ __launch_bounds__(MAXB, 4) void k_merkle_leaf_pairs(MerkleArgs a) {
  __shared__ uint64_t sm[8][MAXB];
  const uint32_t tid = threadIdx.x;
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + tid;  // level-1 node
  uint64_t* __restrict__ tree = merkle_tree_ptr(a);
  uint64_t* const root_slot = merkle_root_slot(a);
  uint64_t d[8];
  {
    // both leaves are read (and folded) up front and both digests stored together, so each lane's
    // 32-byte leaf pair and 128-byte digest pair move as whole lines (stored one compression apart,
    // the digest halves were written back to HBM as separate partial lines: 1.19x the algorithmic
    // bytes in the PMC pass)
    // (the plain-leaf variant keeps the two-call form: the pair form's schedule takes it from 104
    // to 132 VGPRs, 4 -> 3 waves per SIMD, and the 2^25 tree 13 % slower in the round-4 A/B)
    fe v0, v1;
    if constexpr (FOLD) {
      leaf_value_pair<true>(a, 2 * p, v0, v1);
    } else {
      v0 = leaf_value<false>(a, 2 * p);
      v1 = leaf_value<false>(a, 2 * p + 1);
    }
    // keep the second leaf's read beside the first: the first compression's input is tied to it
    // (the scheduler would sink the read past that compression to save 4 VGPRs, re-touching each
    // lane pair's line ~2000 instructions later)
    asm("" : "+v"(v0.w[0]), "+v"(v0.w[1]), "+v"(v0.w[2]), "+v"(v0.w[3])
        : "v"(v1.w[0]), "v"(v1.w[1]), "v"(v1.w[2]), "v"(v1.w[3]));
    uint64_t l[8], r[8];
    leaf_hash(v0, l);
    leaf_hash(v1, r);
    if (a.drop == 0) {  // lean trees keep no leaf digests
      st_digest(tree + (a.off[1] + 2 * p) * 8, l);
      st_digest(tree + (a.off[1] + 2 * p + 1) * 8, r);
    }
    blake2b_node(l, r, d);
    if (a.drop <= 1) st_digest(tree + (a.off[2] + p) * 8, d);
    if (a.first_level + 1 == a.root_level && root_slot) {
      for (int i = 0; i < 8; ++i) root_slot[i] = d[i];
      merkle_root_publish(a, true);
    }
  }
  uint32_t count = blockDim.x;  // digests of this block at the current level
  for (int lev = 2; lev < a.fuse; ++lev) {
#pragma unroll
    for (int i = 0; i < 8; ++i) sm[i][tid] = d[i];
    __syncthreads();
    count >>= 1;
    if (tid < count) {
      uint64_t l[8], r[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const ulonglong2 lr = *reinterpret_cast<const ulonglong2*>(&sm[i][2 * tid]);
        l[i] = lr.x;
        r[i] = lr.y;
      }
      blake2b_node(l, r, d);
      uint64_t gidx = (uint64_t)blockIdx.x * count + tid;
      if (a.first_level + lev >= a.drop) st_digest(tree + (a.off[lev + 1] + gidx) * 8, d);
      if (a.first_level + lev == a.root_level && root_slot) {
        for (int i = 0; i < 8; ++i) root_slot[i] = d[i];
        merkle_root_publish(a, true);
      }
    }
    __syncthreads();
  }
}

// (round 6: the rejected node-level variants -- a grid-stride pipelined kernel, two nodes per
// lane, the level-2 hand-over by DPP -- were removed; their same-box A/Bs stay in profiles/.)


// ---------------------------------------------------- Merkle: 4 lanes per hash
//
// The top of a tree is latency-bound: a level of a few thousand nodes or less
// cannot fill the chip, and each level waits for the one below.  Here one
// compression is split over a quad of lanes (BLAKE2b's four independent G
// columns): lane q holds column q (v[q], v[4+q], v[8+q], v[12+q]), the
// diagonal step rotates rows 1..3 across the quad with DPP quad_perm moves,
// and message words are read from LDS at the round's sigma positions.
// ~2.4x fewer dependent instructions per level than one lane per hash.

// packed sigma nibbles for one lane of the quad: round r (0..9) occupies bits
// [16r, 16r+16) as (col_x, col_y, diag_x, diag_y) = sigma[r][2q], [2q+1], [8+2q], [9+2q]
struct SigmaPack {
  uint32_t w[5];
};
__host__ __device__ constexpr uint32_t sigma_nib(int r, int q) {
  constexpr uint8_t S[10][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
  return (uint32_t)S[r][2 * q] | ((uint32_t)S[r][2 * q + 1] << 4) | ((uint32_t)S[r][8 + 2 * q] << 8) |
         ((uint32_t)S[r][9 + 2 * q] << 12);
}
__device__ __forceinline__ SigmaPack sigma_pack(int q) {
  SigmaPack p;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    uint32_t v0 = q == 0 ? sigma_nib(2 * k, 0) : q == 1 ? sigma_nib(2 * k, 1) : q == 2 ? sigma_nib(2 * k, 2) : sigma_nib(2 * k, 3);
    uint32_t v1 = q == 0 ? sigma_nib(2 * k + 1, 0) : q == 1 ? sigma_nib(2 * k + 1, 1) : q == 2 ? sigma_nib(2 * k + 1, 2)
                                                                                              : sigma_nib(2 * k + 1, 3);
    p.w[k] = v0 | (v1 << 16);
  }
  return p;
}

template <int CTRL>
__device__ __forceinline__ uint64_t quad_perm64(uint64_t x) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xF, 0xF, true);
  uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, true);
  return ((uint64_t)hi << 32) | lo;
}
// quad_perm encodings: lane i takes lane sel[i]
constexpr int QP_NEXT1 = 1 | (2 << 2) | (3 << 4) | (0 << 6);  // from (q+1)%4
constexpr int QP_NEXT2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // from (q+2)%4
constexpr int QP_NEXT3 = 3 | (0 << 2) | (1 << 4) | (2 << 6);  // from (q+3)%4

#define SG_QG(a, b, c, d, x, y)   \
  a = a + b + (x);                \
  d = rotr64(d ^ a, 32);          \
  c = c + d;                      \
  b = rotr64(b ^ c, 24);          \
  a = a + b + (y);                \
  d = rotr64(d ^ a, 16);          \
  c = c + d;                      \
  b = rotr64(b ^ c, 63);

// One BLAKE2b single-block compression (final block, counter t) computed by a
// quad.  msg: the 16 message words in LDS.  Returns h[q] and h[4+q].
__device__ __forceinline__ void blake2b_quad(const uint64_t* msg, uint64_t t, int q, const SigmaPack& sp,
                                             uint64_t& out_lo, uint64_t& out_hi) {
  const uint64_t ivq = q == 0 ? SG_B2B_IV0 : q == 1 ? SG_B2B_IV1 : q == 2 ? SG_B2B_IV2 : SG_B2B_IV3;
  const uint64_t iv4q = q == 0 ? SG_B2B_IV4 : q == 1 ? SG_B2B_IV5 : q == 2 ? SG_B2B_IV6 : SG_B2B_IV7;
  const uint64_t hq = q == 0 ? (SG_B2B_IV0 ^ 0x01010040ull) : ivq;
  uint64_t a = hq, b = iv4q, c = ivq;
  uint64_t d = iv4q ^ (q == 0 ? t : 0) ^ (q == 2 ? ~0ull : 0);
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    const int rr = r % 10;
    const uint32_t nib = (sp.w[rr >> 1] >> (16 * (rr & 1))) & 0xFFFFu;
    uint64_t mx = msg[nib & 15], my = msg[(nib >> 4) & 15];
    uint64_t dx = msg[(nib >> 8) & 15], dy = msg[nib >> 12];
    SG_QG(a, b, c, d, mx, my)
    b = quad_perm64<QP_NEXT1>(b);
    c = quad_perm64<QP_NEXT2>(c);
    d = quad_perm64<QP_NEXT3>(d);
    SG_QG(a, b, c, d, dx, dy)
    b = quad_perm64<QP_NEXT3>(b);
    c = quad_perm64<QP_NEXT2>(c);
    d = quad_perm64<QP_NEXT1>(d);
  }
  out_lo = hq ^ a ^ c;
  out_hi = iv4q ^ b ^ d;
}

// The `fuse - 1` levels a quad block computes above its first digests (hlo, hhi of node `node`):
// children through LDS, every digest written to the tree, the root published by the level reaching it.
template <int NODES>
__device__ __forceinline__ void quad_upper_levels(const MerkleArgs& a, uint64_t* __restrict__ tree,
                                                  uint64_t* root_slot, uint64_t (*msg)[16], int node, int q,
                                                  const SigmaPack& sp, uint32_t count, uint64_t hlo, uint64_t hhi) {
  for (int lev = 1; lev < a.fuse; ++lev) {
    __syncthreads();  // everyone finished reading msg
    if (node < (int)count) {
      msg[node >> 1][(node & 1) * 8 + q] = hlo;
      msg[node >> 1][(node & 1) * 8 + 4 + q] = hhi;
    }
    __syncthreads();
    count >>= 1;
    if (node < (int)count) {
      blake2b_quad(msg[node], 128, q, sp, hlo, hhi);
      if (a.first_level + lev >= a.drop) {  // lean trees: dropped levels unstored
        uint64_t gidx = (uint64_t)blockIdx.x * count + node;
        uint64_t* dst = tree + (a.off[lev + 1] + gidx) * 8;
        dst[q] = hlo;
        dst[4 + q] = hhi;
      }
      if (a.first_level + lev == a.root_level && root_slot) {
        root_slot[q] = hlo;
        root_slot[4 + q] = hhi;
        merkle_root_publish(a, q == 0);
      }
    }
  }
}

// Node levels with a quad per node: 4 * NODES threads = NODES nodes at the first level,
// `fuse` levels computed (NODES -> 1 at most).  Children of the first level are
// read from HBM (level first_level-1), every produced digest is written to the tree.
// NODES = 64 for wide levels; NODES = 256 takes a tree's last <= 256 nodes to the root
// in one block (one launch fewer per tree than two 64-node steps).
template <int NODES>
__global__ __launch_bounds__(4 * NODES) void k_merkle_quad(MerkleArgs a) {
  __shared__ uint64_t msg[NODES][16];
  const int tid = threadIdx.x;
  const int q = tid & 3;
  const int node = tid >> 2;
  uint64_t* __restrict__ tree = merkle_tree_ptr(a);
  uint64_t* const root_slot = merkle_root_slot(a);
  const SigmaPack sp = sigma_pack(q);
  uint32_t count = blockDim.x >> 2;  // nodes of this block at the current level
  const uint64_t gnode = (uint64_t)blockIdx.x * count + node;
  const bool valid = gnode < a.first_count;
  {
    // message of node gnode = its two children, 16 consecutive words in the child level
    const uint64_t* child = tree + (a.off[0] + 2 * gnode) * 8;
    if (valid) {
      uint4 v0 = reinterpret_cast<const uint4*>(child)[2 * q];
      uint4 v1 = reinterpret_cast<const uint4*>(child)[2 * q + 1];
      msg[node][4 * q + 0] = (uint64_t)v0.x | ((uint64_t)v0.y << 32);
      msg[node][4 * q + 1] = (uint64_t)v0.z | ((uint64_t)v0.w << 32);
      msg[node][4 * q + 2] = (uint64_t)v1.x | ((uint64_t)v1.y << 32);
      msg[node][4 * q + 3] = (uint64_t)v1.z | ((uint64_t)v1.w << 32);
    }
  }
  __syncthreads();
  uint64_t hlo = 0, hhi = 0;
  if (valid) {
    blake2b_quad(msg[node], 128, q, sp, hlo, hhi);
    uint64_t* dst = tree + (a.off[1] + gnode) * 8;
    dst[q] = hlo;
    dst[4 + q] = hhi;
    if (a.first_level == a.root_level && root_slot) {
      root_slot[q] = hlo;
      root_slot[4 + q] = hhi;
      merkle_root_publish(a, q == 0);  // the quad is one wavefront: its fence covers all 4 lanes
    }
  }
  quad_upper_levels<NODES>(a, tree, root_slot, msg, node, q, sp, count, hlo, hhi);
}

// Leaf level of a latency-bound tree (a late FRI round's codeword, C4's small trees, a forest's
// small subtrees) with a quad of lanes per leaf: each lane of the quad converts the leaf to its
// decimal words (the quad shares a wavefront, so the redundant conversion costs no time) and
// stores its four of the 16 message words (decimal words 0..4, zeros above); the quad then
// compresses the single block with t = the string length (merkle_root.rs:7-32 on
// field_element.rs:46-50 bytes), and the node levels above are fused as in k_merkle_quad.
// FOLD: the leaf is the fold of the previous round's codeword (fri.rs:151-159), stored too.
template <int NODES, bool FOLD>
__global__ __launch_bounds__(4 * NODES) void k_merkle_quad_leaves(MerkleArgs a) {
  __shared__ uint64_t msg[NODES][16];
  const int tid = threadIdx.x;
  const int q = tid & 3;
  const int node = tid >> 2;
  uint64_t* __restrict__ tree = merkle_tree_ptr(a);
  uint64_t* const root_slot = merkle_root_slot(a);
  const SigmaPack sp = sigma_pack(q);
  uint32_t count = blockDim.x >> 2;  // leaves of this block
  const uint64_t leaf = (uint64_t)blockIdx.x * count + node;
  const bool valid = leaf < a.first_count;
  uint32_t len = 0;
  if (valid) {
    fe v;
    if constexpr (FOLD) {
      const fe x = ld_fe(a.fold.src + leaf);
      const fe y = ld_fe(a.fold.src + leaf + a.first_count);
      const uint64_t e = leaf << a.fold.shift;
      const fe K = fold_k(a);
      fe t = mont_mul(K, ld_fe(a.fold.Tlo + (e & 4095)));
      t = mont_mul(t, ld_fe(a.fold.Thi + (e >> 12)));
      v = fe_add(fe_halve(fe_add(x, y)), mont_mul(fe_sub(x, y), t));
      if (q == 0) st_fe(a.fold.dst + leaf, v);
    } else {
      v = ld_fe(merkle_leaves_ptr(a) + leaf);
    }
    uint64_t m[5];
    len = fe_decimal_words(v, m);
    msg[node][4 * q + 0] = q == 0 ? m[0] : q == 1 ? m[4] : 0;
    msg[node][4 * q + 1] = q == 0 ? m[1] : 0;
    msg[node][4 * q + 2] = q == 0 ? m[2] : 0;
    msg[node][4 * q + 3] = q == 0 ? m[3] : 0;
  }
  __syncthreads();
  uint64_t hlo = 0, hhi = 0;
  if (valid) {
    blake2b_quad(msg[node], len, q, sp, hlo, hhi);
    if (a.drop == 0) {  // lean trees keep no leaf digests
      uint64_t* dst = tree + (a.off[1] + leaf) * 8;
      dst[q] = hlo;
      dst[4 + q] = hhi;
    }
    if (a.first_level == a.root_level && root_slot) {
      root_slot[q] = hlo;
      root_slot[4 + q] = hhi;
      merkle_root_publish(a, q == 0);
    }
  }
  quad_upper_levels<NODES>(a, tree, root_slot, msg, node, q, sp, count, hlo, hhi);
}

// --------------------------------------------- proof-stream tail serialization

__device__ __forceinline__ void put_be64_dev(uint8_t* o, uint64_t v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (uint8_t)(v >> (56 - 8 * i));
}

// one 64-lane block per object (TailItem in kernels.hpp); lane 0 writes the 9-byte header, lane k
// the k-th element / path entry (a path has log2(n) <= 64 entries).  A lean tree's path (src[2] = K
// <= 3 levels not stored): the aligned 2^K-leaf block holding the opened leaf is rehashed from the
// leaf values (src[1]) into LDS, a quad of lanes per compression (the decimal leaf words as in
// k_merkle_quad_leaves, then the node levels), so its K - 1 dependent steps take quad-lane
// latency; the block's nodes are the path's first K siblings (merkle_root.rs:25-53).
__global__ __launch_bounds__(64) void k_serialize_tail(const TailItem* __restrict__ items,
                                                      const uint64_t* __restrict__ table, uint8_t* __restrict__ out) {
  TailItem it = items[blockIdx.x];
  if (it.sel != kTailLiteral) {  // uniform over the block
    // an index past its object (a table not yet valid: the device sampler's failure, redone from the
    // host) reads element 0 instead of faulting; such a block's bytes are always rewritten
    uint64_t idx = table[it.sel] & it.mask;
    if (it.code == 2) {
      const uint64_t i2 = it.index + idx;
      it.index = i2 < it.n ? i2 : 0;
    } else {
      if (idx >= it.n) idx = 0;
      it.src[0] += 16 * idx;
      it.src[1] += 16 * idx;
      it.src[2] += 16 * idx;
    }
  }
  const uint32_t l = threadIdx.x;
  const bool path = it.code == 2;  // SG_OBJ_PATH
  // The object's bytes are assembled in LDS at the alignment they take in `out` (`a`: the start's
  // offset in its 16-byte word), then stored as whole 16-byte words -- 1 KiB contiguous per store
  // instruction, which `out` in host memory (the pinned stream body) needs for PCIe rate -- with byte
  // stores only in the words where the object starts or ends (their other bytes are other objects').
  __shared__ uint4 sw[(15 + 9 + 72 * 64 + 15) / 16];
  uint8_t* sb = reinterpret_cast<uint8_t*>(sw);
  const uintptr_t g0 = reinterpret_cast<uintptr_t>(out + it.dst);
  const uint32_t a = (uint32_t)(g0 & 15);
  const uint32_t rec = path ? 72u : 16u;
  const uint32_t size = 9 + rec * it.count;
  auto be64 = [&](uint32_t pos, uint64_t v) {
#pragma unroll
    for (int j = 0; j < 8; ++j) sb[pos + j] = (uint8_t)(v >> (8 * (7 - j)));
  };
  if (l == 0) {
    sb[a] = (uint8_t)it.code;
    be64(a + 1, (uint64_t)rec * it.count);
  }
  __shared__ uint64_t msg[8][16];  // level-0 messages (decimal leaf words)
  __shared__ uint64_t mt[16][8];   // the block's levels 0 .. K-1: 2^K + 2^(K-1) + ... digests
  const uint32_t K = path ? (uint32_t)it.src[2] : 0u;  // uniform over the block
  if (K) {
    const fe* lv = reinterpret_cast<const fe*>(it.src[1]);
    const uint64_t base = it.index & ~((1ull << K) - 1);
    const int q = (int)(l & 3), node = (int)(l >> 2);
    const SigmaPack sp = sigma_pack(q);
    const bool on0 = node < (1 << K);
    uint32_t len = 0;
    if (on0) {
      uint64_t m[5];
      len = fe_decimal_words(ld_fe(lv + base + node), m);
      msg[node][4 * q + 0] = q == 0 ? m[0] : q == 1 ? m[4] : 0;
      msg[node][4 * q + 1] = q == 0 ? m[1] : 0;
      msg[node][4 * q + 2] = q == 0 ? m[2] : 0;
      msg[node][4 * q + 3] = q == 0 ? m[3] : 0;
    }
    __syncthreads();
    uint64_t hlo = 0, hhi = 0;
    if (on0) {
      blake2b_quad(msg[node], len, q, sp, hlo, hhi);
      mt[node][q] = hlo;
      mt[node][4 + q] = hhi;
    }
    __syncthreads();
    for (uint32_t lev = 1, off = 0, cnt = 1u << K; lev < K; ++lev) {
      if (node < (int)(cnt >> 1)) {
        blake2b_quad(&mt[off + 2 * node][0], 128, q, sp, hlo, hhi);  // children adjacent: 16 words
        mt[off + cnt + node][q] = hlo;
        mt[off + cnt + node][4 + q] = hhi;
      }
      __syncthreads();
      off += cnt;
      cnt >>= 1;
    }
  }
  if (l < it.count) {
    const uint32_t e = a + 9 + rec * l;
    if (path) {
      be64(e, 64);
      uint64_t h[8];
      if (l < K) {  // sibling at level l inside the rehashed block
        const uint32_t off = (1u << (K + 1)) - (1u << (K + 1 - l));  // 2^K + 2^(K-1) + ... (l terms)
        const uint32_t sib = (uint32_t)(((it.index >> l) ^ 1) & ((1ull << (K - l)) - 1));
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = mt[off + sib][k];
      } else {
        // level l sibling; a lean tree's buffer starts at level K
        const uint64_t d = (2 * it.n - 2 * (it.n >> l)) - (2 * it.n - 2 * (it.n >> K)) + ((it.index >> l) ^ 1);
        ld_digest(reinterpret_cast<const uint64_t*>(it.src[0] + 64 * d), h);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) sb[e + 8 + 8 * k + j] = (uint8_t)(h[k] >> (8 * j));
    } else {
      const fe v = ld_fe(reinterpret_cast<const fe*>(it.src[l]));
      be64(e, fe_hi(v));
      be64(e + 8, fe_lo(v));
    }
  }
  __syncthreads();
  uint4* gw = reinterpret_cast<uint4*>(g0 - a);
  uint8_t* gb = reinterpret_cast<uint8_t*>(g0 - a);
  const uint32_t end = a + size, nd = (end + 15) / 16;
  for (uint32_t i = l; i < nd; i += 64) {
    const uint32_t b0 = 16 * i;
    if (b0 >= a && b0 + 16 <= end) {
      gw[i] = sw[i];
    } else {
      for (uint32_t b = b0 < a ? a : b0; b < b0 + 16 && b < end; ++b) gb[b] = sb[b];
    }
  }
}

hipError_t launch_serialize_tail(const TailItem* items, const uint64_t* table, uint32_t count, uint8_t* out,
                                 uint64_t bytes, hipStream_t s) {
  if (!count) return hipSuccess;
  ProfScope ps("serialize_tail", bytes, s);
  hipLaunchKernelGGL(k_serialize_tail, dim3(count), dim3(64), 0, s, items, table, out);
  return hipGetLastError();
}

hipError_t launch_merkle_lanes(int kind, bool fold, dim3 grid, unsigned bs, hipStream_t s, const MerkleArgs& a) {
  switch (kind) {
    case 0:
      if (fold) hipLaunchKernelGGL((k_merkle_levels<true, 256, true>), grid, dim3(bs), 0, s, a);
      else hipLaunchKernelGGL((k_merkle_levels<true, 256>), grid, dim3(bs), 0, s, a);
      break;
    case 1:
      if (fold) hipLaunchKernelGGL((k_merkle_levels<true, 1024, true>), grid, dim3(bs), 0, s, a);
      else hipLaunchKernelGGL((k_merkle_levels<true, 1024>), grid, dim3(bs), 0, s, a);
      break;
    case 2: hipLaunchKernelGGL((k_merkle_levels<false, 256>), grid, dim3(bs), 0, s, a); break;
    case 6: hipLaunchKernelGGL((k_merkle_levels<false, 512>), grid, dim3(bs), 0, s, a); break;
    case 3: hipLaunchKernelGGL(k_merkle_quad<64>, grid, dim3(bs), 0, s, a); break;
    case 5: hipLaunchKernelGGL(k_merkle_quad<256>, grid, dim3(bs), 0, s, a); break;
    case 7:
      if (fold) hipLaunchKernelGGL((k_merkle_quad_leaves<256, true>), grid, dim3(bs), 0, s, a);
      else hipLaunchKernelGGL((k_merkle_quad_leaves<256, false>), grid, dim3(bs), 0, s, a);
      break;
    case 12:
      if (fold) hipLaunchKernelGGL((k_merkle_quad_leaves<64, true>), grid, dim3(bs), 0, s, a);
      else hipLaunchKernelGGL((k_merkle_quad_leaves<64, false>), grid, dim3(bs), 0, s, a);
      break;
    case 4:
      if (fold) hipLaunchKernelGGL((k_merkle_levels<true, 512, true>), grid, dim3(bs), 0, s, a);
      else hipLaunchKernelGGL((k_merkle_levels<true, 512>), grid, dim3(bs), 0, s, a);
      break;
    case 8:
      if (fold) hipLaunchKernelGGL((k_merkle_leaf_pairs<512, true>), grid, dim3(bs), 0, s, a);
      else hipLaunchKernelGGL((k_merkle_leaf_pairs<512, false>), grid, dim3(bs), 0, s, a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace sg
