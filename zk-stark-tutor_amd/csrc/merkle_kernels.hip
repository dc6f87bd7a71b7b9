// Merkle lane-per-hash kernels: one leaf or node compression per lane (two leaves in
// k_merkle_leaf_pairs), the levels above fused through LDS (merkle_root.rs:7-32).
//
// This translation unit is compiled with LLVM's max-ILP machine scheduler (Makefile): it
// interleaves the four independent G functions of each BLAKE2b half-round, trading VGPRs
// (74 -> 104 for the leaf-pair kernel, 6 -> 4 waves per SIMD) for per-wave instruction-level
// parallelism: 2^25 tree 2.5 % faster (profiles/r03_ab_merkle_max_ilp.log).  The NTT and quad-lane
// kernels stay on the default scheduler (max-ILP spills them).
#include <cstdlib>

#include "merkle_dev.hpp"

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
        const fe K = a.fold.Kp ? ld_fe(a.fold.Kp) : a.fold.K;
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
    st_digest(tree + (a.off[1] + idx) * 8, d);
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
      st_digest(tree + (a.off[lev + 1] + gidx) * 8, d);
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
__global__ __launch_bounds__(MAXB) void k_merkle_leaf_pairs(MerkleArgs a) {
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
    st_digest(tree + (a.off[1] + 2 * p) * 8, l);
    st_digest(tree + (a.off[1] + 2 * p + 1) * 8, r);
    blake2b_node(l, r, d);
    st_digest(tree + (a.off[2] + p) * 8, d);
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
      st_digest(tree + (a.off[lev + 1] + gidx) * 8, d);
      if (a.first_level + lev == a.root_level && root_slot) {
        for (int i = 0; i < 8; ++i) root_slot[i] = d[i];
        merkle_root_publish(a, true);
      }
    }
    __syncthreads();
  }
}

// Node levels as k_merkle_levels<false, MAXB>, but each block walks groups g = blockIdx.x,
// blockIdx.x + gridDim.x, ... (MAXB first-level nodes and their fused levels each) and issues the
// NEXT group's child loads before hashing the current one: the 128 B of children per lane arrive
// while the lane compresses, instead of every block starting with a full HBM round trip (the SQ
// pass of the one-group kernel shows its waves parked on s_waitcnt / barriers 36 % of their
// lifetime, against 25 % for the leaf kernel).  groups = first_count / MAXB (host-checked exact).
template <int MAXB>
__global__ __launch_bounds__(MAXB) void k_merkle_nodes_pipe(MerkleArgs a, uint64_t groups) {
  __shared__ uint64_t sm[8][MAXB];
  const uint32_t tid = threadIdx.x;
  uint64_t* __restrict__ tree = merkle_tree_ptr(a);
  const uint64_t* child = tree + a.off[0] * 8;
  uint64_t nl[8], nr[8];
  uint64_t g = blockIdx.x;
  if (g < groups) {
    const uint64_t idx = g * MAXB + tid;
    ld_digest(child + (2 * idx) * 8, nl);
    ld_digest(child + (2 * idx + 1) * 8, nr);
  }
  for (; g < groups; g += gridDim.x) {
    uint64_t l[8], r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      l[i] = nl[i];
      r[i] = nr[i];
    }
    const uint64_t gn = g + gridDim.x;
    if (gn < groups) {
      const uint64_t idxn = gn * MAXB + tid;
      ld_digest(child + (2 * idxn) * 8, nl);
      ld_digest(child + (2 * idxn + 1) * 8, nr);
    }
    uint64_t d[8];
    blake2b_node(l, r, d);
    st_digest(tree + (a.off[1] + g * MAXB + tid) * 8, d);
    uint32_t count = MAXB;
    for (int lev = 1; lev < a.fuse; ++lev) {
#pragma unroll
      for (int i = 0; i < 8; ++i) sm[i][tid] = d[i];
      __syncthreads();
      count >>= 1;
      if (tid < count) {
        uint64_t cl[8], cr[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const ulonglong2 lr = *reinterpret_cast<const ulonglong2*>(&sm[i][2 * tid]);
          cl[i] = lr.x;
          cr[i] = lr.y;
        }
        blake2b_node(cl, cr, d);
        st_digest(tree + (a.off[lev + 1] + g * count + tid) * 8, d);
      }
      __syncthreads();
    }
  }
}

// Node level with two nodes per lane, as k_merkle_leaf_pairs for the leaves: lane p reads its four
// children (256 contiguous bytes), hashes nodes 2p and 2p + 1 of the first level and their parent
// itself, so the first two levels keep all waves of the block busy (the one-node kernel's fused
// levels leave 4, 2, 1 of 4 waves busy) and each lane has two independent compressions to
// interleave while the other's loads are in flight.  first_count is a multiple of 2 * MAXB
// (host-checked); levels 2 .. fuse-1 follow through LDS.
template <int MAXB>
__global__ __launch_bounds__(MAXB) __attribute__((amdgpu_waves_per_eu(4))) void k_merkle_node_pairs(MerkleArgs a) {
  __shared__ uint64_t sm[8][MAXB];
  const uint32_t tid = threadIdx.x;
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + tid;
  uint64_t* __restrict__ tree = merkle_tree_ptr(a);
  uint64_t* const root_slot = merkle_root_slot(a);
  const uint64_t* child = tree + a.off[0] * 8 + (4 * p) * 8;
  uint64_t d[8];
  {
    uint64_t c0[8], c1[8], c2[8], c3[8];
    ld_digest(child, c0);
    ld_digest(child + 8, c1);
    ld_digest(child + 16, c2);
    ld_digest(child + 24, c3);
    uint64_t l[8], r[8];
    blake2b_node(c0, c1, l);
    blake2b_node(c2, c3, r);
    st_digest(tree + (a.off[1] + 2 * p) * 8, l);
    st_digest(tree + (a.off[1] + 2 * p + 1) * 8, r);
    blake2b_node(l, r, d);
    st_digest(tree + (a.off[2] + p) * 8, d);
    if (a.first_level + 1 == a.root_level && root_slot) {
      for (int i = 0; i < 8; ++i) root_slot[i] = d[i];
      merkle_root_publish(a, true);
    }
  }
  uint32_t count = blockDim.x;
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
      const uint64_t gidx = (uint64_t)blockIdx.x * count + tid;
      st_digest(tree + (a.off[lev + 1] + gidx) * 8, d);
      if (a.first_level + lev == a.root_level && root_slot) {
        for (int i = 0; i < 8; ++i) root_slot[i] = d[i];
        merkle_root_publish(a, true);
      }
    }
    __syncthreads();
  }
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
    case 9: {
      // pipelined node levels: grid.x = the groups, run by at most `cap` resident blocks per tree
      const uint64_t groups = grid.x;
      static const uint64_t cap = [] {
        const char* v = getenv("SG_MERKLE_NODE_PIPE_BLOCKS");  // blocks per launch row (A/B knob)
        return (uint64_t)(v && atoi(v) > 0 ? atoi(v) : 1024);
      }();
      dim3 g2((unsigned)(groups < cap ? groups : cap), grid.y);
      hipLaunchKernelGGL((k_merkle_nodes_pipe<256>), g2, dim3(bs), 0, s, a, groups);
      break;
    }
    case 6: hipLaunchKernelGGL((k_merkle_levels<false, 512>), grid, dim3(bs), 0, s, a); break;
    case 10: hipLaunchKernelGGL((k_merkle_node_pairs<256>), grid, dim3(bs), 0, s, a); break;
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
