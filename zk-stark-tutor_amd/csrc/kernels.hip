// HIP kernels for gfx950 (MI355X): NTT / LDE, Merkle tree, FRI fold.
//
// NTT: the reference's radix-2 DIT graph (fft/ntt.rs:7-49) executed exactly:
// bit-reversal gather, then log2(n) stages where stage S (size 2^S) combines
// (j, j + 2^(S-1)) with twiddle powtable[k * n/2^S], k = j mod 2^(S-1).
// Stages are grouped into passes over LDS tiles (up to 4096 elements = 64 KiB)
// and, inside a pass, into radix-8/4/2 register steps (three consecutive
// radix-2 stages on 8 elements).  Every butterfly sees the same operands and
// twiddle as in the reference, so the output is bit-identical for ANY root,
// primitive or not.
//
// Merkle: leaf = BLAKE2b(decimal(v)), node = BLAKE2b(left || right)
// (merkle_root.rs:7-32).  One launch hashes one level from HBM and fuses up to
// three more levels through LDS; every level's digests are written to a
// retained tree buffer (levels concatenated, 64 B per digest) so openings are
// O(log n) gathers.
//
// FRI fold (fri.rs:150-159): c'[i] = (c[i] + c[i+h])/2 + K*w^-i*(c[i] - c[i+h])
// with K = alpha * offset^-1 / 2 in Montgomery form; w^-i advanced by one
// Montgomery product per grid-stride step, no per-element inverse or pow.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include "fe128.hpp"
#include "dev_util.hpp"
#include "blake2b.hpp"
#include "leaf_decimal.hpp"
#include "kernels.hpp"
#include "profiler.hpp"
#include "knobs.hpp"
#include "merkle_dev.hpp"

// SG_NTT_WPE: minimum waves per SIMD the NTT passes' launch bounds ask for (1: the compiler's choice,
// 118-126 VGPRs, 4 waves).  (Round 6 built the verdict's interleaved-carry butterflies as generated
// inline asm, tools/gen_fe_asm.py: 78 % fewer s_nop wait states in k_ntt_pass_rr<11>, C2 unchanged,
// and kernel faults from SGPR hazards between the asm and hipcc's own code -- removed)
#ifndef SG_NTT_WPE
#define SG_NTT_WPE 1
#endif
namespace sg {

thread_local KernelProfiler* g_prof = nullptr;


// ------------------------------------------------------------------ helpers


// ------------------------------------------------------------- twiddles

// tw[e] = A[e & 4095] * B[e >> 12] (both Montgomery) => Montgomery of root^e
__global__ void k_pow_table(fe* __restrict__ tw, const fe* __restrict__ A, const fe* __restrict__ B, uint64_t count) {
  uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  st_fe(tw + e, mont_mul(ld_fe(A + (e & 4095)), ld_fe(B + (e >> 12))));
}

// Twiddle plan of a 2^logn transform (one buffer, built once per (root, logn)):
//  * stage-major entries for stages S = 1..s_cut: entries [2^(S-1) - 1, 2^S - 1)
//    hold Montgomery(root^(k * n / 2^S)), k < 2^(S-1), so a pass reads consecutive
//    k with consecutive lanes (coalesced);
//  * then A[e] = Montgomery(root^e), e < 4096, and B[e] = Montgomery(root^(4096 e)),
//    e < max(n / 2^13, 1): a twiddle of a stage above s_cut is A[e & 4095] * B[e >> 12]
//    with e = k * n / 2^S -- one Montgomery product instead of streaming a table of
//    n/2 entries (512 MB at 2^25) that no cache holds.
// A and B are the caller's (A: 4096 entries, B: n/2^13 entries, Montgomery form).
__global__ void k_stage_twiddles(fe* __restrict__ out, const fe* __restrict__ A, const fe* __restrict__ B, int logn,
                                 int s_cut) {
  uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // < 2^s_cut - 1
  if (idx + 1 >= ((uint64_t)1 << s_cut)) return;
  int S = 63 - __builtin_clzll(idx + 1) + 1;  // idx in [2^(S-1) - 1, 2^S - 1)
  uint64_t k = idx + 1 - ((uint64_t)1 << (S - 1));
  uint64_t e = k << (logn - S);
  st_fe(out + idx, mont_mul(ld_fe(A + (e & 4095)), ld_fe(B + (e >> 12))));
}

// --------------------------------------------------- bit reversal (+ LDE scale)

// out[j] = x[rev(j)] (* offset^rev(j) when sA != nullptr), zero beyond n_in.
// skip > 0 (requires n_in <= n >> skip): the first `skip` DIT stages only see
// (a, 0) pairs, and a butterfly (a, 0) -> (a + 0*w, a - 0*w) = (a, a) exactly,
// so their output is x[rev(j & ~(2^skip - 1))] replicated; the caller starts
// the butterflies at stage skip + 1.
struct GatherArgs {
  fe* out[kMaxBatch];
  const fe* in[kMaxBatch];
  uint64_t in_ys, out_ys;  // != 0: strided rows, row blockIdx.y at in[0] + y * in_ys / out[0] + y * out_ys
  uint64_t in_es;          // element stride of an input row (1; R for R interleaved rows, in_ys = 1)
};

__global__ void k_bitrev_gather(GatherArgs ga, uint64_t n_in, int logn, const fe* __restrict__ sA,
                                const fe* __restrict__ sB, int skip) {
  fe* __restrict__ out = ga.out_ys ? ga.out[0] + (uint64_t)blockIdx.y * ga.out_ys : ga.out[blockIdx.y];
  const fe* __restrict__ in = ga.in_ys ? ga.in[0] + (uint64_t)blockIdx.y * ga.in_ys : ga.in[blockIdx.y];
  uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >> logn) return;
  uint64_t jj = (j >> skip) << skip;
  uint64_t i = logn ? (__builtin_bitreverse64(jj) >> (64 - logn)) : 0;
  fe v = fe_zero();
  if (i < n_in) {
    v = ld_fe(in + i * ga.in_es);
    if (sA) {
      fe f = mont_mul(ld_fe(sA + (i & 4095)), ld_fe(sB + (i >> 12)));  // Montgomery of offset^i
      v = mont_mul(v, f);
    }
  }
  st_fe(out + j, v);
}

// ------------------------------------------------------------- NTT passes

// An LDS slot of one element, 16-byte aligned so every tile access is one
// ds_read_b128 / ds_write_b128 (fe itself is 4-byte aligned: the compiler would
// split it into two ds_read2_b32, twice the LDS cycles and 4-way bank conflicts
// on the C = 16-column tiles that b128 banking serves conflict-free).
struct alignas(16) fe_lds {
  uint32_t w[4];
  __device__ __forceinline__ operator fe() const {
    const uint4 v = *reinterpret_cast<const uint4*>(w);
    fe r = {{v.x, v.y, v.z, v.w}};
    return r;
  }
  __device__ __forceinline__ fe_lds& operator=(const fe& a) {
    *reinterpret_cast<uint4*>(w) = make_uint4(a.w[0], a.w[1], a.w[2], a.w[3]);
    return *this;
  }
};

// transforms of >= 2^24 elements (>= 256 MiB, the MALL's size) stream their data with the
// non-temporal hint (2^25 fwd+inv 2.42 -> 2.35 ms; at 2^22 the plain access is faster)
constexpr int kStreamLogN = 24;

struct PassArgs {
  fe* data[kMaxBatch];  // one transform per blockIdx.y
  const fe* tw;        // stage-major twiddles (see ntt_stage_twiddles), Montgomery form
  const fe* post;      // optional Montgomery constant applied on store (INTT n^-1)
  int logn;
  int b0;              // index bits below the group bits (= first stage of the pass - 1)
  int L;               // stages in this pass (group bits [b0, b0+L))
  int logC;            // columns per tile (consecutive low-bit indices), C <= 2^b0
  int s_cut;           // stages above s_cut compute their twiddles from the A/B tables
  uint64_t ys;         // != 0: strided rows, transform blockIdx.y at data[0] + y * ys
  // four-step epilogue of a transform's last pass (ep_out != nullptr, strided rows): output k of
  // row r = ep_row0 + blockIdx.y is multiplied by w^((ep_j0 + r) k) and stored to the all-to-all
  // send buffer [k >> ep_logR][r][k & (2^ep_logR - 1)] instead of back in place
  fe* ep_out;
  const fe* ep_T0;
  const fe* ep_T1;
  const fe* ep_T2;
  uint64_t ep_row0, ep_j0, ep_rows;
  int ep_logR;
  // batched four-step (ep_k vectors, 2^ep_vlog rows each, one exchange): row r is row r & (2^ep_vlog
  // - 1) of vector r >> ep_vlog, stored at [k >> ep_logR][row][vector][k & (2^ep_logR - 1)];
  // ep_k = 1, ep_vlog = 63 for one vector
  int ep_vlog;
  uint64_t ep_k;
};

// the four-step epilogue's store of output k of (batched) row r: times w^((ep_j0 + row) k), to the
// all-to-all send buffer (PassArgs / FirstArgs)
template <class Args>
__device__ __forceinline__ void ep_store(const Args& a, uint64_t r, uint64_t k, const fe& v) {
  const uint64_t rl = r & ((1ull << a.ep_vlog) - 1), vv = r >> a.ep_vlog;
  const uint64_t e = (a.ep_j0 + rl) * k;  // < 2^36 (host-checked)
  const fe w = mont_mul(mont_mul(ld_fe(a.ep_T0 + (e & 4095)), ld_fe(a.ep_T1 + ((e >> 12) & 4095))),
                        ld_fe(a.ep_T2 + (e >> 24)));
  const uint64_t R = (uint64_t)1 << a.ep_logR;
  st_fe(a.ep_out + (((k >> a.ep_logR) * a.ep_rows + rl) * a.ep_k + vv) * R + (k & (R - 1)), mont_mul(v, w));
}

// store of a transform's element k (row pointer `row`) at the end of a pass
__device__ __forceinline__ void pass_store(const PassArgs& a, fe* row, uint64_t k, fe v, bool post, bool last,
                                           const fe& pc) {
  if (last && a.ep_out) {
    ep_store(a, a.ep_row0 + blockIdx.y, k, v);
    return;
  }
  if (post) v = mont_mul(v, pc);
  else if (last) v = fe_canon(v);
  st_fe_stream(row + k, v, a.logn >= kStreamLogN);
}

// twiddle of global stage S (1-based) for index k < 2^(S-1): Montgomery(root^(k n / 2^S)),
// from the stage-major table (S <= s_cut) or as A[e & 4095] * B[e >> 12], e = k n / 2^S
__device__ __forceinline__ fe twiddle_tab(const PassArgs& a, int S, uint64_t k) {
  return ld_fe(a.tw + (((uint64_t)1 << (S - 1)) - 1) + k);
}
__device__ __forceinline__ fe twiddle_comp(const PassArgs& a, int S, uint64_t k) {
  const fe* tA = a.tw + (((uint64_t)1 << a.s_cut) - 1);
  const uint64_t e = k << (a.logn - S);
  return mont_mul(ld_fe(tA + (e & 4095)), ld_fe(tA + 4096 + (e >> 12)));
}

// One radix-2 butterfly of the reference's DIT graph (fft/ntt.rs:26-46): o = x * w (Montgomery,
// w a Montgomery twiddle), e <- e + o, x <- e - o, lazily reduced (fe128.hpp).
__device__ __forceinline__ void butterfly(fe& e, fe& x, const fe& w) {
  fe o = mont_mul(x, w);
  fe ev = e;
  e = fe_add_lazy(ev, o);
  x = fe_sub_lazy(ev, o);
}
// twiddle 1: o = x (canonical), e <- e + x, x <- e - x
__device__ __forceinline__ void butterfly_unit(fe& e, fe& x) {
  fe ev = e;
  e = fe_add_lazy(ev, x);
  x = fe_sub_lazy(ev, x);
}

// R radix-2 stages (tile-local stages t+1 .. t+R) on the 2^R elements of one group held
// in registers: x[m] is tile row g0 + m * 2^t with g_low = g0 mod 2^t; `low` = the index
// bits below b0 (cb*C + c; 0 when the columns are independent transforms).
// COMP: every twiddle of the step computed from A/B (the step reaches above s_cut), else
// every twiddle from the table -- one uniform choice per step, so the step's twiddle loads
// stay branch-free and are issued together.
#ifndef SG_NTT_STAGE_TW
#define SG_NTT_STAGE_TW 0
#endif
template <int R, bool COMP>
__device__ __forceinline__ void radix_regs_impl(fe* x, const PassArgs& a, int t, uint32_t g_low, uint64_t low) {
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int S = a.b0 + t + u + 1;  // global stage, 1-based
#if SG_NTT_STAGE_TW
    // one stage's twiddles live at a time (2^(R-1) x 4 VGPRs instead of R 2^(R-1) x 4): the
    // scheduling barrier keeps the compiler from hoisting the next stage's loads above this one
    fe w[1 << (R - 1)];
#pragma unroll
    for (int m = 0, j = 0; m < (1 << R); ++m) {
      if (m & (1 << u)) continue;
      uint64_t gmod = (uint64_t)g_low + ((uint64_t)(m & ((1 << u) - 1)) << t);
      uint64_t k = (gmod << a.b0) + low;
      w[j++] = COMP ? twiddle_comp(a, S, k) : twiddle_tab(a, S, k);
    }
#pragma unroll
    for (int m = 0, j = 0; m < (1 << R); ++m) {
      if (m & (1 << u)) continue;
      fe o = mont_mul(x[m + (1 << u)], w[j++]);
      fe ev = x[m];
      x[m] = fe_add_lazy(ev, o);
      x[m + (1 << u)] = fe_sub_lazy(ev, o);
#if SG_NTT_STAGE_TW == 2
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
    __builtin_amdgcn_sched_barrier(0);
#else
#pragma unroll
    for (int m = 0; m < (1 << R); ++m) {
      if (m & (1 << u)) continue;
      uint64_t gmod = (uint64_t)g_low + ((uint64_t)(m & ((1 << u) - 1)) << t);
      uint64_t k = (gmod << a.b0) + low;
      fe w = COMP ? twiddle_comp(a, S, k) : twiddle_tab(a, S, k);
      butterfly(x[m], x[m + (1 << u)], w);  // tile values stay in [0, 2^128) until the last store
    }
#endif
  }
}

// The first radix-8 step of a whole transform (stages 1..3: t = 0, b0 = 0, no column bits):
// k = m mod 2^u is known at compile time, and 7 of its 12 twiddles are root^0 = 1.  A product
// by Montgomery(1) is the canonical residue, so those butterflies take fe_canon(x) (stage 1:
// x itself -- the gathered inputs are canonical) instead of a Montgomery product: same values.
__device__ __forceinline__ void radix8_first(fe* x, const PassArgs& a) {
#pragma unroll
  for (int u = 0; u < 3; ++u) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if (m & (1 << u)) continue;
      const int k = m & ((1 << u) - 1);
      if (k == 0) {
        if (u != 0) x[m + (1 << u)] = fe_canon(x[m + (1 << u)]);
        butterfly_unit(x[m], x[m + (1 << u)]);
      } else {
        butterfly(x[m], x[m + (1 << u)], twiddle_tab(a, u + 1, (uint64_t)k));
      }
    }
  }
}

// MAYCOMP = false: the caller's stages never exceed s_cut (the first pass: <= 9 < 12 <= s_cut)
template <int R, bool MAYCOMP = true>
__device__ __forceinline__ void radix_regs(fe* x, const PassArgs& a, int t, uint32_t g_low, uint64_t low) {
  if (!MAYCOMP || a.b0 + t + R <= a.s_cut) radix_regs_impl<R, false>(x, a, t, g_low, low);
  else radix_regs_impl<R, true>(x, a, t, g_low, low);
}

// COLK: the tile's columns are consecutive low index bits (they enter the twiddle
// index k); false when the columns are independent transforms' tiles (first pass).
template <int R, bool COLK = true>
__device__ __forceinline__ void radix_step(fe_lds* lds, const PassArgs& a, int t, uint64_t lowbase) {
  const int logC = a.logC;
  const uint32_t C = 1u << logC;
  const uint32_t groups = (1u << (a.L + logC)) >> R;
  for (uint32_t q = threadIdx.x; q < groups; q += blockDim.x) {
    uint32_t c = q & (C - 1);
    uint32_t qq = q >> logC;
    uint32_t g_low = qq & ((1u << t) - 1);
    uint32_t g_high = qq >> t;
    uint32_t g0 = (g_high << (t + R)) | g_low;
    fe x[1 << R];
#pragma unroll
    for (int m = 0; m < (1 << R); ++m) x[m] = lds[((g0 + ((uint32_t)m << t)) << logC) + c];
    radix_regs<R, COLK>(x, a, t, g_low, COLK ? lowbase + c : 0);
#pragma unroll
    for (int m = 0; m < (1 << R); ++m) lds[((g0 + ((uint32_t)m << t)) << logC) + c] = x[m];
  }
  __syncthreads();
}

// One pass: load a 2^L x C tile into LDS, run L radix-2 stages as radix-8/4/2
// register steps, store.  TL > 0: the tile is exactly 2^TL elements handled
// by 256 threads, so the loads/stores are unrolled (all 2^TL/256 global loads
// of a thread in flight at once); TL == 0: generic loop for small transforms.
template <int TL>
__global__ __launch_bounds__(256) void k_ntt_pass(PassArgs a) {
  extern __shared__ fe_lds lds[];
  const int logC = a.logC;
  const uint32_t C = 1u << logC;
  const uint32_t tile = 1u << (a.L + logC);
  // tile id -> (h, cb)
  const uint64_t ncb = (uint64_t)1 << (a.b0 - logC);
  const uint64_t h = blockIdx.x / ncb;
  const uint64_t cb = blockIdx.x % ncb;
  const uint64_t base = (h << (a.b0 + a.L)) + cb * C;
  fe* __restrict__ data = a.ys ? a.data[0] + (uint64_t)blockIdx.y * a.ys : a.data[blockIdx.y];
  if constexpr (TL > 0) {
    constexpr int PER = (1 << TL) / 256;
    fe v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      uint32_t l = threadIdx.x + 256u * k;
      uint32_t g = l >> logC, c = l & (C - 1);
      v[k] = ld_fe(data + base + ((uint64_t)g << a.b0) + c);
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) lds[threadIdx.x + 256u * k] = v[k];
  } else {
    for (uint32_t l = threadIdx.x; l < tile; l += blockDim.x) {
      uint32_t g = l >> logC, c = l & (C - 1);
      lds[l] = ld_fe(data + base + ((uint64_t)g << a.b0) + c);
    }
  }
  __syncthreads();
  int t = 0;
  while (t < a.L) {
    int rem = a.L - t;
    if (rem >= 3) { radix_step<3>(lds, a, t, cb * C); t += 3; }
    else if (rem == 2) { radix_step<2>(lds, a, t, cb * C); t += 2; }
    else { radix_step<1>(lds, a, t, cb * C); t += 1; }
  }
  const bool post = a.post != nullptr;
  const bool last = a.b0 + a.L == a.logn;  // the transform's last pass stores canonical values
  fe pc = post ? ld_fe(a.post) : fe_zero();
  if constexpr (TL > 0) {
    constexpr int PER = (1 << TL) / 256;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      uint32_t l = threadIdx.x + 256u * k;
      uint32_t g = l >> logC, c = l & (C - 1);
      pass_store(a, data, base + ((uint64_t)g << a.b0) + c, lds[l], post, last, pc);
    }
  } else {
    for (uint32_t l = threadIdx.x; l < tile; l += blockDim.x) {
      uint32_t g = l >> logC, c = l & (C - 1);
      pass_store(a, data, base + ((uint64_t)g << a.b0) + c, lds[l], post, last, pc);
    }
  }
}

// A 2048-element pass (256 threads, L >= 6 stages) whose first and last radix-8 steps
// run straight out of / into HBM: each thread loads the 8 rows of its first-step group
// (rows 8 qq + m of column c), and stores the 8 rows of its last-step group (rows
// qq + m 2^(L-3)).  Only the middle stages go through LDS: one LDS write + one read per
// element plus a round trip per middle step, and L/3 barriers fewer than k_ntt_pass.
template <int TL>
__global__ __launch_bounds__(1 << (TL - 3), SG_NTT_WPE) void k_ntt_pass_rr(PassArgs a) {
  static_assert(TL >= 10 && TL <= 13, "2^TL-element tiles, 2^(TL-3) threads");
  extern __shared__ fe_lds lds[];
  const int logC = a.logC, L = a.L;
  const uint32_t C = 1u << logC;
  const uint64_t ncb = (uint64_t)1 << (a.b0 - logC);
  const uint64_t h = blockIdx.x / ncb;
  const uint64_t cb = blockIdx.x % ncb;
  const uint64_t base = (h << (a.b0 + L)) + cb * C;
  fe* __restrict__ data = a.ys ? a.data[0] + (uint64_t)blockIdx.y * a.ys : a.data[blockIdx.y];
  const uint32_t c = threadIdx.x & (C - 1), qq = threadIdx.x >> logC;  // qq < 2^(L-3)
  const uint64_t low = cb * C + c;
  fe x[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) x[m] = ld_fe_stream(data + base + ((uint64_t)(8 * qq + m) << a.b0) + c, a.logn >= kStreamLogN);
  radix_regs<3>(x, a, 0, 0, low);
#pragma unroll
  for (int m = 0; m < 8; ++m) lds[((8 * qq + m) << logC) + c] = x[m];
  __syncthreads();
  int t = 3;
  while (t < L - 3) {
    int rem = L - 3 - t;
    if (rem >= 3) { radix_step<3>(lds, a, t, cb * C); t += 3; }
    else if (rem == 2) { radix_step<2>(lds, a, t, cb * C); t += 2; }
    else { radix_step<1>(lds, a, t, cb * C); t += 1; }
  }
  const int tl = L - 3;
#pragma unroll
  for (int m = 0; m < 8; ++m) x[m] = lds[((qq + ((uint32_t)m << tl)) << logC) + c];
  radix_regs<3>(x, a, tl, qq, low);
  const bool post = a.post != nullptr;
  const bool last = a.b0 + L == a.logn;  // the transform's last pass stores canonical values
  const fe pc = post ? ld_fe(a.post) : fe_zero();
#pragma unroll
  for (int m = 0; m < 8; ++m)
    pass_store(a, data, base + ((uint64_t)(qq + ((uint32_t)m << tl)) << a.b0) + c, x[m], post, last, pc);
}

// First pass with the bit-reversal fused in (fft/ntt.rs:14 bit_reverse_copy).
// Positions j = h*2^L + t of the bit-reversed array hold x[rev_m(j)] =
// x[rev_{m-L}(h) + rev_L(t) * 2^(m-L)], so the C = 2^logC tiles whose
// c = rev_{m-L}(h) are consecutive read C-element runs of x per row u = rev_L(t).
// Rows past n_in are zero; with skip leading trivial stages (n_in <= n >> skip)
// only rows u < 2^(L-skip) can be non-zero and each lands replicated on 2^skip
// positions (a butterfly (a, 0) is (a, a) exactly).  Optional LDE scale by
// offset^index (Montgomery tables sA/sB).  Stages skip+1..L then run in LDS and
// every tile is written back as one contiguous 2^L run.
struct FirstArgs {
  fe* out[kMaxBatch];
  const fe* in[kMaxBatch];
  const fe* tw;
  const fe* sA;
  const fe* sB;
  uint64_t n_in;
  int logn;
  int L;
  int logC;
  int skip;
  int s_cut;
  uint64_t in_ys, out_ys;  // != 0: strided rows (see GatherArgs)
  // != 0: the rows are interleaved, row y's element i at in[0] + i * in_il + y; the tile's C
  // columns are then C consecutive rows at one bit-reversed position h (64-byte runs across rows)
  // instead of C positions of one row -- the butterflies are the same (columns are independent)
  uint64_t in_il;
  // k_ntt_first<11, WHOLE = true>: the pass runs all logn = L stages of small transforms, the
  // tile's C columns being C whole rows (rows blockIdx.y C + k), and stores the final values:
  // times *post (INTT n^-1, POST), or canonical, or through the four-step epilogue (EP, as
  // pass_store) -- the bit-reversal gather and the generic all-LDS pass of a small transform in
  // one launch
  const fe* post;
  fe* ep_out;
  const fe* ep_T0;
  const fe* ep_T1;
  const fe* ep_T2;
  uint64_t ep_row0, ep_j0, ep_rows;
  int ep_logR;
  int ep_vlog;  // as PassArgs
  uint64_t ep_k;
};

// WHOLE variants: EP = the four-step epilogue store, POST = times *post (INTT n^-1), else canonical
template <int TL, bool WHOLE = false, bool EP = false, bool POST = false>
__global__ __launch_bounds__(1 << (TL - 3), TL == 11 ? SG_NTT_WPE : 1) void k_ntt_first(FirstArgs a) {
  extern __shared__ fe_lds lds[];
  const int L = a.L, logC = a.logC, m = a.logn;
  const uint32_t C = 1u << logC;
  const int skip = a.skip < L ? a.skip : L;
  // XCD-aware: workgroups are dealt round-robin to the 8 XCDs, so give each XCD
  // a contiguous range of column groups; neighbouring C-runs then share its L2
  uint32_t bx = blockIdx.x;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  const bool il = a.in_il != 0;
  const bool rowcols = il || WHOLE;  // the tile's columns are rows (interleaved, or whole transforms)
  // column k of the tile: position h = hcol(k) of row ycol(k)
  const uint64_t c0 = rowcols ? (uint64_t)bx : (uint64_t)bx << logC;
  const uint64_t y0 = rowcols ? (uint64_t)blockIdx.y << logC : (uint64_t)blockIdx.y;
  auto hcol = [&](uint64_t k) { return rowcols ? c0 : c0 + k; };
  auto ycol = [&](uint64_t k) { return rowcols ? y0 + k : y0; };
  // element idx of column k's row
  // (WHOLE launches have strided rows: ntt_small_whole requires them)
  auto in_at = [&](uint64_t k, uint64_t idx) -> const fe* {
    if (il) return a.in[0] + idx * a.in_il + ycol(k);
    if constexpr (WHOLE) return a.in[0] + ycol(k) * a.in_ys + idx;
    return (a.in_ys ? a.in[0] + ycol(k) * a.in_ys : a.in[ycol(k)]) + idx;
  };
  auto out_row = [&](uint64_t k) -> fe* {
    const uint64_t y = ycol(k);
    if constexpr (WHOLE) return a.out[0] + y * a.out_ys;
    return a.out_ys ? a.out[0] + y * a.out_ys : a.out[y];
  };
  PassArgs pa;
  pa.tw = a.tw;
  pa.post = nullptr;
  pa.logn = m;
  pa.b0 = 0;
  pa.L = L;
  pa.logC = logC;
  pa.s_cut = a.s_cut;
  pa.ep_out = nullptr;
  // one radix-8 group per thread in the first and last steps (column c, group qq)
  const bool regs = L >= 6 && ((1u << (L - 3)) << logC) == blockDim.x;
  int t = skip;
  if (regs && skip == 0) {
    // first radix-8 step straight from HBM: tile row 8 qq + j holds x[rev_L(8 qq + j)]
    const uint32_t c = threadIdx.x & (C - 1), qq = threadIdx.x >> logC;
    fe x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t u = __builtin_bitreverse32(8 * qq + j) >> (32 - L);
      const uint64_t idx = hcol(c) + ((uint64_t)u << (m - L));
      x[j] = fe_zero();
      if (idx < a.n_in) {
        x[j] = ld_fe_stream(in_at(c, idx), m >= kStreamLogN);
        if (a.sA) x[j] = mont_mul(x[j], mont_mul(ld_fe(a.sA + (idx & 4095)), ld_fe(a.sB + (idx >> 12))));
      }
    }
    radix8_first(x, pa);
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[((8 * qq + j) << logC) + c] = x[j];
    t = 3;
  } else {
    const uint32_t rows = 1u << (L - skip);
    const uint32_t rep = 1u << skip;
    for (uint32_t l = threadIdx.x; l < rows * C; l += blockDim.x) {
      const uint32_t k = l & (C - 1), u = l >> logC;
      const uint64_t idx = hcol(k) + ((uint64_t)u << (m - L));
      fe v = fe_zero();
      if (idx < a.n_in) {
        v = ld_fe(in_at(k, idx));
        if (a.sA) v = mont_mul(v, mont_mul(ld_fe(a.sA + (idx & 4095)), ld_fe(a.sB + (idx >> 12))));
      }
      const uint32_t tr = __builtin_bitreverse32(u) >> (32 - L);
      for (uint32_t r = 0; r < rep; ++r) lds[((tr + r) << logC) + k] = v;
    }
  }
  __syncthreads();
  if (regs && L - t >= 3) {
    // remainder step first, radix-8 steps, and the last radix-8 step (rows qq + m 2^(L-3)
    // of column c) straight from registers to HBM: out[(h << L) + row]
    const int r0 = (L - t) % 3;
    if (r0 == 2) { radix_step<2, false>(lds, pa, t, 0); t += 2; }
    else if (r0 == 1) { radix_step<1, false>(lds, pa, t, 0); t += 1; }
    while (t < L - 3) { radix_step<3, false>(lds, pa, t, 0); t += 3; }
    const uint32_t c = threadIdx.x & (C - 1), qq = threadIdx.x >> logC;
    const int tl = L - 3;
    fe x[8];
#pragma unroll
    for (int mm = 0; mm < 8; ++mm) x[mm] = lds[((qq + ((uint32_t)mm << tl)) << logC) + c];
    radix_regs<3, false>(x, pa, tl, qq, 0);
    fe* const orow = out_row(c);
    if constexpr (WHOLE) {
      // the transform's final values (m == L): element k = qq + mm 2^tl of row ycol(c)
      const fe pc = POST ? ld_fe(a.post) : fe_zero();
#pragma unroll
      for (int mm = 0; mm < 8; ++mm) {
        const uint64_t k = qq + ((uint32_t)mm << tl);
        if constexpr (EP) {
          ep_store(a, a.ep_row0 + ycol(c), k, x[mm]);
        } else {
          st_fe(orow + k, POST ? mont_mul(x[mm], pc) : fe_canon(x[mm]));
        }
      }
      return;
    }
    const uint64_t h = __builtin_bitreverse64(hcol(c)) >> (64 - (m - L));
#pragma unroll
    for (int mm = 0; mm < 8; ++mm) st_fe_stream(orow + (h << L) + qq + ((uint32_t)mm << tl), x[mm], m >= kStreamLogN);
    return;
  }
  while (t < L) {
    int rem = L - t;
    if (rem >= 3) { radix_step<3, false>(lds, pa, t, 0); t += 3; }
    else if (rem == 2) { radix_step<2, false>(lds, pa, t, 0); t += 2; }
    else { radix_step<1, false>(lds, pa, t, 0); t += 1; }
  }
  const uint32_t tile = 1u << (L + logC);
  for (uint32_t l = threadIdx.x; l < tile; l += blockDim.x) {
    const uint32_t tt = l & ((1u << L) - 1), k = l >> L;
    // (whole transforms take the register path above: the host launches them with L - skip >= 3)
    const uint64_t h = m > L ? __builtin_bitreverse64(hcol(k)) >> (64 - (m - L)) : 0;
    st_fe(out_row(k) + (h << L) + tt, lds[(tt << logC) + k]);
  }
}

// elementwise v *= Montgomery constant (used for tiny INTTs)
__global__ void k_scale_const(fe* __restrict__ data, uint64_t n, const fe* __restrict__ cst) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_fe(data + i, mont_mul(ld_fe(data + i), ld_fe(cst)));
}

// ------------------------------------------------------------- Merkle

// ---------------------------------------------- row-sharded helpers (four-step)
//
// Multi-GPU transforms work on 2-D shards: rows x cols of field
// elements, row-major.  These kernels are the local steps around the all-to-all.

// data[r][c] *= base^e, e = (a0 + a1*r)*c + b0 + b1*r < 2^36, via three 4096-entry
// Montgomery power tables (T0: base^i, T1: base^(i<<12), T2: base^(i<<24)).
// Twiddles of the four-step (omega^(j1*k2)) and the coset scale (offset^j) are
// both of this form.
// (nb arrays of rows x cols back to back, each scaled alike)
struct MulPowArgs {
  fe* data;
  uint64_t rows, cols;
  uint64_t a0, a1, b0, b1;
  const fe* T0;
  const fe* T1;
  const fe* T2;
  uint64_t nb;
};

__global__ __launch_bounds__(256) void k_mul_pow(MulPowArgs a) {
  const uint64_t total = a.rows * a.cols * a.nb;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; l < total; l += stride) {
    const uint64_t rr = l / a.cols, c = l - rr * a.cols, r = a.nb > 1 ? rr % a.rows : rr;
    const uint64_t e = (a.a0 + a.a1 * r) * c + a.b0 + a.b1 * r;
    fe w = mont_mul(ld_fe(a.T0 + (e & 4095)), ld_fe(a.T1 + ((e >> 12) & 4095)));
    w = mont_mul(w, ld_fe(a.T2 + (e >> 24)));
    st_fe(a.data + l, mont_mul(ld_fe(a.data + l), w));
  }
}

// out[b][a][c] = in[a][b][c] for an A x B x C array (swap the two outer axes).
// C >= 16: every (a, b) run of C elements is a coalesced copy.  C < 16: 32 x 32
// tiles of (a, b) through LDS so both the reads and the writes are coalesced.
// nb arrays back to back (array v at v A B C in both)
__global__ __launch_bounds__(256) void k_swap01_runs(const fe* __restrict__ in, fe* __restrict__ out, uint64_t A,
                                                     uint64_t B, uint64_t C, uint64_t nb) {
  const uint64_t one = A * B * C, total = one * nb;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; l < total; l += stride) {
    const uint64_t c = l % C, ab = l / C;
    const uint64_t b = ab % B, vaa = ab / B;  // l = (((v A + aa) B) + b) C + c
    const uint64_t v = nb > 1 ? vaa / A : 0, aa = vaa - v * A;
    st_fe(out + v * one + (b * A + aa) * C + c, ld_fe(in + l));
  }
}

__global__ __launch_bounds__(256) void k_swap01_tiled(const fe* __restrict__ in, fe* __restrict__ out, uint64_t A,
                                                      uint64_t B, uint64_t C) {
  __shared__ fe tile[32][33];
  // blockIdx.x: tile over b (32 wide), blockIdx.y: tile over a, blockIdx.z: c + C v (array v)
  const uint64_t b0 = (uint64_t)blockIdx.x * 32, a0 = (uint64_t)blockIdx.y * 32, c = blockIdx.z % C;
  const uint64_t vo = (blockIdx.z / C) * A * B * C;
  in += vo;
  out += vo;
  const uint32_t tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (uint32_t k = ty; k < 32; k += 8) {
    const uint64_t aa = a0 + k, b = b0 + tx;
    if (aa < A && b < B) tile[k][tx] = ld_fe(in + (aa * B + b) * C + c);
  }
  __syncthreads();
  for (uint32_t k = ty; k < 32; k += 8) {
    const uint64_t b = b0 + k, aa = a0 + tx;
    if (aa < A && b < B) st_fe(out + (b * A + aa) * C + c, tile[tx][k]);
  }
}

// FRI fold of a run-sharded codeword (fri.rs:151-159).  Local element l is
// global index i(l) = (l / run) * run_stride + run_off + l % run; its partner
// i + n/2 is local l + half (the caller checks the layout guarantees it).
struct FoldRunsArgs {
  fe* out;
  const fe* in;
  uint64_t half;       // local outputs
  uint64_t run, run_stride, run_off;
  const fe* T0;        // Montgomery(w_r^-e): e & 4095, (e >> 12) & 4095, e >> 24
  const fe* T1;
  const fe* T2;
  fe K;                // Montgomery(alpha * offset_r^-1 * 2^-1)
};

__global__ __launch_bounds__(256) void k_fri_fold_runs(FoldRunsArgs a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; l < a.half; l += stride) {
    const uint64_t q = l / a.run;
    const uint64_t e = q * a.run_stride + a.run_off + (l - q * a.run);
    fe t = mont_mul(a.K, ld_fe(a.T0 + (e & 4095)));
    t = mont_mul(t, ld_fe(a.T1 + ((e >> 12) & 4095)));
    t = mont_mul(t, ld_fe(a.T2 + (e >> 24)));
    const fe x = ld_fe(a.in + l);
    const fe y = ld_fe(a.in + l + a.half);
    st_fe(a.out + l, fe_add(fe_halve(fe_add(x, y)), mont_mul(fe_sub(x, y), t)));
  }
}

// FRI round gate (fri_commit_dev): a round's fold + tree are queued before its challenge exists;
// this one-lane kernel holds the stream until the host has written K (Montgomery, pinned) and
// raised the gate word to `want`, then copies K into device memory for the fold kernel.  The
// wait is bounded (`ticks` of the 100 MHz wall clock): on expiry it raises the timeout word and
// returns, the host reports it as an error.
__global__ void k_fri_gate(const uint64_t* gate, uint64_t want, const uint64_t* Kh, fe* Kd, uint32_t* timeout,
                           uint64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_fetch_or(timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  const uint64_t lo = __hip_atomic_load(Kh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t hi = __hip_atomic_load(Kh + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  fe k;
  k.w[0] = (uint32_t)lo;
  k.w[1] = (uint32_t)(lo >> 32);
  k.w[2] = (uint32_t)hi;
  k.w[3] = (uint32_t)(hi >> 32);
  st_fe(Kd, k);
}

hipError_t launch_fri_gate(const uint64_t* gate, uint64_t want, const uint64_t* Kh, fe* Kd, uint32_t* timeout,
                           double seconds, hipStream_t s) {
  const uint64_t ticks = (uint64_t)(seconds * 1e8);  // wall_clock64 counts at 100 MHz
  hipLaunchKernelGGL(k_fri_gate, dim3(1), dim3(64), 0, s, gate, want, Kh, Kd, timeout, ticks);
  return hipGetLastError();
}

// roots of `count` strided trees (root digest at tree + y * tree_ys + root_off) -> contiguous
__global__ void k_gather_roots(const uint64_t* __restrict__ tree, uint64_t tree_ys, uint64_t root_off,
                               uint64_t* __restrict__ out, uint64_t count) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  uint64_t d[8];
  ld_digest(tree + i * tree_ys + root_off, d);
  st_digest(out + i * 8, d);
}

// ------------------------------------------------------------- gathers (openings)

__global__ void k_gather_digests(const uint64_t* __restrict__ tree, const uint64_t* __restrict__ idx,
                                 uint64_t* __restrict__ out, uint32_t count) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  uint64_t d[8];
  ld_digest(tree + idx[i] * 8, d);
  st_digest(out + (uint64_t)i * 8, d);
}

// column shard of a replicated coefficient vector: out[r][j] = in[base + r + n1 j] (0 past len)
// (nb vectors: vector v from in + v in_stride into out + v rows row_len)
__global__ void k_gather_cols(fe* __restrict__ out, const fe* __restrict__ in, uint64_t len, uint64_t rows,
                              uint64_t row_len, uint64_t n1, uint64_t base, uint64_t nb, uint64_t in_stride) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t one = rows * row_len;
  if (t >= one * nb) return;
  const uint64_t v = nb > 1 ? t / one : 0, tl = t - v * one;
  const uint64_t r = tl / row_len, j = tl % row_len, src = base + r + n1 * j;
  st_fe(out + t, src < len ? ld_fe(in + v * in_stride + src) : fe_zero());
}

__global__ void k_gather_fe(const fe* __restrict__ src, const uint64_t* __restrict__ idx, fe* __restrict__ out,
                            uint32_t count) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  st_fe(out + i, ld_fe(src + idx[i]));
}

// DIGEST: an address with bit 0 set names a digest a lean tree did not store: bits 1-2 are its
// level lv (0..2), the address (16-byte aligned) the first value of its 2^lv-leaf block, and the
// digest is rehashed -- the leaf (merkle_root.rs:25-30) or the block's subtree root
// (blake2b(left || right) upwards, merkle_root.rs:7-19)
__device__ __forceinline__ void subtree_rehash(const fe* lp, int lv, uint64_t d[8]) {
  if (lv == 0) {
    leaf_hash(ld_fe(lp), d);
    return;
  }
  uint64_t a[8], b[8], n0[8];
  const int pairs = 1 << (lv - 1);  // lv 1: one node over 2 leaves; lv 2: two nodes, then the root
  for (int k = 0; k < pairs; ++k) {
    leaf_hash(ld_fe(lp + 2 * k), a);
    leaf_hash(ld_fe(lp + 2 * k + 1), b);
    if (k == 0) blake2b_node(a, b, n0);
    else blake2b_node(a, b, d);
  }
  if (lv == 1) {
#pragma unroll
    for (int w = 0; w < 8; ++w) d[w] = n0[w];
  } else {
#pragma unroll
    for (int w = 0; w < 8; ++w) b[w] = d[w];
    blake2b_node(n0, b, d);
  }
}

template <bool DIGEST>
__global__ void k_gather_abs(const uint64_t* __restrict__ addr, void* __restrict__ out, uint32_t count) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  if constexpr (DIGEST) {
    uint64_t d[8];
    const uint64_t ad = addr[i];
    if (ad & 1) subtree_rehash(reinterpret_cast<const fe*>(ad & ~15ull), (int)((ad >> 1) & 3), d);
    else ld_digest(reinterpret_cast<const uint64_t*>(ad), d);
    st_digest(static_cast<uint64_t*>(out) + (uint64_t)i * 8, d);
  } else {
    st_fe(static_cast<fe*>(out) + i, ld_fe(reinterpret_cast<const fe*>(addr[i])));
  }
}


// HBM copy probe (measurement only): one 16-byte element per lane, non-temporal loads and stores
// (streamed data: no cache keeps it).  tools/microbench_copy.hip measured this flat form fastest
// (6.6 TB/s read + write over 2 GiB; grid-stride and chunked forms 4.7-5.6 TB/s).
__global__ void __launch_bounds__(256) k_copy16(const sg_u32x4* __restrict__ src, sg_u32x4* __restrict__ dst,
                                                uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// grid-stride form (the probe's comparison point: a fixed grid of `blocks`)
__global__ void __launch_bounds__(256) k_copy16_stride(const sg_u32x4* __restrict__ src, sg_u32x4* __restrict__ dst,
                                                       uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// gather from a list of absolute device addresses (one launch for every round's openings)
// ------------------------------------------------------------- launchers


hipError_t launch_gather_digests(const uint64_t* tree, const uint64_t* idx, uint64_t* out, uint32_t count,
                                 hipStream_t s) {
  if (!count) return hipSuccess;
  ProfScope ps("gather_digests", 128ull * count, s);
  hipLaunchKernelGGL(k_gather_digests, dim3((count + 255) / 256), dim3(256), 0, s, tree, idx, out, count);
  return hipGetLastError();
}


hipError_t launch_gather_abs(const uint64_t* addr, void* out, uint32_t count, bool digest, hipStream_t s) {
  if (!count) return hipSuccess;
  ProfScope ps(digest ? "gather_digests" : "gather_fe", (digest ? 72ull : 24ull) * count, s);
  if (digest)
    hipLaunchKernelGGL(k_gather_abs<true>, dim3((count + 255) / 256), dim3(256), 0, s, addr, out, count);
  else
    hipLaunchKernelGGL(k_gather_abs<false>, dim3((count + 255) / 256), dim3(256), 0, s, addr, out, count);
  return hipGetLastError();
}

hipError_t launch_gather_cols(fe* out, const fe* in, uint64_t len, uint64_t rows, uint64_t row_len, uint64_t n1,
                              uint64_t base, hipStream_t s, uint64_t nb, uint64_t in_stride) {
  const uint64_t total = rows * row_len * nb;
  if (!total) return hipSuccess;
  if ((total + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  ProfScope ps("gather_cols", 32 * total, s);
  hipLaunchKernelGGL(k_gather_cols, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, out, in, len, rows, row_len,
                     n1, base, nb, in_stride);
  return hipGetLastError();
}

hipError_t launch_gather_fe(const fe* src, const uint64_t* idx, fe* out, uint32_t count, hipStream_t s) {
  if (!count) return hipSuccess;
  ProfScope ps("gather_fe", 32ull * count, s);
  hipLaunchKernelGGL(k_gather_fe, dim3((count + 255) / 256), dim3(256), 0, s, src, idx, out, count);
  return hipGetLastError();
}

static inline unsigned nblocks(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }


hipError_t launch_copy16(const void* src, void* dst, uint64_t bytes, unsigned blocks, hipStream_t s) {
  if (bytes < 16) return hipSuccess;
  const uint64_t n = bytes / 16;
  ProfScope ps("copy16", 2 * bytes, s);
  if (blocks == 0) {
    if ((n + 255) / 256 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_copy16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       static_cast<const sg_u32x4*>(src), static_cast<sg_u32x4*>(dst), n);
  } else {
    hipLaunchKernelGGL(k_copy16_stride, dim3(blocks), dim3(256), 0, s, static_cast<const sg_u32x4*>(src),
                       static_cast<sg_u32x4*>(dst), n);
  }
  return hipGetLastError();
}

hipError_t launch_pow_table(fe* tw, const fe* A, const fe* B, uint64_t count, hipStream_t s) {
  if (count == 0) return hipSuccess;
  ProfScope ps("pow_table", 16 * count, s);
  hipLaunchKernelGGL(k_pow_table, dim3(nblocks(count, 256)), dim3(256), 0, s, tw, A, B, count);
  return hipGetLastError();
}

int ntt_tw_cut(int logn) {
  // the top SG_NTT_TWTOP (default 3) stages of a transform of >= 2^15 points compute their
  // twiddles: A/B on MI355X (tools/ab_ntt_tw.sh) -- at 2^22 and 2^25 the top three stages'
  // n/2 + n/4 + n/8 table entries cost more HBM time than one Montgomery product per twiddle,
  // deeper cuts trade too much VALU.  SG_NTT_TWCUT forces an absolute cut (experiments).
  static const int top = SG_KNOB(NTT_TWTOP, 3);
  static const int forced = SG_KNOB(NTT_TWCUT, 0);
  int c = forced > 0 ? forced : (logn >= 15 ? logn - top : logn);
  if (c < 12) c = 12;
  return logn < c ? logn : c;
}

uint64_t ntt_tw_entries(int logn) {
  const int c = ntt_tw_cut(logn);
  if (c == logn) return logn ? ((uint64_t)1 << logn) - 1 : 1;
  const uint64_t nb = logn > 13 ? (uint64_t)1 << (logn - 13) : 1;
  return (((uint64_t)1 << c) - 1) + 4096 + nb;
}

hipError_t launch_stage_twiddles(fe* out, const fe* A, const fe* B, int logn, hipStream_t s) {
  const int c = ntt_tw_cut(logn);
  uint64_t cnt = ((uint64_t)1 << c) - 1;
  if (cnt == 0) return hipSuccess;
  ProfScope ps("stage_twiddles", 16 * cnt, s);
  hipLaunchKernelGGL(k_stage_twiddles, dim3(nblocks(cnt, 256)), dim3(256), 0, s, out, A, B, logn, c);
  return hipGetLastError();
}

static bool batch_ok(int batch, uint64_t ys) {
  return batch >= 1 && (ys ? batch <= 65535 : batch <= kMaxBatch);
}

hipError_t launch_bitrev_gather(fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn,
                                const fe* sA, const fe* sB, int skip, hipStream_t s, uint64_t in_ys,
                                uint64_t out_ys, uint64_t in_es) {
  if (!batch_ok(batch, out_ys) || (in_ys != 0) != (out_ys != 0)) return hipErrorInvalidValue;
  uint64_t n = (uint64_t)1 << logn;
  GatherArgs ga;
  const int np = out_ys ? 1 : batch;
  for (int b = 0; b < kMaxBatch; ++b) {
    ga.out[b] = b < np ? out[b] : nullptr;
    ga.in[b] = b < np ? in[b] : nullptr;
  }
  ga.in_ys = in_ys;
  ga.out_ys = out_ys;
  ga.in_es = in_es ? in_es : 1;
  ProfScope ps("bitrev_gather", batch * (16 * (n_in < n ? n_in : n) + 16 * n), s, (uint64_t)batch * n);
  hipLaunchKernelGGL(k_bitrev_gather, dim3(nblocks(n, 256), batch), dim3(256), 0, s, ga, n_in, logn, sA, sB, skip);
  return hipGetLastError();
}

hipError_t launch_scale_const(fe* data, uint64_t n, const fe* cst, hipStream_t s) {
  ProfScope ps("scale_const", 32 * n, s);
  hipLaunchKernelGGL(k_scale_const, dim3(nblocks(n, 256)), dim3(256), 0, s, data, n, cst);
  return hipGetLastError();
}

// Stage plan from `first_b0` (stages first_b0+1 .. logn): each pass runs L
// stages on 2^L x C tiles (<= 4096 elements = 64 KiB of LDS), with C
// consecutive low-bit indices per tile so global accesses are C*16-byte runs.
// dynamic-LDS limits of the NTT kernels (> 64 KiB for the 8192-element tiles), set once per
// process; a function-local static, so concurrent first calls from several host threads are safe
static hipError_t ntt_lds_attributes() {
  static const hipError_t err = [] {
    const auto set = [](const void* f, int bytes) {
      return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    };
    hipError_t e = set((const void*)k_ntt_pass<0>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_pass<12>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_pass<11>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_pass_rr<10>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_pass_rr<11>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_pass_rr<12>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_pass_rr<13>, 131072);
    if (e == hipSuccess) e = set((const void*)k_ntt_first<10>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_first<11>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_first<12>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_first<13>, 131072);
    if (e == hipSuccess) e = set((const void*)k_ntt_first<11, true, false, false>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_first<11, true, false, true>, 65536);
    if (e == hipSuccess) e = set((const void*)k_ntt_first<11, true, true>, 65536);
    return e;
  }();
  return err;
}

hipError_t launch_ntt_dit(fe* const* data, int batch, const fe* tw, int logn, const fe* post, int first_b0,
                          hipStream_t s, uint64_t ys, const NttEpilogue* ep, int big_tl) {
  if (!batch_ok(batch, ys)) return hipErrorInvalidValue;
  if (ep && (!ys || post || first_b0 >= logn)) return hipErrorInvalidValue;  // the epilogue needs a last pass
  if (ys && ys != ((uint64_t)1 << logn)) return hipErrorInvalidValue;  // rows are contiguous transforms
  const int np = ys ? 1 : batch;
  if (const hipError_t e = ntt_lds_attributes(); e != hipSuccess) return e;
  static const bool use_rr = SG_KNOB(NTT_RR, 1) != 0;  // register-direct first/last steps
  const int big = big_tl;
  static const int tile_log = [] {
    int t = SG_KNOB(NTT_TILE_LOG, 11);  // A/B knob: 10, 11 or 12
    return (t >= 10 && t <= 12) ? t : 11;
  }();
  if (first_b0 >= logn) {
    for (int b = 0; post && b < np; ++b) {
      hipError_t e = launch_scale_const(data[b], ((uint64_t)1 << logn) * (ys ? (uint64_t)batch : 1), post, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // Balanced plan: as few passes as the tile allows (columns >= 8, i.e. 128-byte
  // runs), then the stages spread evenly, e.g. 2^25 after a 9-stage first pass
  // runs 8 + 8 instead of 7 + 7 + 2 (a whole HBM round trip for two stages).
  int b0 = first_b0;
  int pi = 0;
  while (b0 < logn) {
    PassArgs a;
    for (int b = 0; b < kMaxBatch; ++b) a.data[b] = b < np ? data[b] : nullptr;
    a.ys = ys;
    a.tw = tw;
    a.logn = logn;
    a.s_cut = ntt_tw_cut(logn);
    a.b0 = b0;
    int rem = logn - b0;
    int lmax = tile_log - (b0 < 3 ? b0 : 3);
    int passes = (rem + lmax - 1) / lmax;
    a.L = (rem + passes - 1) / passes;
    a.logC = b0 < tile_log - a.L ? b0 : tile_log - a.L;
    // one pass on a 2^big-element tile for all the remaining stages (columns: >= 64-byte runs on
    // 2^13 tiles, >= 32 on 2^12), 2^(big - 3) threads
    const bool big_pass = (big == 12 || big == 13) && use_rr && rem >= 6 && rem <= big - (big == 13 ? 2 : 1) &&
                          b0 >= big - rem && !ep;
    if (big_pass) {
      a.L = rem;
      a.logC = big - rem;
    }
    a.post = (b0 + a.L == logn) ? post : nullptr;
    a.ep_out = (ep && b0 + a.L == logn) ? ep->out : nullptr;
    if (a.ep_out) {
      a.ep_T0 = ep->T0;
      a.ep_T1 = ep->T1;
      a.ep_T2 = ep->T2;
      a.ep_row0 = ep->row0;
      a.ep_j0 = ep->j0;
      a.ep_rows = ep->rows;
      a.ep_logR = ep->logR;
      a.ep_vlog = ep->vlog;
      a.ep_k = ep->k;
    }
    uint64_t tile = (uint64_t)1 << (a.L + a.logC);
    uint64_t ntiles = ((uint64_t)1 << logn) / tile;
    unsigned threads = tile >= 2048 ? 256 : (unsigned)(tile / 8 > 64 ? tile / 8 : 64);
    size_t lds = tile * sizeof(fe);
    static const char* names[] = {"ntt_pass1", "ntt_pass2", "ntt_pass3", "ntt_pass4", "ntt_pass5"};
    ProfScope ps(names[pi < 4 ? pi : 4], batch * 32 * ((uint64_t)1 << logn), s);
    ++pi;
    dim3 grid((unsigned)ntiles, batch);
    if (big_pass && big == 13)
      hipLaunchKernelGGL(k_ntt_pass_rr<13>, grid, dim3(1024), lds, s, a);
    else if (big_pass)
      hipLaunchKernelGGL(k_ntt_pass_rr<12>, grid, dim3(512), lds, s, a);
    else if (tile == 4096 && threads == 256)
      hipLaunchKernelGGL(k_ntt_pass<12>, grid, dim3(256), lds, s, a);
    else if (tile == 2048 && threads == 256 && a.L >= 6 && use_rr)
      hipLaunchKernelGGL(k_ntt_pass_rr<11>, grid, dim3(256), lds, s, a);
    else if (tile == 1024 && threads == 128 && a.L >= 6 && use_rr)
      hipLaunchKernelGGL(k_ntt_pass_rr<10>, grid, dim3(128), lds, s, a);
    else if (tile == 2048 && threads == 256)
      hipLaunchKernelGGL(k_ntt_pass<11>, grid, dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL(k_ntt_pass<0>, grid, dim3(threads), lds, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    b0 += a.L;
  }
  return hipSuccess;
}

// Whole transform: fused bit-reversal first pass (when logn leaves room for a
// later pass), then launch_ntt_dit from stage L1 + 1.  `out` must not alias `in`.
bool ntt_small_whole(int logn, int batch, int skip, bool strided) {
  static const bool on = SG_KNOB(NTT_SMALL_WHOLE, 1) != 0;
  return on && strided && logn >= 6 && logn <= 11 && skip <= logn - 3 && batch % (1 << (11 - logn)) == 0;
}

hipError_t launch_ntt_fused(fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn, const fe* tw,
                            const fe* sA, const fe* sB, int skip, const fe* post, hipStream_t s, uint64_t in_ys,
                            uint64_t out_ys, uint64_t in_il, const NttEpilogue* ep) {
  if (!batch_ok(batch, out_ys) || (in_ys != 0) != (out_ys != 0)) return hipErrorInvalidValue;
  if (in_il && (!out_ys || (batch & 3))) return hipErrorInvalidValue;  // interleaved rows: strided, 4 per tile
  const int np = out_ys ? 1 : batch;
  if (const hipError_t e = ntt_lds_attributes(); e != hipSuccess) return e;
  // mid-size transforms: two passes on 2^12 / 2^13-element tiles (11 stages + the rest) instead of
  // three on 2048-element tiles (the multi-GPU interleaved gather and epilogue keep the latter)
  const int TL = (!in_il && !ep) ? ntt_first_tile(logn) : 11;
  const int LOGC1 = TL == 12 ? 1 : 2, L1 = TL - LOGC1;
  FirstArgs a;
  a.post = nullptr;
  a.ep_out = nullptr;
  if (logn <= L1 + LOGC1 || logn - L1 > 63) {
    // small transforms (2^6 .. 2^11 points) whole in one k_ntt_first<11> launch, 2^(11 - logn) rows
    // per 256-lane tile: the gather, every stage and the final store (canonical / n^-1 / four-step
    // epilogue) without the bit-reversal pass and the all-LDS generic pass (SG_NTT_SMALL_WHOLE=0:
    // the latter, A/B)
    const int logCw = 11 - logn;
    if (ntt_small_whole(logn, batch, skip, out_ys != 0)) {
      for (int b = 0; b < kMaxBatch; ++b) {
        a.out[b] = b < np ? out[b] : nullptr;
        a.in[b] = b < np ? in[b] : nullptr;
      }
      a.in_ys = in_il ? 0 : in_ys;
      a.out_ys = out_ys;
      a.tw = tw;
      a.sA = sA;
      a.sB = sB;
      a.n_in = n_in;
      a.logn = logn;
      a.L = logn;
      a.logC = logCw;
      a.skip = skip;
      a.s_cut = ntt_tw_cut(logn);
      a.in_il = in_il;
      a.post = post;
      if (ep) {
        a.ep_out = ep->out;
        a.ep_T0 = ep->T0;
        a.ep_T1 = ep->T1;
        a.ep_T2 = ep->T2;
        a.ep_row0 = ep->row0;
        a.ep_j0 = ep->j0;
        a.ep_rows = ep->rows;
        a.ep_logR = ep->logR;
        a.ep_vlog = ep->vlog;
        a.ep_k = ep->k;
      }
      const uint64_t n = (uint64_t)1 << logn;
      ProfScope ps("ntt_small", batch * (16 * (n_in < n ? n_in : n) + 16 * n), s, (uint64_t)batch * n);
      const dim3 grid(1, (unsigned)(batch >> logCw));
      if (ep) hipLaunchKernelGGL((k_ntt_first<11, true, true>), grid, dim3(256), (size_t)16 << 11, s, a);
      else if (post) hipLaunchKernelGGL((k_ntt_first<11, true, false, true>), grid, dim3(256), (size_t)16 << 11, s, a);
      else hipLaunchKernelGGL((k_ntt_first<11, true, false, false>), grid, dim3(256), (size_t)16 << 11, s, a);
      return hipGetLastError();
    }
    hipError_t e = launch_bitrev_gather(out, in, batch, n_in, logn, sA, sB, skip, s, in_il ? 1 : in_ys, out_ys,
                                        in_il);
    if (e != hipSuccess) return e;
    return launch_ntt_dit(out, batch, tw, logn, post, skip, s, out_ys, ep);
  }
  for (int b = 0; b < kMaxBatch; ++b) {
    a.out[b] = b < np ? out[b] : nullptr;
    a.in[b] = b < np ? in[b] : nullptr;
  }
  a.in_ys = in_ys;
  a.out_ys = out_ys;
  a.tw = tw;
  a.sA = sA;
  a.sB = sB;
  a.n_in = n_in;
  a.logn = logn;
  a.L = L1;
  a.logC = LOGC1;
  a.skip = skip;
  a.s_cut = ntt_tw_cut(logn);
  a.in_il = in_il;
  uint64_t n = (uint64_t)1 << logn;
  {
    ProfScope ps("ntt_first", batch * (16 * (n_in < n ? n_in : n) + 16 * n), s, (uint64_t)batch * n);
    // interleaved rows: a tile is 4 rows at one position (grid: positions x row quads)
    const dim3 grid = in_il ? dim3((unsigned)(n >> L1), (unsigned)(batch >> LOGC1)) : dim3((unsigned)(n >> TL), batch);
    if (TL == 10)
      hipLaunchKernelGGL(k_ntt_first<10>, grid, dim3(128), (size_t)16 << 10, s, a);
    else if (TL == 13)
      hipLaunchKernelGGL(k_ntt_first<13>, grid, dim3(1024), (size_t)16 << 13, s, a);
    else if (TL == 12)
      hipLaunchKernelGGL(k_ntt_first<12>, grid, dim3(512), (size_t)16 << 12, s, a);
    else
      hipLaunchKernelGGL(k_ntt_first<11>, grid, dim3(256), (size_t)16 << 11, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  // trivial stages beyond L1 are not replicated across tiles: later passes run
  // them as real butterflies on zeros, (a, 0) -> (a, a), which is exact
  return launch_ntt_dit(out, batch, tw, logn, post, L1, s, out_ys, ep, TL > 11 ? TL : 0);
}

int ntt_first_tile(int logn) {
  // fwd+inv on MI355X (tools/ab_big.sh, tools/ab_big2.sh; profiles/r02_ab_ntt_tiles.log):
  // 2^18-2^20 fastest with 2^12 tiles (11 + 7..9 stages: 2^20 0.148 -> 0.115 ms), 2^21 with 2^13
  // tiles (11 + 10: 0.202 -> 0.184 ms); at 2^22 and above the three-pass plan on 2048-element
  // tiles (4 blocks per CU) wins, and below 2^18 the launch count no longer matters
  static const bool on = SG_KNOB(NTT_TILES, 1) != 0;
  static const int forced = SG_KNOB(NTT_FIRST_TILE, 0);  // A/B knob: 10 .. 13 for every size
  if (forced >= 10 && forced <= 13) return forced;
  if (!on) return 11;
  if (logn >= 18 && logn <= 20) return 12;
  if (logn == 21) return 13;
  return 11;
}

uint64_t merkle_tree_digests(uint64_t n) { return 2 * n - 1; }


hipError_t launch_merkle_tree(const fe* const* leaves, uint64_t* const* tree, int batch, uint64_t n,
                              uint64_t* const* root_host, hipStream_t s, uint64_t leaves_ys, uint64_t tree_ys,
                              int start_level, uint64_t* const* root_flag, uint64_t root_seq,
                              const FoldLeaves* fold, int drop) {
  if (!batch_ok(batch, tree_ys) || (start_level == 0 && (leaves_ys != 0) != (tree_ys != 0))) return hipErrorInvalidValue;
  const int np = tree_ys ? 1 : batch;
  // Launch plan.  Levels 0..logn; level k has n >> k digests at offset 2n - 2(n >> k).
  //  * leaves: one lane per leaf (decimal + hash) in 512-lane blocks; 3 more levels
  //    fused through LDS (512 -> 64 lanes: every active wave full) when the tree is
  //    large enough to be throughput-bound, else the leaf level only;
  //    a tree of <= 1024 leaves with nothing above runs in one 1024-thread block;
  //    latency-bound leaf levels (< 2^17 leaves over the launch's trees) take a quad of lanes
  //    per leaf instead, 256 leaves per block, every level up to the block's digest fused;
  //  * node levels with >= kQuadBelow digests: one lane per node, 3 levels fused;
  //  * smaller levels (latency-bound): a quad of lanes per node, up to 7 levels fused.
  // SG_MERKLE_QUAD_BELOW = log2 of the threshold (A/B only)
  static const uint64_t kQuadBelow = (uint64_t)1 << SG_KNOB(MERKLE_QUAD_BELOW, 16);
  // forests (the sharded prove's run subtrees: thousands of trees of ~2^10 leaves per launch):
  // a node level with <= 2^SG_MERKLE_FOREST_QUAD digests per tree goes to the quad-lane kernel,
  // every level to each tree's root in one launch, however many trees the launch holds -- the
  // one-lane-per-node kernel would run blocks of count (< 64) lanes, i.e. partial waves, and
  // need two more launches per forest.  0 disables it (A/B knob).
  static const int kForestQuad = SG_KNOB(MERKLE_FOREST_QUAD, 6);
  int logn = 0;
  while (((uint64_t)1 << logn) < n) ++logn;
  int level = start_level;
  while (level <= logn) {
    uint64_t count = n >> level;
    MerkleArgs a;
    for (int b = 0; b < kMaxBatch; ++b) {
      a.leaves[b] = (level == 0 && b < np) ? leaves[b] : nullptr;
      a.tree[b] = b < np ? tree[b] : nullptr;
      a.root_host[b] = (root_host && b < np && !tree_ys) ? root_host[b] : nullptr;
      a.root_flag[b] = (a.root_host[b] && root_flag) ? root_flag[b] : nullptr;
    }
    a.root_seq = root_seq;
    a.drop = (uint32_t)(drop > 0 ? drop : 0);
    const bool fold_here = fold && level == 0;
    a.fold.src = fold_here ? fold->src : nullptr;
    a.fold.dst = fold_here ? fold->dst : nullptr;
    a.fold.Tlo = fold_here ? fold->Tlo : nullptr;
    a.fold.Thi = fold_here ? fold->Thi : nullptr;
    a.fold.shift = fold_here ? fold->shift : 0;
    a.fold.K = fold_here ? fold->K : fe_zero();
    a.fold.Kp = fold_here ? fold->Kp : nullptr;
    a.leaves_ys = leaves_ys;
    a.tree_ys = tree_ys;
    a.root_level = (uint64_t)logn;
    a.first_level = level;
    a.first_count = count;
    int fuse;
    unsigned bs;
    int kind;  // 0: leaf 256, 1: leaf tail 1024, 2: node 256, 3: quad 64, 4: leaf 512, 5: quad 256, 6: node 512, 8: leaf pairs 512,
              // 7: quad leaves 256, 12: quad leaves 64
    // SG_MERKLE_QUAD_LEAF_BELOW = log2 of the leaf count (all trees of the launch) under which the
    // leaf level takes a quad per leaf (k_merkle_quad_leaves); 0 disables it (A/B knob)
    static const int env_qleaf = SG_KNOB(MERKLE_QUAD_LEAF_BELOW, 17);
    if (level == 0 && env_qleaf > 0 && count * (uint64_t)batch < ((uint64_t)1 << env_qleaf)) {
      // latency-bound leaf level: up to 256 leaves per 1024-lane block, every level fused up to
      // the block's single digest (the whole tree when it has <= 256 leaves)
      // SG_MERKLE_QUAD_LEAF_NODES = leaves per block (256 or 64; A/B knob): a 256-leaf block puts
      // 16 waves on one CU, whose first levels then run at that CU's issue rate
      static const int env_qln = SG_KNOB(MERKLE_QUAD_LEAF_NODES, 256);
      const uint64_t qcap = env_qln == 64 ? 64 : 256;
      kind = qcap == 64 ? 12 : 7;
      const uint64_t nodes = count < qcap ? count : qcap;
      bs = (unsigned)(4 * nodes);
      int lg = 0;
      while (((uint64_t)1 << lg) < nodes) ++lg;
      fuse = lg + 1;
    } else if (level == 0) {
      if (count <= 64) {
        kind = 1; bs = (unsigned)count; fuse = logn + 1;
      } else {
        static const int env_bs = SG_KNOB(MERKLE_LEAF_BS, 512);
        static const int env_fuse = SG_KNOB(MERKLE_LEAF_FUSE, 4);
        unsigned lbs = env_bs == 512 ? 512u : 256u;
        kind = lbs == 512 ? 4 : 0;
        bs = count < lbs ? (unsigned)count : lbs;
        // leaf levels of >= 2^SG_MERKLE_LEAF_FUSE_MIN leaves (all trees of the launch together, a
        // forest's subtrees included) fuse node levels (A/B knob)
        static const int env_fmin = SG_KNOB(MERKLE_LEAF_FUSE_MIN, 18);
        fuse = count * (uint64_t)batch >= ((uint64_t)1 << env_fmin) ? env_fuse : 1;
        if (fuse < drop + 1) fuse = drop + 1;  // a lean tree's leaf launch reaches a stored level
        if (bs < lbs) kind = 0;
        {
          int lg = 0;  // a block's fused levels end at its single digest
          while ((1u << lg) < bs) ++lg;
          if (fuse > lg + 1) fuse = lg + 1;
        }
        // two leaves per lane (k_merkle_leaf_pairs), 512 lanes per 1024 leaves, the same levels fused:
        // 2^25 tree 4.13 -> 4.08 ms, prove -0.15 ms (profiles/r03_ab_leaf_pairs.log).
        // SG_MERKLE_LEAF_PAIRS = 0 restores one leaf per lane; k > 1 fuses k - 1 levels more (A/B knob)
        static const int env_pairs = SG_KNOB(MERKLE_LEAF_PAIRS, 1);
        if (env_pairs > 0 && fuse >= 2 && count % 1024 == 0) {
          kind = 8;
          bs = 512;
          fuse = fuse + env_pairs - 1;
          if (fuse > 11) fuse = 11;  // leaf + level 1 in the lane, then 512 -> 1 through LDS
        }
      }
    } else if (count * (uint64_t)batch >= kQuadBelow && count >= 2 &&
               !(kForestQuad > 0 && batch > 1 && count <= ((uint64_t)1 << kForestQuad))) {
      // 2 levels per launch: same-box A/Bs put 3 ahead of 4 (round 3, profiles/r03_ab_merkle_nodes.log,
      // r03_ab_nodes.log) and 2 ahead of 3 (round 4, r04_ab_node_fuse_*.log: every fused level above
      // the first parks half of the block's remaining waves at a barrier); coalesced child loads
      // staged through LDS were slower (4.22-4.27 ms) and were dropped.  The level is
      // throughput-bound when all its trees together have >= kQuadBelow nodes (a forest of many
      // small subtrees included): one lane per node, blocks no larger than a tree's level.
      // (rejected and removed in round 6, their A/B logs kept: a grid-stride kernel prefetching the
      // next group's children, r04_ab_node_pipe*; two nodes per lane, r04_ab_node_pairs*; the
      // level-2 hand-over by DPP, r05_ab_node_dpp_* -- none beat this plan on the same box)
      static const int env_nfuse = SG_KNOB(MERKLE_NODE_FUSE, 2);
      static const int env_nbs = SG_KNOB(MERKLE_NODE_BS, 256);  // A/B knob: 256 or 512
      kind = env_nbs == 512 ? 6 : 2; bs = env_nbs == 512 ? 512u : 256u; fuse = env_nfuse;
      if (count < bs) {
        kind = 2;
        bs = (unsigned)count;  // a power of two (tree levels)
        int lg = 0;
        while ((1u << lg) < bs) ++lg;
        if (fuse > lg + 1) fuse = lg + 1;
      }
    } else {
      // the last <= 256 nodes of a tree go to the root in one 1024-lane block
      // (SG_MERKLE_QUAD_TOP=0: 64-node blocks only)
      static const int env_top = SG_KNOB(MERKLE_QUAD_TOP, 1);
      // SG_MERKLE_QUAD_TOP_MAX = the largest level that one block takes to the root (A/B knob)
      static const uint64_t top_max = (uint64_t)SG_KNOB(MERKLE_QUAD_TOP_MAX, 256);
      const uint64_t cap = (env_top && count <= top_max && count <= 256) ? 256 : 64;
      kind = cap == 256 ? 5 : 3;
      uint64_t nodes = count < cap ? count : cap;
      bs = (unsigned)(4 * nodes);
      int lg = 0;
      while (((uint64_t)1 << lg) < nodes) ++lg;
      fuse = lg + 1;
    }
    // a lean tree's leaf launch reaches level `drop` (or the root): no later launch reads a dropped level
    if (level == 0 && drop > 0 && fuse < drop + 1 && fuse < logn + 1) return hipErrorInvalidValue;
    if (level + fuse - 1 > logn) fuse = logn - level + 1;
    if (fuse < 1 || fuse > kMaxFuse) return hipErrorInvalidValue;
    a.fuse = fuse;
    // digest offsets in the buffer: a lean tree's buffer starts at level `drop` (the dropped levels
    // are never stored or read)
    const uint64_t dropped = drop > 0 ? 2 * n - 2 * (n >> drop) : 0;
    for (int k = 0; k <= kMaxFuse; ++k) {
      int lv = level - 1 + k;
      a.off[k] = (lv < 0 || lv > logn || lv < drop) ? 0 : (2 * n - 2 * (n >> lv)) - dropped;
    }
    // algorithmic bytes (Merkle(n) = 16 n + 64 (2n - 1)): leaves read once (16 B) +
    // 64 B per digest of these levels -- a lean tree's leaf digests count although they are not
    // stored (the figure prices the algorithm; its PMC traffic is then below it)
    uint64_t digests = 0;
    for (int k = 0; k < fuse; ++k) digests += count >> k;
    // a fused fold reads 2 source elements and writes the folded one instead of reading the leaf
    // quad kernels: 4 lanes per node; leaf pairs: 2 leaves per lane
    const uint64_t per_block = kind == 3 || kind == 5 || kind == 7 || kind == 12 ? bs / 4 : kind == 8 || kind == 10 ? 2 * bs : bs;
    dim3 grid((unsigned)((count + per_block - 1) / per_block), batch);
    // elems = lanes launched (the rocprofv3 Grid_Size of this dispatch), so per-wave PMC
    // instruction counts scale to any launch population
    ProfScope ps(kind == 7 || kind == 12 ? "merkle_leaves_quad"
                 : level == 0 ? (fold_here ? "merkle_fold_leaves" : "merkle_leaves")
                            : (kind == 3 || kind == 5 ? "merkle_nodes_quad" : "merkle_nodes"),
                 batch * ((level == 0 ? (fold_here ? 48 : 16) * count : 0) + 64 * digests), s,
                 (uint64_t)grid.x * grid.y * bs);
    hipError_t e = launch_merkle_lanes(kind, fold_here, grid, bs, s, a);
    if (e != hipSuccess) return e;
    level += fuse;
  }
  return hipSuccess;
}



// ---------------------------------------------- row-sharded helpers: launchers

static unsigned grid_stride_blocks(uint64_t n) {
  uint64_t blocks = (n + 255) / 256;
  const uint64_t cap = 256 * 16;
  return (unsigned)(blocks < cap ? (blocks ? blocks : 1) : cap);
}

hipError_t launch_mul_pow(fe* data, uint64_t rows, uint64_t cols, uint64_t a0, uint64_t a1, uint64_t b0,
                          uint64_t b1, const fe* T0, const fe* T1, const fe* T2, hipStream_t s, uint64_t nb) {
  if (rows * cols * nb == 0) return hipSuccess;
  MulPowArgs a{data, rows, cols, a0, a1, b0, b1, T0, T1, T2, nb};
  ProfScope ps("mul_pow", 32 * rows * cols * nb, s);
  hipLaunchKernelGGL(k_mul_pow, dim3(grid_stride_blocks(rows * cols * nb)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_swap01(const fe* in, fe* out, uint64_t A, uint64_t B, uint64_t C, hipStream_t s, uint64_t nb) {
  if (A * B * C * nb == 0) return hipSuccess;
  ProfScope ps("transpose", 32 * A * B * C * nb, s);
  if (C >= 16 || A == 1 || B == 1) {
    hipLaunchKernelGGL(k_swap01_runs, dim3(grid_stride_blocks(A * B * C * nb)), dim3(256), 0, s, in, out, A, B, C,
                       nb);
  } else {
    uint64_t gx = (B + 31) / 32, gy = (A + 31) / 32;
    if (gx > 0x7FFFFFFFull || gy > 65535 || C * nb > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_swap01_tiled, dim3((unsigned)gx, (unsigned)gy, (unsigned)(C * nb)), dim3(256), 0, s, in,
                       out, A, B, C);
  }
  return hipGetLastError();
}

hipError_t launch_fri_fold_runs(fe* out, const fe* in, uint64_t half, uint64_t run, uint64_t run_stride,
                                uint64_t run_off, const fe* T0, const fe* T1, const fe* T2, const fe& K,
                                hipStream_t s) {
  if (half == 0) return hipSuccess;
  FoldRunsArgs a{out, in, half, run, run_stride, run_off, T0, T1, T2, K};
  ProfScope ps("fri_fold", 48 * half, s);
  hipLaunchKernelGGL(k_fri_fold_runs, dim3(grid_stride_blocks(half)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_gather_roots(const uint64_t* tree, uint64_t tree_ys, uint64_t root_off, uint64_t* out,
                               uint64_t count, hipStream_t s) {
  if (count == 0) return hipSuccess;
  ProfScope ps("gather_roots", 128 * count, s);
  hipLaunchKernelGGL(k_gather_roots, dim3(nblocks(count, 256)), dim3(256), 0, s, tree, tree_ys, root_off, out, count);
  return hipGetLastError();
}

}  // namespace sg
