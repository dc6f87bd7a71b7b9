// Host-side launchers for the gfx950 kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "fe128.hpp"

namespace sg {

hipError_t launch_stage_twiddles(fe* out, const fe* pw, int logn, hipStream_t s);
hipError_t launch_pow_table(fe* tw, const fe* A, const fe* B, uint64_t count, hipStream_t s);
// batched over up to 4 independent transforms / trees (one per blockIdx.y)
hipError_t launch_bitrev_gather(fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn,
                                const fe* sA, const fe* sB, int skip, hipStream_t s);
hipError_t launch_scale_const(fe* data, uint64_t n, const fe* cst, hipStream_t s);
hipError_t launch_ntt_dit(fe* const* data, int batch, const fe* tw, int logn, const fe* post, int first_b0,
                          hipStream_t s);
// bit-reversal (+ LDE scale, + `skip` trivial stages) fused into the first pass; out must not alias in
hipError_t launch_ntt_fused(fe* const* out, const fe* const* in, int batch, uint64_t n_in, int logn, const fe* tw,
                            const fe* sA, const fe* sB, int skip, const fe* post, hipStream_t s);
uint64_t merkle_tree_digests(uint64_t n);
// root_host (optional, per tree): host-coherent 64-byte slots that receive the root
hipError_t launch_merkle_tree(const fe* const* leaves, uint64_t* const* tree, int batch, uint64_t n,
                              uint64_t* const* root_host, hipStream_t s);
hipError_t launch_fri_fold(fe* out, const fe* in, uint64_t half, const fe* Tlo, const fe* Thi, int shift,
                           const fe& K, const fe& Wstride, unsigned grid, hipStream_t s);
unsigned fri_fold_grid(uint64_t half);
hipError_t launch_gather_digests(const uint64_t* tree, const uint64_t* idx, uint64_t* out, uint32_t count,
                                 hipStream_t s);
hipError_t launch_gather_digest_ptrs(const uint64_t* addrs, uint64_t* out, uint32_t count, hipStream_t s);
hipError_t launch_gather_fe_ptrs(const uint64_t* addrs, fe* out, uint32_t count, hipStream_t s);
hipError_t launch_gather_fe(const fe* src, const uint64_t* idx, fe* out, uint32_t count, hipStream_t s);

}  // namespace sg
