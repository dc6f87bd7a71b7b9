/*
 * stark_gpu.h -- C ABI of the MI355X-native STARK hot path (libstarkgpu.so).
 *
 * Drop-in boundary for the reference crate SpekalsG3/zk-stark-tutor (Rust).
 * Each entry point replaces one reference function; the citation after each
 * declaration is the file:line (under the reference's src/) of the Rust item
 * whose signature and semantics it keeps.  A Rust `extern "C"` shim (see
 * INTEGRATION.md) marshals Vec<FieldElement> into packed sg_fe arrays and maps
 * negative return codes to the reference's panic!/Err paths.
 *
 * Conventions
 *   - sg_fe is a canonical field element (value < p = 1 + 407*2^119) as two
 *     little-endian u64 limbs.  Inputs >= p are rejected (SG_ERR_NONCANONICAL)
 *     where the library reads them on the host, otherwise undefined.
 *   - The caller owns every host buffer; the library owns device memory it
 *     allocates.  `_dev` variants take device pointers (hipMalloc'd) and run on
 *     the context's stream; all calls return after their work is complete.
 *   - Return value: 0 on success, < 0 on error (sg_last_error() has the text).
 *     The library never aborts the process.
 *   - A context is not thread-safe: one context per host thread.
 */
#ifndef STARK_GPU_H
#define STARK_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_OK 0
#define SG_ERR_INVALID (-1)      /* argument the reference rejects with panic!/assert */
#define SG_ERR_HIP (-2)          /* HIP runtime error */
#define SG_ERR_NONCANONICAL (-3) /* field element >= p */
#define SG_ERR_CALLBACK (-4)     /* a proof-stream callback returned non-zero */
#define SG_ERR_NOMEM (-5)        /* device (or host) memory exhausted; the context stays usable */
/* A failed call leaves no HIP error behind on the calling thread (its hipGetLastError is cleared), so
 * the caller's own HIP work (e.g. torch's) is unaffected; sg_last_error(ctx) holds the message. */

typedef struct {
  uint64_t lo, hi;
} sg_fe;

typedef struct sg_ctx sg_ctx;

/* ------------------------------------------------------------ context */
int sg_ctx_create(int device, sg_ctx** out);
void sg_ctx_destroy(sg_ctx* ctx);
const char* sg_last_error(const sg_ctx* ctx);
/* hipStream_t the context launches on (for callers that time or chain work) */
void* sg_ctx_stream(sg_ctx* ctx);
/* release cached device buffers and twiddle tables */
int sg_ctx_trim(sg_ctx* ctx);
/* instrumentation, no reference counterpart: the number of public tables the context keeps
 * (domain / AIR coset tables, twiddle plans, interpolation kernels) -- constant across proofs
 * on one (AIR, domain), also when the constraints are rebuilt for every proof */
int sg_ctx_cached_tables(const sg_ctx* ctx, size_t* domain_tables, size_t* twiddle_tables);
/* Options of a context (no reference counterpart; every setting writes the same proof bytes --
 * tests compare the equivalent paths this way, and no environment variable switches them):
 *   "domain_cache"   1 (default; 0 also by SG_NO_DOMAIN_CACHE=1 at creation): public domain /
 *                    AIR tables kept across calls, else recomputed in every call
 *   "air_generic"    0 (default): the Rescue-Prime AIR in its factored form; 1: its expanded groups
 *   "geo_decimate"   1 (default): decimated geometric interpolation; 0: the full group
 *   "lean_trees"     1 (default): the retained prove / FRI trees drop their lowest levels
 *   "stream_pin"     1 (default): a native proof stream's buffer is page-locked for device copies
 *   "world1_sharded" 0 (default): a one-rank communicator proves through the single-GPU plan; 1:
 *                    through the four-step path (tests of the sharded machinery over RCCL)
 *   "lean_drop"      3 (default): the most levels a lean tree drops (0..3; 0 = keep every level)
 *   "fri_gate"       1 (default): FRI::commit queues round r+1's fold + tree behind a device gate
 *                    before round r's challenge exists (the host raises the gate after writing K;
 *                    a gate left 60 s raises an error); 0: each round is launched after its challenge
 *   "fri_gate_timeout_ms" 60000 (default): how long a gate waits for its challenge before the call
 *                    fails with SG_ERR_HIP (a test sets it low to exercise the deadline)
 * SG_ERR_INVALID for an unknown name. */
int sg_ctx_set_option(sg_ctx* ctx, const char* name, int64_t value);
/* Device memory (no reference counterpart): `live` = bytes of the context's buffer pool in use,
 * `peak` = their high-water mark since creation or the last reset (the working set of the calls
 * in between: codewords, retained trees, scratch), `pooled` = returned buffers the pool caches,
 * device_used / device_total = hipMemGetInfo of the context's device (every process, every
 * allocation: cached tables included).  reset_peak != 0 restarts the high-water mark at `live`. */
int sg_ctx_memory(sg_ctx* ctx, uint64_t* live, uint64_t* peak, uint64_t* pooled, uint64_t* device_used,
                  uint64_t* device_total, int reset_peak);
/* HBM probe (measurement, no reference counterpart): read + write GB/s of a dwordx4 streaming
 * device copy of `bytes` (multiple of 16), best of `iters`; blocks = 0: one 16-byte element per
 * lane, else a grid-stride copy over blocks x 256 lanes */
int sg_hbm_copy_probe(sg_ctx* ctx, size_t bytes, int iters, unsigned blocks, double* gbs);
/* per-kernel HIP-event timing on the context stream (instrumentation, no reference counterpart):
 * enable resets the totals; the report is JSON {kernel: {launches, ms, bytes}} where bytes are
 * the algorithmic bytes of the launches; len receives the size incl. the NUL. */
/* Device-pointer transforms (sg_ntt_dev, sg_intt_dev, sg_fast_coset_evaluate*_dev) return
 * after their work completes (default) or, with async enabled, once it is enqueued on the
 * context's stream: later library calls on the same context are ordered after it, and
 * sg_ctx_synchronize waits for everything (needed before reading results elsewhere). */
int sg_ctx_set_async(sg_ctx* ctx, int enable);
int sg_ctx_synchronize(sg_ctx* ctx);
int sg_ctx_profile(sg_ctx* ctx, int enable);
/* restrict the timing to launches of one kernel name (NULL or "" = all) to keep event overhead low */
int sg_ctx_profile_only(sg_ctx* ctx, const char* kernel);
int sg_ctx_profile_report(sg_ctx* ctx, char* buf, size_t cap, size_t* len);

/* ------------------------------------------------------------ field (field/field.rs) */
sg_fe sg_field_prime(void);                               /* field/field.rs:10 FIELD_PRIME */
sg_fe sg_field_generator(void);                           /* field/field.rs:41-44 Field::generator */
int sg_primitive_nth_root(uint64_t n, sg_fe* out);        /* field/field.rs:58-71 Field::primitive_nth_root */
sg_fe sg_field_sample(const uint8_t* bytes, size_t len);  /* field/field.rs:87-99 Field::sample */
sg_fe sg_fe_mul(sg_fe a, sg_fe b);                        /* field/field_element.rs:70-78 Mul */
sg_fe sg_fe_inverse(sg_fe a);                             /* field/field_element.rs:35-40 inverse */
sg_fe sg_fe_pow(sg_fe a, uint64_t e);                     /* field/field_element.rs:127-143 BitXor<usize> */

/* ------------------------------------------------------------ transforms (fft/) */
/* fft/ntt.rs:7-49  pub fn ntt(root, inputs: Vec<FieldElement>) -> Vec<FieldElement>
 * out receives next_pow2(n_in) elements (zero padding as bit_reverse_copy does). */
int sg_ntt(sg_ctx* ctx, sg_fe root, const sg_fe* inputs, size_t n_in, sg_fe* out);
/* fft/ntt.rs:51-68  pub fn intt(root, input) -> Vec<FieldElement>; n_in < 2 returns the input */
int sg_intt(sg_ctx* ctx, sg_fe root, const sg_fe* inputs, size_t n_in, sg_fe* out);
/* fft/ntt_arithmetics.rs:161-170  pub fn fast_coset_evaluate(generator, root_order, offset, polynomial)
 * out receives next_pow2(root_order) elements; d > root_order is SG_ERR_INVALID (reference panics). */
int sg_fast_coset_evaluate(sg_ctx* ctx, sg_fe generator, uint64_t root_order, sg_fe offset,
                           const sg_fe* coeffs, size_t d, sg_fe* out);
/* same, with device pointers (inputs resident in HBM) */
int sg_ntt_dev(sg_ctx* ctx, sg_fe root, const sg_fe* d_inputs, size_t n_in, sg_fe* d_out);
int sg_intt_dev(sg_ctx* ctx, sg_fe root, const sg_fe* d_inputs, size_t n_in, sg_fe* d_out);
int sg_fast_coset_evaluate_dev(sg_ctx* ctx, sg_fe generator, uint64_t root_order, sg_fe offset,
                               const sg_fe* d_coeffs, size_t d, sg_fe* d_out);
/* batch (1..4) independent LDEs of equal length in one launch sequence -- stark/stark.rs:367-386
 * evaluates one boundary quotient per register with identical (generator, root_order, offset) */
int sg_fast_coset_evaluate_batch_dev(sg_ctx* ctx, sg_fe generator, uint64_t root_order, sg_fe offset,
                                     const sg_fe* const* d_coeffs, size_t d, sg_fe* const* d_out, size_t batch);

/* ------------------------------------------------------------ Merkle (merkle_root.rs) */
typedef struct sg_tree sg_tree; /* retained device tree: all 2n-1 digests */

/* merkle_root.rs:21-32  MerkleRoot::commit(leafs: &[FieldElement]) -> Bytes (64 bytes) */
int sg_merkle_commit(sg_ctx* ctx, const sg_fe* leaves, size_t n, uint8_t root[64]);
/* merkle_root.rs:55-66  MerkleRoot::open(index, leafs) -> Vec<Bytes>; path gets log2(n) x 64 bytes */
int sg_merkle_open(sg_ctx* ctx, size_t index, const sg_fe* leaves, size_t n, uint8_t* path, size_t* path_len);
/* merkle_root.rs:89-95  MerkleRoot::verify(root, index, path, leaf) -> bool: returns 1/0, < 0 on error */
int sg_merkle_verify(const uint8_t root[64], size_t index, const uint8_t* path, size_t path_len, sg_fe leaf);
/* device-resident tree: build once, open in O(log n) */
int sg_merkle_build_dev(sg_ctx* ctx, const sg_fe* d_leaves, size_t n, sg_tree** out);
/* batch (1..4) equal-size trees built together (stark/stark.rs:380 commits one per register) */
int sg_merkle_build_batch_dev(sg_ctx* ctx, const sg_fe* const* d_leaves, size_t n, size_t batch, sg_tree** out);
int sg_tree_root(const sg_tree* t, uint8_t root[64]);
size_t sg_tree_leaves(const sg_tree* t);
int sg_tree_open(sg_ctx* ctx, const sg_tree* t, size_t index, uint8_t* path, size_t* path_len);
void sg_tree_free(sg_ctx* ctx, sg_tree* t);

/* ------------------------------------------------------------ proof stream (proof_stream.rs) */
/* Object codes = StarkProofStreamEnum discriminants (stark/proof_stream_enum.rs:8-15);
 * payload = the to_bytes() serialization (stark/proof_stream_enum.rs:67-127). */
#define SG_OBJ_ROOT 0
#define SG_OBJ_CODEWORD 1
#define SG_OBJ_PATH 2
#define SG_OBJ_LEAFS 3
#define SG_OBJ_VALUE 4

/* Callback view of any ProofStream impl (proof_stream.rs:6-12): push + fiat_shamir_prover. */
typedef struct {
  void* user;
  int (*push)(void* user, uint8_t code, const uint8_t* payload, size_t len);
  int (*fiat_shamir_prover)(void* user, size_t num_bytes, uint8_t* out);
} sg_proof_stream;

/* Native streams: IndependentProofStream (proof_stream.rs:15-78) and
 * SignatureProofStream (rescue_prime/proof_stream.rs:9-61, prefix = blake2b(document)). */
typedef struct sg_stream sg_stream;
sg_stream* sg_stream_create(void);
sg_stream* sg_stream_create_signature(const uint8_t* document, size_t doc_len);
void sg_stream_destroy(sg_stream* s);
sg_proof_stream sg_stream_callbacks(sg_stream* s);
int sg_stream_push(sg_stream* s, uint8_t code, const uint8_t* payload, size_t len);
size_t sg_stream_count(const sg_stream* s);
/* stark/proof_stream_enum.rs:161-190 digest(): pass out=NULL to query the size */
int sg_stream_digest(const sg_stream* s, uint8_t* out, size_t cap, size_t* len);
int sg_stream_fiat_shamir_prover(const sg_stream* s, size_t num_bytes, uint8_t* out);
int sg_stream_fiat_shamir_verifier(const sg_stream* s, size_t num_bytes, uint8_t* out);
/* proof_stream.rs:54-64 pull(): returns a view valid until the stream is modified */
int sg_stream_pull(sg_stream* s, uint8_t* code, const uint8_t** payload, size_t* len);
/* stark/stark.rs:30-67 deser_independent_proof_stream */
int sg_stream_deserialize(const uint8_t* bytes, size_t len, sg_stream** out);

/* ------------------------------------------------------------ FRI (fri.rs) */
typedef struct {
  sg_fe offset;                   /* fri.rs:23-29 FRI::new(offset, omega, domain_length, */
  sg_fe omega;                    /*                       expansion_factor,               */
  uint64_t domain_length;         /*                       num_colinearity_tests)          */
  uint64_t expansion_factor;
  uint64_t num_colinearity_tests;
} sg_fri;

typedef struct sg_fri_state sg_fri_state; /* retained codewords + trees of every round */

size_t sg_fri_num_rounds(const sg_fri* fri); /* fri.rs:40-50 */
/* fri.rs:115-172  FRI::commit: Root per round, alpha = sample(fiat_shamir_prover(32)),
 * fold, final Codeword.  keep != NULL retains the rounds for sg_fri_query. */
int sg_fri_commit(sg_ctx* ctx, const sg_fri* fri, const sg_fe* codeword, size_t n,
                  const sg_proof_stream* ps, sg_fri_state** keep);
int sg_fri_commit_dev(sg_ctx* ctx, const sg_fri* fri, const sg_fe* d_codeword, size_t n,
                      const sg_proof_stream* ps, sg_fri_state** keep);
/* fri.rs:210-248  FRI::prove: commit + sample_indices + query per round.
 * top_indices receives num_colinearity_tests indices. */
int sg_fri_prove(sg_ctx* ctx, const sg_fri* fri, const sg_fe* codeword, size_t n,
                 const sg_proof_stream* ps, size_t* top_indices);
int sg_fri_prove_dev(sg_ctx* ctx, const sg_fri* fri, const sg_fe* d_codeword, size_t n,
                     const sg_proof_stream* ps, size_t* top_indices);
void sg_fri_state_free(sg_ctx* ctx, sg_fri_state* st);
/* fri.rs:88-113  FRI::sample_indices */
int sg_fri_sample_indices(const uint8_t* seed, size_t seed_len, size_t size, size_t reduced_size,
                          size_t number, size_t* out);


/* ------------------------------------------------ row-sharded blocks (multi-GPU)
 * the four-step NTT, the sharded Merkle commit and the FRI fold
 * over a codeword distributed as runs.  The reference is single-threaded and has
 * no counterpart; these are the local steps a multi-GPU Rust caller (or
 * starkgpu/dist.py) composes around one all-to-all and per-tree all-gathers.
 * Shards are row-major arrays of canonical elements in device memory. */
typedef struct sg_forest sg_forest; /* `runs` Merkle trees of `run` leaves each */

/* `rows` independent ntt()s (fft/ntt.rs:7-49 per row): row r reads n_in elements at
 * d_in + r*n_in (zero-padded to n) and writes n at d_out + r*n.  Output must not
 * alias the input. */
int sg_ntt_rows_dev(sg_ctx* ctx, sg_fe root, const sg_fe* d_in, size_t n_in, size_t rows,
                    sg_fe* d_out, size_t n);
/* d[i] *= c for i < n (the n^-1 of an inverse transform, fft/ntt.rs:62-67) */
int sg_scale_dev(sg_ctx* ctx, sg_fe* d_data, size_t n, sg_fe c);
/* d[r][c] *= base^((a0 + a1 r) c + b0 + b1 r), exponents < 2^36: four-step twiddles
 * omega^(j1 k2) and the coset scale offset^j (field/polynomial.rs:109-121) */
int sg_mul_pow_dev(sg_ctx* ctx, sg_fe base, sg_fe* d_data, size_t rows, size_t cols,
                   uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1);
/* out[b][a][c] = in[a][b][c] for an A x B x C array */
int sg_transpose_dev(sg_ctx* ctx, const sg_fe* d_in, sg_fe* d_out, size_t A, size_t B, size_t C);
/* merkle_root.rs:21-32 on each of `runs` consecutive runs of `run` leaves (retained) */
int sg_merkle_forest_dev(sg_ctx* ctx, const sg_fe* d_leaves, size_t run, size_t runs, sg_forest** out);
/* the runs' roots, 64 bytes each, into device memory (runs x 64 bytes) */
int sg_forest_roots_dev(sg_ctx* ctx, const sg_forest* f, uint8_t* d_roots);
/* merkle_root.rs:34-53 path of leaf `index` inside tree `tree` of the forest */
int sg_forest_open(sg_ctx* ctx, const sg_forest* f, size_t tree, size_t index, uint8_t* path,
                   size_t* path_len);
void sg_forest_free(sg_ctx* ctx, sg_forest* f);
/* merkle_root.rs:7-19 node levels over n given digests (device, n x 64 bytes): the
 * top of a tree whose lower levels are the runs' subtrees.  Root via sg_tree_root. */
int sg_merkle_top_dev(sg_ctx* ctx, const uint8_t* d_digests, size_t n, sg_tree** out);
/* fri.rs:151-159 fold of a run-sharded codeword of global length n_global with this
 * round's omega / offset and alpha: local element l is global index
 * (l / run) * run_stride + run_off + l % run and its partner (global + n_global/2)
 * must be local l + n_local/2.  Writes n_local/2 elements. */
int sg_fri_fold_runs_dev(sg_ctx* ctx, sg_fe omega, sg_fe offset, sg_fe alpha, const sg_fe* d_in,
                         size_t n_local, size_t run, size_t run_stride, size_t run_off,
                         size_t n_global, sg_fe* d_out);

/* ------------------------------------------------ multi-GPU (one process per GPU)
 * a Rust (or any) caller shards the LDE / NTT / Merkle / FRI commit
 * without torch.  A communicator binds a context to RCCL over xGMI (sg_dist_create, from a
 * unique id the caller distributes: rank 0 calls sg_dist_unique_id) or to a host-staged
 * transport the caller implements (sg_dist_create_transport: MPI, gloo, sockets, tests).
 * Shards (device, canonical elements), rank g of G, n = N1 N2 (sg_dist_plan):
 *   column shard [N1/G][row_len]  row r = x[(g N1/G + r) + N1 j], j < row_len <= N2, zero beyond
 *   run shard    [N1][N2/G]       element [k1][c] = X[k1 N2 + g N2/G + c]
 * The data exchange of a transform is ONE all-to-all (the four-step transpose); the Merkle
 * commit all-gathers N1 64-byte run roots; FRI folds are rank-local.  Outputs equal the
 * single-GPU / reference results bit for bit (roots of order exactly n). */
#define SG_DIST_ID_BYTES 128
typedef struct sg_dist sg_dist;
typedef struct {
  void* user;
  /* host buffers: send = nranks blocks of `bytes` (block h goes to rank h); recv = nranks blocks
   * (block h came from rank h).  Return 0 on success. */
  int (*all_to_all)(void* user, const void* send, void* recv, size_t bytes);
  /* send = one block of `bytes`; recv = every rank's block in rank order */
  int (*all_gather)(void* user, const void* send, void* recv, size_t bytes);
  /* optional (may be NULL): called once when a call fails on this rank and the communicator is
   * poisoned, so the caller can end the peers' pending exchanges (e.g. tear its group down).
   * The library cannot interrupt a callback that blocks: a caller transport bounds its own waits. */
  void (*abort)(void* user);
} sg_dist_transport;
int sg_dist_unique_id(uint8_t* id /* SG_DIST_ID_BYTES */);                   /* ncclGetUniqueId */
int sg_dist_create(sg_ctx* ctx, const uint8_t* id, int nranks, int rank, sg_dist** out); /* RCCL */
int sg_dist_create_transport(sg_ctx* ctx, int nranks, int rank, const sg_dist_transport* t,
                             sg_dist** out);
void sg_dist_destroy(sg_dist* d);
/* Failure containment (no reference counterpart; the reference is single-process).  Every
 * sg_dist_* call below is collective.  When one fails on a rank -- an error of its own, a failing
 * proof-stream or transport callback, an RCCL asynchronous error, or a host wait that outlasts the
 * deadline -- the communicator is POISONED on that rank: RCCL's is aborted with ncclCommAbort, a
 * caller transport's abort hook runs, and every later call on it returns SG_ERR_INVALID.  Destroy
 * it and create a new one.  ncclCommAbort is local; so that the peers of an RCCL communicator
 * learn of it, the failing rank also raises an out-of-band flag -- a node-local file named from
 * the unique id, /dev/shm/sg_dist_abort_<FNV-1a of the id> -- that every rank's host waits poll
 * about every 10 ms: a peer waiting inside a call then poisons its own communicator (aborting its
 * collectives) and returns SG_ERR_HIP ("a peer rank failed (rank r of G: reason)") within
 * milliseconds.  Ranks on other nodes (no shared /dev/shm) fail at their deadline instead.
 * Host-blocking RCCL calls (ncclCommInitRank, the connection set-up inside ncclGroupEnd) are not
 * watched.  A caller transport gets the abort hook instead of the flag (e.g. tear its group down).
 * Deadline: SG_DIST_TIMEOUT_S at creation (default 30 s) or sg_dist_set_timeout (per rank): the
 * longest one host wait inside a communicator call may last (the prove's longest is well under a
 * second at the headline size, a few seconds at 2^27 rows over 8 ranks). */
int sg_dist_set_timeout(sg_dist* d, double seconds);
int sg_dist_poisoned(const sg_dist* d); /* 1 when poisoned */
/* instrumentation: collectives this communicator issued, transition quotients and trace columns
 * whose coset work / interpolation sg_dist_stark_prove ran on run shards (the rest ran replicated) */
int sg_dist_counters(const sg_dist* d, uint64_t* collectives, uint64_t* sharded_quotients,
                     uint64_t* sharded_interpolations);
/* Collective: the codeword size (log2 elements, <= 0: never) at which a sharded FRI commit hands
 * over to the single-GPU rounds (default SG_DIST_FRI_TAIL at creation, else 20).  It decides the
 * collective schedule, so every rank passes the same value; the call all-gathers it and fails
 * (poisoning) when they differ.  Creation checks the environment's value the same way. */
int sg_dist_set_fri_tail(sg_dist* d, int log2_elements);
/* N1 = 2^floor(log2 n / 2), N2 = n / N1; needs N1 >= G and N2 >= 4 G */
int sg_dist_plan(size_t n, int nranks, size_t* n1, size_t* n2);
/* fft/ntt.rs:7-49 over the ranks: column shard in, run shard out */
int sg_dist_ntt(sg_dist* d, sg_fe root, const sg_fe* d_cols, size_t row_len, size_t n,
                sg_fe* d_runs);
/* fft/ntt.rs:51-68: run shard in, column shard (rows of N2) out */
int sg_dist_intt(sg_dist* d, sg_fe root, const sg_fe* d_runs, size_t n, sg_fe* d_cols);
/* fft/ntt_arithmetics.rs:161-170: coefficients as a column shard, codeword as a run shard */
int sg_dist_coset_evaluate(sg_dist* d, sg_fe generator, size_t root_order, sg_fe offset,
                           const sg_fe* d_cols, size_t row_len, sg_fe* d_runs);
/* merkle_root.rs:21-32 of the natural-order codeword held as run shards (same root on every rank) */
int sg_dist_merkle_root(sg_dist* d, const sg_fe* d_runs, size_t n, uint8_t* root);
/* fri.rs:115-172 FRI::commit of a run-sharded codeword: every rank writes the same stream bytes */
int sg_dist_fri_commit(sg_dist* d, const sg_fri* fri, const sg_fe* d_runs, size_t n,
                       const sg_proof_stream* ps);
/* fri.rs:210-248 FRI::prove of a run-sharded codeword (replaces FRI::prove when the codeword is
 * sharded): the sharded commit keeps every round's runs, forests and top trees; each query opening
 * comes from the rank that owns the leaf's run (value + subtree path, one all-gather per round)
 * plus the top path every rank holds.  Every rank writes the same proof-stream bytes as the
 * single-GPU sg_fri_prove and receives the same c top-level indices in top. */
int sg_dist_fri_prove(sg_dist* d, const sg_fri* fri, const sg_fe* d_runs, size_t n, const sg_proof_stream* ps,
                      size_t* top);

/* ------------------------------------------- polynomial algebra (fft/ntt_arithmetics.rs)
 * A polynomial is a device-resident coefficient vector owned by the library
 * (field/polynomial.rs Polynomial: never trimmed; degree() skips trailing zeros).
 * Outputs are the reference's exact vectors (same length, same values). */
typedef struct sg_poly sg_poly;
int sg_poly_create(sg_ctx* ctx, const sg_fe* coeffs, size_t len, sg_poly** out);        /* Polynomial::new */
int sg_poly_create_dev(sg_ctx* ctx, const sg_fe* d_coeffs, size_t len, sg_poly** out);
size_t sg_poly_len(const sg_poly* p);                                                     /* coefficients.len() */
const sg_fe* sg_poly_data_dev(const sg_poly* p);
int sg_poly_read(sg_ctx* ctx, const sg_poly* p, sg_fe* out);                              /* len() elements */
int sg_poly_degree(sg_ctx* ctx, const sg_poly* p, int64_t* out); /* polynomial.rs:41-58 (-1 = None) */
void sg_poly_free(sg_poly* p);
/* ntt_arithmetics.rs:5-64 fast_multiply(root, root_order, lhs, rhs) */
int sg_fast_multiply(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_poly* lhs, const sg_poly* rhs,
                     sg_poly** out);
/* ntt_arithmetics.rs:239-310 fast_coset_divide(root, root_order, offset, lhs, rhs);
 * a zero divisor value fails like the reference's "divide by zero" panic */
int sg_fast_coset_divide(sg_ctx* ctx, sg_fe root, uint64_t root_order, sg_fe offset, const sg_poly* lhs,
                         const sg_poly* rhs, sg_poly** out);
/* ntt_arithmetics.rs:66-113 fast_zerofier(root, root_order, domain): geometric domains
 * (domain[i] = root^i) in closed form on the GPU; any other domain of any size by a GPU product
 * tree (exact below root_order; above it the reference's wrapped recursion is reproduced) */
int sg_fast_zerofier(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_fe* domain, size_t n, sg_poly** out);
/* ntt_arithmetics.rs:172-237 fast_interpolate_domain(root, root_order, domain, values) */
int sg_fast_interpolate_domain(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_fe* domain,
                               const sg_fe* values, size_t n, sg_poly** out);
/* the geometric-domain forms of the two above (domain root^0 .. root^(n-1), n <= root_order) */
int sg_fast_zerofier_geometric(sg_ctx* ctx, sg_fe root, uint64_t root_order, size_t n, sg_poly** out);
int sg_fast_interpolate_geometric_dev(sg_ctx* ctx, sg_fe root, uint64_t root_order, const sg_fe* d_values,
                                      size_t n, sg_poly** out);

/* ------------------------------------------- multivariate polynomials (m_polynomial.rs)
 * MPolynomial {exponent vector: coefficient}; zero coefficients are kept as keys (the
 * STARK's degree bounds read the keys, stark.rs:117-160).  Stored grouped by the
 * register exponents (variables 1..) with a dense coefficient vector in variable 0. */
typedef struct sg_mpoly sg_mpoly;
/* MPolynomial::new(dict): nterms keys of nvars exponents each (variable 0 first) */
int sg_mpoly_create(sg_ctx* ctx, size_t nvars, size_t nterms, const uint32_t* exps, const sg_fe* coeffs,
                    sg_mpoly** out);
int sg_mpoly_constant(sg_ctx* ctx, sg_fe c, sg_mpoly** out);                            /* m_polynomial.rs:37-44 */
int sg_mpoly_variable(sg_ctx* ctx, size_t num_variables, size_t index, sg_mpoly** out); /* :49-64 variables()[i] */
int sg_mpoly_lift(sg_ctx* ctx, const sg_fe* coeffs, size_t len, size_t variable_index, sg_mpoly** out); /* :66-81 */
int sg_mpoly_lift_poly(sg_ctx* ctx, const sg_poly* p, size_t variable_index, sg_mpoly** out);
int sg_mpoly_neg(sg_ctx* ctx, const sg_mpoly* a, sg_mpoly** out);                          /* :170-181 */
int sg_mpoly_add(sg_ctx* ctx, const sg_mpoly* a, const sg_mpoly* b, sg_mpoly** out);       /* :183-222 */
int sg_mpoly_sub(sg_ctx* ctx, const sg_mpoly* a, const sg_mpoly* b, sg_mpoly** out);       /* :224-229 */
int sg_mpoly_mul(sg_ctx* ctx, const sg_mpoly* a, const sg_mpoly* b, sg_mpoly** out);       /* :231-262 */
int sg_mpoly_pow(sg_ctx* ctx, const sg_mpoly* a, sg_fe exponent, sg_mpoly** out);          /* :265-298 (u128) */
int sg_mpoly_is_zero(const sg_mpoly* a);                                                   /* :83-93 (1/0) */
int sg_mpoly_evaluate(sg_ctx* ctx, const sg_mpoly* a, const sg_fe* point, size_t n, sg_fe* out); /* :95-122 */
/* grouped view: ngroups groups of (nvars - 1 register exponents, x-vector length, coefficients) */
int sg_mpoly_shape(const sg_mpoly* a, size_t* nvars, size_t* ngroups, size_t* ncoeffs);
int sg_mpoly_export(const sg_mpoly* a, uint32_t* exps, uint64_t* lens, sg_fe* coeffs);
void sg_mpoly_free(sg_mpoly* a);

/* ------------------------------------------- Rescue-Prime (rescue_prime/rescue_prime.rs) */
typedef struct sg_rescue sg_rescue;
typedef struct {
  uint64_t cycle;
  uint64_t reg;
  sg_fe value;
} sg_boundary; /* (cycle, register, value) boundary constraint (stark.rs:279) */
int sg_rescue_create(sg_ctx* ctx, size_t m, size_t capacity, size_t security_level, size_t N,
                     sg_rescue** out); /* rescue_prime.rs:111-128 RescuePrime::new */
void sg_rescue_free(sg_rescue* rp);
/* alpha / alpha_inv exponents (u128 in an sg_fe), MDS and MDS^-1 (m x m row-major), 2 m N round constants */
int sg_rescue_info(const sg_rescue* rp, sg_fe* alpha, sg_fe* alpha_inv, sg_fe* mds, sg_fe* mds_inv,
                   sg_fe* round_constants);
int sg_rescue_hash(sg_ctx* ctx, const sg_rescue* rp, sg_fe input, sg_fe* out);   /* rescue_prime.rs:183-190 */
int sg_rescue_trace(sg_ctx* ctx, const sg_rescue* rp, sg_fe input, sg_fe* trace); /* :192-204, (N+1) x m */
/* rescue_prime.rs:206-283 transition_constraints(omicron, omicron_domain_length): m polynomials */
int sg_rescue_transition_constraints(sg_ctx* ctx, const sg_rescue* rp, sg_fe omicron,
                                     uint64_t omicron_domain_length, sg_mpoly** out);
int sg_rescue_boundary_constraints(const sg_rescue* rp, sg_fe output, sg_boundary* out); /* :285-290, 2 */

/* ------------------------------------------- STARK (stark/stark.rs) */
typedef struct sg_stark sg_stark;
/* stark.rs:71-114 Stark::new */
int sg_stark_create(sg_ctx* ctx, size_t expansion_factor, size_t num_colinearity_checks, size_t security_level,
                    size_t num_registers, size_t num_cycles, size_t transition_constraints_degree, sg_stark** out);
void sg_stark_free(sg_stark* st);
int sg_stark_params(const sg_stark* st, sg_fe* omicron, uint64_t* omicron_domain_length, sg_fri* fri,
                    size_t* num_randomizers);
/* stark.rs:171-186 max_degree (the randomizer polynomial has max_degree + 1 coefficients) */
int sg_stark_max_degree(sg_ctx* ctx, const sg_stark* st, const sg_mpoly* const* tcs, size_t ntcs, uint64_t* out);
/* stark.rs:117-160 transition_degree_bounds */
int sg_stark_degree_bounds(sg_ctx* ctx, const sg_stark* st, const sg_mpoly* const* tcs, size_t ntcs,
                           uint64_t* transition_bounds);
/* stark.rs:276-562 Stark::prove.  The thread_rng draws are explicit: trace_randomizers =
 * num_randomizers x num_registers field elements (stark.rs:285-301, row-major), then the
 * randomizer polynomial's max_degree + 1 coefficients (stark.rs:425-433).  The proof is the
 * stream's digest(); SG_ERR_INVALID with the reference's Err text where it returns Err. */
int sg_stark_prove(sg_ctx* ctx, const sg_stark* st, const sg_fe* trace, size_t rows, const sg_mpoly* const* tcs,
                   size_t ntcs, const sg_boundary* boundary, size_t nb, const sg_fe* trace_randomizers,
                   const sg_fe* randomizer_coeffs, size_t n_rc, const sg_proof_stream* ps);
/* the same with the trace, the trace randomizers and the randomizer coefficients in device memory */
int sg_stark_prove_dev(sg_ctx* ctx, const sg_stark* st, const sg_fe* d_trace, size_t rows,
                       const sg_mpoly* const* tcs, size_t ntcs, const sg_boundary* boundary, size_t nb,
                       const sg_fe* d_trace_randomizers, const sg_fe* d_randomizer_coeffs, size_t n_rc,
                       const sg_proof_stream* ps);
/* stark.rs:276-562 Stark::prove with the codeword domain sharded over the communicator (replaces
 * Stark::prove when the FRI domain is split across GPUs).  Every rank passes the same arguments
 * (st and tcs created on the communicator's context, sg_dist_ctx) and writes the same proof-stream
 * bytes as sg_stark_prove: the trace-domain algebra is replicated, the four LDEs, the three
 * commitments, FRI::prove and the openings run on run shards of N_fri / world elements.  A FRI
 * domain too small to split (sg_dist_plan fails) is proved whole by every rank. */
int sg_dist_stark_prove(sg_dist* d, const sg_stark* st, const sg_fe* trace, size_t rows, const sg_mpoly* const* tcs,
                        size_t ntcs, const sg_boundary* boundary, size_t nb, const sg_fe* trace_randomizers,
                        const sg_fe* randomizer_coeffs, size_t n_rc, const sg_proof_stream* ps);
int sg_dist_stark_prove_dev(sg_dist* d, const sg_stark* st, const sg_fe* d_trace, size_t rows,
                            const sg_mpoly* const* tcs, size_t ntcs, const sg_boundary* boundary, size_t nb,
                            const sg_fe* d_trace_randomizers, const sg_fe* d_randomizer_coeffs, size_t n_rc,
                            const sg_proof_stream* ps);

#ifdef __cplusplus
}
#endif
#endif /* STARK_GPU_H */
