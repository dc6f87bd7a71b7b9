/*
 * prove_rescue.c -- a compiled host calling libstarkgpu through its C ABI only (no Python, no
 * torch): what the reference crate's Stark::prove (stark/stark.rs:276-562) does for the
 * Rescue-Prime signature statement (rescue_prime/rescue_prime.rs, stark.rs:823-840), with the
 * two thread_rng draws read from a file so the bytes can be compared with another prover's.
 *
 *   prove_rescue N expansion colinearity security tcd input_lo input_hi randomness.bin proof.bin
 *                [--dist id_file rank nranks [nonce]] [--document text]
 *
 * With --document the proof goes through a SignatureProofStream of that document
 * (rescue_prime/proof_stream.rs:9-52: every Fiat-Shamir draw is prefixed by blake2b(document)):
 * RPSSS::sign (rpsss.rs:74-78), e.g. the reference's published configuration
 * `27 4 64 128 3 ... --document "Hello, World!"` (rpsss.rs:103-108, 1 156 888 bytes).
 *
 * With --dist the proof is computed with the FRI domain sharded over `nranks` processes, one GPU
 * each (sg_dist_stark_prove over RCCL, rank r on GPU r): rank 0 writes the RCCL unique id to
 * id_file, the other ranks wait for it; every rank writes the same bytes.  `nonce` (any 64-bit
 * number the launcher picks per run and passes to every rank) is written before the id, and the
 * other ranks accept only a file carrying it: an id file left over from an earlier run is never
 * read as this run's id.  With nranks > 1 the nonce is required (a missing or zero nonce is a
 * usage error).
 *
 * randomness.bin: 16-byte little-endian (lo, hi) field elements -- num_randomizers x 2 trace
 * randomizer rows (stark.rs:285-301), then max_degree + 1 randomizer coefficients
 * (stark.rs:425-433).  proof.bin receives the proof stream's digest() (stark.rs:562).
 * Prints "proof <bytes> num_randomizers <r> randomizer_coefficients <k> fri_domain <n>".
 * Exit status 0 on success; 2 when randomness.bin is too short (it prints how many elements
 * it needs first, so a caller can size the file); 1 on any library error.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "stark_gpu.h"

#define CHECK(call)                                                                      \
  do {                                                                                   \
    int rc_ = (call);                                                                    \
    if (rc_ != 0) {                                                                      \
      fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, ctx ? sg_last_error(ctx) : ""); \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

int main(int argc, char** argv) {
  int dist = 0, bad = argc < 10;
  const char *id_path = NULL, *document = NULL;
  int rank = 0, nranks = 1;
  uint64_t nonce = 0;
  for (int i = 10; i < argc && !bad;) {
    if (strcmp(argv[i], "--document") == 0 && i + 1 < argc) {
      document = argv[i + 1];
      i += 2;
    } else if (strcmp(argv[i], "--dist") == 0 && i + 3 < argc) {
      dist = 1;
      id_path = argv[i + 1];
      rank = atoi(argv[i + 2]);
      nranks = atoi(argv[i + 3]);
      i += 4;
      if (i < argc && strncmp(argv[i], "--", 2) != 0) nonce = strtoull(argv[i++], NULL, 0);
    } else {
      bad = 1;
    }
  }
  if (dist && nranks > 1 && nonce == 0) {
    /* the nonce is what keeps a stale id file from an earlier run from being read as this run's */
    fprintf(stderr, "--dist with nranks > 1 needs a non-zero nonce (the same on every rank)\n");
    bad = 1;
  }
  if (bad) {
    fprintf(stderr,
            "usage: %s N expansion colinearity security tcd input_lo input_hi randomness.bin proof.bin"
            " [--dist id_file rank nranks [nonce]] [--document text]\n",
            argv[0]);
    return 1;
  }
  const size_t N = strtoull(argv[1], NULL, 10), exp = strtoull(argv[2], NULL, 10);
  const size_t c = strtoull(argv[3], NULL, 10), sec = strtoull(argv[4], NULL, 10);
  const size_t tcd = strtoull(argv[5], NULL, 10);
  const sg_fe input = {strtoull(argv[6], NULL, 0), strtoull(argv[7], NULL, 0)};
  sg_ctx* ctx = NULL;
  CHECK(sg_ctx_create(dist ? rank : 0, &ctx));  /* one GPU per rank of the node */
  sg_dist* comm = NULL;
  if (dist) {
    uint8_t id[SG_DIST_ID_BYTES];
    if (rank == 0) {
      CHECK(sg_dist_unique_id(id));
      char tmp[4096];
      snprintf(tmp, sizeof tmp, "%s.tmp", id_path);
      FILE* f = fopen(tmp, "wb");
      if (!f || fwrite(&nonce, 1, sizeof nonce, f) != sizeof nonce || fwrite(id, 1, sizeof id, f) != sizeof id ||
          fclose(f) != 0 || rename(tmp, id_path) != 0) {
        fprintf(stderr, "cannot write %s\n", id_path);
        return 1;
      }
    } else {
      int have = 0;
      for (int tries = 0; tries < 6000 && !have; ++tries) {  /* up to 60 s for rank 0 */
        FILE* f = fopen(id_path, "rb");
        uint64_t got = 0;
        if (f) {
          have = fread(&got, 1, sizeof got, f) == sizeof got && got == nonce && fread(id, 1, sizeof id, f) == sizeof id;
          fclose(f);
        }
        if (!have) {
          struct timespec ts = {0, 10000000};
          nanosleep(&ts, NULL);
        }
      }
      if (!have) {
        fprintf(stderr, "no id for this run (nonce %llu) in %s\n", (unsigned long long)nonce, id_path);
        return 1;
      }
    }
    CHECK(sg_dist_create(ctx, id, nranks, rank, &comm));
  }
  sg_rescue* rp = NULL;
  CHECK(sg_rescue_create(ctx, 2, 1, sec, N, &rp));  /* RescuePrime::new(m = 2, capacity 1, ...) */
  sg_fe output;
  CHECK(sg_rescue_hash(ctx, rp, input, &output));
  sg_fe* trace = malloc((N + 1) * 2 * sizeof(sg_fe));
  CHECK(sg_rescue_trace(ctx, rp, input, trace));
  sg_boundary bnd[2];
  CHECK(sg_rescue_boundary_constraints(rp, output, bnd));
  sg_stark* st = NULL;
  CHECK(sg_stark_create(ctx, exp, c, sec, 2, N + 1, tcd, &st));
  sg_fe omicron;
  uint64_t D = 0;
  sg_fri fri;
  size_t nr = 0;
  CHECK(sg_stark_params(st, &omicron, &D, &fri, &nr));
  sg_mpoly* tcs[2] = {NULL, NULL};
  CHECK(sg_rescue_transition_constraints(ctx, rp, omicron, D, tcs));
  uint64_t md = 0;
  CHECK(sg_stark_max_degree(ctx, st, (const sg_mpoly* const*)tcs, 2, &md));
  const size_t nrc = (size_t)md + 1, need = 2 * nr + nrc;
  printf("needs %zu randomness elements\n", need);
  FILE* f = fopen(argv[8], "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", argv[8]);
    return 1;
  }
  sg_fe* rnd = malloc(need * sizeof(sg_fe));
  const size_t got = fread(rnd, sizeof(sg_fe), need, f);
  fclose(f);
  if (got != need) {
    fprintf(stderr, "%s holds %zu elements, %zu needed\n", argv[8], got, need);
    return 2;
  }
  sg_stream* s = document ? sg_stream_create_signature((const uint8_t*)document, strlen(document))
                          : sg_stream_create();
  const sg_proof_stream cb = sg_stream_callbacks(s);
  if (comm)
    CHECK(sg_dist_stark_prove(comm, st, trace, N + 1, (const sg_mpoly* const*)tcs, 2, bnd, 2, rnd, rnd + 2 * nr, nrc,
                              &cb));
  else
    CHECK(sg_stark_prove(ctx, st, trace, N + 1, (const sg_mpoly* const*)tcs, 2, bnd, 2, rnd, rnd + 2 * nr, nrc,
                         &cb));
  size_t len = 0;
  CHECK(sg_stream_digest(s, NULL, 0, &len));
  uint8_t* proof = malloc(len);
  CHECK(sg_stream_digest(s, proof, len, &len));
  FILE* o = fopen(argv[9], "wb");
  if (!o || fwrite(proof, 1, len, o) != len) {
    fprintf(stderr, "cannot write %s\n", argv[9]);
    return 1;
  }
  fclose(o);
  printf("proof %zu num_randomizers %zu randomizer_coefficients %zu fri_domain %llu\n", len, nr, nrc,
         (unsigned long long)fri.domain_length);
  free(proof);
  free(rnd);
  free(trace);
  sg_stream_destroy(s);
  sg_mpoly_free(tcs[0]);
  sg_mpoly_free(tcs[1]);
  sg_stark_free(st);
  sg_rescue_free(rp);
  if (comm) sg_dist_destroy(comm);
  sg_ctx_destroy(ctx);
  return 0;
}
