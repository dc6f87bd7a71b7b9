"""The reference's one published end-to-end fixture: the Rescue-Prime STARK signature scheme at
`RPSSS::new(field, 4, 64, 128, 3)` (/root/reference/src/rpsss.rs:103), i.e. Rescue-Prime
`RescuePrime::new(field, 2, 1, 128, 27)` (rpsss.rs:23) under `Stark::new(field, 4, 64, 128, m = 2,
N + 1 = 28, 3)` (rpsss.rs:24-33): 256 randomizer rows, omicron domain 1024, FRI domain 4096,
64 colinearity checks, signed through a `SignatureProofStream(b"Hello, World!")`
(rpsss.rs:75-78, rescue_prime/proof_stream.rs:9-52).  The reference pins the signature's size at
1 156 888 bytes (rpsss.rs:89) and checks that it verifies for the document and not for
b"Malicious document" (rpsss.rs:113-131).

TEST INFRASTRUCTURE (tests/ and bench.py's side leg only).  The three `thread_rng` draws --
keygen's 17 bytes (rpsss.rs:66-72) and `Stark::prove`'s trace randomizers / randomizer
coefficients (stark.rs:286-301, 425-433) -- come from seeded SHAKE256 streams so the GPU, the
oracle and the CPU checker see the same inputs.
"""
import stark_oracle as o
import stark_prove_oracle as e

EXPANSION, CHECKS, SECURITY, TCD = 4, 64, 128, 3   # rpsss.rs:103
RESCUE = (2, 1, SECURITY, 27)                      # rpsss.rs:23
DOCUMENT = b"Hello, World!"                        # rpsss.rs:108
FORGED = b"Malicious document"                     # rpsss.rs:127
PROOF_LEN = 1156888                                # rpsss.rs:89


class Case:
    """keygen + the inputs of `RPSSS::stark_prove` (rpsss.rs:37-50), oracle objects."""

    def __init__(self, seed: bytes = b"rpsss"):
        self.rp = e.RescuePrime(*RESCUE)
        self.st = e.Stark(EXPANSION, CHECKS, SECURITY, self.rp.m, self.rp.N + 1, TCD)
        self.sk = o.sample(o.shake256(b"rpsss-keygen" + seed, 17))   # rpsss.rs:66-72
        self.pk = self.rp.hash(self.sk)
        self.air = self.rp.transition_constraints(self.st.omicron, self.st.omicron_domain_length)
        self.trace = self.rp.trace(self.sk)
        self.boundary = self.rp.boundary_constraints(self.pk)
        m = self.rp.m
        nrc = self.st.num_randomizer_coefficients(self.air)
        r = e.randomness_from_seed(seed, m * self.st.num_randomizers + nrc)
        self.trace_randomizers = [r[m * i:m * i + m] for i in range(self.st.num_randomizers)]
        self.randomizer_coefficients = r[m * self.st.num_randomizers:]

    def oracle_sign(self, document: bytes = DOCUMENT) -> bytes:
        """RPSSS::sign (rpsss.rs:74-78) through the oracle's Stark.prove."""
        return self.st.prove(self.trace, self.air, self.boundary, o.SignatureProofStream(document),
                             self.trace_randomizers, self.randomizer_coefficients)

    def oracle_verify(self, document: bytes, signature: bytes):
        """RPSSS::verify (rpsss.rs:80-85): (ok, error)."""
        sps = o.SignatureProofStream(document, o.deserialize(signature))
        return self.st.verify(self.air, self.rp.boundary_constraints(self.pk), sps)
