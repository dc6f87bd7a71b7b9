"""A mid-size `Stark::prove` pinned to the Python oracle itself (round-5 verdict, missing #5): the
statement sits between the reference's published RPSSS configuration (T = 284, FRI domain 4096,
tests/rpsss_case.py) and the full-size cases, which are held only to the CPU checker
(oracle/fast_cpu.cpp).

Rescue-Prime `RescuePrime::new(field, 2, 1, 128, N = 1000)` (rescue_prime/rescue_prime.rs:107-114,
trace :194-204) under `Stark::new(field, 8, 64, 128, m = 2, N + 1, 3)` (stark/stark.rs:71-114):
trace T = 1001 + 4 * 64 = 1257 rows, omicron domain 2^bitlen(3 T) = 4096, FRI domain 2^15,
expansion 8, 64 colinearity checks, transition degree 3, an IndependentProofStream.  The
`thread_rng` draws (stark.rs:286-301, 425-433) come from a seeded SHAKE256 stream
(stark_prove_oracle.randomness_from_seed), the secret input from `Field::sample` of a seeded
SHAKE256 output.

TEST INFRASTRUCTURE (tests/ only).  `tests/golden/make_midsize.py` runs the oracle's prove once in
the build container (a few minutes of Python) and commits the proof's length and SHA-256 in
`tests/golden/midsize_proof.json`; the GPU test and the CPU-checker test compare against that digest.
"""
import stark_oracle as o
import stark_prove_oracle as e

RESCUE = (2, 1, 128, 1000)          # m, capacity, security level, N (rescue_prime.rs:107)
EXPANSION, CHECKS, SECURITY, TCD = 8, 64, 128, 3
SEED = b"midsize"
OMICRON_DOMAIN, FRI_DOMAIN = 4096, 1 << 15


def inputs(seed: bytes = SEED):
    """(rp, st, air, trace, boundary, trace_randomizers, randomizer_coefficients), oracle objects."""
    rp = e.RescuePrime(*RESCUE)
    st = e.Stark(EXPANSION, CHECKS, SECURITY, rp.m, rp.N + 1, TCD)
    assert (st.omicron_domain_length, st.omicron_domain_length * EXPANSION) == (OMICRON_DOMAIN, FRI_DOMAIN)
    air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
    secret = o.sample(o.shake256(b"midsize-input" + seed, 17))
    m = rp.m
    nrc = st.num_randomizer_coefficients(air)
    r = e.randomness_from_seed(seed, m * st.num_randomizers + nrc)
    tr = [r[m * i:m * i + m] for i in range(st.num_randomizers)]
    return rp, st, air, rp.trace(secret), rp.boundary_constraints(rp.hash(secret)), tr, r[m * st.num_randomizers:]


def light_inputs(seed: bytes = SEED):
    """The same statement without the oracle's expanded AIR (O(N^2) Python to build): the randomizer
    count comes from the AIR's key structure (stark_prove_oracle.RescueAirAtPoint, whose degree
    bounds equal the expanded AIR's -- tests/test_oracle_fast.py).  Returns
    (rp, st, trace, boundary, trace_randomizers, randomizer_coefficients)."""
    rp = e.RescuePrime(*RESCUE)
    st = e.Stark(EXPANSION, CHECKS, SECURITY, rp.m, rp.N + 1, TCD)
    sair = [e.RescueAirAtPoint(rp, i, None) for i in range(rp.m)]
    secret = o.sample(o.shake256(b"midsize-input" + seed, 17))
    m = rp.m
    nrc = st.max_degree(sair) + 1
    r = e.randomness_from_seed(seed, m * st.num_randomizers + nrc)
    tr = [r[m * i:m * i + m] for i in range(st.num_randomizers)]
    return rp, st, rp.trace(secret), rp.boundary_constraints(rp.hash(secret)), tr, r[m * st.num_randomizers:]

