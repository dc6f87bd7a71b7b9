"""The optimized CPU checker (oracle/fast_cpu.cpp: Montgomery, OpenMP) agrees with the
reference's known-answer vectors and with the Python restatement, so it
can stand in for the oracle at sizes Python cannot reach (2^22..2^27 transforms, 2^24
FRI proofs, trace-2^20 verification)."""
import os
import subprocess

import numpy as np
import pytest

import stark_oracle as o
import stark_prove_oracle as e

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fc():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    import fast_cpu
    return fast_cpu


def test_fast_checker_kats(fc, kats):
    for v in kats["ntt"]:
        root = o.primitive_nth_root(v["n"])
        assert fc.ints(fc.ntt(root, [int(x) for x in v["input"]])) == [int(x) for x in v["output"]], v["src"]
    for v in kats["intt"]:
        root = o.primitive_nth_root(v["n"])
        assert fc.ints(fc.intt(root, [int(x) for x in v["input"]])) == [int(x) for x in v["output"]], v["src"]
    for v in kats["merkle_commit"]:
        assert fc.merkle_commit([int(x) for x in v["leaves"]]).hex() == v["root_hex"], v["src"]
    for v in kats["blake2b512"]:
        assert fc.blake2b512(bytes.fromhex(v["in_hex"])).hex() == v["out_hex"], v["src"]
    for v in kats["fe_mul"]:
        a, b = fc.arr([int(v["a"])]), fc.arr([int(v["b"])])
        out = fc.arr([0])
        fc.lib().fc_mul(fc._p(a), fc._p(b), fc._p(out))
        assert fc.ints(out)[0] == int(v["out"]), v["src"]
    for v in kats["fe_inverse"]:
        a, out = fc.arr([int(v["a"])]), fc.arr([0])
        fc.lib().fc_inv(fc._p(a), fc._p(out))
        assert fc.ints(out)[0] == int(v["out"]), v["src"]
    # SHAKE256 vs hashlib over rate-boundary lengths (the KATs' inputs are Debug strings)
    import hashlib
    for n in (0, 1, 135, 136, 137, 300):
        d = bytes(range(256)) * 2
        assert fc.shake256(d[:n], 77) == hashlib.shake_256(d[:n]).digest(77)
    for n in (0, 1, 127, 128, 129, 300):
        d = bytes((7 * i) & 255 for i in range(n))
        assert fc.blake2b512(d) == hashlib.blake2b(d, digest_size=64).digest()


@pytest.mark.parametrize("logn", [0, 1, 2, 5, 10, 12, 13, 14])
def test_fast_ntt_matches_oracle(fc, logn):
    n = 1 << logn
    x = o.synthetic_elements(logn, b"fast", n)
    w = o.primitive_nth_root(n)
    assert fc.ints(fc.ntt(w, x)) == o.ntt(w, x)
    if n >= 2:
        assert fc.ints(fc.intt(w, x)) == o.intt(w, x)
        # zero padding (ntt.rs:14 bit_reverse_copy) and a non-primitive root (same DIT graph)
        assert fc.ints(fc.ntt(w, x[: n // 2 + 1])) == o.ntt(w, x[: n // 2 + 1])
        w2 = o.fpow(w, 2)
        assert fc.ints(fc.ntt(w2, x)) == o.ntt(w2, x)
    d = max(n // 8, 1)
    assert fc.ints(fc.fast_coset_evaluate(w, n, o.GENERATOR, x[:d])) == o.fast_coset_evaluate(w, n, o.GENERATOR, x[:d])
    assert fc.merkle_commit(x) == o.merkle_commit(x)


def test_fast_edge_values(fc):
    n = 1 << 10
    w = o.primitive_nth_root(n)
    for x in ([0] * n, [o.P - 1] * n, [1] + [0] * (n - 1), [0] * (n - 1) + [1]):
        assert fc.ints(fc.ntt(w, x)) == o.ntt(w, x)
        assert fc.merkle_commit(x) == o.merkle_commit(x)
    assert fc.ints(fc.intt(w, [5])) == [5]  # ntt.rs:55-57: fewer than two elements unchanged


@pytest.mark.parametrize("n,exp,c", [(1 << 11, 8, 16), (1 << 12, 4, 17), (1 << 13, 8, 64)])
def test_fast_fri_prove_stream(fc, n, exp, c):
    w = o.primitive_nth_root(n)
    cw = o.fast_coset_evaluate(w, n, o.GENERATOR, o.synthetic_elements(3, b"fri", n // exp))
    prefix = [(o.ROOT, bytes(range(64)))]
    ps = o.IndependentProofStream(prefix)
    top = o.FRI(o.GENERATOR, w, n, exp, c).prove(cw, ps)
    data, ftop = fc.fri_prove(o.GENERATOR, w, cw, exp, c, prefix=o.serialize(prefix))
    assert ftop == top
    assert data == ps.digest()


def test_fast_barycentric_and_zerofier(fc):
    q = o.primitive_nth_root(1 << 8)
    n = 100
    cols = [o.synthetic_elements(1, b"c1", n), o.synthetic_elements(2, b"c2", n)]
    xs = [o.GENERATOR, 12345, o.fpow(q, 150), o.fpow(q, 7)]  # off-domain points, then a node q^7
    bary = e.GeometricBarycentric(q, n, {0: cols[0], 1: cols[1]})
    got = fc.geometric_bary(q, cols, xs)
    for j, x in enumerate(xs[:3]):
        assert got[j] == [bary.value(x, 0), bary.value(x, 1)]
    assert got[3] == [cols[0][7], cols[1][7]]  # at a node the interpolant takes the node's value
    dom = [o.fpow(q, r) for r in range(n)]
    for x, z in zip(xs, fc.geometric_prod(q, n, xs)):
        want = 1
        for d in dom:
            want = want * (x - d) % o.P
        assert z == want


def test_fast_barycentric_handle(fc):
    q = o.primitive_nth_root(1 << 9)
    n = 300
    cols = {"a": o.synthetic_elements(4, b"a", n), "b": o.synthetic_elements(5, b"b", n)}
    ref = e.GeometricBarycentric(q, n, cols)
    fast = fc.Barycentric(q, n, {k: fc.arr(v) for k, v in cols.items()})
    for x in (o.GENERATOR, 777, o.fpow(o.GENERATOR, 5)):
        for k in cols:
            assert fast.value(x, k) == ref.value(x, k)


def test_fast_verifier_pieces_verify_oracle_proof(fc):
    """The accelerated verifier pieces the trace-2^20 GPU test uses (Rescue AIR at a point with
    C++ barycentric interpolants, transition zerofier by C++ products) accept a proof made by the
    oracle prover at the reference test's size (stark.rs:823-840) and reject a false claim."""
    rp = e.RescuePrime(2, 1, 2, 27)
    st = e.Stark(4, 2, 2, 2, 28, 2)
    air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
    inp = o.sample(b"fastverify")
    out = rp.hash(inp)
    trace, bnd = rp.trace(inp), rp.boundary_constraints(out)
    r = e.randomness_from_seed(b"fv", 2 * st.num_randomizers + st.num_randomizer_coefficients(air))
    tr = [r[2 * i:2 * i + 2] for i in range(st.num_randomizers)]
    rc = r[2 * st.num_randomizers:]
    ps = o.IndependentProofStream()
    st.prove(trace, air, bnd, ps, tr, rc)
    vst = fc.verifier_stark(4, 2, 2, 2, 28, 2)
    sair = fc.rescue_air_at_point(rp, vst.omicron)
    assert vst.transition_degree_bounds(sair) == st.transition_degree_bounds(air)
    ok, err = vst.verify(sair, bnd, o.IndependentProofStream(ps.objects))
    assert ok, err
    ok, _ = vst.verify(sair, rp.boundary_constraints(o.add_mod(out, 1)), o.IndependentProofStream(ps.objects))
    assert not ok


def test_fast_cpu_arbitrary_domain_checkers_vs_oracle(fc):
    """The O(n^2) exact product and the Horner evaluator the arbitrary-domain GPU tests check
    against agree with the oracle's fast_zerofier / fast_interpolate_domain recursion."""
    import random
    rng = random.Random(5)
    for n in (1, 2, 7, 33, 100):
        dom = [rng.randrange(o.P) for _ in range(n)]
        vals = [rng.randrange(o.P) for _ in range(n)]
        w = o.primitive_nth_root(256)
        assert fc.ints(fc.poly_from_roots(dom)) == e.fast_zerofier(w, 256, dom)
        ip = e.fast_interpolate_domain(w, 256, dom, vals)
        assert fc.ints(fc.eval_points(ip, dom)) == vals


# --------------------------------------------------------- Stark::prove (the end-to-end checker)

def _rescue_case(N, exp, c, sec, tcd, seed, m=2):
    rp = e.RescuePrime(m, 1, sec, N)
    st = e.Stark(exp, c, sec, m, N + 1, tcd)
    air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
    inp = o.sample(seed)
    nrc = st.num_randomizer_coefficients(air)
    r = e.randomness_from_seed(seed, m * st.num_randomizers + nrc)
    tr = [r[m * i:m * i + m] for i in range(st.num_randomizers)]
    return rp, st, air, rp.trace(inp), rp.boundary_constraints(rp.hash(inp)), tr, r[m * st.num_randomizers:]


def test_fast_geometric_interpolation_and_zerofier_vs_oracle(fc):
    """The checker's building blocks against fast_interpolate_domain / fast_zerofier
    (ntt_arithmetics.rs:66-113, 172-237) on prefixes of <q>: the same coefficient vectors."""
    D = 128
    q = o.primitive_nth_root(D)
    for n in (1, 2, 3, 17, 64, 100, 127, 128):
        vals = o.synthetic_elements(n, b"geo", n)
        dom = [o.fpow(q, i) for i in range(n)]
        assert fc.ints(fc.geo_interpolate(q, D, vals)) == e.fast_interpolate_domain(q, D, dom, vals), n
        if n < D:
            assert fc.ints(fc.geo_zerofier(q, n)) == e.fast_zerofier(q, D, dom), n


@pytest.mark.parametrize("N,exp,c,sec,tcd", [(27, 4, 2, 2, 2), (27, 8, 4, 8, 3), (40, 4, 3, 4, 2), (9, 16, 2, 4, 4)])
def test_fast_stark_prove_equals_oracle(fc, N, exp, c, sec, tcd):
    """stark.rs:276-562: the CPU checker's proof bytes equal the oracle's (the GPU tests' parameter
    sets; (40, 4, 3, 4, 2) has max_degree >= the omicron order, where the reference's products wrap),
    and its degree bounds (from the AIR's key structure) equal the expanded AIR's."""
    rp, st, air, trace, bnd, tr, rc = _rescue_case(N, exp, c, sec, tcd, b"case-%d" % N)
    want = st.prove(trace, air, bnd, o.IndependentProofStream(), tr, rc)
    bounds = fc.rescue_degree_bounds(rp, st)
    assert bounds == (st.transition_quotient_degree_bounds(air), st.max_degree(air))
    assert fc.stark_prove_rescue(rp, st, trace, bnd, tr, rc) == want


def test_fast_stark_prove_false_witness_and_errors(fc):
    """stark.rs:845-880 false witnesses (inexact transition division: the reference's truncated
    quotient) give the oracle's bytes; the reference's Err / panics map to ValueError."""
    for (N, exp, c, sec, tcd, seed, row, reg, delta) in (
            (27, 4, 2, 2, 2, b"bad", 22, 1, 17274817952119230544216945715808633996),
            (40, 4, 3, 4, 2, b"factored-air", 17, 0, 5)):
        rp, st, air, trace, bnd, tr, rc = _rescue_case(N, exp, c, sec, tcd, seed)
        bad = [list(r) for r in trace]
        bad[row][reg] = o.add_mod(bad[row][reg], delta)
        assert fc.stark_prove_rescue(rp, st, bad, bnd, tr, rc) == \
            st.prove(bad, air, bnd, o.IndependentProofStream(), tr, rc)
    with pytest.raises(ValueError, match="max_degree"):
        fc.stark_prove_rescue(rp, st, trace, bnd, tr, rc[:-1])


def test_fast_stark_prove_rpsss_published_configuration(fc):
    """The reference's published end-to-end fixture (rpsss.rs:89,103,113-131; tests/rpsss_case.py):
    RPSSS::new(field, 4, 64, 128, 3) signing b"Hello, World!" through a SignatureProofStream.
    The CPU checker (with the stream's Fiat-Shamir prefix) writes the oracle's bytes, the length is
    the reference's 1 156 888, the oracle verifier accepts the document and rejects the forgery,
    and the bytes are the committed golden digest (tests/golden/make_rpsss.py)."""
    import hashlib
    import json
    import rpsss_case as R
    with open(os.path.join(ROOT, "tests", "golden", "rpsss_published.json")) as f:
        g = json.load(f)
    c = R.Case(g["seed"].encode())
    assert (c.sk, c.pk) == (int(g["sk"]), int(g["pk"]))
    want = c.oracle_sign()
    assert len(want) == R.PROOF_LEN == g["proof_len"], "rpsss.rs:89"
    assert hashlib.sha256(want).hexdigest() == g["proof_sha256"]
    got = fc.stark_prove_rescue(c.rp, c.st, c.trace, c.boundary, c.trace_randomizers,
                                c.randomizer_coefficients, document=R.DOCUMENT)
    assert got == want
    # an IndependentProofStream's Fiat-Shamir draws differ: same length, different bytes
    plain = fc.stark_prove_rescue(c.rp, c.st, c.trace, c.boundary, c.trace_randomizers, c.randomizer_coefficients)
    assert len(plain) == len(want) and plain != want
    assert c.oracle_verify(R.DOCUMENT, want) == (True, "")
    ok, err = c.oracle_verify(R.FORGED, want)
    assert not ok, "rpsss.rs:127-131"
    assert o.serialize(o.deserialize(want)) == want


def test_fast_stark_prove_midsize_equals_oracle_digest(fc):
    """The CPU checker on the mid-size statement pinned to the Python oracle (tests/midsize_case.py:
    trace 1257 rows, FRI domain 2^15, c = 64): its proof bytes hash to the oracle's committed digest
    (tests/golden/midsize_proof.json, tests/golden/make_midsize.py), the link between the
    published-configuration pin (FRI domain 4096) and the checker's full-size use."""
    import hashlib
    import json
    import midsize_case as M
    with open(os.path.join(ROOT, "tests", "golden", "midsize_proof.json")) as f:
        g = json.load(f)
    rp, st, trace, bnd, tr, rc = M.light_inputs()
    got = fc.stark_prove_rescue(rp, st, trace, bnd, tr, rc)
    assert len(got) == g["proof_len"]
    assert hashlib.sha256(got).hexdigest() == g["proof_sha256"]


def test_fast_cpu_fullsize_equals_python_oracle_digests(fc):
    """The CPU checker at BASELINE's full sizes against the Python oracle itself: C2 (2^22 NTT and a
    ragged input, fft/ntt.rs:7-68) and C3 (LDE 2^21 -> 2^24 + FRI::prove, fri.rs:210-248) hash to the
    digests tests/golden/make_fullsize.py computed with oracle/stark_oracle.py (~16 s here)."""
    import hashlib
    import json
    import os
    G = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_digests.json")))

    def d(a):
        return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()

    n = 1 << 22
    root = o.primitive_nth_root(n)
    x = _synth_np(b"c2", n)
    assert d(x) == G["c2"]["input"]["sha256"]
    assert d(fc.ntt(root, x)) == G["c2"]["ntt"]["sha256"]
    assert d(fc.ntt(root, x[: n - 5])) == G["c2"]["ragged_ntt_n_minus_5"]["sha256"]
    N = 1 << 24
    w = o.primitive_nth_root(N)
    coeffs = _synth_np(b"c3", N // 8)
    assert d(coeffs) == G["c3"]["coeffs"]["sha256"]
    cw = fc.fast_coset_evaluate(w, N, o.GENERATOR, coeffs)
    assert d(cw) == G["c3"]["lde"]["sha256"]
    proof, top = fc.fri_prove(o.GENERATOR, w, cw, 8, 64)
    assert len(proof) == G["c3"]["proof_len"] and hashlib.sha256(proof).hexdigest() == G["c3"]["proof_sha256"]
    assert list(top) == G["c3"]["top_indices"]


def _synth_np(tag: bytes, n: int) -> np.ndarray:
    """o.synthetic_elements(0, tag, n) as an (n, 2) u64 array, vectorized (one conditional subtraction
    of p: a 128-bit value is < 2p)."""
    import hashlib
    P = o.P
    raw = hashlib.shake_256(b"sg-bench" + (0).to_bytes(8, "big") + tag).digest(16 * n)
    be = np.frombuffer(raw, dtype=">u8").reshape(n, 2)
    hi, lo = be[:, 0].astype(np.uint64), be[:, 1].astype(np.uint64)
    p_hi, p_lo = np.uint64(P >> 64), np.uint64(P & (2**64 - 1))
    ge = (hi > p_hi) | ((hi == p_hi) & (lo >= p_lo))
    borrow = (lo < p_lo) & ge
    lo = np.where(ge, lo - p_lo, lo)
    hi = np.where(ge, hi - p_hi - borrow.astype(np.uint64), hi)
    return np.ascontiguousarray(np.stack([lo, hi], axis=1))
