"""CPU-side checks of the C ABI: the library loads, exports every symbol the
header declares, and its host-only logic (field constants, transcript,
sample_indices, Merkle verify) matches the oracle.  No GPU compute here."""
import os
import re

import stark_oracle as o
import starkgpu as sg
from starkgpu import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "stark_gpu.h")).read()
    return sorted(set(re.findall(r"\b(sg_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol():
    lib = sg.lib()
    syms = header_symbols()
    assert len(syms) >= 40
    for s in syms:
        assert hasattr(lib, s), f"libstarkgpu.so does not export {s}"
    assert set(syms) == set(_lib.PROTOTYPES), "ctypes prototypes out of sync with the header"


def test_one_rccl_and_one_hip_runtime_in_a_torch_process():
    """libstarkgpu's NEEDED librccl.so.1 / libamdhip64.so.7 carry the same sonames as the copies
    torch ships; loaded after torch (starkgpu._lib does that), the loader reuses torch's, so the
    library's communicator and torch.distributed's share one RCCL and one HIP runtime."""
    sg.lib()
    for tag in ("librccl", "libamdhip64"):
        paths = {line.split()[-1] for line in open("/proc/self/maps") if tag in line and "/" in line}
        assert len(paths) <= 1, f"{tag} mapped from more than one file: {paths}"


def test_host_field_matches_oracle(kats):
    assert sg.generator() == o.GENERATOR
    for v in kats["fe_mul"]:
        assert sg.fe_mul(int(v["a"]), int(v["b"])) == int(v["out"]), v["src"]
    for v in kats["fe_div"]:
        assert sg.fe_mul(int(v["a"]), sg.fe_inverse(int(v["b"]))) == int(v["out"]), v["src"]
    for v in kats["fe_pow"]:
        assert sg.fe_pow(int(v["a"]), int(v["e"])) == int(v["out"]), v["src"]
    for v in kats["primitive_nth_root"]:
        assert sg.primitive_nth_root(int(v["n"])) == int(v["out"]), v["src"]
    for v in kats["sample"]:
        assert sg.sample(bytes.fromhex(v["bytes_hex"])) == int(v["out"]), v["src"]
    assert sg.fe_inverse(0) == 0
    for x in o.synthetic_elements(1, b"inv", 50):
        assert sg.fe_inverse(x) == o.inv(x)
        assert sg.fe_mul(x, x) == o.mul_mod(x, x)


def test_host_sample_indices(kats):
    for v in kats["fri_sample_indices"]:
        assert sg.FRI.sample_indices(bytes.fromhex(v["seed_hex"]), v["size"], v["reduced_size"],
                                     v["number"]) == v["out"], v["src"]
    seed = o.shake256(b"seed", 32)
    f = o.FRI(o.GENERATOR, o.primitive_nth_root(1 << 12), 1 << 12, 8, 64)
    assert sg.FRI.sample_indices(seed, 2048, 512, 64) == f.sample_indices(seed, 2048, 512, 64)


def test_host_merkle_verify(kats):
    path = [bytes.fromhex(h) for h in kats["merkle_verify_path_hex"]]
    for v in kats["merkle_verify"]:
        assert sg.MerkleRoot.verify(bytes.fromhex(v["root_hex"]), v["index"], path, int(v["leaf"])) == v["expect"]


def test_host_transcript_matches_oracle():
    objs = [(o.ROOT, bytes(range(64))), (o.ROOT, bytes(64)), (o.CODEWORD, [3, o.P - 1]),
            (o.PATH, [bytes([1] * 64)]), (o.LEAFS, (7, 8, 9)), (o.VALUE, 11)]
    s = sg.IndependentProofStream()
    ostream = o.IndependentProofStream()
    for k, ob in enumerate(objs):
        s.push(ob)
        ostream.push(ob)
        assert s.digest() == ostream.digest()
        assert s.fiat_shamir_prover(32) == ostream.fiat_shamir_prover(32)
    assert s.pull() == objs[0]
    ostream.pull()
    assert s.fiat_shamir_verifier(64) == ostream.fiat_shamir_verifier(64)
    back = sg.IndependentProofStream.deserialize(s.digest())
    assert back.objects() == objs
    # an empty IndependentProofStream digests to a 16-byte zero field header
    assert sg.IndependentProofStream().digest() == bytes(16)


def test_host_transcript_long_streams_match_oracle():
    """Streams past several sponge blocks and arena growth steps, both stream kinds,
    repeated so released arenas are reused (proof_stream.rs:15-78, rescue_prime/proof_stream.rs:9-61)."""
    import random
    rng = random.Random(7)

    def rand_obj():
        k = rng.randrange(5)
        if k == 0:
            return (o.ROOT, rng.randbytes(64))
        if k == 1:
            return (o.PATH, [rng.randbytes(64) for _ in range(rng.randrange(1, 12))])
        if k == 2:
            return (o.CODEWORD, [rng.randrange(o.P) for _ in range(rng.randrange(0, 40))])
        if k == 3:
            return (o.LEAFS, tuple(rng.randrange(o.P) for _ in range(3)))
        return (o.VALUE, rng.randrange(o.P))

    for rep in range(3):
        doc = rng.randbytes(rng.randrange(0, 200))
        pairs = [(sg.IndependentProofStream(), o.IndependentProofStream()),
                 (sg.SignatureProofStream(doc), o.SignatureProofStream(doc))]
        for s, ref in pairs:
            for i in range(120):
                ob = rand_obj()
                s.push(ob)
                ref.push(ob)
                if i % 7 == 0:
                    assert s.fiat_shamir_prover(32) == ref.fiat_shamir_prover(32)
            assert s.fiat_shamir_prover(64) == ref.fiat_shamir_prover(64)
            assert s.digest() == ref.digest()
            for _ in range(50):
                assert o.serialize([s.pull()]) == o.serialize([ref.pull()])
            assert s.fiat_shamir_verifier(48) == ref.fiat_shamir_verifier(48)


# ---------------------------------------------------------------- host-only native logic

def test_host_rescue_prime_matches_reference_kats():
    """RescuePrime::new / hash / trace through the library's host path (no device)."""
    import json
    import stark_prove_oracle as e
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats_e2e.json")) as f:
        k = json.load(f)
    h = sg.HostContext()
    rp = sg.RescuePrime(2, 1, 128, 27, ctx=h)
    r = k["rescue_new"]
    assert rp.alpha == r["alpha"] and rp.alpha_inv == int(r["alpha_inv"]), r["src"]
    assert rp.MDS == [[int(x) for x in row] for row in r["mds"]], r["src"]
    assert rp.MDS_inv == [[int(x) for x in row] for row in r["mds_inv"]], r["src"]
    assert rp.round_constants == [int(x) for x in r["round_constants"]], r["src"]
    assert rp.hash(int(k["rescue_hash"]["input"])) == int(k["rescue_hash"]["output"])
    t = rp.trace(int(k["rescue_trace"]["input"]))
    assert t[-1][0] == int(k["rescue_trace"]["last_rate"])
    for (m, N) in ((3, 7), (2, 60)):
        a, b = sg.RescuePrime(m, 1, 2, N, ctx=h), e.RescuePrime(m, 1, 2, N)
        assert a.MDS == b.MDS and a.MDS_inv == b.MDS_inv and a.round_constants == b.round_constants
        assert a.trace(99) == b.trace(99)
    import pytest
    with pytest.raises(sg.StarkGpuError, match="GPU context"):
        rp.transition_constraints(1, 2)


def test_host_mpolynomial_and_degree_bounds_match_oracle():
    """MPolynomial arithmetic (small, host) and Stark's key-based degree bounds vs the oracle."""
    import random
    import stark_prove_oracle as e
    h = sg.HostContext()

    def grouped(d):
        out = {}
        for key, c in d.items():
            v = out.setdefault(tuple(key[1:]), [])
            v.extend([0] * (key[0] + 1 - len(v)))
            v[key[0]] = (v[key[0]] + c) % o.P
        return (len(next(iter(d))) if d else 0), out

    rng = random.Random(11)
    for _ in range(6):
        nv = rng.randrange(1, 5)
        da = {tuple(rng.randrange(4) for _ in range(nv)): rng.choice([0, rng.randrange(o.P)]) for _ in range(5)}
        db = {tuple(rng.randrange(3) for _ in range(nv)): rng.randrange(o.P) for _ in range(4)}
        A, B = sg.MPolynomial.new(da, ctx=h), sg.MPolynomial.new(db, ctx=h)
        oa, ob = e.MPolynomial(da), e.MPolynomial(db)
        assert (A * B).groups() == grouped((oa * ob).d)
        assert (A - B).groups() == grouped((oa - ob).d)
        assert (A ** 3).groups() == grouped((oa ** 3).d)
        pt = [rng.randrange(o.P) for _ in range(nv)]
        assert A.evaluate(pt) == oa.evaluate(pt)
    # the oracle's Rescue AIR, handed to the library as dictionaries: same key-based bounds
    st_o = e.Stark(4, 2, 2, 2, 28, 2)
    st_h = sg.Stark(4, 2, 2, 2, 28, 2, ctx=h)
    assert (st_h.omicron, st_h.omicron_domain_length, st_h.num_randomizers, st_h.fri_domain_length) == \
        (st_o.omicron, st_o.omicron_domain_length, st_o.num_randomizers, st_o.fri.domain_length)
    air_o = e.RescuePrime(2, 1, 2, 27).transition_constraints(st_o.omicron, st_o.omicron_domain_length)
    air_h = [sg.MPolynomial.new(a.d, ctx=h) for a in air_o]
    assert st_h.transition_degree_bounds(air_h) == st_o.transition_degree_bounds(air_o)
    assert st_h.max_degree(air_h) == st_o.max_degree(air_o)


def test_c_host_example_builds_and_links():
    """examples/prove_rescue.c compiles against include/stark_gpu.h alone and links libstarkgpu.so
    (no Python in that binary); without arguments it prints its usage (no GPU touched)."""
    import subprocess
    import tempfile
    out = os.path.join(tempfile.mkdtemp(prefix="sg_chost_"), "prove_rescue")
    pkg = os.path.join(ROOT, "zk-stark-tutor_amd", "starkgpu")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "prove_rescue.c"), "-L", pkg, "-lstarkgpu",
                    "-Wl,-rpath," + pkg, "-Wl,-rpath,/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib", "-o", out],
                   check=True)
    res = subprocess.run([out], capture_output=True, text=True, timeout=60)
    assert res.returncode == 1 and "usage" in res.stderr
