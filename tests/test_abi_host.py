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
