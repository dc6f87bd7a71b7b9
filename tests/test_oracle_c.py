"""The C restatement (oracle/ref_cpu.c) agrees with the reference KATs and with
the Python restatement: two independent CPU oracles for the same path."""
import os
import subprocess

import pytest

import stark_oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rc():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    import ref_cpu
    return ref_cpu


def ints(a):
    return [(int(h) << 64) | int(l) for l, h in a.tolist()]


def test_c_oracle_kats(rc, kats):
    for v in kats["ntt"]:
        root = o.primitive_nth_root(v["n"])
        assert ints(rc.ntt(root, [int(x) for x in v["input"]])) == [int(x) for x in v["output"]], v["src"]
    for v in kats["intt"]:
        root = o.primitive_nth_root(v["n"])
        assert ints(rc.intt(root, [int(x) for x in v["input"]])) == [int(x) for x in v["output"]], v["src"]
    for v in kats["merkle_commit"]:
        assert rc.merkle_commit([int(x) for x in v["leaves"]]).hex() == v["root_hex"], v["src"]
    for v in kats["merkle_open"]:
        assert [p.hex() for p in rc.merkle_open(v["index"], [int(x) for x in v["leaves"]])] == v["path_hex"]


@pytest.mark.parametrize("logn", [1, 4, 9, 12])
def test_c_oracle_matches_python_oracle(rc, logn):
    n = 1 << logn
    x = o.synthetic_elements(logn, b"c", n)
    w = o.primitive_nth_root(n)
    assert ints(rc.ntt(w, x)) == o.ntt(w, x)
    assert ints(rc.fast_coset_evaluate(w, n, o.GENERATOR, x[: max(n // 8, 1)])) == \
        o.fast_coset_evaluate(w, n, o.GENERATOR, x[: max(n // 8, 1)])
    assert rc.merkle_commit(x) == o.merkle_commit(x)


def test_c_oracle_fri_commit_stream(rc):
    n, exp, c = 1 << 11, 8, 16
    w = o.primitive_nth_root(n)
    cw = o.fast_coset_evaluate(w, n, o.GENERATOR, o.synthetic_elements(5, b"fri", n // exp))
    prefix_objs = [(o.ROOT, bytes(range(64)))]
    ps = o.IndependentProofStream(prefix_objs)
    codewords = o.FRI(o.GENERATOR, w, n, exp, c).commit(cw, ps)
    stream, roots, cws = rc.fri_commit(o.GENERATOR, w, cw, exp, c, prefix=o.serialize(prefix_objs),
                                       want_codewords=True)
    assert stream == ps.digest()
    assert [ints(a) for a in cws] == codewords
    assert roots == [ob[1] for ob in ps.objects if ob[0] == o.ROOT][1:]
