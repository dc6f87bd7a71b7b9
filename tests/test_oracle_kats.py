"""Pin the CPU oracle (oracle/stark_oracle.py) to the reference's own known-answer tests.

Every vector comes from tests/golden/reference_kats.json, transcribed from the
reference's #[cfg(test)] assertions (file:line in each entry).
"""
import stark_oracle as o


def I(s):
    return int(s)


def test_constants(kats):
    assert o.P == I(kats["prime"])
    assert o.GENERATOR == I(kats["generator"])


def test_field_ops(kats):
    for v in kats["field_mul_mod"] + kats["fe_mul"]:
        assert o.mul_mod(I(v["a"]), I(v["b"])) == I(v["out"]), v["src"]
    for v in kats["fe_div"]:
        assert o.div(I(v["a"]), I(v["b"])) == I(v["out"]), v["src"]
    for v in kats["fe_inverse"]:
        assert o.inv(I(v["a"])) == I(v["out"]), v["src"]
    for v in kats["fe_add"]:
        assert o.add_mod(I(v["a"]), I(v["b"])) == I(v["out"]), v["src"]
    for v in kats["fe_sub"]:
        assert o.sub_mod(I(v["a"]), I(v["b"])) == I(v["out"]), v["src"]
    for v in kats["fe_neg"]:
        assert o.neg_mod(I(v["a"])) == I(v["out"]), v["src"]
    for v in kats["fe_pow"]:
        assert o.fpow(I(v["a"]), I(v["e"])) == I(v["out"]), v["src"]
    for v in kats["u_xgcd"]:
        assert o.u_xgcd(I(v["a"]), I(v["b"])) == tuple(I(x) for x in v["out"]), v["src"]
    # field_element.rs:210-220: x * x^-1 == 1
    for x in (8, o.P - 2):
        assert o.mul_mod(x, o.inv(x)) == 1
    assert o.inv(0) == 0  # u_xgcd(0, p) -> (0, 1, p)


def test_roots_and_sample(kats):
    for v in kats["primitive_nth_root"]:
        assert o.primitive_nth_root(I(v["n"])) == I(v["out"]), v["src"]
    for v in kats["sample"]:
        assert o.sample(bytes.fromhex(v["bytes_hex"])) == I(v["out"]), v["src"]
    z = o.primitive_nth_root(256)  # field.rs:201-216
    assert o.fpow(z, 256) == 1 and o.fpow(z, 128) != 1


def test_ntt_intt(kats):
    for v in kats["ntt"]:
        root = o.primitive_nth_root(v["n"])
        assert o.ntt(root, [I(x) for x in v["input"]]) == [I(x) for x in v["output"]], v["src"]
    for v in kats["intt"]:
        root = o.primitive_nth_root(v["n"])
        assert o.intt(root, [I(x) for x in v["input"]]) == [I(x) for x in v["output"]], v["src"]
    # fft/ntt.rs:98-104: the ntt equals evaluation on the powers of the root
    v = kats["ntt"][0]
    root = o.primitive_nth_root(16)
    xs = [I(x) for x in v["input"]]
    assert [o.evaluate(xs, o.fpow(root, i)) for i in range(16)] == [I(x) for x in v["output"]]


def test_hashes(kats):
    for v in kats["blake2b512"]:
        assert o.blake2b512(bytes.fromhex(v["in_hex"])).hex() == v["out_hex"], v["src"]
    for v in kats["shake256"]:
        assert o.shake256(v["in_ascii"].encode(), v["num_bytes"]).hex() == v["out_hex"], v["src"]


def test_merkle(kats):
    for v in kats["merkle_commit"]:
        assert o.merkle_commit([I(x) for x in v["leaves"]]).hex() == v["root_hex"], v["src"]
    for v in kats["merkle_open"]:
        path = o.merkle_open(v["index"], [I(x) for x in v["leaves"]])
        assert [p.hex() for p in path] == v["path_hex"], v["src"]
    path = [bytes.fromhex(h) for h in kats["merkle_verify_path_hex"]]
    for v in kats["merkle_verify"]:
        assert o.merkle_verify(bytes.fromhex(v["root_hex"]), v["index"], path, I(v["leaf"])) == v["expect"], v["src"]


def test_sample_indices(kats):
    for v in kats["fri_sample_indices"]:
        fri = o.FRI(o.GENERATOR, o.primitive_nth_root(v["n"]), v["n"], v["expansion_factor"],
                    v["num_colinearity_tests"])
        got = fri.sample_indices(bytes.fromhex(v["seed_hex"]), v["size"], v["reduced_size"], v["number"])
        assert got == v["out"], v["src"]


def test_serialization_layout(kats):
    objs = []
    for kind, val in kats["serialize_roundtrip"]["objects"]:
        if kind == "root":
            objs.append((o.ROOT, bytes.fromhex(val)))
        elif kind == "codeword":
            objs.append((o.CODEWORD, [I(x) for x in val]))
        elif kind == "path":
            objs.append((o.PATH, [bytes.fromhex(x) for x in val]))
        elif kind == "leafs":
            objs.append((o.LEAFS, tuple(I(x) for x in val)))
        else:
            objs.append((o.VALUE, I(val)))
    b = o.serialize(objs)
    # field prefix: 16-byte BE prime since codeword/leafs/value carry the field
    assert b[:16] == o.P.to_bytes(16, "big")
    # first object: code 0, len 4 (u64 BE), payload
    assert b[16:16 + 13] == bytes([0]) + (4).to_bytes(8, "big") + bytes.fromhex("496e2074")
    # a stream of roots only has a zero field prefix
    assert o.serialize([(o.ROOT, b"\x01" * 64)])[:16] == bytes(16)


def test_fri_roundtrip_small():
    """fri.rs:450-531: degree 63, expansion 4, 17 tests, domain 256; prove -> verify, tamper -> reject."""
    n, exp, c = 256, 4, 17
    omega = o.primitive_nth_root(n)
    fri = o.FRI(o.GENERATOR, omega, n, exp, c)
    poly = list(range(64))
    codeword = [o.evaluate(poly, o.fpow(omega, i)) for i in range(n)]
    ps = o.IndependentProofStream()
    fri.prove(codeword, ps)
    ok, err, points = fri.verify(ps)
    assert ok, err
    for x, y in points:
        assert o.evaluate(poly, o.fpow(omega, x)) == y
    bad = list(codeword)
    for i in range(63 // 3):
        bad[i] = 0
    ps = o.IndependentProofStream()
    fri.prove(bad, ps)
    ok, _, _ = fri.verify(ps)
    assert not ok


def test_coset_evaluate_matches_direct():
    """fft/ntt_arithmetics.rs:472-492: LDE on the coset 5*w^i equals direct evaluation (n=64)."""
    n = 64
    w = o.primitive_nth_root(n)
    coeffs = o.synthetic_elements(7, b"lde", 40)
    got = o.fast_coset_evaluate(w, n, 5, coeffs)
    assert got == [o.evaluate(coeffs, o.mul_mod(5, o.fpow(w, i))) for i in range(n)]
