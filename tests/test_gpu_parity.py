"""GPU parity: libstarkgpu (HIP, gfx950) vs the CPU oracle, bit-exact.

Runs on an MI355X (`pytest -m gpu`).  Every comparison is exact equality of
field elements / digest bytes / proof-stream bytes.  The oracle restates the
reference (oracle/stark_oracle.py) and is pinned by tests/test_oracle_kats.py.
"""
import random

import numpy as np
import pytest

import stark_oracle as o
import starkgpu as sg

pytestmark = pytest.mark.gpu

P = o.P


def rnd(seed, n, tag=b"t"):
    return o.synthetic_elements(seed, tag, n)


EDGE_VALUES = [0, 1, 2, 9, 10, 99, 100, 10**8 - 1, 10**8, 10**16, 10**19 - 1, 10**19, 2**64 - 1, 2**64,
               10**32 - 1, 10**32, 10**38 - 1, 10**38, P - 2, P - 1]


# ------------------------------------------------------------------ field / host

def test_field_host_kats(kats):
    for v in kats["fe_mul"]:
        assert sg.fe_mul(int(v["a"]), int(v["b"])) == int(v["out"]), v["src"]
    for v in kats["fe_inverse"]:
        assert sg.fe_inverse(int(v["a"])) == int(v["out"])
    for v in kats["primitive_nth_root"]:
        assert sg.primitive_nth_root(int(v["n"])) == int(v["out"])
    for v in kats["sample"]:
        assert sg.sample(bytes.fromhex(v["bytes_hex"])) == int(v["out"])


# ------------------------------------------------------------------ NTT

def test_ntt_kats(kats):
    for v in kats["ntt"]:
        root = o.primitive_nth_root(v["n"])
        got = sg.to_ints(sg.ntt(root, [int(x) for x in v["input"]]))
        assert got == [int(x) for x in v["output"]], v["src"]
    for v in kats["intt"]:
        root = o.primitive_nth_root(v["n"])
        got = sg.to_ints(sg.intt(root, [int(x) for x in v["input"]]))
        assert got == [int(x) for x in v["output"]], v["src"]


@pytest.mark.parametrize("logn", list(range(0, 15)))
def test_ntt_vs_oracle(logn):
    n = 1 << logn
    x = rnd(logn, n)
    root = o.primitive_nth_root(n)
    assert sg.to_ints(sg.ntt(root, x)) == o.ntt(root, x)


@pytest.mark.parametrize("n_in", [1, 2, 3, 5, 7, 100, 1000, 4097])
def test_ntt_zero_padding(n_in):
    """bit_reverse_copy pads to next_pow2 (utils/bit_reverse_copy.rs:8-17)."""
    x = rnd(n_in, n_in, b"pad")
    n = 1 << (n_in - 1).bit_length() if n_in > 1 else 1
    root = o.primitive_nth_root(n)
    assert sg.to_ints(sg.ntt(root, x)) == o.ntt(root, x)


@pytest.mark.parametrize("logn,root", [(4, 5), (10, 12345678901234567890), (13, 3)])
def test_ntt_non_primitive_root_same_graph(logn, root):
    """The DIT butterfly graph is the reference's, so even a non-primitive root matches."""
    n = 1 << logn
    x = rnd(7, n, b"np")
    assert sg.to_ints(sg.ntt(root, x)) == o.ntt(root, x)


def test_ntt_edge_values():
    x = (EDGE_VALUES * 4)[:64]
    root = o.primitive_nth_root(64)
    assert sg.to_ints(sg.ntt(root, x)) == o.ntt(root, x)
    assert sg.to_ints(sg.ntt(root, [P - 1] * 64)) == o.ntt(root, [P - 1] * 64)
    imp = [0] * 64
    imp[63] = 1
    assert sg.to_ints(sg.ntt(root, imp)) == o.ntt(root, imp)


@pytest.mark.parametrize("n_in", [1, 2, 16, 1000, 4096, 8192])
def test_intt_vs_oracle(n_in):
    x = rnd(n_in, n_in, b"intt")
    n = 1 << (n_in - 1).bit_length() if n_in > 1 else 1
    root = o.primitive_nth_root(n)
    assert sg.to_ints(sg.intt(root, x)) == o.intt(root, x)


def test_ntt_intt_empty_input():
    """fft/ntt.rs:11 indexes inputs[0] (the reference panics on an empty ntt input: an error here);
    intt returns an input shorter than 2 unchanged (fft/ntt.rs:51-68), the empty one included."""
    root = o.primitive_nth_root(4)
    with pytest.raises(ValueError):  # the Python mirror checks first; the C ABI returns SG_ERR_INVALID
        sg.ntt(root, [])
    assert len(sg.intt(root, [])) == 0
    assert sg.to_ints(sg.intt(root, [12345])) == [12345]


def test_ntt_rejects_noncanonical():
    with pytest.raises(sg.StarkGpuError) as e:
        sg.ntt(o.primitive_nth_root(4), [P, 0, 0, 0])
    assert e.value.code == -3
    arr = sg.fe_array([0, 0, 0, 0])
    arr[0, 1] = np.uint64(0xFFFFFFFFFFFFFFFF)
    with pytest.raises(sg.StarkGpuError):
        sg.ntt(o.primitive_nth_root(4), arr)


# ------------------------------------------------------------------ LDE

@pytest.mark.parametrize("d,N", [(0, 16), (1, 16), (5, 16), (64, 64), (100, 512), (1 << 10, 1 << 13),
                                 (3000, 1 << 14), (1 << 12, 1 << 15)])
def test_coset_evaluate_vs_oracle(d, N):
    coeffs = rnd(d, d, b"lde")
    w = o.primitive_nth_root(N)
    got = sg.to_ints(sg.fast_coset_evaluate(w, N, o.GENERATOR, coeffs))
    assert got == o.fast_coset_evaluate(w, N, o.GENERATOR, coeffs)


def test_coset_evaluate_non_pow2_root_order():
    coeffs = rnd(1, 7, b"lde")
    w = o.primitive_nth_root(16)
    assert sg.to_ints(sg.fast_coset_evaluate(w, 12, 5, coeffs)) == o.fast_coset_evaluate(w, 12, 5, coeffs)


def test_coset_evaluate_rejects_long_polynomial():
    with pytest.raises(ValueError):
        sg.fast_coset_evaluate(o.primitive_nth_root(4), 4, 5, [1, 2, 3, 4, 5])


# ------------------------------------------------------------------ Merkle

def test_merkle_kats(kats):
    for v in kats["merkle_commit"]:
        assert sg.MerkleRoot.commit([int(x) for x in v["leaves"]]).hex() == v["root_hex"], v["src"]
    for v in kats["merkle_open"]:
        path = sg.MerkleRoot.open(v["index"], [int(x) for x in v["leaves"]])
        assert [p.hex() for p in path] == v["path_hex"], v["src"]


def test_merkle_decimal_leaf_lengths():
    """Every decimal length 1..39 (field_element.rs:46-50) hashes like the reference."""
    vals = [0] + [10**k for k in range(1, 39)] + [10**k - 1 for k in range(1, 39)] + EDGE_VALUES
    vals = [v for v in vals if v < P]
    n = 1 << (len(vals) - 1).bit_length()
    vals = (vals + EDGE_VALUES * 8)[:n]
    levels = o.merkle_levels(vals)
    assert sg.MerkleRoot.commit(vals) == levels[-1][0]
    for i in (0, 1, n // 2, n - 1):
        assert sg.MerkleRoot.open(i, vals) == o.merkle_open(i, vals)


@pytest.mark.parametrize("logn", [0, 1, 2, 3, 5, 8, 9, 10, 12, 13, 16])
def test_merkle_commit_vs_oracle(logn):
    n = 1 << logn
    vals = rnd(logn, n, b"mk")
    assert sg.MerkleRoot.commit(vals) == o.merkle_commit(vals)


def test_merkle_open_verify_roundtrip():
    vals = rnd(3, 1 << 11, b"open")
    root = o.merkle_commit(vals)
    rng = random.Random(5)
    for i in [0, 1, 1023, 1024, 2047] + [rng.randrange(2048) for _ in range(8)]:
        path = sg.MerkleRoot.open(i, vals)
        assert path == o.merkle_open(i, vals)
        assert sg.MerkleRoot.verify(root, i, path, vals[i])
        assert not sg.MerkleRoot.verify(root, i, path, (vals[i] + 1) % P)


def test_merkle_rejects_non_pow2():
    with pytest.raises(sg.StarkGpuError):
        sg.MerkleRoot.commit([1, 2, 3])


def test_entry_points_under_a_pool_cap(monkeypatch):
    """Every hot-path entry point on a context whose buffer pool is capped at 512 KiB
    (SG_POOL_LIMIT_BYTES, a test knob): inputs past the cap fail with SG_ERR_NOMEM -- ntt / intt /
    fast_coset_evaluate at 2^16, a 2^14-leaf Merkle commit, FRI::prove on a 2^14 codeword -- each
    leaves no pool buffer behind, and the same calls at sizes under the cap (with any tree layout,
    lean trees off included, in the alternate-paths suite) then equal the oracle's."""
    from starkgpu._lib import SG_ERR_NOMEM
    monkeypatch.setenv("SG_POOL_LIMIT_BYTES", str(512 << 10))
    ctx = sg.Context(0)
    monkeypatch.delenv("SG_POOL_LIMIT_BYTES")
    big = rnd(11, 1 << 16, b"cap")
    r16 = o.primitive_nth_root(1 << 16)
    omega, cw = _fri_case(1 << 14, 8, 16, 1 << 14)
    calls = [lambda: sg.ntt(r16, big, ctx=ctx), lambda: sg.intt(r16, big, ctx=ctx),
             lambda: sg.fast_coset_evaluate(r16, 1 << 16, o.GENERATOR, big[:1 << 12], ctx=ctx),
             lambda: sg.MerkleRoot.commit(big[:1 << 14], ctx=ctx),
             lambda: sg.FRI(o.GENERATOR, omega, 1 << 14, 8, 16, ctx=ctx).prove(cw, sg.IndependentProofStream())]
    for call in calls:
        live = ctx.memory()["live"]
        with pytest.raises(sg.StarkGpuError) as err:
            call()
        assert err.value.code == SG_ERR_NOMEM, err.value
        assert ctx.memory()["live"] == live
    small = big[:256]
    r8 = o.primitive_nth_root(256)
    assert sg.to_ints(sg.ntt(r8, small, ctx=ctx)) == o.ntt(r8, small)
    assert sg.to_ints(sg.intt(r8, small, ctx=ctx)) == o.intt(r8, small)
    w10 = o.primitive_nth_root(1 << 10)
    assert sg.to_ints(sg.fast_coset_evaluate(w10, 1 << 10, o.GENERATOR, small[:100], ctx=ctx)) == \
        o.fast_coset_evaluate(w10, 1 << 10, o.GENERATOR, small[:100])
    assert sg.MerkleRoot.commit(small, ctx=ctx) == o.merkle_commit(small)
    omega, cw = _fri_case(256, 4, 2, 256)
    ops = o.IndependentProofStream()
    otop = o.FRI(o.GENERATOR, omega, 256, 4, 2).prove(cw, ops)
    gps = sg.IndependentProofStream()
    assert sg.FRI(o.GENERATOR, omega, 256, 4, 2, ctx=ctx).prove(cw, gps) == otop
    assert gps.digest() == ops.digest()


def test_merkle_tree_beyond_device_memory_is_nomem():
    """A tree that cannot fit: 2^32 device-resident leaves (a 64 GiB codeword) whose digests would
    take 512 GiB, above the GPU's 288 GB.  sg_merkle_build_dev returns SG_ERR_NOMEM (the ABI never
    aborts), holds nothing afterwards, and the same context then builds a tree whose root and
    path equal the oracle's (merkle_root.rs:21-32, 55-66)."""
    import torch
    ctx = sg.Context(0)
    n = 1 << 32
    big = torch.empty((n, 2), dtype=torch.int64, device=torch.device("cuda", 0))  # in bounds, never hashed
    live = ctx.memory()["live"]
    with pytest.raises(sg.StarkGpuError) as err:
        sg.DeviceTree(big.data_ptr(), n, ctx=ctx)
    from starkgpu._lib import SG_ERR_NOMEM
    assert err.value.code == SG_ERR_NOMEM, err.value
    assert ctx.memory()["live"] == live
    del big
    vals = rnd(7, 1 << 10, b"after-nomem")
    small = torch.from_numpy(sg.fe_array(vals).view(np.int64)).to(torch.device("cuda", 0))
    t = sg.DeviceTree(small.data_ptr(), len(vals), ctx=ctx)
    assert t.root() == o.merkle_commit(vals)
    assert t.open(333) == o.merkle_open(333, vals)
    t.free()


# ------------------------------------------------------------------ proof stream

def test_stream_serialization_matches_oracle():
    objs = [(o.ROOT, bytes(range(64))), (o.CODEWORD, [20, 100, P - 1]), (o.PATH, [bytes(64), bytes([7] * 64)]),
            (o.LEAFS, (1, 5, 10)), (o.VALUE, 2)]
    s = sg.IndependentProofStream()
    for ob in objs:
        s.push(ob)
    assert s.digest() == o.serialize(objs)
    assert s.fiat_shamir_prover(32) == o.shake256(o.serialize(objs), 32)
    back = sg.IndependentProofStream.deserialize(s.digest())
    assert back.objects() == objs
    sig = sg.SignatureProofStream(b"document")
    osig = o.SignatureProofStream(b"document")
    for ob in objs[:2]:
        sig.push(ob)
        osig.push(ob)
    assert sig.fiat_shamir_prover(32) == osig.fiat_shamir_prover(32)


# ------------------------------------------------------------------ FRI

def _fri_case(n, exp, c, seed):
    omega = o.primitive_nth_root(n)
    d = n // exp
    coeffs = rnd(seed, d, b"fri")
    codeword = o.fast_coset_evaluate(omega, n, o.GENERATOR, coeffs)
    return omega, codeword


@pytest.mark.parametrize("n,exp,c", [(256, 4, 17), (1024, 8, 2), (1 << 12, 8, 16), (1 << 14, 8, 64)])
def test_fri_prove_stream_bytes_match_oracle(n, exp, c):
    omega, cw = _fri_case(n, exp, c, n)
    ofri = o.FRI(o.GENERATOR, omega, n, exp, c)
    ops = o.IndependentProofStream()
    otop = ofri.prove(cw, ops)
    gfri = sg.FRI(o.GENERATOR, omega, n, exp, c)
    gps = sg.IndependentProofStream()
    gtop = gfri.prove(cw, gps)
    assert gtop == otop
    assert gps.digest() == ops.digest()
    ok, err, _ = ofri.verify(o.IndependentProofStream(gps.objects()))
    assert ok, err


def test_fri_commit_matches_oracle_and_callback_stream():
    n, exp, c = 1 << 10, 4, 8
    omega, cw = _fri_case(n, exp, c, 11)
    ofri = o.FRI(o.GENERATOR, omega, n, exp, c)
    ops = o.IndependentProofStream()
    ofri.commit(cw, ops)
    # a foreign ProofStream implementation driven through the callback ABI
    cps = o.IndependentProofStream()
    sg.FRI(o.GENERATOR, omega, n, exp, c).commit(cw, cps)
    assert cps.digest() == ops.digest()


@pytest.mark.parametrize("stream_kind", ["callback", "native_unpinned"])
def test_fri_prove_tail_paths_match_oracle(stream_kind, monkeypatch):
    """The proof tail (query-phase Leafs/Path objects, serialized on the device) reaches a foreign
    ProofStream through the push callback, and a native stream whose body cannot be page-locked
    through pinned staging -- byte-identical to the oracle either way."""
    n, exp, c = 1 << 11, 8, 12
    omega, cw = _fri_case(n, exp, c, 23)
    ofri = o.FRI(o.GENERATOR, omega, n, exp, c)
    ops = o.IndependentProofStream()
    otop = ofri.prove(cw, ops)
    gfri = sg.FRI(o.GENERATOR, omega, n, exp, c)
    if stream_kind == "callback":
        gps = o.IndependentProofStream()
        gtop = gfri.prove(cw, gps)
    else:
        gps = sg.IndependentProofStream()
        with sg.Context.default().option("stream_pin", 0, 1):  # the staging fallback
            gtop = gfri.prove(cw, gps)
    assert gtop == otop
    assert gps.digest() == ops.digest()


class _FsFailsAfter(o.IndependentProofStream):
    """A foreign proof stream whose Fiat-Shamir callback raises from its (after+1)-th call on."""

    def __init__(self, after):
        super().__init__()
        self.calls, self.after = 0, after

    def fiat_shamir_prover(self, num_bytes):
        self.calls += 1
        if self.calls > self.after:
            raise RuntimeError("injected Fiat-Shamir failure")
        return super().fiat_shamir_prover(num_bytes)


def test_fri_gate_bytes_and_release_on_callback_failure():
    """Option fri_gate (default on): round r + 1's fold + tree are queued behind a device gate
    (k_fri_gate) before round r's challenge exists, and the host raises the gate once it has
    written K.  Gate on and off write the oracle's bytes.  A Fiat-Shamir callback failing while a
    gated round is queued (first, second, fourth challenge; and the query seed, after the last
    round) raises at once -- the pending gate is released, the stream drains instead of waiting
    for the gate's 60 s deadline -- and the context proves the oracle's bytes afterwards."""
    import time
    n, exp, c = 1 << 14, 8, 64
    omega, cw = _fri_case(n, exp, c, 41)
    ofri = o.FRI(o.GENERATOR, omega, n, exp, c)
    ops = o.IndependentProofStream()
    otop = ofri.prove(cw, ops)
    gfri = sg.FRI(o.GENERATOR, omega, n, exp, c)
    ctx = sg.Context.default()
    for gate in (1, 0):
        with ctx.option("fri_gate", gate, 1):
            gps = sg.IndependentProofStream()
            assert gfri.prove(cw, gps) == otop
            assert gps.digest() == ops.digest()
    # 2^14 -> 2^8: six rounds, five challenges, then the query seed (the sixth call)
    for after in (0, 1, 3, 5):
        t0 = time.perf_counter()
        bad = _FsFailsAfter(after)
        with pytest.raises(RuntimeError, match="injected"):  # the callback's own exception, re-raised
            gfri.prove(cw, bad)
        assert time.perf_counter() - t0 < 10, "the pending gate was not released"
        assert bad.calls == after + 1
    gps = sg.IndependentProofStream()
    assert gfri.prove(cw, gps) == otop
    assert gps.digest() == ops.digest()


class _FsSlowAt(o.IndependentProofStream):
    """A foreign proof stream whose k-th Fiat-Shamir call sleeps `seconds` first."""

    def __init__(self, k, seconds):
        super().__init__()
        self.calls, self.k, self.seconds = 0, k, seconds

    def fiat_shamir_prover(self, num_bytes):
        import time
        self.calls += 1
        if self.calls == self.k:
            time.sleep(self.seconds)
        return super().fiat_shamir_prover(num_bytes)


def test_fri_gate_deadline():
    """A gated round whose challenge comes later than the gate's deadline (context option
    fri_gate_timeout_ms, 60 s by default; 20 ms here against a 0.3 s callback) fails the call with
    the gate's timeout -- never a proof folded with a stale challenge -- and the context then
    proves the oracle's bytes again."""
    n, exp, c = 1 << 14, 8, 64
    omega, cw = _fri_case(n, exp, c, 43)
    ofri = o.FRI(o.GENERATOR, omega, n, exp, c)
    ops = o.IndependentProofStream()
    otop = ofri.prove(cw, ops)
    gfri = sg.FRI(o.GENERATOR, omega, n, exp, c)
    ctx = sg.Context.default()
    with ctx.option("fri_gate_timeout_ms", 20, 60000):
        with pytest.raises(sg.StarkGpuError, match="gate timed out"):
            gfri.prove(cw, _FsSlowAt(2, 0.3))
        gps = sg.IndependentProofStream()  # a prompt stream under the short deadline
        assert gfri.prove(cw, gps) == otop and gps.digest() == ops.digest()
    gps = sg.IndependentProofStream()
    assert gfri.prove(cw, gps) == otop and gps.digest() == ops.digest()


def test_fri_tampered_codeword_rejected():
    """fri.rs:514-528: zeroing a third of the low-degree positions makes verify fail."""
    n, exp, c = 256, 4, 17
    omega, cw = _fri_case(n, exp, c, 3)
    bad = list(cw)
    for i in range(63 // 3):
        bad[i] = 0
    gps = sg.IndependentProofStream()
    sg.FRI(o.GENERATOR, omega, n, exp, c).prove(bad, gps)
    ok, _, _ = o.FRI(o.GENERATOR, omega, n, exp, c).verify(o.IndependentProofStream(gps.objects()))
    assert not ok


# ------------------------------------------------------------------ large sizes: algebraic properties

def test_large_ntt_roundtrip_and_spot_checks():
    logn = 22
    n = 1 << logn
    x = np.random.default_rng(1).integers(0, 2**63, size=(n, 2), dtype=np.uint64)
    x[:, 1] &= np.uint64((1 << 63) - 1)
    x[:, 1] %= np.uint64(0xCB80000000000000)  # keep < p
    root = o.primitive_nth_root(n)
    X = sg.ntt(root, x)
    back = sg.intt(root, X)
    assert np.array_equal(back, x)
    rng = random.Random(9)
    xs = sg.to_ints(x)
    for k in [0, 1, n - 1] + [rng.randrange(n) for _ in range(3)]:
        wk = o.fpow(root, k)
        assert sg.to_ints(X[k:k + 1])[0] == o.evaluate(xs, wk)


def _sparse(n, nnz, seed):
    """(n, 2) limb array with nnz random field values at random positions, and those terms."""
    rng = random.Random(seed)
    terms = {rng.randrange(n): rng.randrange(o.P) for _ in range(nnz)}
    x = np.zeros((n, 2), dtype=np.uint64)
    for j, v in terms.items():
        x[j, 0], x[j, 1] = v & (2**64 - 1), v >> 64
    return x, terms


def test_prove_size_ntt_and_lde_spot_checks():
    """The prove's largest transforms (2^25 NTT, degree-2^22 LDE onto 2^25 coset points)
    on sparse inputs whose outputs are cheap sums on the host: every stage's twiddles and
    the whole pass plan enter each checked output; plus a dense 2^25 round trip."""
    logn = 25
    n = 1 << logn
    w = o.primitive_nth_root(n)
    rng = random.Random(25)
    ks = [0, 1, n - 1, n // 2 + 3] + [rng.randrange(n) for _ in range(4)]
    x, terms = _sparse(n, 40, 251)
    X = sg.ntt(w, x)
    for k in ks:
        assert sg.to_ints(X[k:k + 1])[0] == sum(c * o.fpow(w, j * k) for j, c in terms.items()) % o.P
    d = 1 << 22
    c, cterms = _sparse(d, 40, 252)
    out = sg.fast_coset_evaluate(w, n, o.GENERATOR, c)
    for k in ks:
        pt = o.GENERATOR * o.fpow(w, k) % o.P
        assert sg.to_ints(out[k:k + 1])[0] == sum(v * o.fpow(pt, j) for j, v in cterms.items()) % o.P
    dense = np.random.default_rng(253).integers(0, 2**63, size=(n, 2), dtype=np.uint64)
    dense[:, 1] %= np.uint64(0xCB80000000000000)
    assert np.array_equal(sg.intt(w, sg.ntt(w, dense)), dense)


def test_batched_lde_and_trees_match_single():
    """sg_fast_coset_evaluate_batch_dev / sg_merkle_build_batch_dev == per-item calls == oracle."""
    import torch
    dev = torch.device("cuda", 0)
    N, d = 1 << 12, 1 << 9
    w = o.primitive_nth_root(N)
    polys = [rnd(s, d, b"batch") for s in range(3)]
    ins = [torch.from_numpy(sg.fe_array(p).view(np.int64)).to(dev) for p in polys]
    outs = [torch.empty((N, 2), dtype=torch.int64, device=dev) for _ in polys]
    sg.fast_coset_evaluate_batch_dev(w, N, o.GENERATOR, [t.data_ptr() for t in ins], d,
                                     [t.data_ptr() for t in outs])
    torch.cuda.synchronize()
    expect = [o.fast_coset_evaluate(w, N, o.GENERATOR, p) for p in polys]
    for out, e in zip(outs, expect):
        assert sg.to_ints(out.cpu().numpy().view(np.uint64)) == e
    trees = sg.DeviceTree.build_batch([t.data_ptr() for t in outs], N)
    for t, e in zip(trees, expect):
        assert t.root() == o.merkle_commit(e)
        assert t.open(77) == o.merkle_open(77, e)


def test_large_merkle_vs_c_oracle():
    """2^20 leaves exercise every launch kind (fused leaves, 1-lane nodes, quad nodes)."""
    import ref_cpu
    n = 1 << 20
    x = np.random.default_rng(3).integers(0, 2**63, size=(n, 2), dtype=np.uint64)
    x[:, 1] %= np.uint64(0xCB80000000000000)
    root = sg.MerkleRoot.commit(x)
    assert root == ref_cpu.merkle_commit(x)


def test_async_device_transforms_are_stream_ordered():
    """sg_ctx_set_async: LDE + tree build + FRI enqueue back to back; results unchanged."""
    import torch
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    N, d = 1 << 14, 1 << 11
    w = o.primitive_nth_root(N)
    coeffs = rnd(5, d, b"async")
    cin = torch.from_numpy(sg.fe_array(coeffs).view(np.int64)).to(dev)
    cw = torch.empty((N, 2), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ctx.set_async(True)
    try:
        for _ in range(3):
            sg.fast_coset_evaluate_dev(w, N, o.GENERATOR, cin.data_ptr(), d, cw.data_ptr(), ctx=ctx)
            root = sg.DeviceTree(cw.data_ptr(), N, ctx=ctx).root()
            stream = sg.IndependentProofStream()
            top = sg.FRI(o.GENERATOR, w, N, 8, 16, ctx=ctx).prove_dev(cw.data_ptr(), N, stream)
        ctx.synchronize()
    finally:
        ctx.set_async(False)
    expect = o.fast_coset_evaluate(w, N, o.GENERATOR, coeffs)
    assert sg.to_ints(cw.cpu().numpy().view(np.uint64)) == expect
    assert root == o.merkle_commit(expect)
    ref = o.IndependentProofStream()
    assert top == o.FRI(o.GENERATOR, w, N, 8, 16).prove(expect, ref)
    assert stream.digest() == ref.digest()
