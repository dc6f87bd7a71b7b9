"""Parity at BASELINE.json's full sizes (VERDICT r01 task 1), checked against the optimized CPU
restatement (oracle/fast_cpu.cpp, itself pinned to the Python oracle and the reference's KATs by
tests/test_oracle_fast.py) and against the oracle's own verifiers:

* C2: dense 2^22-point forward + inverse NTT, element for element;
* C3: FRI::prove at N = 2^24, expansion 8, 64 colinearity tests on the LDE of a seeded
  degree < 2^21 polynomial: LDE elements, round-0 root and the complete proof-stream bytes equal
  the checker's, the oracle's FRI.verify (fri.rs:250-416) accepts, a tampered codeword is
  rejected (fri.rs:514-528);
* C4 and the bench workload: Stark::prove on Rescue-Prime traces of 2^16 - 1 and 2^20 - 1 randomized
  rows (FRI domains 2^21 and 2^25): the GPU's proof bytes equal the CPU checker's Stark::prove
  (fast_cpu.stark_prove_rescue, itself byte-equal to the oracle's prove at the small parameter sets,
  tests/test_oracle_fast.py), the oracle's Stark.verify (stark.rs:565-770, AIR evaluated from its
  structure) accepts the proof and rejects a false claim;
* C5: the 2^27-point NTT sharded over 2 and 8 ranks (one process per rank on this box's one GPU,
  gloo host-staged exchange) bit-identical to the single-GPU transform and to the checker.

C2 and C3 are also pinned to the Python oracle itself (VERDICT r05 "Next round" 2): the GPU's
outputs hash to the SHA-256 digests tests/golden/make_fullsize.py computed with
oracle/stark_oracle.py (ntt / intt / fast_coset_evaluate / FRI.prove at these exact inputs, 24 min of
Python), stored in tests/golden/fullsize_digests.json.
"""
import hashlib
import os
import shutil
import socket
import tempfile
import time

import numpy as np
import pytest

import json

import stark_oracle as o
import stark_prove_oracle as e
import starkgpu as sg

pytestmark = pytest.mark.gpu
P = o.P
ORACLE = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_digests.json")))


def elem_digest(a: np.ndarray) -> str:
    """SHA-256 of an (n, 2) u64 element array as 16 LE bytes per element (make_fullsize.py's encoding)."""
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def fc():
    import fast_cpu
    fast_cpu.lib()
    return fast_cpu


def synthetic(seed: int, tag: bytes, n: int) -> np.ndarray:
    """SURVEY.md 8(d) value generator: BE 16-byte chunks of SHAKE256(b"sg-bench" || seed || tag) mod p."""
    raw = hashlib.shake_256(b"sg-bench" + seed.to_bytes(8, "big") + tag).digest(16 * n)
    be = np.frombuffer(raw, dtype=">u8").reshape(n, 2)
    hi, lo = be[:, 0].astype(np.uint64), be[:, 1].astype(np.uint64)
    p_hi, p_lo = np.uint64(P >> 64), np.uint64(P & (2**64 - 1))
    ge = (hi > p_hi) | ((hi == p_hi) & (lo >= p_lo))
    borrow = (lo < p_lo) & ge
    lo = np.where(ge, lo - p_lo, lo)
    hi = np.where(ge, hi - p_hi - borrow.astype(np.uint64), hi)
    return np.ascontiguousarray(np.stack([lo, hi], axis=1))


def _const(n: int, v: int) -> np.ndarray:
    x = np.empty((n, 2), dtype=np.uint64)
    x[:, 0], x[:, 1] = v & (2**64 - 1), v >> 64
    return x


# ------------------------------------------------------------------ C2

def test_c2_dense_2p22_ntt_intt_elementwise(fc):
    n = 1 << 22
    root = o.primitive_nth_root(n)
    x = synthetic(0, b"c2", n)
    assert elem_digest(x) == ORACLE["c2"]["input"]["sha256"]
    X = sg.ntt(root, x)
    assert elem_digest(X) == ORACLE["c2"]["ntt"]["sha256"], "ntt 2^22 != the Python oracle's (digest)"
    assert np.array_equal(X, fc.ntt(root, x)), "ntt 2^22 != checker"
    Y = sg.intt(root, X)
    assert np.array_equal(Y, fc.intt(root, X)), "intt 2^22 != checker"
    assert np.array_equal(Y, x)
    # edge fixtures: all p - 1, an impulse at n - 1, a zero-padded length
    for v in (_const(n, P - 1), np.zeros((n, 2), dtype=np.uint64)):
        assert np.array_equal(sg.ntt(root, v), fc.ntt(root, v))
    imp = np.zeros((n, 2), dtype=np.uint64)
    imp[n - 1, 0] = 1
    assert np.array_equal(sg.ntt(root, imp), fc.ntt(root, imp))
    ragged = x[: n - 5]
    R = sg.ntt(root, ragged)
    assert elem_digest(R) == ORACLE["c2"]["ragged_ntt_n_minus_5"]["sha256"], "ragged ntt != oracle digest"
    assert np.array_equal(R, fc.ntt(root, ragged))


@pytest.mark.parametrize("logn", [16, 17, 18, 19, 20, 21, 23])
def test_ntt_tile_plans_elementwise(fc, logn):
    """Every first-pass tile plan (kernels.hip ntt_first_tile: 2048-element tiles and three passes
    at 2^16-2^17 and 2^23, 2^12 tiles + one pass for the rest at 2^18-2^20, 2^13 tiles at 2^21)
    element for element against the checker: forward, inverse, a ragged (zero-padded) input and an
    LDE whose first stages are skipped (fft/ntt.rs:7-68, fft/ntt_arithmetics.rs:161-170)."""
    n = 1 << logn
    root = o.primitive_nth_root(n)
    x = synthetic(logn, b"tiles", n)
    X = sg.ntt(root, x)
    assert np.array_equal(X, fc.ntt(root, x)), f"ntt 2^{logn}"
    assert np.array_equal(sg.intt(root, X), fc.intt(root, X)), f"intt 2^{logn}"
    ragged = x[: n - 3]
    assert np.array_equal(sg.ntt(root, ragged), fc.ntt(root, ragged)), f"ragged ntt 2^{logn}"
    coeffs = x[: n >> 3]
    got = sg.fast_coset_evaluate(root, n, o.GENERATOR, coeffs)
    assert np.array_equal(np.asarray(got), fc.fast_coset_evaluate(root, n, o.GENERATOR, coeffs)), f"LDE 2^{logn}"


# ------------------------------------------------------------------ C3

def test_c3_fri_prove_2p24_exp8_c64(fc):
    N, exp, c = 1 << 24, 8, 64
    d = N // exp
    w = o.primitive_nth_root(N)
    coeffs = synthetic(0, b"c3", d)
    assert elem_digest(coeffs) == ORACLE["c3"]["coeffs"]["sha256"]
    cw = sg.fast_coset_evaluate(w, N, o.GENERATOR, coeffs)
    assert elem_digest(cw) == ORACLE["c3"]["lde"]["sha256"], "LDE 2^21 -> 2^24 != the Python oracle's (digest)"
    assert np.array_equal(cw, fc.fast_coset_evaluate(w, N, o.GENERATOR, coeffs)), "LDE 2^21 -> 2^24 != checker"
    gps = sg.IndependentProofStream()
    top = sg.FRI(o.GENERATOR, w, N, exp, c).prove(cw, gps)
    proof = gps.digest()
    assert len(proof) == ORACLE["c3"]["proof_len"] and hashlib.sha256(proof).hexdigest() == ORACLE["c3"]["proof_sha256"], \
        "FRI::prove bytes != the Python oracle's (digest)"
    assert list(top) == ORACLE["c3"]["top_indices"]
    ref, ref_top = fc.fri_prove(o.GENERATOR, w, cw, exp, c)
    objs = gps.objects()
    assert [ob[1].hex() for ob in objs if ob[0] == o.ROOT] == ORACLE["c3"]["roots"]
    assert objs[0] == (o.ROOT, fc.merkle_commit(cw)), "round-0 root != checker"
    assert top == ref_top
    assert gps.digest() == ref, "FRI::prove proof bytes != checker"
    ofri = o.FRI(o.GENERATOR, w, N, exp, c)
    assert len([ob for ob in objs if ob[0] == o.ROOT]) == ofri.num_rounds() == 16
    ok, err, _ = ofri.verify(o.IndependentProofStream(objs))
    assert ok, err
    # fri.rs:514-528: zero a third of the low-degree positions -> verify fails
    bad = cw.copy()
    bad[: (d - 1) // 3] = 0
    bps = sg.IndependentProofStream()
    sg.FRI(o.GENERATOR, w, N, exp, c).prove(bad, bps)
    ok, _, _ = ofri.verify(o.IndependentProofStream(bps.objects()))
    assert not ok


# ------------------------------------------------------------------ C4 + headline prove

def _prove_gpu_and_checker(fc, log_rows, tag):
    """Stark::prove (stark.rs:276-562) of a Rescue-Prime trace with 2^log_rows - 1 randomized rows,
    expansion 8, c = 64, security 128, transition degree 3, on the GPU and on the CPU checker with
    the same inputs.  Returns (GPU proof stream, checker bytes, oracle RescuePrime, output, gpu Stark)."""
    N = (1 << log_rows) - 2 - 256
    rp_g = sg.RescuePrime(2, 1, 128, N)
    st_g = sg.Stark(8, 64, 128, 2, N + 1, 3)
    assert st_g.fri_domain_length == 1 << (log_rows + 5)
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    rp_o = e.RescuePrime(2, 1, 128, N)
    assert rp_g.round_constants == rp_o.round_constants
    st_o = e.Stark(8, 64, 128, 2, N + 1, 3)
    bounds = fc.rescue_degree_bounds(rp_o, st_o)
    assert st_g.transition_degree_bounds(air_g) == \
        [b + (N + 1 - 1) for b in bounds[0]] and st_g.max_degree(air_g) == bounds[1]
    inp = o.sample(tag)
    trace = rp_g.trace_array(inp)
    out = sg.to_ints(trace[-2:-1])[0]  # last row, register 0: the hash output
    nrc = bounds[1] + 1
    tr = synthetic(0, tag + b"trace-rand", 2 * st_g.num_randomizers)
    rc = synthetic(0, tag + b"rand-poly", nrc)
    bnd = rp_o.boundary_constraints(out)
    ps = sg.IndependentProofStream()
    t0 = time.perf_counter()
    st_g.prove(trace, air_g, bnd, ps, tr, rc)
    t1 = time.perf_counter()
    phases = {}
    want = fc.stark_prove_rescue(rp_o, st_o, trace, bnd, tr, rc, bounds=bounds, phases=phases)
    t2 = time.perf_counter()
    print("trace 2^%d: GPU prove (host buffers) %.1f ms, CPU checker %.1f s (%d threads; %s), %d bytes"
          % (log_rows, (t1 - t0) * 1e3, t2 - t1, fc.threads(),
             ", ".join("%s %.2f" % kv for kv in phases.items()), len(want)))
    return ps, want, rp_o, out, N


@pytest.mark.timeout(900)
def test_c4_proof_bytes_equal_checker(fc):
    """BASELINE config C4 (trace 2^16, FRI domain 2^21): the GPU's proof bytes == the checker's."""
    ps, want, rp_o, out, N = _prove_gpu_and_checker(fc, 16, b"c4-bytes")
    assert ps.digest() == want, "C4 proof bytes differ from the CPU checker's Stark::prove"


@pytest.mark.timeout(1800)
def test_trace_2p20_headline_proof_bytes_and_verified(fc):
    """bench.py's workload: Rescue-Prime m=2, N = 2^20 - 258 rounds (+256 randomizer rows =
    2^20 - 1), expansion 8, c = 64, security 128, transition degree 3: omicron domain 2^22, FRI
    domain 2^25.  Proof bytes == the CPU checker's; the oracle verifier (AIR from its structure,
    C++ barycentric round-constant interpolants and zerofier products) accepts it and rejects a
    false claim."""
    ps, want, rp_o, out, N = _prove_gpu_and_checker(fc, 20, b"headline")
    assert ps.digest() == want, "headline proof bytes differ from the CPU checker's Stark::prove"
    del want
    objs = ps.objects()
    vst = fc.verifier_stark(8, 64, 128, 2, N + 1, 3)
    sair = fc.rescue_air_at_point(rp_o, vst.omicron)
    bnd = rp_o.boundary_constraints(out)
    ok, err = vst.verify(sair, bnd, o.IndependentProofStream(objs))
    assert ok, err
    ok, _ = vst.verify(sair, rp_o.boundary_constraints(o.add_mod(out, 1)), o.IndependentProofStream(objs))
    assert not ok


# ------------------------------------------------------------------ C5 sharded

C5_LOG = 27


@pytest.fixture(scope="module")
def c5_reference(fc):
    """x (2^27 seeded elements) and X = single-GPU sg.ntt(x), checked against the CPU checker."""
    n = 1 << C5_LOG
    tmp = tempfile.mkdtemp(prefix="sg_c5_")
    try:
        rng = np.random.default_rng(2027)
        x = rng.integers(0, 2**63, size=(n, 2), dtype=np.uint64)
        x[:, 1] %= np.uint64(0xCB80000000000000)
        root = o.primitive_nth_root(n)
        X = sg.ntt(root, x)
        assert np.array_equal(X, fc.ntt(root, x)), "single-GPU 2^27 NTT != checker"
        np.save(os.path.join(tmp, "x.npy"), x)
        np.save(os.path.join(tmp, "X.npy"), X)
        del x, X
        yield tmp
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _c5_native_worker(rank, world, port, tmp):
    """C5 through the C ABI (sg_dist_ntt / sg_dist_intt, host-staged transport over gloo)."""
    import torch
    import torch.distributed as dist
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = sg.Context(0)
        nd = D.NativeDist(ctx, transport="host")
        n = 1 << C5_LOG
        n1, n2 = nd.plan(n, world)
        rows, R = n1 // world, n2 // world
        x = np.load(os.path.join(tmp, "x.npy"), mmap_mode="r")
        X = np.load(os.path.join(tmp, "X.npy"), mmap_mode="r")
        cols = np.ascontiguousarray(x.reshape(n2, n1, 2)[:, rank * rows:(rank + 1) * rows].transpose(1, 0, 2))
        dev = torch.device("cuda", 0)
        shard = torch.from_numpy(cols.view(np.int64).reshape(-1)).to(dev)
        root = o.primitive_nth_root(n)
        runs = nd.ntt(root, shard, n2, n)
        got = runs.cpu().numpy().view(np.uint64).reshape(n1, R, 2)
        want = X.reshape(n1, n2, 2)[:, rank * R:(rank + 1) * R]
        ok = bool(np.array_equal(got, want))
        back = nd.intt(root, runs, n)
        ok_inv = bool(torch.equal(back, shard))
        flags = [None] * world
        dist.all_gather_object(flags, (ok, ok_inv))
        assert all(f[0] for f in flags), f"sg_dist_ntt 2^{C5_LOG} differs from the single-GPU transform: {flags}"
        assert all(f[1] for f in flags), f"sg_dist_intt did not invert sg_dist_ntt at 2^{C5_LOG}: {flags}"
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_c5_native_dist_2p27_one_gpu(c5_reference, world):
    """BASELINE config C5 (2^27-point NTT sharded over the ranks) through the C ABI: bit-identical
    to the single-GPU NTT (checked against the CPU checker), and sg_dist_intt inverts it."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_c5_native_worker, args=(world, port, c5_reference), nprocs=world, join=True)


def test_c5_native_dist_2p27_world1_rccl(c5_reference):
    """C5 through sg_dist_ntt / sg_dist_intt on a one-rank RCCL communicator: each collective then
    moves the whole 2 GiB shard per peer, above what one RCCL call carries (dist.cpp exchange:
    kMaxCollBytes chunks) -- bit-identical to the single-GPU transform, and inverted."""
    import torch
    from starkgpu import dist as D
    ctx = sg.Context(0)
    nd = D.NativeDist(ctx, transport="rccl")
    try:
        n = 1 << C5_LOG
        n1, n2 = nd.plan(n, 1)
        x = np.load(os.path.join(c5_reference, "x.npy"), mmap_mode="r")
        X = np.load(os.path.join(c5_reference, "X.npy"), mmap_mode="r")
        cols = np.ascontiguousarray(x.reshape(n2, n1, 2).transpose(1, 0, 2))
        dev = torch.device("cuda", 0)
        shard = torch.from_numpy(cols.view(np.int64).reshape(-1)).to(dev)
        del cols
        root = o.primitive_nth_root(n)
        runs = nd.ntt(root, shard, n2, n)
        assert np.array_equal(runs.cpu().numpy().view(np.uint64).reshape(n, 2), X), "sg_dist_ntt at world 1"
        back = nd.intt(root, runs, n)
        assert torch.equal(back, shard), "sg_dist_intt at world 1"
    finally:
        nd.close()


def _c5_rccl_worker(rank, world, port, logn):
    """One rank per GPU over RCCL: the sharded NTT of a 2^logn input (every rank builds the same
    input) against the single-GPU transform this rank computes of the whole input."""
    import torch
    import torch.distributed as dist
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # carries the RCCL unique id only
    try:
        ctx = sg.Context(rank)
        nd = D.NativeDist(ctx, transport="rccl")
        n = 1 << logn
        rng = np.random.default_rng(2028)
        x = rng.integers(0, 2**63, size=(n, 2), dtype=np.uint64)
        x[:, 1] %= np.uint64(0xCB80000000000000)
        root = o.primitive_nth_root(n)
        X = sg.ntt(root, x, ctx=ctx)
        n1, n2 = nd.plan(n, world)
        rows, R = n1 // world, n2 // world
        cols = np.ascontiguousarray(x.reshape(n2, n1, 2)[:, rank * rows:(rank + 1) * rows].transpose(1, 0, 2))
        del x
        dev = torch.device("cuda", rank)
        shard = torch.from_numpy(cols.view(np.int64).reshape(-1)).to(dev)
        del cols
        runs = nd.ntt(root, shard, n2, n)
        ok = bool(np.array_equal(runs.cpu().numpy().view(np.uint64).reshape(n1, R, 2),
                                 X.reshape(n1, n2, 2)[:, rank * R:(rank + 1) * R]))
        ok_inv = bool(torch.equal(nd.intt(root, runs, n), shard))
        flags = [None] * world
        dist.all_gather_object(flags, (ok, ok_inv))
        assert all(f[0] and f[1] for f in flags), f"RCCL sharded NTT 2^{logn} at world {world}: {flags}"
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_c5_multi_gpu_rccl_chunked_exchange():
    """the RCCL exchange's chunked path at more than one rank.  2^28 points over 2 GPUs
    (one rank each): every rank's all-to-all moves 2 GiB, above the 1 GiB one RCCL call carries
    correctly, so it goes as grouped send / receive chunks between the GPUs --
    bit-identical to the single-GPU transform, and inverted.  Skipped on a one-GPU box."""
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs (one RCCL rank per device)")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_c5_rccl_worker, args=(2, port, 28), nprocs=2, join=True)
