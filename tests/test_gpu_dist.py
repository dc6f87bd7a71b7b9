"""GPU tests of the row-sharded C ABI and the multi-GPU driver (starkgpu/dist.py).

* the new entry points (sg_ntt_rows_dev, sg_mul_pow_dev, sg_transpose_dev,
  sg_merkle_forest_dev / sg_merkle_top_dev, sg_fri_fold_runs_dev) against the
  oracle and the single-GPU path;
* the test model of the sharded path (tests/dist_model.py: DistStark over the row entry points)
  with the HIP backend at world size 1 (in process) and world size 2
  (two processes sharing this box's one GPU over gloo, device tensors staged
  through the host): four-step NTT / INTT, sharded LDE, Merkle root and FRI
  commit proof-stream bytes equal the single-GPU results (which the parity
  suite pins to the oracle).
"""
import ctypes
import json
import os
import socket

import numpy as np
import pytest

import stark_oracle as o

pytestmark = pytest.mark.gpu


def _dev():
    import torch
    return torch.device("cuda", 0)


def _t(arr):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.int64).reshape(-1).copy()).to(_dev())


def _np(t):
    return t.cpu().numpy().view(np.uint64).reshape(-1, 2)


def _rand(seed, n):
    x = np.random.default_rng(seed).integers(0, 2**63, size=(n, 2), dtype=np.uint64)
    x[:, 1] %= np.uint64(0xCB80000000000000)
    return x


def _ints(a):
    import starkgpu as sg
    return sg.to_ints(a)


# ------------------------------------------------------------------ row-sharded ABI

@pytest.mark.parametrize("n,n_in,rows", [(1, 1, 3), (2, 1, 5), (16, 16, 7), (64, 9, 4), (1 << 12, 1 << 12, 3),
                                         (1 << 13, 1 << 10, 2), (1 << 14, 1 << 14, 5),
                                         # 2^6..2^11 points, 2^(11 - log n) rows per tile (the whole-transform
                                         # first pass) and row counts it does not divide (the generic path)
                                         (64, 64, 32), (64, 33, 64), (256, 200, 16), (512, 512, 12),
                                         (1024, 1024, 6), (1024, 77, 3), (2048, 700, 3), (2048, 2048, 1)])
def test_ntt_rows_matches_oracle(n, n_in, rows):
    import torch
    from starkgpu import dist as D
    import dist_model as M
    import ref_cpu
    be = M.GpuRows()
    root = o.primitive_nth_root(n)
    x = _rand(n + rows, rows * n_in)
    src = _t(x)
    dst = torch.empty(2 * rows * n, dtype=torch.int64, device=_dev())
    be.ntt_rows(root, src, n_in, rows, dst, n)
    out = _np(dst)
    for r in range(rows):
        row = np.zeros((n, 2), dtype=np.uint64)
        row[:n_in] = x[r * n_in:(r + 1) * n_in]
        assert np.array_equal(out[r * n:(r + 1) * n], ref_cpu.ntt(root, row)), r


def test_ntt_rows_beyond_grid_limit():
    """70000 rows (> 65535 per launch) of n = 8: chunked launches, every row right."""
    import torch
    from starkgpu import dist as D
    import dist_model as M
    be = M.GpuRows()
    n, rows = 8, 70000
    root = o.primitive_nth_root(n)
    pats = _rand(5, 3 * n).reshape(3, n, 2)
    x = np.concatenate([pats[r % 3] for r in range(rows)])
    dst = torch.empty(2 * rows * n, dtype=torch.int64, device=_dev())
    be.ntt_rows(root, _t(x), n, rows, dst, n)
    out = _np(dst).reshape(rows, n, 2)
    expect = [o.ntt(root, _ints(pats[k])) for k in range(3)]
    for r in [0, 1, 2, 65534, 65535, 65536, 69999]:
        assert _ints(out[r]) == expect[r % 3], r


def test_mul_pow_and_transpose():
    import torch
    from starkgpu import dist as D
    import dist_model as M
    be = M.GpuRows()
    rows, cols = 37, 53
    base = o.synthetic_elements(1, b"base", 1)[0]
    x = _rand(11, rows * cols)
    buf = _t(x)
    a0, a1, b0, b1 = 5, 3, 7, 11
    be.mul_pow(base, buf, rows, cols, a0, a1, b0, b1)
    got = _ints(_np(buf))
    xi = _ints(x)
    for r in (0, 1, 17, 36):
        for c in (0, 1, 30, 52):
            e = (a0 + a1 * r) * c + b0 + b1 * r
            assert got[r * cols + c] == o.mul_mod(xi[r * cols + c], o.fpow(base, e))
    for A, B, C in [(37, 53, 1), (3, 5, 16), (64, 8, 4), (1, 9, 2), (300, 2, 1)]:
        y = _rand(A * B * C, A * B * C)
        dst = torch.empty(2 * A * B * C, dtype=torch.int64, device=_dev())
        be.transpose(_t(y), dst, A, B, C)
        expect = y.reshape(A, B, C, 2).transpose(1, 0, 2, 3).reshape(-1, 2)
        assert np.array_equal(_np(dst), expect), (A, B, C)


def test_forest_top_and_fold_runs():
    import torch
    import starkgpu as sg
    from starkgpu import dist as D
    import dist_model as M
    be = M.GpuRows()
    run, runs = 1 << 10, 8
    x = _rand(21, run * runs)
    buf = _t(x)
    roots = be.forest_roots(buf, run, runs).cpu().numpy().tobytes()
    for k in range(runs):
        assert roots[64 * k:64 * (k + 1)] == sg.MerkleRoot.commit(x[k * run:(k + 1) * run])
    # the top over the run roots (natural run order) is the root of the whole vector
    top = be.top_root(be.forest_roots(buf, run, runs), runs)
    assert top == sg.MerkleRoot.commit(x)
    one = be.top_root(be.forest_roots(buf[:2 * run], run, 1), 1)
    assert one == sg.MerkleRoot.commit(x[:run])
    # fold of the whole codeword as one run == the reference fold (fri.rs:150-159)
    n = 1 << 8
    w = o.primitive_nth_root(n)
    cw = o.synthetic_elements(2, b"fold", n)
    alpha = o.synthetic_elements(3, b"alpha", 1)[0]
    dst = torch.empty(n, dtype=torch.int64, device=_dev())
    be.fold_runs(w, o.GENERATOR, alpha, be.from_ints(cw), n, n // 2, n // 2, 0, n, dst)
    assert be.to_ints(dst) == o.FRI.fold(cw, alpha, w, o.GENERATOR)
    # same fold over a shard holding runs [k1][4] of a 2-rank split (rank 1)
    G, n1 = 2, 16
    n2 = n // n1
    R = n2 // G
    shard = [cw[k1 * n2 + R + c] for k1 in range(n1) for c in range(R)]
    dst2 = torch.empty(n, dtype=torch.int64, device=_dev())
    be.fold_runs(w, o.GENERATOR, alpha, be.from_ints(shard), n1 * R, R, n2, R, n, dst2)
    full = o.FRI.fold(cw, alpha, w, o.GENERATOR)
    assert be.to_ints(dst2, n1 * R // 2) == [full[k1 * n2 + R + c] for k1 in range(n1 // 2) for c in range(R)]


# ------------------------------------------------------------------ DistStark, world size 1

@pytest.mark.parametrize("logn", [12, 16, 20])
def test_dist_world1_ntt_lde_merkle(logn):
    import torch
    import starkgpu as sg
    from starkgpu import dist as D
    import dist_model as M
    ds = M.DistStark(M.GpuRows(), M.Comm())
    n = 1 << logn
    root = sg.primitive_nth_root(n)
    x = _rand(logn, n)
    cols, row = D.scatter_columns_np(x, n, 1, 0)
    out = ds.ntt(root, _t(cols), row, n)
    got = D.gather_runs_np([_np(out)], n, 1)
    ref = torch.empty(2 * n, dtype=torch.int64, device=_dev())
    xt = _t(x)
    sg.ntt_dev(root, xt.data_ptr(), n, ref.data_ptr())
    assert np.array_equal(got, _np(ref))
    back = ds.intt(root, out, n)
    assert np.array_equal(_np(back), cols)
    # LDE d = n/8 on the coset, then the Merkle root of the run shard
    d = n // 8
    coeffs = x[:d]
    cc, crow = D.scatter_columns_np(coeffs, n, 1, 0)
    cw = ds.coset_evaluate(root, n, sg.generator(), _t(cc), crow)
    ref_cw = torch.empty(2 * n, dtype=torch.int64, device=_dev())
    sg.fast_coset_evaluate_dev(root, n, sg.generator(), _t(coeffs).data_ptr(), d, ref_cw.data_ptr())
    assert np.array_equal(D.gather_runs_np([_np(cw)], n, 1), _np(ref_cw))
    n1, n2 = D.plan(n, 1)
    assert ds.merkle_root(cw, n1, n2) == sg.DeviceTree(ref_cw.data_ptr(), n).root()


def test_dist_world1_fri_commit_stream():
    import torch
    import starkgpu as sg
    from starkgpu import dist as D
    import dist_model as M
    ds = M.DistStark(M.GpuRows(), M.Comm())
    n, exp, c = 1 << 14, 8, 16
    w = sg.primitive_nth_root(n)
    cw = _rand(77, n)
    ref = sg.IndependentProofStream()
    sg.FRI(sg.generator(), w, n, exp, c).commit(cw, ref)
    n1, n2 = D.plan(n, 1)
    shard = cw.reshape(n1, n2, 2).reshape(-1, 2)   # world 1: the run shard is the natural order
    got = sg.IndependentProofStream()
    ds.fri_commit(sg.generator(), w, _t(shard), n, exp, c, got)
    assert got.digest() == ref.digest()


# ------------------------------------------------------------------ DistStark, world size 2 on one GPU

def _world2_worker(rank, world, port, logn):
    import torch
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    import dist_model as M
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = sg.Context(0)
        ds = M.DistStark(M.GpuRows(ctx), M.Comm())
        n = 1 << logn
        root = sg.primitive_nth_root(n)
        x = _rand(logn, n)
        cols, row = D.scatter_columns_np(x, n, world, rank)
        out = ds.ntt(root, _t(cols), row, n)
        shards = [None] * world
        dist.all_gather_object(shards, _np(out))
        full = D.gather_runs_np(shards, n, world)
        assert np.array_equal(full, sg.ntt(root, x, ctx=ctx)), "ntt"
        assert np.array_equal(_np(ds.intt(root, out, n)), cols), "intt"
        d = n // 8
        cc, crow = D.scatter_columns_np(x[:d], n, world, rank)
        cw = ds.coset_evaluate(root, n, sg.generator(), _t(cc), crow)
        dist.all_gather_object(shards, _np(cw))
        cw_full = D.gather_runs_np(shards, n, world)
        assert np.array_equal(cw_full, sg.fast_coset_evaluate(root, n, sg.generator(), x[:d], ctx=ctx)), "lde"
        n1, n2 = D.plan(n, world)
        assert ds.merkle_root(cw, n1, n2 // world) == sg.MerkleRoot.commit(cw_full, ctx=ctx), "merkle"
        ref = sg.IndependentProofStream()
        sg.FRI(sg.generator(), root, n, 8, 16, ctx=ctx).commit(cw_full, ref)
        got = sg.IndependentProofStream()
        ds.fri_commit(sg.generator(), root, cw, n, 8, 16, got)
        assert got.digest() == ref.digest(), "fri stream"
    finally:
        dist.destroy_process_group()


def test_dist_world2_one_gpu_gloo():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_world2_worker, args=(2, port, 14), nprocs=2, join=True)


# ------------------------------------------------------------------ the C-ABI communicator (sg_dist_*)

def _native_checks(nd, ctx, world, rank, logn, gather):
    """sg_dist_ntt / intt / coset_evaluate / merkle_root / fri_commit against the single-GPU path
    (itself pinned to the oracle by the parity suite); gather(local ndarray) -> every rank's."""
    import starkgpu as sg
    from starkgpu import dist as D
    n = 1 << logn
    root = sg.primitive_nth_root(n)
    x = _rand(1000 + logn, n)
    cols, row = D.scatter_columns_np(x, n, world, rank)
    runs = nd.ntt(root, _t(cols), row, n)
    full = D.gather_runs_np(gather(_np(runs)), n, world)
    assert np.array_equal(full, sg.ntt(root, x, ctx=ctx)), "ntt"
    assert np.array_equal(_np(nd.intt(root, runs, n)), cols), "intt"
    # a short column shard (zero tails: the row transforms skip stages)
    d = n // 8
    cc, crow = D.scatter_columns_np(x[:d], n, world, rank)
    cw = nd.coset_evaluate(root, n, sg.generator(), _t(cc), crow)
    cw_full = D.gather_runs_np(gather(_np(cw)), n, world)
    assert np.array_equal(cw_full, sg.fast_coset_evaluate(root, n, sg.generator(), x[:d], ctx=ctx)), "lde"
    assert nd.merkle_root(cw, n) == sg.MerkleRoot.commit(cw_full, ctx=ctx), "merkle"
    # FRI: c = 16 folds down to one run per rank and finishes on the gathered codeword; c = n/16
    # (two rounds) ends while still sharded and gathers the last codeword.  SG_DIST_FRI_TAIL: the
    # codeword size at which the sharded rounds hand over to the single-GPU commit (0: never
    # early; logn - 2: after two sharded rounds, with several runs per rank left; logn: at once)
    try:
        for tail in (0, logn - 2, logn):
            nd.set_fri_tail(tail)  # collective: every rank sets the same hand-over size
            for c in (16, n // 16):
                ref = sg.IndependentProofStream()
                sg.FRI(sg.generator(), root, n, 8, c, ctx=ctx).commit(cw_full, ref)
                got = sg.IndependentProofStream()
                nd.fri_commit(sg.generator(), root, cw, n, 8, c, got)
                assert got.digest() == ref.digest(), f"fri stream c={c} tail={tail}"
                # FRI::prove (fri.rs:210-248): openings gathered from the ranks that own the leaves
                ref = sg.IndependentProofStream()
                top = sg.FRI(sg.generator(), root, n, 8, c, ctx=ctx).prove(cw_full, ref)
                got = sg.IndependentProofStream()
                gtop = nd.fri_prove(sg.generator(), root, cw, n, 8, c, got)
                assert gtop == top, f"fri prove top indices c={c} tail={tail}"
                assert got.digest() == ref.digest(), f"fri prove stream c={c} tail={tail}"
    finally:
        nd.set_fri_tail(20)


def test_native_dist_world1_rccl():
    """sg_dist_create from an RCCL unique id (1 rank: the collectives run through RCCL)."""
    import starkgpu as sg
    from starkgpu import dist as D
    ctx = sg.Context(0)
    nd = D.NativeDist(ctx, transport="rccl")
    try:
        _native_checks(nd, ctx, 1, 0, 12, lambda a: [a])
    finally:
        nd.close()


def _native_worker(rank, world, port, logn):
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = sg.Context(0)
        nd = D.NativeDist(ctx, transport="host")

        def gather(a):
            out = [None] * world
            dist.all_gather_object(out, a)
            return out

        _native_checks(nd, ctx, world, rank, logn, gather)
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,logn", [(2, 14), (8, 14), (4, 17)])
def test_native_dist_one_gpu_host_transport(world, logn):
    """world ranks sharing this box's GPU, the library's all-to-all / all-gather staged through
    host buffers over gloo (RCCL refuses two ranks on one device)."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_native_worker, args=(world, port, logn), nprocs=world, join=True)


# ------------------------------------------------------------------ north-star block, sharded FRI::prove

NS_LOG, NS_EXP, NS_C = 24, 8, 64


@pytest.fixture(scope="module")
def north_star_reference():
    """The north-star block on one GPU: LDE of a seeded degree < 2^21 polynomial onto 2^24 points
    (fast_coset_evaluate) + FRI::prove(expansion 8, c = 64): proof bytes and top indices."""
    import shutil
    import tempfile
    import starkgpu as sg
    n = 1 << NS_LOG
    d = n // NS_EXP
    coeffs = _rand(2024, d)
    root = sg.primitive_nth_root(n)
    cw = sg.fast_coset_evaluate(root, n, sg.generator(), coeffs)
    ps = sg.IndependentProofStream()
    top = sg.FRI(sg.generator(), root, n, NS_EXP, NS_C).prove(cw, ps)
    tmp = tempfile.mkdtemp(prefix="sg_ns_")
    try:
        np.save(os.path.join(tmp, "coeffs.npy"), coeffs)
        with open(os.path.join(tmp, "proof.bin"), "wb") as f:
            f.write(ps.digest())
        np.save(os.path.join(tmp, "top.npy"), np.array(top, dtype=np.uint64))
        yield tmp
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _north_star_worker(rank, world, port, tmp, tail):
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SG_DIST_FRI_TAIL"] = tail
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = sg.Context(0)
        nd = D.NativeDist(ctx, transport="host")
        n = 1 << NS_LOG
        root = sg.primitive_nth_root(n)
        coeffs = np.load(os.path.join(tmp, "coeffs.npy"))
        cols, row = D.scatter_columns_np(coeffs, n, world, rank)
        runs = nd.coset_evaluate(root, n, sg.generator(), _t(cols), row)
        ps = sg.IndependentProofStream()
        top = nd.fri_prove(sg.generator(), root, runs, n, NS_EXP, NS_C, ps)
        want = open(os.path.join(tmp, "proof.bin"), "rb").read()
        ok = (ps.digest() == want, top == [int(t) for t in np.load(os.path.join(tmp, "top.npy"))])
        flags = [None] * world
        dist.all_gather_object(flags, ok)
        assert all(f[0] for f in flags), f"sharded FRI::prove bytes differ from the single-GPU proof: {flags}"
        assert all(f[1] for f in flags), f"sharded FRI::prove top indices differ: {flags}"
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("tail", ["20", "0"])
@pytest.mark.parametrize("world", [2, 8])
def test_north_star_sharded_lde_fri_prove(north_star_reference, world, tail):
    """The north-star block sharded over `world` ranks on this box's GPU (host transport over gloo):
    sg_dist_coset_evaluate (2^21 -> 2^24) + sg_dist_fri_prove (expansion 8, c = 64) write the
    single-GPU FRI::prove bytes (fri.rs:210-248) on every rank -- with the default hand-over of the
    rounds <= 2^20 to the single-GPU commit, and with every round sharded (SG_DIST_FRI_TAIL=0)."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_north_star_worker, args=(world, port, north_star_reference, tail), nprocs=world, join=True)


# ------------------------------------------------------------------ sharded Stark::prove

# (N, expansion, colinearity checks, security, transition degree): FRI domains 2^9 .. 2^21, and
# 2^8 (too small to split over 8 ranks: every rank proves it whole)
STARK_CASES = [(40, 4, 3, 4, 2), (27, 8, 4, 8, 3), (100, 8, 8, 16, 3), (65278, 8, 64, 128, 3), (9, 4, 2, 2, 2)]


@pytest.fixture(scope="module")
def stark_reference():
    """Rescue-Prime Stark::prove inputs and expected proof bytes per case: the oracle's bytes for
    the small cases, the single-GPU bytes at C4 (pinned to the CPU checker by
    test_gpu_fullsize.py::test_c4_proof_bytes_equal_checker).  Plus one false witness."""
    import shutil
    import tempfile
    import stark_prove_oracle as e
    import starkgpu as sg
    tmp = tempfile.mkdtemp(prefix="sg_dstark_")
    try:
        for k, (N, exp, c, sec, tcd) in enumerate(STARK_CASES):
            seed = b"dist-stark-%d" % k
            rp_o = e.RescuePrime(2, 1, sec, N)
            st_g = sg.Stark(exp, c, sec, 2, N + 1, tcd)
            rp_g = sg.RescuePrime(2, 1, sec, N)
            air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
            inp = o.sample(seed)
            trace = rp_g.trace_array(inp)
            if k == 1:  # a false witness: the reference still writes a (rejected) proof
                t = sg.to_ints(trace)
                t[9] = o.add_mod(t[9], 3)
                trace = sg.fe_array(t)
            nrc = st_g.num_randomizer_coefficients(air_g)
            r = e.randomness_from_seed(seed, 2 * st_g.num_randomizers + nrc)
            tr, rc = sg.fe_array(r[:2 * st_g.num_randomizers]), sg.fe_array(r[2 * st_g.num_randomizers:])
            bnd = rp_o.boundary_constraints(rp_o.hash(inp))
            if N < 1000:
                st_o = e.Stark(exp, c, sec, 2, N + 1, tcd)
                air_o = rp_o.transition_constraints(st_o.omicron, st_o.omicron_domain_length)
                rows = sg.to_ints(trace)
                want = st_o.prove([rows[2 * i:2 * i + 2] for i in range(len(rows) // 2)], air_o, bnd,
                                  o.IndependentProofStream(), [r[2 * i:2 * i + 2] for i in range(st_g.num_randomizers)],
                                  r[2 * st_g.num_randomizers:])
            else:
                want = st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc)
            np.save(os.path.join(tmp, "trace%d.npy" % k), trace)
            np.save(os.path.join(tmp, "tr%d.npy" % k), tr)
            np.save(os.path.join(tmp, "rc%d.npy" % k), rc)
            with open(os.path.join(tmp, "bnd%d.json" % k), "w") as f:
                json.dump([[int(a), int(b), str(v)] for (a, b, v) in bnd], f)
            with open(os.path.join(tmp, "proof%d.bin" % k), "wb") as f:
                f.write(want)
        yield tmp
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _stark_checks(nd, world, rank, tmp, cases, gather, sharded_algebra=True):
    """Every case proved with sg_dist_stark_prove on this rank: bytes == expected on every rank."""
    import starkgpu as sg
    ok = []
    for k in cases:
        N, exp, c, sec, tcd = STARK_CASES[k]
        st = sg.Stark(exp, c, sec, 2, N + 1, tcd, ctx=nd.ctx)
        air = sg.RescuePrime(2, 1, sec, N, ctx=nd.ctx).transition_constraints(st.omicron, st.omicron_domain_length)
        with open(os.path.join(tmp, "bnd%d.json" % k)) as f:
            bnd = [(a, b, int(v)) for (a, b, v) in json.load(f)]
        trace = np.load(os.path.join(tmp, "trace%d.npy" % k))
        tr, rc = np.load(os.path.join(tmp, "tr%d.npy" % k)), np.load(os.path.join(tmp, "rc%d.npy" % k))
        # small domains: every FRI round sharded (hand-over size 0); C4: the default hand-over
        nd.set_fri_tail(0 if N < 1000 else 20)
        before = nd.counters()
        got = st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc, dist=nd)
        after = nd.counters()
        ok.append((k, got == open(os.path.join(tmp, "proof%d.bin" % k), "rb").read(), after[1] - before[1],
                   after[2] - before[2]))
    flags = gather(ok)
    assert all(f for per_rank in flags for (_, f, _, _) in per_rank), \
        f"world {world}: sharded proof bytes differ: {flags}"
    # the transition quotients' coset work ran on run shards (2 constraints) wherever the coset
    # splits over the ranks: C4 (coset 2^18) at every world > 1, the false witness (coset 2^8,
    # redone from the gathered values) at 2 and 4 ranks; one rank runs the replicated path
    # The boundary quotients' division (order 2^16 at C4, 2^6 for case 1) likewise, and the trace
    # interpolation's transforms (both register columns) where its subgroup (order M = D / f)
    # splits: C4 (M = 2^16) at every world > 1.
    want_sq = {(3, 2): 4, (3, 4): 4, (3, 8): 4, (1, 2): 4, (1, 4): 2}
    for per_rank in flags:
        for (k, _, sq, si) in per_rank:
            if not sharded_algebra:
                assert sq == 0 and si == 0, f"world {world} case {k}: algebra sharded although switched off"
                continue
            if (k, world) in want_sq:
                assert sq == want_sq[(k, world)], f"world {world} case {k}: {sq} sharded quotients"
            if world > 1 and k == 3:
                assert si == 2, f"world {world} case {k}: {si} sharded interpolation columns"
            if world == 1:
                assert sq == 0 and si == 0, f"world 1 case {k}: {sq} / {si} sharded quotients / columns"


@pytest.mark.parametrize("forced", ["1", "0"])
def test_dist_stark_prove_world1_rccl(stark_reference, monkeypatch, forced):
    """sg_dist_stark_prove over a 1-rank RCCL communicator: the single-GPU / oracle proof bytes --
    through the four-step path forced (context option world1_sharded: the sharded machinery over RCCL)
    and through the default one-rank plan (the single-GPU prove)."""
    import starkgpu as sg
    from starkgpu import dist as D
    ctx = sg.Context(0)
    ctx.set_option("world1_sharded", int(forced))
    nd = D.NativeDist(ctx, transport="rccl")
    try:
        _stark_checks(nd, 1, 0, stark_reference, range(len(STARK_CASES)), lambda a: [a])
        st = sg.Stark(4, 3, 4, 2, 41, 2)  # created on another context
        with pytest.raises(ValueError):
            st.prove([[0, 0]], [], [], sg.IndependentProofStream(), [[0, 0]] * st.num_randomizers, [0], dist=nd)
    finally:
        nd.close()


def _stark_worker(rank, world, port, tmp, cases, shard="1"):
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SG_DIST_SHARD_ALGEBRA"] = shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nd = D.NativeDist(sg.Context(0), transport="host")

        def gather(a):
            out = [None] * world
            dist.all_gather_object(out, a)
            return out

        _stark_checks(nd, world, rank, tmp, cases, gather, sharded_algebra=shard != "0")
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,cases,shard", [(2, (0, 1, 2, 3, 4), "1"), (4, (1, 2, 4), "1"), (8, (0, 1, 2, 3, 4), "1"),
                                               (2, (1, 3), "0")])
def test_dist_stark_prove_one_gpu_host_transport(stark_reference, world, cases, shard):
    """Stark::prove (stark.rs:276-562) with the FRI domain sharded over `world` ranks on this box's
    GPU (host transport over gloo): every rank writes the expected proof bytes, C4 included.
    shard = "0": SG_DIST_SHARD_ALGEBRA=0, the trace-domain algebra replicated (no sharded counts)."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_stark_worker, args=(world, port, stark_reference, cases, shard), nprocs=world, join=True)


def _bounded_cache_worker(rank, world, port, tmp, nfill):
    """Rank body of test_dist_prove_with_bounded_cache_full: see there."""
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, exp, c, sec, tcd = STARK_CASES[2]
        trace = np.load(os.path.join(tmp, "trace2.npy"))
        tr, rc = np.load(os.path.join(tmp, "tr2.npy")), np.load(os.path.join(tmp, "rc2.npy"))
        rows = sg.to_ints(trace)

        def bnd(cyc):  # register 0 pinned at cycle 0 (one zerofier for every statement), register 1 at `cyc`
            return [(0, 0, rows[0]), (cyc, 1, rows[2 * cyc + 1])]

        # expected bytes of the last statement: the single-GPU prove on a context of its own
        ref_ctx = sg.Context(0)
        st_r = sg.Stark(exp, c, sec, 2, N + 1, tcd, ctx=ref_ctx)
        air_r = sg.RescuePrime(2, 1, sec, N, ctx=ref_ctx).transition_constraints(st_r.omicron, st_r.omicron_domain_length)
        last = nfill + 2
        want = st_r.prove(trace, air_r, bnd(last), sg.IndependentProofStream(), tr, rc)
        want_first = st_r.prove(trace, air_r, bnd(1), sg.IndependentProofStream(), tr, rc)
        nd = D.NativeDist(sg.Context(0), transport="host")
        nd.set_fri_tail(0)
        st = sg.Stark(exp, c, sec, 2, N + 1, tcd, ctx=nd.ctx)
        air = sg.RescuePrime(2, 1, sec, N, ctx=nd.ctx).transition_constraints(st.omicron, st.omicron_domain_length)
        before = nd.counters()
        ok_first = st.prove(trace, air, bnd(1), sg.IndependentProofStream(), tr, rc, dist=nd) == want_first
        sharded = nd.counters()[1] - before[1]
        for cyc in range(2, last):  # two new bounded tables per statement (register 1's inverse + shard)
            st.prove(trace, air, bnd(cyc), sg.IndependentProofStream(), tr, rc, dist=nd)
        ok_last = st.prove(trace, air, bnd(last), sg.IndependentProofStream(), tr, rc, dist=nd) == want
        tables = nd.ctx.cached_tables()[0]
        flags = [None] * world
        dist.all_gather_object(flags, (ok_first, ok_last, sharded, tables))
        assert all(f[0] and f[1] for f in flags), f"proof bytes differ with the bounded cache full: {flags}"
        assert all(f[2] >= 2 for f in flags), f"the boundary quotients did not run sharded: {flags}"
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dist_prove_with_bounded_cache_full(stark_reference):
    """the sharded boundary quotients hold every register's divisor-inverse
    shard (a bounded, content-keyed table) until their batch is enqueued, while later registers
    insert new tables.  Register 0's zerofier (cycle 0) is the same in every statement, so its
    tables sit at the front of the FIFO once the cache is full; the last statement then hits them
    and inserts register 1's, which would evict (hipFree) the shard still to be read.  The cache is
    pinned for the call (sg::BoundedPin): world 2 on this box's GPU (host transport), the statement
    proved after 32 distinct ones writes the single-GPU prove's bytes, as does the first."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_bounded_cache_worker, args=(2, port, stark_reference, 31), nprocs=2, join=True)


# ----------------------------------------------------------------- failure containment

class _FailingStream(o.IndependentProofStream):
    """A proof stream whose Fiat-Shamir callback fails: the prover has issued collectives by then
    (the randomizer LDE's all-to-all, the forests' run-root all-gathers)."""

    def fiat_shamir_prover(self, num_bytes):
        raise RuntimeError("injected proof-stream failure")


def _load_case(tmp, k):
    N, exp, c, sec, tcd = STARK_CASES[k]
    with open(os.path.join(tmp, "bnd%d.json" % k)) as f:
        bnd = [(a, b, int(v)) for (a, b, v) in json.load(f)]
    return (N, exp, c, sec, tcd), bnd, np.load(os.path.join(tmp, "trace%d.npy" % k)), \
        np.load(os.path.join(tmp, "tr%d.npy" % k)), np.load(os.path.join(tmp, "rc%d.npy" % k))


def test_dist_failure_world1_rccl_poisons(stark_reference, monkeypatch):
    """A call that fails after issuing collectives poisons the RCCL communicator (ncclCommAbort):
    the prove returns an error, sg_dist_poisoned reports it, and every later call fails with
    SG_ERR_INVALID at once instead of issuing collectives out of step with the peers.  (The
    four-step path is forced: a one-rank communicator otherwise proves through the single-GPU plan.)"""
    import starkgpu as sg
    from starkgpu import dist as D
    ctx = sg.Context(0)
    ctx.set_option("world1_sharded", 1)
    nd = D.NativeDist(ctx, transport="rccl")
    try:
        (N, exp, c, sec, tcd), bnd, trace, tr, rc = _load_case(stark_reference, 1)
        st = sg.Stark(exp, c, sec, 2, N + 1, tcd, ctx=ctx)
        air = sg.RescuePrime(2, 1, sec, N, ctx=ctx).transition_constraints(st.omicron, st.omicron_domain_length)
        assert not nd.poisoned
        with pytest.raises(RuntimeError, match="injected"):
            st.prove(trace, air, bnd, _FailingStream(), tr, rc, dist=nd)
        assert nd.poisoned
        with pytest.raises(sg.StarkGpuError) as ei:
            st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc, dist=nd)
        assert ei.value.code == -1 and "poisoned" in str(ei.value)
        with pytest.raises(sg.StarkGpuError):
            nd.set_fri_tail(20)
        # a new communicator on the same context works again and proves the expected bytes
        nd.close()
        nd = D.NativeDist(ctx, transport="rccl")
        got = st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc, dist=nd)
        assert got == open(os.path.join(stark_reference, "proof1.bin"), "rb").read()
    finally:
        nd.close()


def _failure_worker(rank, world, port, tmp):
    import time
    from datetime import timedelta
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    aborted = []

    def on_abort():  # poisoned on this rank: close its pairs so the peers' exchanges fail now
        aborted.append(time.time())
        if dist.is_initialized():
            dist.destroy_process_group()

    out = {"rank": rank}
    try:
        ctx = sg.Context(0)
        nd = D.NativeDist(ctx, transport="host", abort=on_abort)
        (N, exp, c, sec, tcd), bnd, trace, tr, rc = _load_case(tmp, 1)
        st = sg.Stark(exp, c, sec, 2, N + 1, tcd, ctx=ctx)
        air = sg.RescuePrime(2, 1, sec, N, ctx=ctx).transition_constraints(st.omicron, st.omicron_domain_length)
        stream = _FailingStream() if rank == world - 1 else sg.IndependentProofStream()
        t0 = time.time()
        try:
            st.prove(trace, air, bnd, stream, tr, rc, dist=nd)
            out["result"] = "ok"
        except Exception as e:  # noqa: BLE001 - recorded for the parent
            out["result"] = type(e).__name__ + ": " + str(e)
        out["seconds"] = time.time() - t0
        out["poisoned"] = nd.poisoned
        out["aborted"] = bool(aborted)
        try:
            nd.set_fri_tail(20)
            out["after"] = "ok"
        except Exception as e:  # noqa: BLE001
            out["after"] = str(e)
        nd.close()
    finally:
        with open(os.path.join(tmp, "fail_rank%d.json" % rank), "w") as f:
            json.dump(out, f)
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dist_failure_one_rank_host_transport(stark_reference):
    """World 2 on this GPU over the host transport (gloo): rank 1 alone fails mid-prove (its
    Fiat-Shamir callback raises after the commitments' collectives).  Both ranks return an error
    well within the deadline -- rank 1 from its callback, rank 0 from the exchange its peer left --
    both communicators are poisoned, later calls fail at once, and no process is left blocked."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    for r in range(2):
        p = os.path.join(stark_reference, "fail_rank%d.json" % r)
        if os.path.exists(p):
            os.remove(p)
    mp.spawn(_failure_worker, args=(2, port, stark_reference), nprocs=2, join=True)
    res = [json.load(open(os.path.join(stark_reference, "fail_rank%d.json" % r))) for r in range(2)]
    for r in res:
        assert r["result"] != "ok", res
        assert r["poisoned"] and r["aborted"], res
        assert "poisoned" in r["after"], res
        assert r["seconds"] < 30, res  # within the default deadline (SG_DIST_TIMEOUT_S = 30 s)
    assert "injected" in res[1]["result"], res


def _rccl_failure_worker(rank, world, port, tmp, out_dir):
    """One rank per GPU over RCCL: the last rank's Fiat-Shamir callback raises mid-prove."""
    import time
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # carries the RCCL unique id only
    out = {"rank": rank}
    try:
        ctx = sg.Context(rank)
        nd = D.NativeDist(ctx, transport="rccl")
        (N, exp, c, sec, tcd), bnd, trace, tr, rc = _load_case(tmp, 3)  # C4: many collectives per prove
        st = sg.Stark(exp, c, sec, 2, N + 1, tcd, ctx=ctx)
        air = sg.RescuePrime(2, 1, sec, N, ctx=ctx).transition_constraints(st.omicron, st.omicron_domain_length)
        want = open(os.path.join(tmp, "proof3.bin"), "rb").read()
        out["clean"] = st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc, dist=nd) == want
        stream = _FailingStream() if rank == world - 1 else sg.IndependentProofStream()
        t0 = time.time()
        try:
            st.prove(trace, air, bnd, stream, tr, rc, dist=nd)
            out["result"] = "ok"
        except Exception as e:  # noqa: BLE001 - recorded for the parent
            out["result"] = type(e).__name__ + ": " + str(e)
        out["seconds"] = time.time() - t0
        out["poisoned"] = nd.poisoned
        nd.close()
    finally:
        with open(os.path.join(out_dir, "rccl_fail_rank%d.json" % rank), "w") as f:
            json.dump(out, f)
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_dist_failure_multi_gpu_rccl_peers_fail_promptly(stark_reference, tmp_path):
    """One process per GPU over RCCL (every GPU of the box, up to 8; skipped on a one-GPU box --
    RCCL refuses two ranks on one device): a clean sharded C4 prove writes the expected bytes on
    every rank, then the last rank fails mid-prove.  The failing rank poisons its communicator and
    raises the out-of-band abort flag; every peer, blocked in a collective the failed rank never
    joins, reads the flag within ~10 ms of polling, aborts its own communicator and returns
    "a peer rank failed" -- within seconds, not at the 30 s deadline."""
    import torch
    import torch.multiprocessing as mp
    world = min(torch.cuda.device_count(), 8)
    if world < 2:
        pytest.skip("needs >= 2 GPUs (one RCCL rank per device)")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rccl_failure_worker, args=(world, port, stark_reference, str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(os.path.join(str(tmp_path), "rccl_fail_rank%d.json" % r))) for r in range(world)]
    for r in res:
        assert r["clean"], res
        assert r["result"] != "ok" and r["poisoned"], res
        assert r["seconds"] < 10, res
    assert "injected" in res[-1]["result"], res
    assert all("peer rank failed" in r["result"] for r in res[:-1]), res


# ------------------------------------------- the reference's published configuration, sharded

def _rpsss_worker(rank, world, port, tmp):
    import torch.distributed as dist
    import rpsss_case as R
    import starkgpu as sg
    from starkgpu import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = R.Case()
        ctx = sg.Context(0)
        nd = D.NativeDist(ctx, transport="host")
        rp = sg.RescuePrime(*R.RESCUE, ctx=ctx)
        st = sg.Stark(R.EXPANSION, R.CHECKS, R.SECURITY, rp.m, R.RESCUE[3] + 1, R.TCD, ctx=ctx)
        air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
        before = nd.counters()
        got = st.prove(rp.trace_array(c.sk), air, rp.boundary_constraints(c.pk), sg.SignatureProofStream(R.DOCUMENT),
                       sg.fe_array([v for row in c.trace_randomizers for v in row]),
                       sg.fe_array(c.randomizer_coefficients), dist=nd)
        after = nd.counters()
        res = (got == open(os.path.join(tmp, "rpsss.bin"), "rb").read(), after[1] - before[1], after[2] - before[2])
        flags = [None] * world
        dist.all_gather_object(flags, res)
        assert all(f[0] for f in flags), f"sharded RPSSS signature differs from the oracle's: {flags}"
        # FRI domain 4096: transition quotients (coset 1024) and boundary quotients (order 512) on
        # run shards, and the interpolation (subgroup 512) at 2 and 4 ranks
        assert all(f[1] == 4 and f[2] == 2 for f in flags), flags
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_dist_rpsss_published_configuration(tmp_path, world):
    """RPSSS::sign at rpsss.rs:103 (c = 64, FRI domain 4096, SignatureProofStream) with the prove
    sharded over `world` ranks on this GPU (host transport over gloo), the trace-domain algebra on
    run shards: every rank writes the oracle's 1 156 888-byte signature (rpsss.rs:89)."""
    import torch.multiprocessing as mp
    import rpsss_case as R
    want = R.Case().oracle_sign()
    assert len(want) == R.PROOF_LEN
    (tmp_path / "rpsss.bin").write_bytes(want)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rpsss_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)


# ----------------------------------------------------------------- mid-size statement pinned to the oracle

def _midsize_worker(rank, world, port, results):
    import hashlib
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu import dist as D
    import midsize_case as M
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nd = D.NativeDist(sg.Context(0), transport="host")
        rp_o, st_o, trace, bnd, tr, rc = M.light_inputs()
        rp_g = sg.RescuePrime(*M.RESCUE, ctx=nd.ctx)
        st_g = sg.Stark(M.EXPANSION, M.CHECKS, M.SECURITY, rp_g.m, M.RESCUE[3] + 1, M.TCD, ctx=nd.ctx)
        air = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
        nd.set_fri_tail(0)  # every FRI round sharded at this size
        got = st_g.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc, dist=nd)
        out = [None] * world
        dist.all_gather_object(out, (len(got), hashlib.sha256(got).hexdigest(), nd.counters()[1]))
        if rank == 0:
            with open(results, "w") as f:
                json.dump(out, f)
        nd.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_dist_stark_prove_midsize_equals_oracle_digest(world, tmp_path):
    """sg_dist_stark_prove of the mid-size statement (tests/midsize_case.py: trace 1257 rows, FRI
    domain 2^15, c = 64) over `world` ranks on this GPU (host transport): every rank's proof hashes
    to the Python oracle's committed digest (tests/golden/midsize_proof.json) -- the sharded path
    pinned to the oracle itself above the toy sizes, every FRI round sharded."""
    import torch.multiprocessing as mp
    with open(os.path.join(os.path.dirname(__file__), "golden", "midsize_proof.json")) as f:
        g = json.load(f)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    res = str(tmp_path / "midsize.json")
    mp.spawn(_midsize_worker, args=(world, port, res), nprocs=world, join=True)
    out = json.load(open(res))
    assert all(n == g["proof_len"] and h == g["proof_sha256"] for n, h, _ in out), out
    assert all(sq > 0 for _, _, sq in out), "the quotients' coset work should run on run shards"
