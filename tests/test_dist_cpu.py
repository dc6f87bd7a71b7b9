"""Multi-rank logic of the sharded path (the test model tests/dist_model.py) on CPU: gloo, world 2 and 4.

The local row steps come from the oracle (tests/dist_cpu_backend.py); what is
under test is the distribution itself -- the four-step index maps and its one
all-to-all, the inverse with swapped factors, the coset scale on column
shards, run-root gathering for the Merkle root, run-sharded FRI folds, the
gathered tail and the resulting proof-stream bytes -- against the oracle's
single-process results (fft/ntt.rs, ntt_arithmetics.rs:161-170,
merkle_root.rs:21-32, fri.rs:115-172).
"""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import stark_oracle as O


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cases(world):
    from starkgpu import dist as D
    import dist_model as M
    from dist_cpu_backend import CpuRows

    be = CpuRows()
    ds = M.DistStark(be, M.Comm())
    g = ds.g

    def gather(buf):
        vals = be.to_ints(buf)
        allv = [None] * world
        dist.all_gather_object(allv, vals)
        return allv

    # four-step ntt / intt
    for n in (16, 64, 256):
        if n < world * world:
            continue
        root = O.primitive_nth_root(n)
        x = O.synthetic_elements(3, b"dist-ntt", n)
        cols = D.scatter_columns(x, n, world, g)
        shard = be.from_ints([v for row in cols for v in row])
        out = ds.ntt(root, shard, len(cols[0]), n)
        full = D.gather_runs(gather(out), n, world)
        assert full == O.ntt(root, x), f"ntt n={n} world={world}"
        back = ds.intt(root, out, n)
        assert be.to_ints(back) == [v for row in cols for v in row], f"intt n={n}"

    # LDE of d = n/8 coefficients on the coset (fast_coset_evaluate), then its Merkle root
    n, d = 256, 32
    coeffs = O.synthetic_elements(4, b"dist-lde", d)
    omega = O.primitive_nth_root(n)
    cols = D.scatter_columns(coeffs, n, world, g)
    shard = be.from_ints([v for row in cols for v in row])
    cw_shard = ds.coset_evaluate(omega, n, O.GENERATOR, shard, len(cols[0]))
    cw = D.gather_runs(gather(cw_shard), n, world)
    assert cw == O.fast_coset_evaluate(omega, n, O.GENERATOR, coeffs), "coset_evaluate"
    n1, n2 = D.plan(n, world)
    assert ds.merkle_root(cw_shard, n1, n2 // world) == O.merkle_commit(cw), "merkle root"

    # FRI commit: tail after the shards collapse (c = 2), and all rounds sharded (c = 16)
    for expansion, c in ((4, 2), (4, 16)):
        ref = O.IndependentProofStream()
        O.FRI(O.GENERATOR, omega, n, expansion, c).commit(cw, ref)
        got = O.IndependentProofStream()
        ds.fri_commit(O.GENERATOR, omega, cw_shard, n, expansion, c, got)
        assert got.digest() == ref.digest(), f"fri commit stream c={c}"


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _cases(world)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_path_matches_oracle(world):
    mp.spawn(_worker, args=(world, _free_port()), nprocs=world, join=True)


def test_plan_and_scatter_helpers():
    from starkgpu import dist as D
    assert D.plan(1 << 27, 8) == (1 << 13, 1 << 14)
    assert D.plan(256, 4) == (16, 16)
    with pytest.raises(ValueError):
        D.plan(32, 8)
    x = list(range(64))
    n1, n2 = D.plan(64, 2)
    cols = [D.scatter_columns(x, 64, 2, g) for g in range(2)]
    # column shard row r of rank g holds x[(g N1/G + r) + N1 j2]
    assert cols[1][0] == [x[(n1 // 2) + n1 * j2] for j2 in range(n2)]
    runs = [[v for k1 in range(n1) for v in x[k1 * n2 + g * (n2 // 2):k1 * n2 + (g + 1) * (n2 // 2)]]
            for g in range(2)]
    assert D.gather_runs(runs, 64, 2) == x
