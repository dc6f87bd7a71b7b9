#!/usr/bin/env python3
"""Benchmark: end-to-end Stark::prove on a Rescue-Prime trace of 2^20 rows, on MI355X.

Workload (BASELINE.json metric "NTT Gelem/s + prove ms, Rescue-Prime trace 2^20"):
one step = one complete `Stark::prove` (stark/stark.rs:276-562) of a Rescue-Prime
(m = 2, capacity 1, security 128) execution trace with 2^20 - 1 randomized rows
(N = 2^20 - 258 rounds + 256 randomizer rows; the same convention as BASELINE
config C4 at 2^16), expansion factor 8, 64 colinearity checks, transition degree 3
(omicron domain 2^22, FRI domain 2^25):
  trace interpolation -> boundary quotients -> 2 LDEs + Merkle commits ->
  transition polynomials (AIR on a coset) / zerofier division -> randomizer LDE +
  commit -> Fiat-Shamir weights -> combination polynomial -> LDE -> FRI::prove ->
  openings.
The trace, the randomizers (thread_rng draws, injected from a seeded generator)
and the transition constraints are resident in HBM before timing starts; every
step writes a complete proof into a fresh proof stream.
`value` = committed codeword elements per second ((m + 2) x 2^25 per proof);
`prove_ms` = the proof time.

One process per GPU (torchrun); each rank proves its own independent trace
(weak scaling, no collective on the data path).  Rank 0 prints one JSON line.

Side measurements (not the metric): at N = 1 the other BASELINE configs (C2 2^22 fwd+inv NTT,
the 2^24 north-star LDE + FRI commit, C4's prove at trace 2^16, C5's 2^27 NTT) and the sharded
paths on a one-rank RCCL communicator (`c5_dist_world1_ms`, `sharded_prove_world1_ms` with a
byte check against the single-GPU proof); at N > 1 the same sharded paths over all ranks
(C2 and C5 NTTs, the north-star block with FRI::prove, and the headline proof through
sg_dist_stark_prove, `sharded_prove_ms`, bytes checked on every rank).
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time
from datetime import timedelta

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zk-stark-tutor_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import starkgpu as sg  # noqa: E402

P = sg.FIELD_PRIME
LOG_TRACE = 20      # randomized trace rows + 1 (trace 2^20)
EXPANSION = 8       # FRI domain = 8 x omicron domain (2^25 at the headline)
COLINEARITY = 64
REGISTERS = 2       # Rescue-Prime m = 2
HBM_PEAK_GBS = 8000.0
# PMC HBM bytes of this workload's kernels (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes on
# `bench.py --steps 3 --warmup 1 --no-side`, tools/pmc_passes.sh + tools/pmc_traffic.py)
PMC_TRAFFIC_FILE = "r06_pmc_traffic_e2e.json"
PMC_VALU_FILE = "r06_pmc_valu_e2e.json"  # SQ_INSTS_VALU pass (tools/pmc_passes.sh + tools/pmc_valu.py)
VALU_MIX_FILE = "r06_valu_mix.json"  # static full/half-rate mix of the same build (tools/valu_mix.py)
MAX_CLOCK_GHZ = 2.4  # MI355X_MICROARCH.md:34


def synthetic_fe(seed: int, tag: bytes, n: int) -> np.ndarray:
    """SURVEY.md §8(d) generator, vectorized: BE 16-byte chunks of SHAKE256(...) mod p."""
    import hashlib
    raw = hashlib.shake_256(b"sg-bench" + seed.to_bytes(8, "big") + tag).digest(16 * n)
    be = np.frombuffer(raw, dtype=">u8").reshape(n, 2)
    hi = be[:, 0].astype(np.uint64)
    lo = be[:, 1].astype(np.uint64)
    p_hi, p_lo = np.uint64(P >> 64), np.uint64(P & ((1 << 64) - 1))
    ge = (hi > p_hi) | ((hi == p_hi) & (lo >= p_lo))  # v < 2^128 < 2p: one subtraction
    borrow = (lo < p_lo) & ge
    lo = np.where(ge, lo - p_lo, lo)
    hi = np.where(ge, hi - p_hi - borrow.astype(np.uint64), hi)
    return np.ascontiguousarray(np.stack([lo, hi], axis=1))


def to_device(arr: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(arr.view(np.int64).copy()).to(device)


class ProveWorkload:
    """Stark::prove on a Rescue-Prime trace with 2^log_rows - 1 randomized rows (stark.rs:276-562)."""

    def __init__(self, rank: int, device, ctx: sg.Context, log_rows=LOG_TRACE):
        self.ctx = ctx
        self.N = (1 << log_rows) - 2 - 4 * COLINEARITY  # Rescue rounds: trace N + 1 rows
        self.rp = sg.RescuePrime(REGISTERS, 1, 128, self.N, ctx=ctx)
        self.stark = sg.Stark(EXPANSION, COLINEARITY, 128, REGISTERS, self.N + 1, 3, ctx=ctx)
        self.air = self.rp.transition_constraints(self.stark.omicron, self.stark.omicron_domain_length)
        inp = int.from_bytes(hashlib_shake(b"sg-bench-input" + rank.to_bytes(8, "big"), 16), "big") % P
        self.boundary = self.rp.boundary_constraints(self.rp.hash(inp))
        self.trace = to_device(self.rp.trace_array(inp), device)
        self.rows = self.N + 1
        self.nrc = self.stark.num_randomizer_coefficients(self.air)
        self.trace_rand = to_device(synthetic_fe(rank, b"trace-rand", REGISTERS * self.stark.num_randomizers), device)
        self.rcoef = to_device(synthetic_fe(rank, b"rand-poly", self.nrc), device)
        self.fri_len = self.stark.fri_domain_length
        self.last_proof = None

    def step(self, phases=None):
        t0 = time.perf_counter()
        stream = sg.IndependentProofStream()
        self.stark.prove_dev(self.trace.data_ptr(), self.rows, self.air, self.boundary, stream,
                             self.trace_rand.data_ptr(), self.rcoef.data_ptr(), self.nrc)
        # Stark::prove returns the serialized proof (stark.rs:562): part of the step
        self.last_proof_bytes = stream.digest()
        self.last_proof = stream
        if phases is not None:
            phases["prove"] = phases.get("prove", 0.0) + (time.perf_counter() - t0)
        return stream

    def elements_per_step(self) -> int:
        return (REGISTERS + 2) * self.fri_len


def hashlib_shake(data: bytes, n: int) -> bytes:
    import hashlib
    return hashlib.shake_256(data).digest(n)


class BlockWorkload:
    """The LDE + commit block of earlier rounds (side measurement): synthetic 2^20-coefficient
    polynomials, N = 2^23 (stark.rs:367-386, 425-445, 500-522)."""

    def __init__(self, rank: int, device, ctx: sg.Context, log_trace=LOG_TRACE):
        self.ctx = ctx
        self.d = 1 << log_trace
        self.N = self.d * EXPANSION
        self.omega = sg.primitive_nth_root(self.N)
        self.offset = sg.generator()
        tags = [b"bq0", b"bq1", b"rand", b"comb"]
        self.coeffs = [to_device(synthetic_fe(rank, t, self.d), device) for t in tags]
        self.codewords = [torch.empty((self.N, 2), dtype=torch.int64, device=device) for _ in tags]
        self.fri = sg.FRI(self.offset, self.omega, self.N, EXPANSION, COLINEARITY, ctx=ctx)

    def step(self, phases=None):
        # host clocks time the phases (a phase ends when its roots are on the host)
        ctx = self.ctx
        clk = time.perf_counter
        t0 = clk()
        # stream-ordered device transforms: the LDEs return once enqueued and the tree
        # builds / FRI that consume them follow on the same stream (roots are read by
        # spinning on flags the root kernels raise), so no host round trip per stage
        ctx.set_async(True)
        stream = sg.IndependentProofStream()
        # boundary quotients + randomizer: independent, so their LDEs and trees
        # run as one batched launch sequence each (stark.rs:367-386, 435-445)
        k3 = REGISTERS + 1
        a = clk()
        sg.fast_coset_evaluate_batch_dev(self.omega, self.N, self.offset,
                                         [t.data_ptr() for t in self.coeffs[:k3]], self.d,
                                         [t.data_ptr() for t in self.codewords[:k3]], ctx=ctx)
        b = clk()
        trees = sg.DeviceTree.build_batch([t.data_ptr() for t in self.codewords[:k3]], self.N, ctx=ctx)
        for t in trees:
            stream.push((sg.ROOT, t.root()))
        t_lde = b - a
        t_mk = clk() - b
        stream.fiat_shamir_prover(sg.PROOF_BYTES)  # combination weights (stark.rs:447-450)
        c = REGISTERS + 1
        a = clk()
        sg.fast_coset_evaluate_dev(self.omega, self.N, self.offset, self.coeffs[c].data_ptr(), self.d,
                                   self.codewords[c].data_ptr(), ctx=ctx)
        b = clk()
        top = self.fri.prove_dev(self.codewords[c].data_ptr(), self.N, stream)
        e = clk()
        ctx.set_async(False)
        for t in trees:
            t.free()
        if phases is not None:
            for k, v in (("lde", t_lde + (b - a)), ("merkle_commits", t_mk), ("fri_prove", e - b),
                         ("step", clk() - t0)):
                phases[k] = phases.get(k, 0.0) + v
        return stream, top

    def elements_per_step(self) -> int:
        return (REGISTERS + 2) * self.N


def median_of(fn, reps: int) -> float:
    vals = sorted(fn() for _ in range(reps))
    return vals[len(vals) // 2]


def side_measurements(ctx: sg.Context, device, iters: int = 5) -> dict:
    """The other two configs BASELINE.json names, timed the same way (inputs in HBM):
    C2 = 2^22-point forward + inverse NTT; north star = 2^24 LDE (2^21 coefficients) + FRI commit."""
    out = {}
    n = 1 << 22
    x = to_device(synthetic_fe(7, b"c2", n), device)
    y = torch.empty_like(x)
    z = torch.empty_like(x)
    w = sg.primitive_nth_root(n)
    sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
    sg.intt_dev(w, y.data_ptr(), n, z.data_ptr(), ctx=ctx)
    assert torch.equal(x, z), "C2 INTT(NTT(x)) != x"
    torch.cuda.synchronize(device)

    def c2_rep():
        # the inverse is stream-ordered behind the forward (no host round trip between them);
        # every iteration waits for both on the host
        ctx.set_async(True)
        t0 = time.perf_counter()
        for _ in range(iters):
            sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
            sg.intt_dev(w, y.data_ptr(), n, z.data_ptr(), ctx=ctx)
            ctx.synchronize()
        dt = (time.perf_counter() - t0) / iters
        ctx.set_async(False)
        return dt

    # a sub-millisecond figure: the median of 5 repetitions, so one slow moment does not set it
    t = median_of(c2_rep, 5)
    assert torch.equal(x, z), "C2 INTT(NTT(x)) != x (timed loop)"
    out["c2_ntt_fwd_inv_2p22_ms"] = round(t * 1e3, 3)
    out["c2_ntt_gelem_s"] = round(2 * n / t / 1e9, 3)
    del x, y, z
    d, N = 1 << 21, 1 << 24
    coeffs = to_device(synthetic_fe(8, b"ns", d), device)
    cw = torch.empty((N, 2), dtype=torch.int64, device=device)
    wN = sg.primitive_nth_root(N)
    fri = sg.FRI(sg.generator(), wN, N, EXPANSION, COLINEARITY, ctx=ctx)

    def once():
        sg.fast_coset_evaluate_dev(wN, N, sg.generator(), coeffs.data_ptr(), d, cw.data_ptr(), ctx=ctx)
        fri.commit_dev(cw.data_ptr(), N, sg.IndependentProofStream())
    once()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(max(iters // 2, 1)):
        once()
    torch.cuda.synchronize(device)
    t = (time.perf_counter() - t0) / max(iters // 2, 1)
    out["north_star_lde_fri_commit_2p24_ms"] = round(t * 1e3, 3)
    # algorithmic bytes: LDE 16(d+N) + sum of Merkle(n) and fold(n) over the FRI rounds
    rounds, ln, alg = 0, N, 16 * (d + N)
    while ln > EXPANSION and ln > 4 * COLINEARITY:
        ln //= 2
        rounds += 1
    ln = N
    for r in range(rounds):
        alg += 16 * ln + 64 * (2 * ln - 1)
        if r < rounds - 1:
            alg += 24 * ln
        ln //= 2
    out["north_star_alg_bytes"] = alg
    out["north_star_hbm_frac"] = round(alg / t / (HBM_PEAK_GBS * 1e9), 4)
    ctx.trim()
    return out


def block_and_c4(ctx: sg.Context, device, iters: int = 5) -> dict:
    """The LDE+commit block of earlier rounds (N = 2^23) and BASELINE config C4 (Stark::prove on a
    Rescue-Prime trace of 2^16 - 1 randomized rows, FRI domain 2^21)."""
    out = {}
    blk = BlockWorkload(0, device, ctx)
    blk.step()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(iters):
        blk.step()
    torch.cuda.synchronize(device)
    out["lde_commit_block_2p23_ms"] = round((time.perf_counter() - t0) / iters * 1e3, 3)
    del blk
    c4 = ProveWorkload(0, device, ctx, 16)
    c4.step()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(iters):
        c4.step()
    torch.cuda.synchronize(device)
    out["c4_prove_trace_2p16_ms"] = round((time.perf_counter() - t0) / iters * 1e3, 3)
    out["c4_proof_bytes"] = len(c4.last_proof.digest())
    del c4
    ctx.trim()
    return out


RPSSS_PUBLISHED_SIGN_MS = 18913   # rpsss.rs:96-97, the reference's "fast" release build, hardware unstated
RPSSS_PROOF_LEN = 1156888         # rpsss.rs:89


def rpsss_side(ctx: sg.Context, iters: int = 5) -> dict:
    """The reference's one published end-to-end configuration, RPSSS::new(field, 4, 64, 128, 3)
    (rpsss.rs:103): Rescue-Prime N = 27, Stark(4, 64, 128, 2, 28, 3), FRI domain 4096, signing
    b"Hello, World!" through a SignatureProofStream.  `rpsss_sign_ms` = RPSSS::sign as the reference
    runs it (rpsss.rs:37-50, 74-78: hash, trace, transition + boundary constraints rebuilt, prove,
    the serialized signature) from host inputs; `rpsss_prove_ms` = Stark::prove alone with the
    constraints built.  Medians of `iters`; the published 18 913 ms is context, not a baseline
    (its hardware is unstated)."""
    import hashlib
    rp = sg.RescuePrime(2, 1, 128, 27, ctx=ctx)
    st = sg.Stark(4, COLINEARITY, 128, 2, 28, 3, ctx=ctx)
    sk = int.from_bytes(hashlib.shake_256(b"sg-bench-rpsss").digest(17), "big") % P
    air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
    nrc = st.num_randomizer_coefficients(air)
    tr = synthetic_fe(0, b"rpsss-trace-rand", 2 * st.num_randomizers)
    rc = synthetic_fe(0, b"rpsss-rand-poly", nrc)
    doc = b"Hello, World!"

    def sign():
        pk = rp.hash(sk)
        trace = rp.trace_array(sk)
        tcs = rp.transition_constraints(st.omicron, st.omicron_domain_length)
        return st.prove(trace, tcs, rp.boundary_constraints(pk), sg.SignatureProofStream(doc), tr, rc)

    def prove():
        return st.prove(rp.trace_array(sk), air, rp.boundary_constraints(rp.hash(sk)), sg.SignatureProofStream(doc),
                        tr, rc)

    sig = sign()  # first call builds the context's tables
    assert len(sig) == RPSSS_PROOF_LEN, len(sig)
    assert prove() == sig

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        return time.perf_counter() - t0

    t_sign = median_of(lambda: timed(sign), iters)
    t_prove = median_of(lambda: timed(prove), iters)
    return {"rpsss_sign_ms": round(t_sign * 1e3, 3), "rpsss_prove_ms": round(t_prove * 1e3, 3),
            "rpsss_signature_bytes": len(sig), "rpsss_published_sign_ms": RPSSS_PUBLISHED_SIGN_MS,
            "rpsss_note": "RPSSS::new(field, 4, 64, 128, 3) (rpsss.rs:103); sign = hash + trace + "
                          "constraints + Stark::prove + serialized signature from host inputs; the "
                          "published 18 913 ms (rpsss.rs:96-97) is the reference's fast build on "
                          "unstated hardware (context only)"}


def allreduce_max(value: float, device) -> float:
    """max over ranks (device tensor on RCCL, host tensor on gloo)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    on = device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def c5_single_gpu(ctx: sg.Context, device, iters: int = 3) -> dict:
    """C5's transform size (2^27, 2 GiB) as one single-GPU NTT: the 1-GPU point of the C5 curve."""
    n = 1 << 27
    root = sg.primitive_nth_root(n)
    x = to_device(synthetic_fe(0, b"c5", n), device)
    y = torch.empty_like(x)
    sg.ntt_dev(root, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(iters):
        sg.ntt_dev(root, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
    torch.cuda.synchronize(device)
    t = (time.perf_counter() - t0) / iters
    del x, y
    ctx.trim()
    out = {"c5_ntt_2p27_ms": round(t * 1e3, 3), "c5_gelem_s": round(n / t / 1e9, 3), "c5_ranks": 1,
           "c5_alg_hbm_frac": round(32 * n / t / (HBM_PEAK_GBS * 1e9), 4)}
    # the sharded path on one rank (sg_dist_ntt over a 1-rank RCCL communicator): the four-step's
    # own cost -- its passes, the epilogue twiddles, the run-shard transpose -- with no peer
    from starkgpu import dist as D
    nd = D.NativeDist(ctx, transport="rccl")
    n1, n2 = nd.plan(n, 1)
    cols = torch.from_numpy(synthetic_fe(0, b"c5", n).reshape(n2, n1, 2).transpose(1, 0, 2).copy()
                            .view(np.int64).reshape(-1)).to(device)
    runs = nd.ntt(root, cols, n2, n)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(iters):
        runs = nd.ntt(root, cols, n2, n)
    torch.cuda.synchronize(device)
    t = (time.perf_counter() - t0) / iters
    out["c5_dist_world1_ms"] = round(t * 1e3, 3)
    out["c5_dist_world1_gelem_s"] = round(n / t / 1e9, 3)
    del cols, runs
    ctx.trim()
    # the headline proof through sg_dist_stark_prove on the same one-rank communicator: since round 5
    # a one-rank communicator proves through the single-GPU plan (its collectives are identities);
    # the context option world1_sharded forces the four-step path, whose own cost (four-step LDEs, forests,
    # sharded FRI rounds, batched openings) without peers is the second line.  Bytes must equal the
    # single-GPU proof's either way.
    try:
        wl = ProveWorkload(0, device, ctx, LOG_TRACE)
        single = wl.step().digest()

        def sharded():
            ps = sg.IndependentProofStream()
            wl.stark.prove_dev(wl.trace.data_ptr(), wl.rows, wl.air, wl.boundary, ps, wl.trace_rand.data_ptr(),
                               wl.rcoef.data_ptr(), wl.nrc, dist=nd)
            return ps.digest()

        for key, forced in (("sharded_prove_world1", False), ("sharded_prove_world1_fourstep", True)):
            ctx.set_option("world1_sharded", int(forced))
            try:
                same = sharded() == single
                torch.cuda.synchronize(device)
                t0 = time.perf_counter()
                for _ in range(iters):
                    sharded()
                torch.cuda.synchronize(device)
            finally:
                ctx.set_option("world1_sharded", 0)
            out[key + "_ms"] = round((time.perf_counter() - t0) / iters * 1e3, 3)
            out[key + "_bytes_equal_single_gpu"] = same
        del wl
    except Exception as e:  # noqa: BLE001
        out["sharded_prove_world1_error"] = f"{type(e).__name__}: {e}"
    nd.close()
    ctx.trim()
    return out


def side_sharded(ctx: sg.Context, device, world: int, rank: int, iters: int = 3) -> dict:
    """Strong-scaling side measurements over all ranks (BASELINE config C5), through
    the C ABI's communicator (csrc/dist.cpp: sg_dist_*, RCCL over xGMI; SG_BENCH_BACKEND=gloo
    rehearses it with the host-staged transport).

    * C5: one 2^27-point NTT sharded across the ranks: four-step, ONE all-to-all, time = max
      over ranks.
    * the north-star block sharded: LDE 2^21 -> 2^24 on the coset + FRI commit
      (exp 8, c = 64) with run-sharded Merkle trees and folds, and the same with FRI::prove
      (sg_dist_fri_prove: openings gathered from the ranks that own the leaves).
    """
    from starkgpu import dist as D
    backend = dist.get_backend()
    ds = D.NativeDist(ctx, transport="rccl" if backend == "nccl" else "host")
    out = {"sharded_ranks": world, "sharded_path": "C ABI sg_dist_* (" +
           ("RCCL" if backend == "nccl" else "host-staged transport over " + backend) + ")"}

    def timed(fn):
        fn()
        dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize(device)
        return allreduce_max((time.perf_counter() - t0) / iters, device)

    # every rank runs the same code on the same shapes, so an error is raised on all of them
    try:
        # C2's size sharded the same way (the NTT part of the curve at 1/2/4/8)
        n = 1 << 22
        n1, n2 = D.plan(n, world)
        shard = to_device(synthetic_fe(rank, b"c2", (n1 // world) * n2), device).reshape(-1)
        root = sg.primitive_nth_root(n)
        t = timed(lambda: ds.ntt(root, shard, n2, n))
        out["c2_sharded_ntt_2p22_ms"] = round(t * 1e3, 3)
        out["c2_sharded_gelem_s"] = round(n / t / 1e9, 3)
        del shard
    except Exception as e:  # noqa: BLE001
        out["c2_sharded_error"] = f"{type(e).__name__}: {e}"
    try:
        n = 1 << 27
        n1, n2 = D.plan(n, world)
        shard = to_device(synthetic_fe(rank, b"c5", (n1 // world) * n2), device).reshape(-1)
        root = sg.primitive_nth_root(n)
        t = timed(lambda: ds.ntt(root, shard, n2, n))
        out["c5_ntt_2p27_ms"] = round(t * 1e3, 3)
        out["c5_gelem_s"] = round(n / t / 1e9, 3)
        out["c5_plan"] = f"N1=2^{n1.bit_length() - 1} x N2=2^{n2.bit_length() - 1}, one all-to-all of " \
                         f"{16 * n // world // 2**20} MiB per rank"
        del shard
    except Exception as e:  # noqa: BLE001
        out["c5_error"] = f"{type(e).__name__}: {e}"
    try:
        N = 1 << 24
        d = N // EXPANSION
        cols, row = D.scatter_columns_np(synthetic_fe(0, b"ns", d), N, world, rank)
        cs = to_device(cols, device)
        omega, off = sg.primitive_nth_root(N), sg.generator()

        def lde_fri():
            cw = ds.coset_evaluate(omega, N, off, cs.reshape(-1), row)
            ds.fri_commit(off, omega, cw, N, EXPANSION, COLINEARITY, sg.IndependentProofStream())

        out["sharded_lde_fri_commit_2p24_ms"] = round(timed(lde_fri) * 1e3, 3)

        def lde_fri_prove():  # FRI::prove incl. the query phase's openings from the owning ranks
            cw = ds.coset_evaluate(omega, N, off, cs.reshape(-1), row)
            ds.fri_prove(off, omega, cw, N, EXPANSION, COLINEARITY, sg.IndependentProofStream())

        out["sharded_lde_fri_prove_2p24_ms"] = round(timed(lde_fri_prove) * 1e3, 3)
    except Exception as e:  # noqa: BLE001
        out["sharded_lde_fri_error"] = f"{type(e).__name__}: {e}"
    try:
        # the headline Stark::prove with its FRI domain sharded over the ranks (sg_dist_stark_prove):
        # trace-domain algebra replicated, LDEs / commitments / FRI / openings on run shards; every
        # rank proves the same statement and must write the single-GPU proof bytes
        wl = ProveWorkload(0, device, ctx, LOG_TRACE)
        single = wl.step().digest()

        def prove():
            ps = sg.IndependentProofStream()
            wl.stark.prove_dev(wl.trace.data_ptr(), wl.rows, wl.air, wl.boundary, ps, wl.trace_rand.data_ptr(),
                               wl.rcoef.data_ptr(), wl.nrc, dist=ds)
            state["bytes"] = ps.digest()

        state = {}
        t = timed(prove)
        same = -allreduce_max(-1.0 if state["bytes"] == single else 0.0, device) == 1.0
        out["sharded_prove_ms"] = round(t * 1e3, 3)
        out["sharded_prove_gelem_s"] = round(wl.elements_per_step() / t / 1e9, 4)
        out["sharded_prove_bytes_equal_single_gpu"] = same
        out["sharded_prove_workload"] = f"the headline proof (trace 2^{LOG_TRACE}, FRI domain " \
                                        f"2^{wl.fri_len.bit_length() - 1}) sharded over {world} ranks"
        del wl
    except Exception as e:  # noqa: BLE001
        out["sharded_prove_error"] = f"{type(e).__name__}: {e}"
    ds.close()
    ctx.trim()
    return out


def host_cpu_info() -> dict:
    """The GPU box's host CPU as lscpu reports it (model, logical CPUs) and this process's affinity."""
    info = {"affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "CPU(s)", "Socket(s)", "Thread(s) per core"):
                info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def faithful_block_step(rc, o, N: int) -> float:
    """One LDE + commit + FRI block (4 LDEs of N/32 coefficients onto N points, 3 Merkle commits, FRI
    commit + query with the reference's O(n)-per-opening Merkle::open) through oracle/ref_cpu.c; seconds.
    d = N/32 is the headline prove's shape: quotients of degree ~2^20 on a FRI domain of 2^25."""
    d = N // 32
    omega = o.primitive_nth_root(N)
    polys = [synthetic_fe(0, t, d) for t in (b"bq0", b"bq1", b"rand", b"comb")]
    fri = o.FRI(o.GENERATOR, omega, N, EXPANSION, COLINEARITY)
    t0 = time.perf_counter()
    stream = bytes(16)
    for k in range(REGISTERS + 1):
        cw = rc.fast_coset_evaluate(omega, N, o.GENERATOR, polys[k])
        stream += bytes([0]) + (64).to_bytes(8, "big") + rc.merkle_commit(cw)
    o.shake256(stream, o.PROOF_BYTES)  # combination weights
    cw = rc.fast_coset_evaluate(omega, N, o.GENERATOR, polys[3])
    stream, roots, cws = rc.fri_commit(o.GENERATOR, omega, cw, EXPANSION, COLINEARITY, prefix=stream,
                                       want_codewords=True)
    top = fri.sample_indices(o.shake256(stream, o.PROOF_BYTES), len(cws[1]), len(cws[-1]), COLINEARITY)
    idx = list(top)
    for r in range(len(cws) - 1):  # fri.rs:231-245 -> query (fri.rs:174-208)
        half = len(cws[r]) // 2
        idx = [i % half for i in idx]
        for i in idx:
            rc.merkle_open(i, cws[r])
            rc.merkle_open(i + half, cws[r])
            rc.merkle_open(i, cws[r + 1])
    return time.perf_counter() - t0


def _other_physical_core(core: int) -> int:
    """A CPU of this process's affinity on a different physical core than `core` (not its SMT
    sibling), so two single-core legs can run side by side; `core` itself when there is none."""
    def siblings(c):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                out = set()
                for part in f.read().strip().split(","):
                    a, _, b = part.partition("-")
                    out.update(range(int(a), int(b or a) + 1))
                return out
        except OSError:
            return {c}
    busy = siblings(core) | {core}
    for c in sorted(os.sched_getaffinity(0)):
        if c not in busy:
            return c
    return core


def faithful_c2_start(core: int, log_n: int = 22):
    """C2 on the reference's algorithms, timed directly: oracle/ref_cpu.c's ntt and
    intt (fft/ntt.rs:7-68 over field.rs:117-131's bit-serial mul_mod) of 2^22 elements -- the
    bench's C2 input -- on ONE pinned core.  ~30 s per transform on the box's host, so it runs in a
    thread (ctypes drops the GIL) pinned to `core` while the one-core block leg runs on another
    physical core.  Returns (thread, result dict filled when the thread ends)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_cpu as rc
    import stark_oracle as o
    res = {}

    def run():
        try:
            os.sched_setaffinity(threading.get_native_id(), {core})
            n = 1 << log_n
            x = synthetic_fe(7, b"c2", n)
            w = o.primitive_nth_root(n)
            t0 = time.perf_counter()
            y = rc.ntt(w, x)
            t1 = time.perf_counter()
            z = rc.intt(w, y)
            t2 = time.perf_counter()
            res.update({"c2_faithful_ms": round((t2 - t0) * 1e3, 1), "c2_faithful_fwd_ms": round((t1 - t0) * 1e3, 1),
                        "c2_faithful_inv_ms": round((t2 - t1) * 1e3, 1),
                        "c2_faithful_gelem_s": round(2 * n / (t2 - t0) / 1e9, 8),
                        "c2_faithful_roundtrip_ok": bool(np.array_equal(z, x)), "c2_faithful_cpu": core,
                        "c2_faithful_sample": f"2^{log_n} fwd + inv NTT through oracle/ref_cpu.c (bit-serial mul_mod, "
                                              f"the reference's radix-2 DIT), one pinned core, timed directly"})
        except Exception as e:  # noqa: BLE001 - reported in the line, the baseline leg stands
            res["c2_faithful_error"] = f"{type(e).__name__}: {e}"

    th = threading.Thread(target=run, daemon=True)
    th.start()
    return th, res


def cpu_baseline_leg(headline_N: int, log_Ns=(12, 13, 14, 15, 16), with_c2: bool = True) -> dict:
    """The reference-faithful C restatement (oracle/ref_cpu.c: bit-serial mul_mod, xgcd inverse,
    per-element pow + division in the fold, recursive Merkle with to_string leaves and O(n) opens)
    on ONE host core -- the reference is single-threaded.

    The prove's LDE + commit + FRI block is timed at N = 2^12 .. 2^16, one step each, and
    extrapolated to the headline FRI domain N = 2^25 with the block's cost model
    t(N) = a N log2 N + b N (NTTs; hashing, folds and the O(N) opens), fitted by least squares
    (SURVEY.md 8(d)(i)).  The reference's trace interpolation and quotient algebra are O(T^2)
    and are not in this leg (cpu_baseline_e2e times them through the Python restatement).
    Beside it (`with_c2`), C2's 2^22 fwd + inv NTT on the reference's algorithms is timed directly on
    a second pinned core (faithful_c2_start), so the GPU's C2 line has its CPU counterpart.
    """
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_cpu as rc
    import stark_oracle as o
    pts = []
    # the reference is single-threaded: the leg runs pinned to one core (SURVEY.md 8(d)(i) "taskset")
    prev = os.sched_getaffinity(0)
    core = min(prev)
    # C2 on the reference's algorithms, directly at 2^22, on another physical core meanwhile
    c2_thread, c2 = faithful_c2_start(_other_physical_core(core)) if with_c2 else (None, {})
    os.sched_setaffinity(0, {core})
    try:
        for ln in log_Ns:
            pts.append((1 << ln, faithful_block_step(rc, o, 1 << ln)))
    finally:
        os.sched_setaffinity(0, prev)
    if c2_thread is not None:
        c2_thread.join()
    from scipy.optimize import nnls
    A = np.array([[n * np.log2(n), n] for n, _ in pts], dtype=np.float64)
    y = np.array([t for _, t in pts], dtype=np.float64)
    (a, b), _ = nnls(A, y)  # non-negative least squares: both cost terms are real work
    Nh = headline_N
    t_h = a * Nh * np.log2(Nh) + b * Nh
    N_last, t_last = pts[-1]
    return {
        "value": round((REGISTERS + 2) * N_last / t_last / 1e9, 8),
        "unit": "Gelem/s",
        "cores": 1,
        "pinned_cpu": core,
        "kind": "port",
        "sample": f"the prove's LDE+commit+FRI block (4 LDEs, 3 commits, FRI prove, c={COLINEARITY}) at "
                  f"N=2^{N_last.bit_length() - 1} on one core (value), measured at "
                  + ", ".join(f"2^{n.bit_length() - 1}: {t:.2f} s" for n, t in pts)
                  + "; oracle/ref_cpu.c keeps the reference's algorithms",
        "extrapolated_headline": {"N": Nh, "block_s": round(float(t_h), 1),
                                  "value": round((REGISTERS + 2) * Nh / float(t_h) / 1e9, 8),
                                  "model": f"t = {a:.3e} N log2 N + {b:.3e} N (least squares over the "
                                           f"measured points, non-negative)", "label": "extrapolated"},
        "c2": c2 or None,
    }


def cpu_threads() -> tuple:
    """(threads to use, why): the process's CPU affinity, capped by OMP_NUM_THREADS when the
    environment sets it (the GPU pool gives a one-GPU job a 16-CPU share of a 256-CPU host and
    exports OMP_NUM_THREADS=16; nproc there reports the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and 0 < int(env) < aff:
        return int(env), (f"OMP_NUM_THREADS={env}: this job's CPU share on a host whose affinity shows "
                          f"{aff} CPUs (the pool sizes worker pools to the share)")
    return aff, "every CPU in this process's affinity"


def cpu_baseline_allcores(log_rows: int = LOG_TRACE) -> dict:
    """The whole Stark::prove (stark.rs:276-562) on the host CPU at the headline size: the checker
    restatement oracle/fast_cpu.cpp (Montgomery arithmetic, OpenMP; the reference's algorithms where
    they define the bytes, fast ones where the result is unique -- its proof bytes equal the GPU's,
    tests/test_gpu_fullsize.py) on the same Rescue-Prime workload as the headline line, timed once."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import fast_cpu as fc
    import stark_prove_oracle as e
    threads, why = cpu_threads()
    fc.set_threads(threads)
    N = (1 << log_rows) - 2 - 4 * COLINEARITY
    rp_o = e.RescuePrime(REGISTERS, 1, 128, N)
    st_o = e.Stark(EXPANSION, COLINEARITY, 128, REGISTERS, N + 1, 3)
    bounds = fc.rescue_degree_bounds(rp_o, st_o)
    rp = sg.RescuePrime(REGISTERS, 1, 128, N)  # the trace is an input (host code, not timed)
    inp = int.from_bytes(hashlib_shake(b"sg-bench-input" + (0).to_bytes(8, "big"), 16), "big") % P
    trace = rp.trace_array(inp)
    out = sg.to_ints(trace[-2:-1])[0]
    tr = synthetic_fe(0, b"trace-rand", REGISTERS * st_o.num_randomizers)
    rc = synthetic_fe(0, b"rand-poly", bounds[1] + 1)
    phases = {}
    t0 = time.perf_counter()
    proof = fc.stark_prove_rescue(rp_o, st_o, trace, rp_o.boundary_constraints(out), tr, rc, bounds=bounds,
                                  phases=phases)
    t = time.perf_counter() - t0
    nf = st_o.fri.domain_length
    return {
        "value": round((REGISTERS + 2) * nf / t / 1e9, 6),
        "unit": "Gelem/s",
        "cores": threads,
        "cores_note": why,
        "kind": "port",
        "prove_ms": round(t * 1e3, 1),
        "proof_bytes": len(proof),
        "phases_s": {k: round(v, 3) for k, v in phases.items()},
        "sample": f"one complete Stark::prove of the headline workload (trace 2^{log_rows} - 1 rows, FRI domain "
                  f"2^{nf.bit_length() - 1}) through oracle/fast_cpu.cpp on {threads} threads: {t:.1f} s",
        "host": host_cpu_info(),
    }


def cpu_baseline_e2e(seconds_budget: float = 6.0) -> dict:
    """The whole Stark::prove through the oracle's restatement (oracle/stark_prove_oracle.py: the
    reference's O(n^2) polynomial algebra, pure Python) at the reference test's size: Rescue-Prime
    N = 27, expansion 4, c = 2 (stark.rs:823-840), one core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import stark_oracle as o
    import stark_prove_oracle as e
    rp = e.RescuePrime(2, 1, 2, 27)
    st = e.Stark(4, 2, 2, 2, 28, 2)
    air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
    inp = o.sample(b"deadbeef")
    trace, bnd = rp.trace(inp), rp.boundary_constraints(rp.hash(inp))
    r = e.randomness_from_seed(b"cpu", 2 * st.num_randomizers + st.num_randomizer_coefficients(air))
    tr = [r[2 * i:2 * i + 2] for i in range(st.num_randomizers)]
    rc = r[2 * st.num_randomizers:]
    n, t0 = 0, time.perf_counter()
    while True:
        st.prove(trace, air, bnd, o.IndependentProofStream(), tr, rc)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds_budget or n >= 50:
            break
    per = el / n
    return {"value": round(4 * st.fri.domain_length / per / 1e9, 9), "unit": "Gelem/s", "cores": 1, "kind": "port",
            "sample": f"Stark::prove, Rescue-Prime N=27 (reference test size, FRI domain 512), {n} proofs, "
                      f"{per * 1e3:.1f} ms/proof; Python restatement of the reference's algorithms"}


def hbm_copy_gbs(ctx: sg.Context, mib: int = 2048, iters: int = 10) -> dict:
    """HBM rate of the library's dwordx4 streaming copy kernel (sg_hbm_copy_probe: non-temporal
    16-byte loads/stores) over a 2 GiB buffer (bytes read + bytes written per second, best of
    `iters`, HIP events on the library's stream): one element per lane, and a grid-stride form."""
    out = {}
    for blocks in (0, 4096):
        out[blocks] = ctx.hbm_copy_gbs(mib << 20, iters, blocks)
    best = max(out.values())
    return {"gbs": round(best, 1),
            "per_form": {("one element per lane" if k == 0 else f"grid-stride {k} blocks"): round(v, 1)
                         for k, v in out.items()},
            "kernel": "sg_hbm_copy_probe (k_copy16)", "bytes": mib << 20}


def standalone_launch(ctx, device, name: str, n: int):
    """Event-timed launches of the dominant kernel alone on the chip: a tree over n seeded leaves."""
    if name != "merkle_leaves":
        return None
    g = torch.Generator(device=device).manual_seed(7)
    leaves = torch.randint(0, 1 << 62, (n, 2), dtype=torch.int64, device=device, generator=g)  # < 2^126 < p
    sg.DeviceTree.build_batch([leaves.data_ptr()], n, ctx=ctx)
    torch.cuda.synchronize(device)
    ctx.profile_only(name)
    ctx.profile(True)
    for _ in range(3):
        sg.DeviceTree.build_batch([leaves.data_ptr()], n, ctx=ctx)
    torch.cuda.synchronize(device)
    rep = ctx.profile_report()[name]
    ctx.profile(False)
    ctx.profile_only(None)
    ms = rep["ms"] / rep["launches"]
    gbs = rep["bytes"] / (rep["ms"] * 1e-3) / 1e9
    return {"leaves": n, "avg_launch_ms": round(ms, 4), "achieved": round(gbs, 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4)}


def prove_valu_budget(breakdown, ms_per_step):
    """Whole-prove VALU issue: every timed launch of one prove (the last warmup step) priced at its
    kernel's SQ_INSTS_VALU per wave (PMC pass of this build) times the waves it ran, summed and set
    against the prove's wall time -- the chip-wide counterpart of roofline.valu, for a job whose two
    streams overlap kernels (a kernel's own live rate then says little about the chip).

    waves: Merkle scopes record the lanes they launch; the NTT passes hold 8 elements per lane
    (2048 / 4096 / 8192-element tiles on 256 / 512 / 1024 lanes), so lanes = elements / 8.
    peak = 1 wave64 instruction / SIMD / 2 clk x 1024 SIMDs at the 2.4 GHz maximum clock (the clock the
    chip holds under this load is lower, so the fractions are lower bounds); mix roof = each kernel's
    full/half-rate mix (clk per instruction per SIMD, tools/valu_mix.py) summed over its instructions."""
    vf = os.path.join(ROOT, "profiles", PMC_VALU_FILE)
    mf = os.path.join(ROOT, "profiles", VALU_MIX_FILE)
    if not (os.path.exists(vf) and os.path.exists(mf)):
        return None
    per_wave = json.load(open(vf))["kernels"]
    mix = json.load(open(mf))["kernels"]
    blake_clk = mix.get("merkle_nodes", {}).get("clk_per_wave_instr_per_simd")
    instr = simd_clk = covered_ms = total_ms = 0.0
    kinds = {}
    for k, v in breakdown.items():
        total_ms += v["ms"]
        key = "ntt_pass" if k.startswith("ntt_pass") else k
        if key not in per_wave:
            continue
        if key == "ntt_pass":
            lanes = v["bytes"] / 32.0 / 8.0
        elif key == "ntt_first":
            lanes = v.get("elems", 0) / 8.0
        else:
            lanes = v.get("elems", 0)
        if lanes <= 0:
            continue
        n = per_wave[key]["valu_instr_per_wave"] * lanes / 64.0
        # the quad-lane tree kernels run the same BLAKE2b body as the node kernel
        clk = mix.get(key, {}).get("clk_per_wave_instr_per_simd") or blake_clk
        instr += n
        simd_clk += n * clk
        covered_ms += v["ms"]
        kinds[k] = int(n)
    if instr <= 0 or ms_per_step <= 0:
        return None
    t = ms_per_step * 1e-3
    hz = MAX_CLOCK_GHZ * 1e9
    peak = 1024 * hz / 2.0
    rate = instr / t
    # SIMD-clk the instructions need at their mix / SIMD-clk the prove's wall time holds
    mix_frac = simd_clk / (1024 * hz * t)
    # the clock the chip held in the PMC pass of the dominant (leaf) kernel, under the same load
    load_ghz = per_wave.get("merkle_leaves", {}).get("clock_ghz")
    return {"wave_instr_per_prove": int(instr), "per_kernel": kinds,
            "mix_frac_at_load_clock": round(simd_clk / (1024 * load_ghz * 1e9 * t), 4) if load_ghz else None,
            "load_clock_ghz": round(load_ghz, 3) if load_ghz else None,
            "achieved": round(rate, -6), "peak": round(peak, -6), "frac": round(rate / peak, 4),
            "mix_frac": round(mix_frac, 4), "clock_ghz": MAX_CLOCK_GHZ,
            "mix_floor_ms": round(simd_clk / (1024 * hz) * 1e3, 3),
            "covered_device_ms_frac": round(covered_ms / total_ms, 4) if total_ms > 0 else None,
            "unit": "wave64 VALU instr/s",
            "source": f"profiles/{PMC_VALU_FILE} (instructions per wave) x the waves of every launch of the last "
                      f"warmup prove; profiles/{VALU_MIX_FILE} (full/half-rate mix); peak and mix_floor_ms at the "
                      f"{MAX_CLOCK_GHZ} GHz maximum clock (MI355X_MICROARCH.md:34), so frac / mix_frac are lower bounds",
            "definition": "the whole prove's VALU instructions (kernels covering covered_device_ms_frac of its device "
                          "time) over its wall time; mix_frac = the SIMD cycles those instructions need at their "
                          "measured full/half-rate costs / the SIMD cycles of the wall time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-trace", type=int, default=LOG_TRACE, help="log2 of the randomized trace rows + 1")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-side", action="store_true", help="skip the side measurements (C2, C4, C5, block, 2^24)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; SG_BENCH_BACKEND=gloo (host-staged) lets a one-GPU box rehearse N > 1
    backend = os.environ.get("SG_BENCH_BACKEND", "nccl")
    gpu = local_rank % max(torch.cuda.device_count(), 1)
    device = torch.device("cuda", gpu)
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=timedelta(seconds=600))
        else:
            dist.init_process_group(backend, timeout=timedelta(seconds=600))

    ctx = sg.Context(gpu)
    wl = ProveWorkload(rank, device, ctx, args.log_trace)
    # warmup; the last warmup step runs with every launch timed, which yields the
    # per-kernel breakdown and picks the dominant kernel for the roofline
    breakdown = {}
    for i in range(max(args.warmup, 1)):
        if i == max(args.warmup, 1) - 1:
            ctx.profile(True)
        wl.step()
    breakdown = ctx.profile_report()
    ctx.profile(False)
    dominant = max(breakdown.items(), key=lambda kv: kv[1]["ms"])[0]

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)

    barrier()
    # the timed region records HIP events (on the library's stream) around the
    # dominant kernel's launches only, so the instrumentation barely perturbs it
    profiled = os.environ.get("SG_BENCH_NO_PROFILE") != "1"
    ctx.profile_only(dominant)
    ctx.profile(profiled)
    host_phases = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step(host_phases)
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    barrier()
    prof = ctx.profile_report() if profiled else {dominant: breakdown[dominant]}
    ctx.profile(False)
    ctx.profile_only(None)

    elapsed = allreduce_max(t1 - t0, device)
    ms_per_step = elapsed / args.steps * 1e3
    total_elems = wl.elements_per_step() * args.steps * world

    # roofline of the dominant kernel: its algorithmic bytes over its event-timed device time
    name, st = dominant, prof[dominant]
    achieved = st["bytes"] / (st["ms"] * 1e-3) / 1e9
    # measured HBM bytes per launch of that kernel (rocprofv3 PMC passes on this code, committed under
    # profiles/; the live bench cannot collect PMC counters itself)
    traffic, traffic_src = None, None
    pmc_file = os.path.join(ROOT, "profiles", PMC_TRAFFIC_FILE)
    if os.path.exists(pmc_file) and args.log_trace == LOG_TRACE:
        pmc = json.load(open(pmc_file))["kernels"].get(name)
        if pmc and pmc.get("hbm_bytes_per_lane") and st.get("elems"):
            traffic = int(pmc["hbm_bytes_per_lane"] * st["elems"] / st["launches"])
            traffic_src = (f"profiles/{PMC_TRAFFIC_FILE} (FETCH_SIZE x2 + WRITE_SIZE per lane of the same workload, "
                           f"scaled to the live launches' lanes)")
    # VALU issue of the dominant kernel: instructions per wave from a rocprofv3 SQ_INSTS_VALU pass on
    # this workload (tools/pmc_valu.py), times the waves the live launches ran (their lane count),
    # over their live duration -- one launch population.  The kernels are integer-VALU-bound, so this
    # is the roof that actually binds them.
    valu = None
    valu_file = os.path.join(ROOT, "profiles", PMC_VALU_FILE)
    if os.path.exists(valu_file) and st.get("elems"):
        vk = json.load(open(valu_file))["kernels"].get(name)
        if vk:
            inst = vk["valu_instr_per_wave"] * st["elems"] / 64.0
            live = inst / (st["ms"] * 1e-3)
            valu = {"unit": "wave64 VALU instr/s", "instr_per_launch": int(inst / st["launches"]),
                    "instr_per_wave": round(vk["valu_instr_per_wave"], 1),
                    "achieved": round(live, -6), "peak": round(vk["peak_wave_instr_per_s"], -6),
                    "frac": round(live / vk["peak_wave_instr_per_s"], 4),
                    "mix_roof": round(vk.get("mix_roof_wave_instr_per_s", 0.0), -6) or None,
                    "mix_frac": round(live / vk["mix_roof_wave_instr_per_s"], 4)
                    if vk.get("mix_roof_wave_instr_per_s") else None,
                    "clock_ghz": round(vk["clock_ghz"], 3),
                    "source": f"profiles/{PMC_VALU_FILE} (SQ_INSTS_VALU per wave); peak = 1 wave64 instr / SIMD / "
                              f"2 clk (SIMD-32) x 1024 SIMDs at the PMC pass's clock; mix_roof = the kernel's "
                              f"full/half-rate instruction mix at the measured per-op rates (tools/valu_mix.py); "
                              f"achieved = per-wave count x the live launches' waves / their live time"}
    # the HBM rate a plain device copy reaches on this box (1 GiB read + 1 GiB written), beside the
    # 8 TB/s spec the contract prices against ("measure actual HBM with a copy kernel")
    copy = hbm_copy_gbs(ctx)
    copy_gbs = copy["gbs"]
    # the same kernel alone on the chip (in the prove, the boundary-quotient and randomizer
    # trees share the CUs with the main stream's algebra, which stretches their launches)
    alone = standalone_launch(ctx, device, name, wl.fri_len)
    phases = {k: {"launches": v["launches"], "ms_per_step": round(v["ms"], 4),
                  "GBps": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] > 0 else None}
              for k, v in sorted(breakdown.items(), key=lambda kv: -kv[1]["ms"])}
    # the workload's own NTT throughput: transform elements of every NTT/INTT/LDE in one prove over
    # the device time of all their passes (last warmup step, every launch event-timed)
    ntt_keys = [k for k in breakdown if k.startswith(("ntt_", "bitrev_gather", "scale_const"))]
    ntt_ms = sum(breakdown[k]["ms"] for k in ntt_keys)
    ntt_elems = sum(breakdown[k].get("elems", 0) for k in ntt_keys)
    ntt_stats = {"ntt_gelem_s": round(ntt_elems / (ntt_ms * 1e-3) / 1e9, 3) if ntt_ms > 0 else None,
                 "ntt_elements_per_prove": int(ntt_elems), "ntt_device_ms_per_prove": round(ntt_ms, 3),
                 "definition": "sum of transform lengths (NTT, INTT, LDE) in one prove / device time of their "
                               "passes, each launch timed with HIP events in the last warmup step"}

    result = {
        "metric": "NTT Gelem/s + prove ms, Rescue-Prime trace 2^20, at 1/2/4/8 MI355X",
        "value": round(total_elems / elapsed / 1e9, 4),
        "unit": "Gelem/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "prove_ms": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u128 (F_p, p = 1 + 407*2^119)",
        "data": "synthetic: Rescue-Prime execution trace of a seeded input; randomizers from a seeded "
                "SHAKE256 stream (SURVEY.md 8(d))",
        "ntt": ntt_stats,
        "prove_valu": prove_valu_budget(breakdown, ms_per_step) if args.log_trace == LOG_TRACE else None,
        "config": {"workload": f"Stark::prove, Rescue-Prime m={REGISTERS} trace {wl.rows} rows "
                               f"(+{wl.stark.num_randomizers} randomizers = 2^{args.log_trace} - 1), "
                               f"expansion {EXPANSION}, c={COLINEARITY}, security 128, transition degree 3 "
                               f"(omicron domain 2^{wl.stark.omicron_domain_length.bit_length() - 1}, "
                               f"FRI domain 2^{wl.fri_len.bit_length() - 1})",
                   "codeword_elements_per_step_per_gpu": wl.elements_per_step(),
                   "value_definition": "Gelem/s = committed codeword elements per second over all ranks: "
                                       "(m + 2) codewords of the FRI domain per proof (2 boundary quotients, the "
                                       "randomizer, the combination) x proofs / wall time; prove_ms = ms per "
                                       "proof; the workload's NTT rate is ntt.ntt_gelem_s",
                   "proof_bytes": len(wl.last_proof.digest()) if wl.last_proof is not None else None,
                   "plans": "twiddle plans and public domain/AIR tables (zerofier transforms, their coset values "
                            "and inverses, AIR x-polynomial coset values) are built by the first (warmup) proof and "
                            "kept in the context, like FFT plans; witness- and transcript-dependent work is all "
                            "redone every step (DESIGN.md section 5; SG_NO_DOMAIN_CACHE=1 disables the tables)",
                   "parallelism": f"replicas x{world} (independent traces, no data-path collective)"},
        "roofline": {"kernel": name, "bound": "hbm", "binding": "valu" if valu else "hbm",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "avg_launch_ms": round(st["ms"] / st["launches"], 4),
                     "launches": st["launches"],
                     "alg_bytes_per_launch": int(st["bytes"] / st["launches"]),
                     "note": "achieved/peak/frac are the contract's HBM roofline (algorithmic bytes / live launch "
                             "time vs 8 TB/s); the roof that binds this integer kernel is VALU issue "
                             "(binding = valu): roofline.valu gives its fraction of the SIMD-32 peak and of its "
                             "instruction-mix roof (DESIGN.md section 4); launches overlap other kernels (side "
                             "stream), standalone = alone on the chip",
                     "valu": valu,
                     "standalone": alone,
                     "hbm_copy_measured_gbs": copy_gbs,
                     "hbm_copy_probe": copy,
                     "frac_of_measured_copy": round(achieved / copy_gbs, 4) if copy_gbs else None},
        "kernels_one_step": phases,  # every launch timed, last warmup step
        "host_phases_ms": {k: round(v / args.steps * 1e3, 3) for k, v in host_phases.items()},
    }
    fri_len = wl.fri_len
    if world == 1 and not args.no_side:
        del wl
        ctx.trim()
        result["side"] = side_measurements(ctx, device)
        result["side"].update(block_and_c4(ctx, device))
        result["side"].update(rpsss_side(ctx))
        result["side"].update(c5_single_gpu(ctx, device))
    if world > 1 and not args.no_side:
        # a hang in a collective must not cost the main line: rank 0 prints it, and every rank
        # exits on its own timer (a rank left blocked in a collective would hold the launcher)
        # A hang exits NON-ZERO (a stuck collective on a process that has touched the GPU is a failure
        # the launcher must see); the lock makes the timer and the main thread mutually exclusive,
        # so at most one of them emits the JSON line.
        emit_lock = threading.Lock()
        state = {"done": False}

        def on_timeout():
            with emit_lock:
                if state["done"]:
                    return
                state["done"] = True
                if rank == 0:
                    result["side"] = {"error": "sharded side measurements timed out"}
                    print(json.dumps(result), flush=True)
            os._exit(3)
        watchdog = threading.Timer(150.0 + (0 if rank == 0 else 15.0), on_timeout)
        watchdog.daemon = True
        watchdog.start()
        try:
            side = side_sharded(ctx, device, world, rank)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line, main metric stands
            side = {"error": f"{type(e).__name__}: {e}"}
        with emit_lock:
            if state["done"]:  # the timer already reported and is exiting the process
                return
            state["done"] = True
            watchdog.cancel()
            result["side"] = side
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_leg(fri_len)
        result["cpu_baseline_allcores"] = cpu_baseline_allcores(args.log_trace)
        result["cpu_baseline_e2e"] = cpu_baseline_e2e()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
