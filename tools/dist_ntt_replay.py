#!/usr/bin/env python3
"""Per-rank device time of the sharded NTT (sg_dist_ntt + sg_dist_intt, fft/ntt.rs:7-68 as the
four-step of csrc/dist.cpp) at world G, rank 0 alone on the GPU -- the NTT counterpart of
tools/dist_rank_replay.py (the curve at 1/2/4/8 for the C2-sized and C5 NTTs;
round-5 verdict item 5).  No multi-GPU box reaches the builder, so:

  record G LOGN DIR [STEPS]  world G on this one GPU (host transport over gloo, spawned ranks):
                             every rank runs STEPS + 1 forward + inverse transforms of its column
                             shard of a seeded 2^LOGN vector; rank 0 writes every collective's
                             receive buffer, in call order, and its last run shard (the forward
                             transform's output) to DIR.
  replay G LOGN DIR [STEPS]  rank 0 by itself: the same calls over a transport that hands back the
                             recorded receive buffers -- exactly rank 0's kernel sequence at world
                             G.  Checks that its run shard equals the recording AND the single-GPU
                             transform's slice, and that the inverse gives back its column shard.
  single LOGN [STEPS]        the single-GPU forward + inverse (sg_ntt_dev / sg_intt_dev) with the
                             same idle gaps, for the baseline column.

Steps are separated by 500 ms of idle, so `tools/ntt_replay_table.py` (gap 300 ms)
splits a `rocprofv3 --kernel-trace` of the replay (or of `single`) into per-step device time.
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zk-stark-tutor_amd")]


def _input(logn):
    """Seeded canonical elements (numpy generator: fast enough for 2^27)."""
    x = np.random.default_rng(2000 + logn).integers(0, 2**63, size=(1 << logn, 2), dtype=np.uint64)
    x[:, 1] %= np.uint64(0xCB80000000000000)  # hi < P's hi word: every value < p
    return x


def _shards(logn, world, rank):
    from starkgpu import dist as D
    x = _input(logn)
    cols, row = D.scatter_columns_np(x, 1 << logn, world, rank)
    return x, cols, row


def _run(lib, ctx, h, root, cols_t, row, n, runs_t, back_t):
    import starkgpu as sg
    ctx.check(lib.sg_dist_ntt(h, sg.api._fe(root), ctypes.c_void_p(cols_t.data_ptr()), row, n,
                              ctypes.c_void_p(runs_t.data_ptr())))
    ctx.check(lib.sg_dist_intt(h, sg.api._fe(root), ctypes.c_void_p(runs_t.data_ptr()), n,
                               ctypes.c_void_p(back_t.data_ptr())))


def _buffers(n, world, cols):
    import torch
    from starkgpu import dist as D
    dev = torch.device("cuda", 0)
    n1, n2 = D.plan(n, world)
    cols_t = torch.from_numpy(np.ascontiguousarray(cols).view(np.int64).reshape(-1).copy()).to(dev)
    runs_t = torch.empty(2 * n1 * (n2 // world), dtype=torch.int64, device=dev)
    back_t = torch.empty(2 * (n1 // world) * n2, dtype=torch.int64, device=dev)
    return cols_t, runs_t, back_t


def _record_worker(rank, world, port, logn, out, steps):
    import torch
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu._lib import A2A_CB, ABORT_CB, sg_dist_transport
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seq = [0]

    def view(ptr, nbytes):
        return torch.from_numpy(np.ctypeslib.as_array((ctypes.c_int64 * (nbytes // 8)).from_address(ptr)))

    def save(recv, nbytes):
        if rank == 0:
            np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(recv)).tofile(
                os.path.join(out, "c%06d.bin" % seq[0]))
        seq[0] += 1

    def a2a(_user, send, recv, nbytes):
        dist.all_to_all_single(view(recv, nbytes * world), view(send, nbytes * world))
        save(recv, nbytes * world)
        return 0

    def ag(_user, send, recv, nbytes):
        dist.all_gather(list(view(recv, nbytes * world).chunk(world)), view(send, nbytes).clone())
        save(recv, nbytes * world)
        return 0

    ctx = sg.Context(0)
    cbs = (A2A_CB(a2a), A2A_CB(ag), ABORT_CB(lambda u: None))
    tr = sg_dist_transport(None, cbs[0], cbs[1], cbs[2])
    h = ctypes.c_void_p()
    lib = sg.lib()
    ctx.check(lib.sg_dist_create_transport(ctx.handle, world, rank, ctypes.byref(tr), ctypes.byref(h)))
    n = 1 << logn
    _, cols, row = _shards(logn, world, rank)
    cols_t, runs_t, back_t = _buffers(n, world, cols)
    root = sg.primitive_nth_root(n)
    for _ in range(steps + 1):
        _run(lib, ctx, h, root, cols_t, row, n, runs_t, back_t)
    torch.cuda.synchronize()
    assert torch.equal(back_t, cols_t), "inverse did not give back the column shard"
    if rank == 0:
        runs_t.cpu().numpy().tofile(os.path.join(out, "runs.bin"))
    print(f"rank {rank}: {seq[0]} collectives over {steps + 1} fwd+inv steps", flush=True)
    lib.sg_dist_destroy(h)
    dist.destroy_process_group()


def record(world, logn, out, steps):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.makedirs(out, exist_ok=True)
    mp.spawn(_record_worker, args=(world, port, logn, out, steps), nprocs=world, join=True)


def replay(world, logn, out, steps):
    import torch
    import starkgpu as sg
    from starkgpu import dist as D
    from starkgpu._lib import A2A_CB, ABORT_CB, sg_dist_transport
    bufs = [np.fromfile(os.path.join(out, f), dtype=np.uint8) for f in sorted(os.listdir(out)) if f.startswith("c")]
    seq = [0]

    def cb(user, send, recv, nbytes):
        if seq[0] >= len(bufs) or bufs[seq[0]].size != nbytes * world:
            print(f"replay: collective {seq[0]} not recorded at this size", flush=True)
            return 1
        ctypes.memmove(recv, bufs[seq[0]].ctypes.data, bufs[seq[0]].size)
        seq[0] += 1
        return 0

    ctx = sg.Context(0)
    cbs = (A2A_CB(cb), A2A_CB(cb), ABORT_CB(lambda u: None))
    tr = sg_dist_transport(None, cbs[0], cbs[1], cbs[2])
    h = ctypes.c_void_p()
    lib = sg.lib()
    ctx.check(lib.sg_dist_create_transport(ctx.handle, world, 0, ctypes.byref(tr), ctypes.byref(h)))
    n = 1 << logn
    x, cols, row = _shards(logn, world, 0)
    cols_t, runs_t, back_t = _buffers(n, world, cols)
    root = sg.primitive_nth_root(n)
    _run(lib, ctx, h, root, cols_t, row, n, runs_t, back_t)  # the first step builds the plans
    torch.cuda.synchronize()
    dt = 0.0
    for _ in range(steps):
        time.sleep(0.5)  # idle gaps separate the steps in a kernel trace (gap 300 ms: the host memmoves
        #                  of the replayed 2^27 exchanges take ~100 ms inside a step)
        t0 = time.perf_counter()
        _run(lib, ctx, h, root, cols_t, row, n, runs_t, back_t)
        torch.cuda.synchronize()
        dt += time.perf_counter() - t0
    time.sleep(0.5)  # the check's own single-GPU transform must not join the last step's trace segment
    got = runs_t.cpu().numpy()
    rec = np.fromfile(os.path.join(out, "runs.bin"), dtype=np.int64)
    # rank 0's run shard [k1][c] = X[k1 N2 + c], c < R, of the single-GPU transform
    X = sg.ntt(root, x, ctx=ctx)
    n1, n2 = D.plan(n, world)
    R = n2 // world
    want = np.ascontiguousarray(X.reshape(n1, n2, 2)[:, :R]).view(np.int64).reshape(-1)
    equal = bool(np.array_equal(got, rec) and np.array_equal(got, want) and torch.equal(back_t, cols_t))
    print(f"world {world} 2^{logn} rank 0 alone: {dt / steps * 1e3:.3f} ms per fwd+inv (host wall; exchanges "
          f"replayed from host memory); {seq[0]} collectives; run shard == recording == single-GPU slice and "
          f"inverse == column shard: {equal}", flush=True)
    assert equal
    lib.sg_dist_destroy(h)


def single(logn, steps):
    import torch
    import starkgpu as sg
    n = 1 << logn
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    x = torch.from_numpy(_input(logn).view(np.int64).reshape(-1).copy()).to(dev)
    y, z = torch.empty_like(x), torch.empty_like(x)
    w = sg.primitive_nth_root(n)

    def step():
        sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
        sg.intt_dev(w, y.data_ptr(), n, z.data_ptr(), ctx=ctx)

    step()
    torch.cuda.synchronize()
    dt = 0.0
    for _ in range(steps):
        time.sleep(0.5)
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        dt += time.perf_counter() - t0
    assert torch.equal(x, z)
    print(f"single GPU 2^{logn}: {dt / steps * 1e3:.3f} ms per fwd+inv (host wall)", flush=True)


def main():
    mode = sys.argv[1]
    if mode == "record":
        record(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]) if len(sys.argv) > 5 else 2)
    elif mode == "replay":
        replay(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]) if len(sys.argv) > 5 else 2)
    elif mode == "single":
        single(int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 2)
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
