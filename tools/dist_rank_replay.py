#!/usr/bin/env python3
"""One rank of the sharded headline Stark::prove (sg_dist_stark_prove) ALONE on the GPU: the
per-rank device time at world G (verdict r3 item 2), without the other ranks'
kernels sharing the card.

  record G DIR [STEPS]   world G on this one GPU (host transport over gloo, spawned ranks): every
                         rank proves the headline statement STEPS + 1 times (the first builds the
                         context's tables) and writes each collective's receive buffer, in call
                         order, to DIR/rank<g>/; rank 0 also writes the proof bytes.
  replay G R DIR [STEPS] rank R by itself, in this process: the same prove calls over a transport
                         that hands back the recorded receive buffers in order -- exactly rank R's
                         kernel sequence at world G, alone on the card.  Prints the per-prove time
                         and checks the proof bytes against the recording.  Run it under
                         `rocprofv3 --kernel-trace --stats -- python3 tools/dist_rank_replay.py replay ...`
                         for rank R's per-kernel device time.

The replay's sends are not compared with the recording (a rank's sends are the peers' inputs);
its proof bytes are, and they only come out right if every received buffer matched its request.
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zk-stark-tutor_amd")]


def _workload(dev, ctx):
    import bench  # SG_REPLAY_LOG: trace 2^LOG (default the headline's 2^20)
    return bench.ProveWorkload(0, dev, ctx, int(os.environ.get("SG_REPLAY_LOG", bench.LOG_TRACE)))


def _prove(wl, nd):
    import starkgpu as sg
    ps = sg.IndependentProofStream()
    wl.stark.prove_dev(wl.trace.data_ptr(), wl.rows, wl.air, wl.boundary, ps, wl.trace_rand.data_ptr(),
                       wl.rcoef.data_ptr(), wl.nrc, dist=nd)
    return ps.digest()


def _record_worker(rank, world, port, out, steps):
    import torch
    import torch.distributed as dist
    import starkgpu as sg
    from starkgpu._lib import A2A_CB, ABORT_CB, sg_dist_transport
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = os.path.join(out, "rank%d" % rank)
    os.makedirs(d, exist_ok=True)
    seq = [0]

    def view(ptr, nbytes):
        return torch.from_numpy(np.ctypeslib.as_array((ctypes.c_int64 * (nbytes // 8)).from_address(ptr)))

    def save(recv, nbytes):
        np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(recv)).tofile(
            os.path.join(d, "c%06d.bin" % seq[0]))
        seq[0] += 1

    def a2a(_user, send, recv, nbytes):  # the same exchanges as starkgpu.dist.NativeDist("host")
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
    nd = _ND(ctx, h)
    wl = _workload(torch.device("cuda", 0), ctx)
    single = wl.step().digest() if rank == 0 else None
    for _ in range(steps + 1):
        got = _prove(wl, nd)
        if rank == 0:
            assert got == single, "sharded proof bytes differ from the single-GPU proof"
    if rank == 0:
        with open(os.path.join(out, "proof.bin"), "wb") as f:
            f.write(single)
    print(f"rank {rank}: {seq[0]} collectives recorded over {steps + 1} proves", flush=True)
    lib.sg_dist_destroy(h)
    dist.destroy_process_group()


class _ND:
    """The NativeDist surface Stark.prove_dev uses (context, handle, torch drain)."""

    def __init__(self, ctx, handle):
        import torch
        self.ctx, self.handle = ctx, handle
        self._torch_ready = lambda: torch.cuda.synchronize()


def record(world, out, steps):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.makedirs(out, exist_ok=True)
    mp.spawn(_record_worker, args=(world, port, out, steps), nprocs=world, join=True)


def replay(world, rank, out, steps):
    import torch
    import starkgpu as sg
    from starkgpu._lib import A2A_CB, ABORT_CB, sg_dist_transport
    d = os.path.join(out, "rank%d" % rank)
    # every recorded buffer in memory before the first prove: the replay reads no file while timed
    bufs = [np.fromfile(os.path.join(d, f), dtype=np.uint8) for f in sorted(os.listdir(d)) if f.startswith("c")]
    seq = [0]

    def cb(user, send, recv, nbytes):
        if seq[0] >= len(bufs):
            print(f"replay: collective {seq[0]} was not recorded", flush=True)
            return 1
        data = bufs[seq[0]]
        if data.size != nbytes * world:
            print(f"replay: collective {seq[0]} asks {nbytes * world} bytes, recorded {data.size}", flush=True)
            return 1
        ctypes.memmove(recv, data.ctypes.data, data.size)
        seq[0] += 1
        return 0

    ctx = sg.Context(0)
    cbs = (A2A_CB(cb), A2A_CB(cb), ABORT_CB(lambda u: None))
    tr = sg_dist_transport(None, cbs[0], cbs[1], cbs[2])
    h = ctypes.c_void_p()
    lib = sg.lib()
    ctx.check(lib.sg_dist_create_transport(ctx.handle, world, rank, ctypes.byref(tr), ctypes.byref(h)))

    nd = _ND(ctx, h)
    wl = _workload(torch.device("cuda", 0), ctx)
    want = open(os.path.join(out, "proof.bin"), "rb").read()
    assert _prove(wl, nd) == want, "replayed proof bytes differ (first prove)"
    torch.cuda.synchronize()
    dt = 0.0
    for _ in range(steps):
        time.sleep(0.1)  # idle gaps separate the proves in a kernel trace (tools/trace_sum.py)
        t0 = time.perf_counter()
        assert _prove(wl, nd) == want, "replayed proof bytes differ"
        torch.cuda.synchronize()
        dt += time.perf_counter() - t0
    dt /= steps
    print(f"world {world} rank {rank} alone: {dt * 1e3:.3f} ms/prove (host wall; exchanges replayed from host "
          f"memory through the staged transport); {seq[0]} collectives", flush=True)
    lib.sg_dist_destroy(h)


def main():
    mode = sys.argv[1]
    if mode == "record":
        record(int(sys.argv[2]), sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 2)
    elif mode == "replay":
        replay(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]) if len(sys.argv) > 5 else 2)
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
