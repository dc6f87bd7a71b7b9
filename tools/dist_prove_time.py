#!/usr/bin/env python3
"""The headline Stark::prove through sg_dist_stark_prove on a one-rank RCCL communicator next to the
single-GPU sg_stark_prove on the same box: the sharded path's own cost (four-step LDEs, forests +
top trees, sharded FRI rounds, owner-rank openings) without peers.

usage: dist_prove_time.py [steps] [log_trace] [only]   (only = single | sharded_world1)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

sg = bench.sg


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    log_trace = int(sys.argv[2]) if len(sys.argv) > 2 else bench.LOG_TRACE
    only = sys.argv[3] if len(sys.argv) > 3 else None
    from starkgpu import dist as D
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    nd = D.NativeDist(ctx, transport="rccl")
    wl = bench.ProveWorkload(0, dev, ctx, log_trace)

    def single():
        return wl.step().digest()

    def sharded():
        ps = sg.IndependentProofStream()
        wl.stark.prove_dev(wl.trace.data_ptr(), wl.rows, wl.air, wl.boundary, ps, wl.trace_rand.data_ptr(),
                           wl.rcoef.data_ptr(), wl.nrc, dist=nd)
        return ps.digest()

    a, b = single(), sharded()
    assert a == b, "sharded proof bytes differ from the single-GPU proof"
    gap = os.environ.get("SG_PROVE_GAPS") == "1"  # idle gaps between proves (tools/trace_sum.py)
    for name, fn in (("single", single), ("sharded_world1", sharded), ("single", single),
                     ("sharded_world1", sharded)):
        if only and name != only:
            continue
        torch.cuda.synchronize(dev)
        dt = 0.0
        for _ in range(steps):
            if gap:
                time.sleep(0.1)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            dt += time.perf_counter() - t0
        print(f"{name}: {dt / steps * 1e3:.3f} ms/prove", flush=True)
    nd.close()


if __name__ == "__main__":
    main()
