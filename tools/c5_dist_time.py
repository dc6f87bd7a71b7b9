#!/usr/bin/env python3
"""The distributed four-step NTT (sg_dist_ntt) of 2^LOG points on a one-rank RCCL communicator, as
bench.py's `c5_dist_world1_ms` side leg times it (for tools/ab.sh c5dist A/Bs).

usage: c5_dist_time.py [log=27] [iters=5]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zk-stark-tutor_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    log = int(sys.argv[1]) if len(sys.argv) > 1 else 27
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    sg = bench.sg
    from starkgpu import dist as D
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    n = 1 << log
    root = sg.primitive_nth_root(n)
    nd = D.NativeDist(ctx, transport="rccl")
    n1, n2 = nd.plan(n, 1)
    x = bench.synthetic_fe(0, b"c5", n)
    cols = torch.from_numpy(x.reshape(n2, n1, 2).transpose(1, 0, 2).copy().view(np.int64).reshape(-1)).to(dev)
    runs = nd.ntt(root, cols, n2, n)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        runs = nd.ntt(root, cols, n2, n)
    torch.cuda.synchronize(dev)
    t = (time.perf_counter() - t0) / iters
    # world 1: the run shard is the natural-order transform
    y = torch.empty_like(cols)
    xt = torch.from_numpy(x.view(np.int64).reshape(-1)).to(dev)
    sg.ntt_dev(root, xt.data_ptr(), n, y.data_ptr(), ctx=ctx)
    torch.cuda.synchronize(dev)
    same = torch.equal(runs.reshape(-1), y.reshape(-1))
    print(f"2^{log} (N1 2^{n1.bit_length() - 1}, N2 2^{n2.bit_length() - 1}): {t * 1e3:.3f} ms  equal {same}",
          flush=True)
    nd.close()


if __name__ == "__main__":
    main()
