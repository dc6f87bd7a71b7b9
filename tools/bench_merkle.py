#!/usr/bin/env python3
"""Merkle tree build timing (per-kernel) for one size through libstarkgpu's profiler.

usage: bench_merkle.py [logn] [batch]   (plan knobs: SG_MERKLE_LEAF_BS, SG_MERKLE_LEAF_FUSE)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-stark-tutor_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import starkgpu as sg  # noqa: E402


def main():
    logn = int(sys.argv[1]) if len(sys.argv) > 1 else 23
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    n = 1 << logn
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    xs = [bench.to_device(bench.synthetic_fe(b, b"mk", n), dev) for b in range(batch)]
    ptrs = [x.data_ptr() for x in xs]
    roots = [t.root() for t in sg.DeviceTree.build_batch(ptrs, n, ctx=ctx)]
    it = 5
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(it):
        trees = sg.DeviceTree.build_batch(ptrs, n, ctx=ctx)
        assert [t.root() for t in trees] == roots
        del trees
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / it
    rep = ctx.profile_report()
    comp = batch * (2 * n - 1)
    dev_ms = sum(v["ms"] for v in rep.values()) / it
    print(f"2^{logn} x{batch} [{os.environ.get('SG_MERKLE_LEAF_BS', '256')}/{os.environ.get('SG_MERKLE_LEAF_FUSE', '4')}]: "
          f"{t*1e3:.3f} ms/build  device {dev_ms:.3f} ms  {comp/dev_ms/1e6:.2f} G compressions/s  root {roots[0][:8].hex()}")
    for k, v in sorted(rep.items(), key=lambda kv: -kv[1]["ms"]):
        print(f"  {k:18s} launches/iter {v['launches']/it:.0f}  ms/iter {v['ms']/it:.4f}")


if __name__ == "__main__":
    main()
