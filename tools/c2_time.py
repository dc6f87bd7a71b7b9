#!/usr/bin/env python3
"""C2-style timing of one transform size: forward + inverse NTT stream-ordered, median of 5 x 5 iterations
(bench.py side_measurements' method), plus the round-trip check.  usage: c2_time.py [logn]"""
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
    logn = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    n = 1 << logn
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    x = bench.to_device(bench.synthetic_fe(7, b"c2", n), dev)
    y, z = torch.empty_like(x), torch.empty_like(x)
    w = sg.primitive_nth_root(n)
    sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
    sg.intt_dev(w, y.data_ptr(), n, z.data_ptr(), ctx=ctx)
    assert torch.equal(x, z)

    def rep():
        ctx.set_async(True)
        t0 = time.perf_counter()
        for _ in range(5):
            sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
            sg.intt_dev(w, y.data_ptr(), n, z.data_ptr(), ctx=ctx)
            ctx.synchronize()
        dt = (time.perf_counter() - t0) / 5
        ctx.set_async(False)
        return dt

    t = bench.median_of(rep, 5)
    assert torch.equal(x, z)
    print(f"2^{logn} fwd+inv {t * 1e3:.3f} ms  {2 * n / t / 1e9:.2f} Gelem/s  SG_NTT_BIG={os.environ.get('SG_NTT_BIG', '0')}")


if __name__ == "__main__":
    main()
