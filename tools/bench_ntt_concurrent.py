#!/usr/bin/env python3
"""k independent 2^logn forward NTTs enqueued on k library contexts (one HIP stream each) at
once vs one after another: whether concurrent transforms fill what one transform leaves idle."""
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
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    n = 1 << logn
    dev = torch.device("cuda", 0)
    ctxs = [sg.Context(0) for _ in range(k)]
    for c in ctxs:
        c.set_async(True)
    xs = [bench.to_device(bench.synthetic_fe(i, b"cc", n), dev) for i in range(k)]
    ys = [torch.empty_like(x) for x in xs]
    w = sg.primitive_nth_root(n)

    def run(concurrent: bool, it=10):
        for c, x, y in zip(ctxs, xs, ys):
            sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=c)
        for c in ctxs:
            c.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            for c, x, y in zip(ctxs, xs, ys):
                sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=c)
                if not concurrent:
                    c.synchronize()
            for c in ctxs:
                c.synchronize()
        return (time.perf_counter() - t0) / it

    for _ in range(2):
        s = run(False)
        c = run(True)
        print(f"2^{logn} x{k}: serial {s * 1e3:.3f} ms  concurrent {c * 1e3:.3f} ms  ratio {c / s:.3f}")


if __name__ == "__main__":
    main()
