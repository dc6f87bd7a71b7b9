#!/usr/bin/env python3
"""Per-kernel timing of one NTT size (forward + inverse) through libstarkgpu's profiler."""
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
    x = bench.to_device(bench.synthetic_fe(1, b"nt", n), dev)
    y, z = torch.empty_like(x), torch.empty_like(x)
    w = sg.primitive_nth_root(n)
    for _ in range(2):
        sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
        sg.intt_dev(w, y.data_ptr(), n, z.data_ptr(), ctx=ctx)
    if not os.environ.get("SG_NO_CHECK"):
        assert torch.equal(x, z)
    ctx.profile(True)
    it = 5
    t0 = time.perf_counter()
    for _ in range(it):
        sg.ntt_dev(w, x.data_ptr(), n, y.data_ptr(), ctx=ctx)
        sg.intt_dev(w, y.data_ptr(), n, z.data_ptr(), ctx=ctx)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / it
    rep = ctx.profile_report()
    print(f"2^{logn}: fwd+inv {t*1e3:.3f} ms (profiled)  {2*n/t/1e9:.2f} Gelem/s")
    for k, v in sorted(rep.items(), key=lambda kv: -kv[1]["ms"]):
        print(f"  {k:16s} launches/iter {v['launches']/it:.0f}  ms/iter {v['ms']/it:.4f}  "
              f"GB/s {v['bytes']/(v['ms']*1e-3)/1e9:.0f}")


if __name__ == "__main__":
    main()
