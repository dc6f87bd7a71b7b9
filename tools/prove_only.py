#!/usr/bin/env python3
"""The bench's prove step alone (for rocprofv3 traces): build the trace-2^20 workload, prove `steps` times.

usage: prove_only.py [steps] [log_trace]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    log_trace = int(sys.argv[2]) if len(sys.argv) > 2 else bench.LOG_TRACE
    dev = torch.device("cuda", 0)
    ctx = bench.sg.Context(0)
    wl = bench.ProveWorkload(0, dev, ctx, log_trace)
    wl.step()
    torch.cuda.synchronize(dev)
    time.sleep(0.05)  # a gap that separates the warmup from the traced steps
    gap = os.environ.get("SG_PROVE_GAPS") == "1"  # idle gaps between proves (tools/trace_sum.py)
    dt = 0.0
    for _ in range(steps):
        if gap:
            time.sleep(0.1)
        t0 = time.perf_counter()
        wl.step()
        torch.cuda.synchronize(dev)
        dt += time.perf_counter() - t0
    print(f"{dt / steps * 1e3:.3f} ms/prove")


if __name__ == "__main__":
    main()
