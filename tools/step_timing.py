#!/usr/bin/env python3
"""Host-side split of the bench's prove step: proof-stream creation, the prove call (returns once the
proof is complete), and the serialized-proof copy (stream.digest()), per step."""
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
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    wl = bench.ProveWorkload(0, dev, ctx, log_trace)
    wl.step()
    wl.step()
    torch.cuda.synchronize(dev)
    tot = {"create": 0.0, "prove": 0.0, "digest": 0.0, "step": 0.0}
    for _ in range(steps):
        t0 = time.perf_counter()
        stream = sg.IndependentProofStream()
        t1 = time.perf_counter()
        wl.stark.prove_dev(wl.trace.data_ptr(), wl.rows, wl.air, wl.boundary, stream, wl.trace_rand.data_ptr(),
                           wl.rcoef.data_ptr(), wl.nrc)
        t2 = time.perf_counter()
        wl.last_proof_bytes = stream.digest()
        t3 = time.perf_counter()
        wl.last_proof = stream
        t4 = time.perf_counter()
        for k, v in (("create", t1 - t0), ("prove", t2 - t1), ("digest", t3 - t2), ("step", t4 - t0)):
            tot[k] += v
    print("  ".join(f"{k} {v / steps * 1e3:.3f} ms" for k, v in tot.items()))


if __name__ == "__main__":
    main()
