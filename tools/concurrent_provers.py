#!/usr/bin/env python3
"""Several provers in flight on one GPU: k host threads, each with its own context (its own streams
and buffer pool) proving its own trace-2^20 workload, against the same proofs run one at a time.

A serving deployment keeps more than one proof in flight per GPU: one proof's latency-bound tail
(the small FRI rounds, the combination's LDE alone on the chip) then shares the chip with another
proof's throughput-bound trees.  Checks that every concurrent proof's bytes equal the sequential
proof of the same trace (contexts share nothing but the device).

usage: concurrent_provers.py [k] [rounds] [log_trace]
"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    log_trace = int(sys.argv[3]) if len(sys.argv) > 3 else bench.LOG_TRACE
    dev = torch.device("cuda", 0)
    ctxs = [bench.sg.Context(0) for _ in range(k)]
    wls = [bench.ProveWorkload(i, dev, ctxs[i], log_trace) for i in range(k)]
    # warmup (plans and domain tables) and the sequential reference bytes
    ref = []
    for wl in wls:
        wl.step()
        wl.step()
        ref.append(wl.last_proof_bytes)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(rounds):
        for wl in wls:
            wl.step()
    torch.cuda.synchronize(dev)
    seq = (time.perf_counter() - t0) / (rounds * k)
    print(f"sequential: {seq * 1e3:.3f} ms per proof", flush=True)

    errs = []
    same = [True] * k
    barrier = threading.Barrier(k + 1)

    def worker(i):
        try:
            torch.cuda.set_device(dev)
            barrier.wait()
            for _ in range(rounds):
                wls[i].step()
                if wls[i].last_proof_bytes != ref[i]:
                    same[i] = False
            barrier.wait()
        except Exception as e:  # surfaced below; the barrier is aborted so main does not wait forever
            errs.append(repr(e))
            barrier.abort()

    th = [threading.Thread(target=worker, args=(i,)) for i in range(k)]
    for t in th:
        t.start()
    try:
        barrier.wait()
        t0 = time.perf_counter()
        barrier.wait()
        conc = (time.perf_counter() - t0) / (rounds * k)
    except threading.BrokenBarrierError:
        conc = None
    for t in th:
        t.join()
    if errs or conc is None:
        print("error:", errs)
        sys.exit(1)
    print(f"{k} in flight: {conc * 1e3:.3f} ms per proof (amortized), {seq / conc:.3f}x the sequential "
          f"throughput; bytes equal to the sequential proofs: {all(same)}", flush=True)
    if not all(same):
        sys.exit(1)


if __name__ == "__main__":
    main()
