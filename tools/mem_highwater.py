#!/usr/bin/env python3
"""Device-memory high-water mark of the bench's Stark::prove (round-5 verdict item 7: where sharding
becomes necessary).  For each trace size 2^L (L from argv, default 16 18 20): a fresh context builds
the workload and proves once (the warmup proof builds the public tables), then the pool's peak is
reset and a second proof runs; the line reports

  peak      the buffer pool's high-water mark during the second proof (codewords, retained FRI and
            commitment trees, scratch: everything a proof allocates and frees)
  resident  device bytes held across proofs: hipMemGetInfo used after the proof minus used before
            the context existed, minus the pool's free cache (twiddle plans, domain / AIR tables,
            the trace and randomizers in torch tensors)
  total     peak + resident = the device memory one proof of this size needs

and, after the sweep, the linear fit total ~ a * 2^L + b and the largest 2^L whose total fits the
device (hipMemGetInfo total).  usage: mem_highwater.py [L ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def one(L: int, dev) -> dict:
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    free0, total = torch.cuda.mem_get_info(dev)
    ctx = bench.sg.Context(0)
    wl = bench.ProveWorkload(0, dev, ctx, L)
    wl.step()
    torch.cuda.synchronize(dev)
    ctx.memory(reset_peak=True)
    wl.step()
    torch.cuda.synchronize(dev)
    m = ctx.memory()
    used0 = total - free0
    resident = m["device_used"] - used0 - m["pooled"] - m["live"]
    out = {"log_trace": L, "fri_domain": wl.fri_len, "peak": m["peak"], "resident": resident,
           "total": m["peak"] + resident, "device_total": m["device_total"],
           "bytes_per_fri_element": round((m["peak"] + resident) / wl.fri_len, 1)}
    del wl
    ctx.trim()
    ctx.close()
    del ctx
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return out


def main():
    Ls = [int(a) for a in sys.argv[1:]] or [16, 18, 20]
    dev = torch.device("cuda", 0)
    rows = []
    for L in Ls:
        r = one(L, dev)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if len(rows) >= 2:
        import numpy as np
        x = np.array([r["fri_domain"] for r in rows], dtype=np.float64)
        y = np.array([r["total"] for r in rows], dtype=np.float64)
        a, b = np.polyfit(x, y, 1)
        cap = rows[-1]["device_total"]
        fit = {"model": f"total = {a:.1f} B x FRI-domain elements + {b / 2**20:.1f} MiB", "a": a, "b": b,
               "device_total": cap}
        # FRI domain = 8 x 2^(L + 2) for this workload (transition degree 3, expansion 8)
        best = None
        for L in range(10, 40):
            nf = 1 << (L + 5)
            if a * nf + b <= cap:
                best = L
        fit["largest_log_trace_one_gpu"] = best
        print(json.dumps({"fit": fit}), flush=True)


if __name__ == "__main__":
    main()
