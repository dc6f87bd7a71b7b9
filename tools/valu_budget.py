#!/usr/bin/env python3
"""Whole-prove VALU budget (bench.prove_valu_budget) at several trace sizes: one prove per size with
every launch event-timed, priced at the PMC instructions per wave of profiles/<bench.PMC_VALU_FILE>,
set against the median wall time of `steps` unprofiled proves.  Shows where the prove stops being
bound by VALU issue and becomes bound by per-level latency (the small FRI rounds, tree tops).

usage: valu_budget.py [log_trace ...]   (default 16 18 20)
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    logs = [int(a) for a in sys.argv[1:]] or [16, 18, 20]
    dev = torch.device("cuda", 0)
    for lg in logs:
        ctx = bench.sg.Context(0)
        wl = bench.ProveWorkload(0, dev, ctx, lg)
        wl.step()
        wl.step()
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            wl.step()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        ms = statistics.median(ts) * 1e3
        ctx.profile(True)
        wl.step()
        torch.cuda.synchronize(dev)
        rep = ctx.profile_report()
        ctx.profile(False)
        b = bench.prove_valu_budget(rep, ms)
        print(f"trace 2^{lg} (FRI domain 2^{wl.fri_len.bit_length() - 1}): prove {ms:.3f} ms  "
              f"VALU {b['wave_instr_per_prove'] / 1e9:.3f} G wave-instr  mix floor {b['mix_floor_ms']:.3f} ms "
              f"(2.4 GHz)  mix_frac {b['mix_frac']:.3f}  at load clock {b['mix_frac_at_load_clock']:.3f}  "
              f"covered {b['covered_device_ms_frac']:.3f}", flush=True)
        del wl
        ctx.close()


if __name__ == "__main__":
    main()
