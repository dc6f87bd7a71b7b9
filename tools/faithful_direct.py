#!/usr/bin/env python3
"""The reference-faithful CPU baseline measured directly at a large N (verdict r3 item 8;
SURVEY.md 8(d)(i)): bench.py's faithful_block_step (oracle/ref_cpu.c: the reference's bit-serial
mul_mod, xgcd inverse, per-element pow + division in the fold, recursive Merkle with O(n) opens;
fri.rs:151-159, merkle_root.rs:34-66) on ONE pinned core at N = 2^12..2^16 (the bench's fit points)
and directly at N = 2^logN, against the t = a N log2 N + b N model fitted on the small points.

usage: tools/faithful_direct.py [logN=20]     (run under tools/hb.sh on the GPU box: one step at
2^20 takes minutes with no output)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
from scipy.optimize import nnls  # noqa: E402

import bench  # noqa: E402
import ref_cpu as rc  # noqa: E402
import stark_oracle as o  # noqa: E402


def main():
    logN = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    prev = os.sched_getaffinity(0)
    core = min(prev)
    os.sched_setaffinity(0, {core})
    pts = []
    for ln in (12, 13, 14, 15, 16):
        t = bench.faithful_block_step(rc, o, 1 << ln)
        pts.append((1 << ln, t))
        print(f"2^{ln}: {t:.3f} s", flush=True)
    A = np.array([[n * np.log2(n), n] for n, _ in pts], dtype=np.float64)
    y = np.array([t for _, t in pts], dtype=np.float64)
    (a, b), _ = nnls(A, y)
    N = 1 << logN
    pred = a * N * np.log2(N) + b * N
    print(f"model t = {a:.4e} N log2 N + {b:.4e} N -> predicted 2^{logN}: {pred:.1f} s", flush=True)
    t0 = time.perf_counter()
    t = bench.faithful_block_step(rc, o, N)
    wall = time.perf_counter() - t0
    os.sched_setaffinity(0, prev)
    out = {"pinned_cpu": core, "points_s": {f"2^{n.bit_length() - 1}": round(v, 3) for n, v in pts},
           "model": {"a": a, "b": b}, "logN": logN, "predicted_s": round(float(pred), 2),
           "measured_s": round(t, 2), "wall_s": round(wall, 2),
           "measured_over_predicted": round(t / float(pred), 4),
           "value_gelem_s": (bench.REGISTERS + 2) * N / t / 1e9,
           "host": bench.host_cpu_info()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
