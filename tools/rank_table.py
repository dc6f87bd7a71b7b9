#!/usr/bin/env python3
"""Markdown table of per-prove device time by kernel category from tools/trace_sum.py JSON outputs
(the single-GPU prove and rank 0 of sharded proves replayed alone).

usage: rank_table.py LABEL=trace_sum.json [LABEL=trace_sum.json ...]   (the first is the baseline)
"""
import json
import sys

CATS = [("merkle", "Merkle kernels"), ("ntt", "NTT kernels"), ("other kernels", "other library kernels")]


def main():
    cols = []
    for arg in sys.argv[1:]:
        label, path = arg.split("=", 1)
        d = json.load(open(path))
        seg = d["segments"][-1]
        cols.append((label, d["categories_last"], seg))
    base = cols[0][1]
    base_lib = sum(base.get(c, 0.0) for c, _ in CATS)
    print("| per prove, device time (ms) | " + " | ".join(lbl for lbl, _, _ in cols) + " |")
    print("|---|" + "---|" * len(cols))
    for key, name in CATS:
        print(f"| {name} | " + " | ".join(f"{c.get(key, 0.0):.2f}" for _, c, _ in cols) + " |")
    libs = [sum(c.get(k, 0.0) for k, _ in CATS) for _, c, _ in cols]
    print("| **library kernels (ratio to the first column)** | "
          + " | ".join(f"**{v:.2f} ({v / base_lib:.2f})**" for v in libs) + " |")
    print("| runtime copies / fills | " + " | ".join(f"{c.get('runtime copy/fill', 0.0):.2f}" for _, c, _ in cols)
          + " |")
    print("| all kernels (sum); busy union | "
          + " | ".join(f"{s['kernel_sum_ms']:.1f}; {s['busy_ms']:.1f}" for _, _, s in cols) + " |")


if __name__ == "__main__":
    main()
