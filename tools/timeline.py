#!/usr/bin/env python3
"""Kernel timeline from a rocprofv3 --kernel-trace sqlite db: per-kernel busy time and the idle gaps
between consecutive dispatches (where the GPU waits for the host).

usage: timeline.py run_results.db [last_n_dispatches]
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    if len(sys.argv) > 2:
        rows = rows[-int(sys.argv[2]):]
    busy = defaultdict(float)
    gaps_after = defaultdict(list)
    total_gap = 0.0
    for i, (name, s, e) in enumerate(rows):
        short = name.split("(")[0].replace("void ", "")[:40]
        busy[short] += (e - s) / 1e3
        if i + 1 < len(rows):
            g = max(0, rows[i + 1][1] - e) / 1e3
            gaps_after[short].append(g)
            total_gap += g
    span = (rows[-1][2] - rows[0][1]) / 1e3
    print(f"dispatches {len(rows)}  span {span:.1f} us  busy {sum(busy.values()):.1f} us  idle {total_gap:.1f} us")
    for k in sorted(busy, key=lambda k: -busy[k]):
        g = gaps_after[k]
        print(f"  {k:42s} busy {busy[k]:9.1f} us  n {len(g):4d}  idle-after total {sum(g):8.1f} us "
              f"mean {sum(g) / max(len(g), 1):6.1f}")


if __name__ == "__main__":
    main()
