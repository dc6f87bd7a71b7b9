#!/usr/bin/env python3
"""Align the FRI commit's host stamps (SG_FRI_TIMING=1, A/B build) with a rocprofv3 kernel trace.

For the last prove of the run: per gated round, where the ~10 us between a round's tree and the
next round's fold goes -- tree end -> host sees the root (device -> host), host sees the root ->
gate raised (host Fiat-Shamir), gate raised -> gate kernel ends (host -> device), and when the
gate kernel started.  The clock domain of the trace is taken from whichever host clock
(CLOCK_MONOTONIC or CLOCK_BOOTTIME) puts the stamps inside the traced kernels' span.

usage: fri_gate_timing.py run_kernel_trace.csv stderr.log
"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sg::", ""))
                for r in rows)
    marks = []
    for line in open(sys.argv[2]):
        m = re.match(r"sg-fri (\d+) (-?\d+) (-?\d+) (-?\d+) boot (-?\d+)", line)
        if m:
            marks.append(tuple(int(g) for g in m.groups()))
    # the last commit: rounds restart at 0
    starts = [i for i, m in enumerate(marks) if m[0] == 0]
    last = marks[starts[-1]:]
    lo, hi = ks[0][0], ks[-1][1]
    mono_in = lo <= last[0][2] <= hi
    off = 0
    if not mono_in:  # the trace is on CLOCK_BOOTTIME: shift the monotonic stamps by the clocks' offset
        off = last[0][4] - last[0][2]
    print(f"clock: {'monotonic' if mono_in else 'boottime (offset %.3f ms)' % (off / 1e6)}")
    gates = [k for k in ks if k[2] == "k_fri_gate"]
    print(" r  tree_end->seen  seen->gate_raised  raised->gate_end  gate_start-tree_end  gate_end->next_start (us)")
    tot = [0.0] * 5
    n = 0
    for r, ws, seen, raised, _ in last:
        seen += off
        raised += off
        ws += off
        # the kernel that finished last before the host saw the root: the tree's top
        before = [k for k in ks if k[1] <= seen + 2000]
        if not before:
            continue
        tree_end = max(k[1] for k in before if k[2] != "k_fri_gate")
        g = [k for k in gates if k[0] >= tree_end - 1000 and k[1] >= raised - 1000]
        if raised <= 0 or not g:
            print(f"{r:2d}  {(seen - tree_end) / 1e3:8.2f}")
            continue
        gk = g[0]
        nxt = [k for k in ks if k[0] >= gk[1]]
        v = [(seen - tree_end) / 1e3, (raised - seen) / 1e3, (gk[1] - raised) / 1e3, (gk[0] - tree_end) / 1e3,
             ((nxt[0][0] - gk[1]) / 1e3) if nxt else 0.0]
        tot = [a + b for a, b in zip(tot, v)]
        n += 1
        print(f"{r:2d}  {v[0]:8.2f}  {v[1]:8.2f}  {v[2]:8.2f}  {v[3]:8.2f}  {v[4]:8.2f}")
    if n:
        print("mean " + "  ".join(f"{t / n:8.2f}" for t in tot))


if __name__ == "__main__":
    main()
