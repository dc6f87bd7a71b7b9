#!/usr/bin/env python3
"""Device time per prove from a rocprofv3 kernel trace (<dir>/run_kernel_trace.csv): the kernels are
split into segments at idle gaps of at least GAP ms (the callers sleep between proves:
tools/dist_rank_replay.py, SG_PROVE_GAPS=1 tools/prove_only.py); per segment it prints the kernel
count, the SUM of kernel durations (device time; overlapping kernels of two streams both count),
the busy time (union of kernel intervals) and the span, plus the top kernels of the last segment.

usage: trace_sum.py run_kernel_trace.csv [GAP_ms=20] [json_out]
"""
import collections
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    segs, cur, seg_end = [], [], 0
    for k in ks:
        if cur and k[0] - seg_end > gap * 1e6:
            segs.append(cur)
            cur = []
        seg_end = max(seg_end, k[1]) if cur else k[1]
        cur.append(k)
    if cur:
        segs.append(cur)
    out = []
    for i, sgm in enumerate(segs):
        tot = sum(e - s for s, e, _ in sgm)
        busy, ce = 0, None
        for s, e, _ in sgm:
            if ce is None or s > ce:
                busy += e - s
                ce = e
            elif e > ce:
                busy += e - ce
                ce = e
        span = max(e for _, e, _ in sgm) - sgm[0][0]
        out.append({"segment": i, "kernels": len(sgm), "kernel_sum_ms": tot / 1e6, "busy_ms": busy / 1e6,
                    "span_ms": span / 1e6})
        print(f"segment {i}: {len(sgm):5d} kernels  sum {tot / 1e6:8.3f} ms  busy {busy / 1e6:8.3f} ms  "
              f"span {span / 1e6:8.3f} ms")
    top = collections.Counter()
    for s, e, n in segs[-1]:
        top[n.split("(")[0].replace("void ", "")[:60]] += e - s
    # per-category kernel sums of the last segment: runtime copies / fills (the host transport's
    # staging copies land here) apart from the library's kernels
    cats = collections.Counter()
    for n, v in top.items():
        c = ("runtime copy/fill" if n.startswith("__amd_rocclr") else "merkle" if "merkle" in n
             else "ntt" if ("ntt" in n or "bitrev" in n) else "other kernels")
        cats[c] += v
    print("last segment by category (ms): " + ", ".join(f"{c} {v / 1e6:.3f}" for c, v in cats.most_common()))
    print("last segment, top kernels (ms):")
    for n, v in top.most_common(15):
        print(f"  {v / 1e6:8.3f}  {n}")
    if len(sys.argv) > 3:
        json.dump({"segments": out, "top_last": {n: v / 1e6 for n, v in top.most_common(30)},
                   "categories_last": {c: v / 1e6 for c, v in cats.items()}},
                  open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
