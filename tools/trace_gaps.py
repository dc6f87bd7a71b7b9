#!/usr/bin/env python3
"""Busy time, per-kernel totals and the largest idle gaps of the last prove in a rocprofv3
--kernel-trace csv (the final burst of dispatches split into `steps` equal parts).  With
kernels on two streams, "busy" is the union of the dispatch intervals.

usage: trace_gaps.py run_kernel_trace.csv [steps]
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs, cur, end = [], [rows[0]], int(rows[0]["End_Timestamp"])
    for b in rows[1:]:
        if int(b["Start_Timestamp"]) - end > 2e6:
            segs.append(cur)
            cur = []
        cur.append(b)
        end = max(end, int(b["End_Timestamp"]))
    segs.append(cur)
    last = segs[-1]
    seg = last[-(len(last) // steps):]
    t0 = int(seg[0]["Start_Timestamp"])
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    # union of intervals and the idle gaps between them
    busy, gaps, cur_end, prev = 0, [], None, None
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur_end is None or s > cur_end:
            if cur_end is not None and (s - cur_end) / 1e3 > 20:
                gaps.append(((s - cur_end) / 1e3, (cur_end - t0) / 1e3, prev["Kernel_Name"][:28], r["Kernel_Name"][:28]))
            if cur_end is not None:
                busy += 0
            cur_start, cur_end = s, e
            busy += e - s
        elif e > cur_end:
            busy += e - cur_end
            cur_end = e
        prev = r if prev is None or int(r["End_Timestamp"]) >= int(prev["End_Timestamp"]) else prev
    span = max(int(r["End_Timestamp"]) for r in seg) - t0
    print(f"dispatches/prove {len(seg)}  span {span / 1e6:.3f} ms  busy (union) {busy / 1e6:.3f} ms  "
          f"kernel time (sum) {sum(map(dur, seg)) / 1e6:.3f} ms")
    agg = defaultdict(float)
    for r in seg:
        agg[r["Kernel_Name"].split("(")[0].replace("void ", "")[:45]] += dur(r) / 1e6
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {k:45s} {v:7.3f} ms")
    print(f"gaps > 20 us: {len(gaps)}, {sum(g[0] for g in gaps):.1f} us")
    for g in sorted(gaps, reverse=True)[:15]:
        print(f"  {g[0]:7.1f} us at {g[1]:9.1f}  after {g[2]:28s} before {g[3]}")


if __name__ == "__main__":
    main()
