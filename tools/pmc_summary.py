#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc sqlite output: per kernel name, mean counter value per dispatch.

usage: pmc_summary.py run_results.db [name-filter]
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sqlite3.connect(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = db.execute("select dispatch_id, kernel_name, counter_name, value, duration, vgpr_count, lds_block_size "
                      "from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(list))
    meta = {}
    for d, k, cn, v, dur, vg, lds in rows:
        if flt not in k:
            continue
        short = k.split("(")[0][:60]
        per[short][cn].append(v)
        per[short]["_dur_ns"].append(dur)
        meta[short] = (vg, lds)
    for k, cs in per.items():
        print(f"{k}  vgpr={meta[k][0]} lds={meta[k][1]}  dispatches={len(cs[next(iter(cs))])}")
        for cn in sorted(cs):
            vals = cs[cn]
            print(f"    {cn:24s} {sum(vals) / len(vals):16.1f}")


if __name__ == "__main__":
    main()
