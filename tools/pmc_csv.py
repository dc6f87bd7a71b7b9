#!/usr/bin/env python3
"""Mean counter value per dispatch, per kernel, from rocprofv3 --pmc csv output
(<dir>/<name>_counter_collection.csv).

usage: pmc_csv.py counter_collection.csv [kernel-substring]
"""
import csv
import sys
from collections import defaultdict


def main():
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    meta = {}
    for r in csv.DictReader(open(sys.argv[1])):
        k = r["Kernel_Name"]
        if flt not in k:
            continue
        short = k.split("(")[0].replace("void ", "")[:60]
        d = r["Dispatch_Id"]
        per[short][r["Counter_Name"]][d] = per[short][r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
        meta[short] = (r.get("VGPR_Count", r.get("Arch_VGPR_Count", "?")), r.get("LDS_Block_Size", "?"))
    for k, cs in per.items():
        nd = len(next(iter(cs.values())))
        print(f"{k}  vgpr={meta[k][0]} lds={meta[k][1]}  dispatches={nd}")
        for cn in sorted(cs):
            vals = list(cs[cn].values())
            print(f"    {cn:26s} {sum(vals) / len(vals):18.1f}")


if __name__ == "__main__":
    main()
