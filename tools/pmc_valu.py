#!/usr/bin/env python3
"""Per-kernel VALU issue from a rocprofv3 --pmc pass (SQ_INSTS_VALU, GRBM_GUI_ACTIVE).

SQ_INSTS_VALU counts wave-level VALU instructions (all SEs); GRBM_GUI_ACTIVE is the GPU
busy-cycle count summed over the 8 XCDs, so clock = GRBM_GUI_ACTIVE / 8 / duration.
The issue roof used here is one wave64 VALU instruction per SIMD per 4 cycles
(16-lane SIMDs; 1024 SIMDs on MI355X) at the measured clock: the non-VOP2 integer
ops the BLAKE2b / Montgomery kernels are made of issue at that rate
(profiles/r01_microbench_int_v2.txt); plain VOP2 ops (xor/add/shift) issue faster,
so a pure-VOP2 kernel could exceed 1.0.

usage: pmc_valu.py COUNTER_CSV KERNEL_TRACE_CSV OUT_JSON
"""
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import alias  # noqa: E402

SIMDS = 1024


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(sys.argv[1])):
        a = alias(r["Kernel_Name"])
        if a:
            vals[(a, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for r in csv.DictReader(open(sys.argv[2])):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = collections.defaultdict(list)
    for (a, d), c in vals.items():
        if d in dur and dur[d] > 0 and "SQ_INSTS_VALU" in c:
            per[a].append((c["SQ_INSTS_VALU"], c.get("GRBM_GUI_ACTIVE", 0.0), dur[d]))
    res = {}
    for a, lst in sorted(per.items()):
        n = len(lst)
        inst = sum(x[0] for x in lst) / n
        t = sum(x[2] for x in lst) / n
        clk = sum(x[1] for x in lst) / 8 / sum(x[2] for x in lst)
        peak = SIMDS * clk / 4
        res[a] = {"launches": n, "valu_wave_instr_per_launch": inst, "avg_ms": t * 1e3, "clock_ghz": clk / 1e9,
                  "achieved_wave_instr_per_s": inst / t, "peak_wave_instr_per_s": peak,
                  "frac": inst / t / peak}
    json.dump({"source": "rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE (+ --kernel-trace durations)",
               "roof": "1 wave64 VALU instruction / SIMD / 4 cycles, 1024 SIMDs, measured clock",
               "kernels": res}, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
