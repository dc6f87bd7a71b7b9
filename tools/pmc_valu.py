#!/usr/bin/env python3
"""Per-kernel VALU issue from a rocprofv3 --pmc pass (SQ_INSTS_VALU, GRBM_GUI_ACTIVE).

SQ_INSTS_VALU counts wave-level VALU instructions; GRBM_GUI_ACTIVE is the busy-cycle
count summed over the 8 XCDs, so clock = GRBM_GUI_ACTIVE / 8 / duration.  Everything is
reduced per WAVE (Grid_Size / 64 of each dispatch), so the figure applies to any launch
population (bench.py scales it by the lanes its live launches ran).

Roofs (wave64 VALU instructions per second at the measured clock, 1024 SIMDs):
  peak     -- the SIMD-32 issue rate, 1 instruction / 2 clk (MI355X_MICROARCH.md:54,473)
  mix_roof -- the kernel's static full/half-rate mix (tools/valu_mix.py) at the measured
              per-op rates (profiles/r01_microbench_int_v2.txt)

usage: pmc_valu.py COUNTER_CSV MIX_JSON OUT_JSON
"""
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import alias  # noqa: E402

SIMDS = 1024


def main():
    rows = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(sys.argv[1])):
        a = alias(r["Kernel_Name"])
        if not a:
            continue
        d = r["Dispatch_Id"]
        rows[(a, d)][r["Counter_Name"]] = rows[(a, d)].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[(a, d)] = (int(r["Grid_Size"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    mix = json.load(open(sys.argv[2]))["kernels"]
    per = collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0.0, 0])  # instr, waves, dur, busy, n
    for key, c in rows.items():
        grid, dur = meta[key]
        if dur <= 0 or "SQ_INSTS_VALU" not in c:
            continue
        acc = per[key[0]]
        acc[0] += c["SQ_INSTS_VALU"]
        acc[1] += grid / 64.0
        acc[2] += dur
        acc[3] += c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        acc[4] += 1
    res = {}
    for a, (inst, waves, dur, busy, n) in sorted(per.items()):
        clk = busy / dur
        rate = inst / dur
        peak = SIMDS * clk / 2.0
        e = {"launches": n, "valu_instr_per_wave": inst / waves, "clock_ghz": clk / 1e9,
             "achieved_wave_instr_per_s": rate, "peak_wave_instr_per_s": peak, "frac": rate / peak}
        if a in mix:
            roof = SIMDS * clk / mix[a]["clk_per_wave_instr_per_simd"]
            e.update({"mix_roof_wave_instr_per_s": roof, "mix_frac": rate / roof, "half_rate_frac": mix[a]["half_frac"]})
        res[a] = e
    json.dump({"source": "rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE (per-dispatch Grid_Size, timestamps)",
               "roof": "peak = 1 wave64 VALU instr / SIMD / 2 clk x 1024 SIMDs at the measured clock; "
                       "mix_roof = the kernel's static full/half-rate mix at the measured per-op rates",
               "kernels": res}, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
