#!/usr/bin/env python3
"""Per-step device time of the sharded NTT replays (tools/dist_ntt_replay.py) from their rocprofv3
kernel traces: the trace is cut into steps at idle gaps >= 300 ms; the steps are the segments made
of library kernels (sg::...); the first one (plan building) is dropped -- and in a replay the last segment, the check's own single-GPU
transform -- and the rest averaged.
Prints a markdown table per transform size: single GPU vs rank 0 at world G -- library kernels by
class (NTT passes, four-step transposes, other library kernels), runtime copies / fills (the host
transport's staging), and the library total's ratio to the single-GPU transform.

usage: ntt_replay_table.py DIR   (DIR/single_<L>/ and DIR/replay_<L>_<G>/ hold run_kernel_trace.csv)
"""
import csv
import glob
import json
import os
import sys

GAP_NS = 300e6


def steps(path, replay):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    segs, cur, end = [], [], 0
    for k in rows:
        if cur and k[0] - end > GAP_NS:
            segs.append(cur)
            cur = []
        end = max(end, k[1]) if cur else k[1]
        cur.append(k)
    if cur:
        segs.append(cur)
    lib = [s for s in segs if any(n.startswith(("sg::", "void sg::")) for _, _, n in s)]
    # drop the first step (plan building) and, in a replay, the last segment: the check's single-GPU
    # transform (tools/dist_ntt_replay.py sleeps before it)
    return lib[1:-1] if replay else lib[1:]


def classify(name):
    n = name.replace("void ", "")
    if n.startswith("__amd_rocclr"):
        return "copies"
    if not n.startswith("sg::"):
        return None
    if "ntt" in n or "bitrev" in n:
        return "ntt"
    if "swap01" in n:
        return "transpose"
    return "other"


def summarize(path, replay):
    sts = steps(path, replay)
    acc = {"ntt": 0.0, "transpose": 0.0, "other": 0.0, "copies": 0.0}
    for s in sts:
        for a, b, n in s:
            c = classify(n)
            if c:
                acc[c] += (b - a) / 1e6
    k = max(len(sts), 1)
    out = {c: v / k for c, v in acc.items()}
    out["library"] = out["ntt"] + out["transpose"] + out["other"]
    out["steps"] = len(sts)
    return out


def main():
    d = sys.argv[1]
    res = {}
    for p in sorted(glob.glob(os.path.join(d, "*", "*kernel_trace.csv"))):
        name = os.path.basename(os.path.dirname(p))
        res[name] = summarize(p, name.startswith("replay"))
    for L in sorted({int(k.split("_")[1]) for k in res}):
        cols = [("single GPU", res.get(f"single_{L}"))] + [(f"world {G}, rank 0", res.get(f"replay_{L}_{G}"))
                                                            for G in (2, 4, 8)]
        cols = [(lbl, r) for lbl, r in cols if r]
        if not cols:
            continue
        base = cols[0][1]["library"]
        print(f"\n2^{L} fwd + inv, device time per step (ms)\n")
        print("| | " + " | ".join(lbl for lbl, _ in cols) + " |")
        print("|---|" + "---|" * len(cols))
        for key, name in (("ntt", "NTT passes"), ("transpose", "four-step transposes"),
                          ("other", "other library kernels")):
            print(f"| {name} | " + " | ".join(f"{r[key]:.3f}" for _, r in cols) + " |")
        print("| **library kernels (ratio to single GPU)** | "
              + " | ".join(f"**{r['library']:.3f} ({r['library'] / base:.2f})**" for _, r in cols) + " |")
        print("| runtime copies / fills (host-transport staging) | "
              + " | ".join(f"{r['copies']:.3f}" for _, r in cols) + " |")
    json.dump(res, open(os.path.join(d, "ntt_replay_table.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
