#!/usr/bin/env python3
"""Critical path of one prove from a rocprofv3 kernel trace (VERDICT r05 "Next round" 4).

The proves of the traced run are separated by idle gaps (SG_PROVE_GAPS=1 tools/prove_only.py); the
last one is taken.  Walking back from its last kernel, each step goes to the kernel (either stream)
that ended last before the current one started -- the chain of work that could not start earlier.
Between two chain kernels the chip was either running other (off-chain) kernels or idle (host round
trips: Fiat-Shamir, degree checks, launches).  Printed: the chain kernel by kernel (start, duration,
stream, the idle time before it) and a summary by kernel family, plus the prove's span / busy time.

usage: critical_path.py run_kernel_trace.csv [gap_ms=20] [json_out]
"""
import collections
import csv
import json
import re
import sys


def family(name: str) -> str:
    n = name
    for key, fam in (("merkle_leaf_pairs", "tree leaves"), ("merkle_quad_leaves", "tree leaves (small)"),
                     ("merkle_levels<true", "tree leaves"), ("merkle_quad", "tree tops"), ("merkle_levels", "tree nodes"),
                     ("ntt_pass", "NTT"), ("ntt_first", "NTT"), ("bitrev", "NTT"), ("air", "AIR"),
                     ("batch_div", "quotient division"), ("fri_fold", "FRI fold"), ("serialize", "openings"),
                     ("gather", "gathers"), ("geo", "interpolation"), ("tree_", "interpolation"), ("copy", "copies")):
        if key in n:
            return fam
    return "other algebra"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sg::", ""), r["Queue_Id"])
                for r in rows)
    segs, cur, end = [], [], 0
    for k in ks:
        if cur and k[0] - end > gap * 1e6:
            segs.append(cur)
            cur = []
        end = max(end, k[1]) if cur else k[1]
        cur.append(k)
    segs.append(cur)
    seg = segs[-1]
    t0 = seg[0][0]
    span = max(e for _, e, _, _ in seg) - t0
    busy, ce = 0, None
    for s, e, _, _ in seg:
        if ce is None or s > ce:
            busy += e - s
            ce = e
        elif e > ce:
            busy += e - ce
            ce = e
    # walk back
    by_end = sorted(seg, key=lambda k: k[1])
    chain = [by_end[-1]]
    while True:
        s = chain[-1][0]
        prev = [k for k in by_end if k[1] <= s]
        if not prev:
            break
        chain.append(prev[-1])
    chain.reverse()
    print("prove: %d kernels, span %.3f ms, busy %.3f ms (%.0f %%), chain of %d kernels" %
          (len(seg), span / 1e6, busy / 1e6, 100 * busy / span, len(chain)))
    print("%9s %8s %8s %6s  %s" % ("start_ms", "dur_us", "idle_us", "queue", "kernel"))
    fam_t, fam_n, idle_tot, last_end = collections.Counter(), collections.Counter(), 0, t0
    lines = []
    for s, e, n, q in chain:
        idle = max(0, s - last_end)
        idle_tot += idle
        fam_t[family(n)] += e - s
        fam_n[family(n)] += 1
        lines.append({"start_ms": round((s - t0) / 1e6, 4), "dur_us": round((e - s) / 1e3, 2),
                      "idle_before_us": round(idle / 1e3, 2), "queue": q, "kernel": n})
        print("%9.4f %8.2f %8.2f %6s  %s" % ((s - t0) / 1e6, (e - s) / 1e3, idle / 1e3, q, n[:70]))
        last_end = e
    print("\nchain by family (ms, kernels):")
    for f, t in fam_t.most_common():
        print("  %-22s %7.3f  %4d" % (f, t / 1e6, fam_n[f]))
    print("  %-22s %7.3f" % ("idle between (host)", idle_tot / 1e6))
    # all kernels of the prove by family (device time on either stream)
    allf = collections.Counter()
    for s, e, n, q in seg:
        allf[family(n)] += e - s
    print("\nwhole prove by family (device ms, both streams):")
    for f, t in allf.most_common():
        print("  %-22s %7.3f" % (f, t / 1e6))
    if len(sys.argv) > 3:
        json.dump({"span_ms": span / 1e6, "busy_ms": busy / 1e6, "chain": lines,
                   "chain_by_family_ms": {f: t / 1e6 for f, t in fam_t.items()}, "chain_idle_ms": idle_tot / 1e6,
                   "all_by_family_ms": {f: t / 1e6 for f, t in allf.items()}}, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
