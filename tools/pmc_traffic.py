#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is
exact for 16-byte-per-lane streaming stores.  Kernels are keyed by the name the bench
reports (merkle_leaves = k_merkle_levels<true,...>, ...).

usage: pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON
"""
import collections
import csv
import json
import sys

ALIASES = [("k_merkle_leaf_pairs<512, true>", "merkle_fold_leaves"), ("k_merkle_leaf_pairs", "merkle_leaves"),
           ("k_merkle_levels<true, 256, true>", "merkle_fold_leaves"),
           ("k_merkle_levels<true, 512, true>", "merkle_fold_leaves"),
           ("k_merkle_levels<true, 1024, true>", "merkle_fold_leaves"), ("k_merkle_levels<true", "merkle_leaves"), ("k_merkle_levels<false", "merkle_nodes"),
           ("k_merkle_quad_leaves", "merkle_leaves_quad"), ("k_merkle_quad", "merkle_nodes_quad"), ("k_ntt_pass", "ntt_pass"), ("k_ntt_first", "ntt_first"),
           ("k_bitrev_gather", "bitrev_gather")]


def alias(name):
    for k, v in ALIASES:
        if k in name:
            return v
    return None


def load(fn):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(fn)):
        a = alias(r["Kernel_Name"])
        if a:
            out[a].append((float(r["Counter_Value"]) * 1024.0, int(r["Grid_Size"])))
    return out


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    res = {}
    for k in sorted(set(fetch) & set(write)):
        n = min(len(fetch[k]), len(write[k]))
        rd = 2.0 * sum(v for v, _ in fetch[k][:n])
        wr = sum(v for v, _ in write[k][:n])
        lanes = sum(g for _, g in fetch[k][:n])
        # per launch (this pass's population) and per lane (Grid_Size), so bench.py can scale the
        # measured bytes to the lanes its own live launches ran
        res[k] = {"launches": n, "read_bytes_per_launch": rd / n, "write_bytes_per_launch": wr / n,
                  "hbm_bytes_per_launch": (rd + wr) / n, "hbm_bytes_per_lane": (rd + wr) / lanes}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; read = 2*FETCH_SIZE",
               "kernels": res}, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
