#!/usr/bin/env python3
"""Summary of a tools/ab.sh log: per variant, the numbers of each round (the first float on each
'LABEL: ...' line, or the regex's first group when given, e.g. 'step ([0-9.]+)' for a prove log or
'([0-9.]+) ms/build' for a Merkle log) and their median.

usage: ab_summary.py LOG [regex]
"""
import re
import statistics
import sys
from collections import OrderedDict


def main():
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"([0-9]+\.[0-9]+)")
    vals = OrderedDict()
    for line in open(sys.argv[1]):
        m = re.match(r"^(\w[\w.-]*): (.*)$", line.strip())
        if not m:
            continue
        lab, rest = m.groups()
        mm = pat.search(rest)
        if mm:
            vals.setdefault(lab, []).append(float(mm.group(1)))
    for lab, v in vals.items():
        print(f"{lab:10s} median {statistics.median(v):9.4f}  rounds {' / '.join(f'{x:.4f}' for x in v)}")


if __name__ == "__main__":
    main()
