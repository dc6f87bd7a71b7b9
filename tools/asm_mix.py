#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing (gfx950).

usage: asm_mix.py LISTING.s NAME_SUBSTRING [top]
"""
import collections
import re
import sys


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r'^(_Z\w+):', line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur:
            if line.startswith('.Lfunc_end'):
                yield cur, body
                cur, body = None, []
            else:
                body.append(line)


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    for name, body in kernels(path):
        if sub not in name:
            continue
        c = collections.Counter()
        for line in body:
            t = line.strip()
            if not t or t[0] in '.;_' or t.endswith(':'):
                continue
            c[t.split()[0]] += 1
        valu = sum(v for k, v in c.items() if k.startswith('v_'))
        print(f"{name}: VALU {valu}, SALU {sum(v for k, v in c.items() if k.startswith('s_'))}, "
              f"LDS {sum(v for k, v in c.items() if k.startswith('ds_'))}, "
              f"VMEM {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_')))}")
        for k, v in c.most_common(top):
            print(f"   {k:28s} {v}")


if __name__ == '__main__':
    main()
