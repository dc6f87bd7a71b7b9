"""Counts VALU instructions, s_nop instructions and the wait states they pad, per kernel, in a gfx950
listing (make -C zk-stark-tutor_amd asm), and classifies the nops by the instructions around them.

  python tools/asm_nops.py zk-stark-tutor_amd/build/kernels-only-gfx950.s [kernel-substring ...]
"""
import collections
import sys


def kernels(path):
    name, body = None, []
    for raw in open(path):
        l = raw.strip()
        head = l.split(" ", 1)[0]
        if head.endswith(":") and head.startswith("_Z"):
            name, body = head[:-1], []
            continue
        if name and l.startswith(".Lfunc_end"):
            yield name, body
            name = None
            continue
        if name and l and ((not l.startswith((";", ".")) and not l.endswith(":")) or l.startswith(";;#ASM")):
            body.append(l)


def stats(body):
    nops = states = valu = 0
    ctx = collections.Counter()
    for i, l in enumerate(body):
        op = l.split()[0]
        if op.startswith("v_"):
            valu += 1
        elif op == "s_nop":
            n = int(l.split()[1].rstrip(",")) + 1
            nops += 1
            states += n
            ctx[(body[i - 1].split()[0], body[i + 1].split()[0] if i + 1 < len(body) else "")] += n
    return valu, nops, states, ctx


if __name__ == "__main__":
    path, pats = sys.argv[1], sys.argv[2:] or ["k_ntt_pass_rr", "k_ntt_first"]
    for name, body in kernels(path):
        if not any(p in name for p in pats):
            continue
        valu, nops, states, ctx = stats(body)
        print("%-70s valu %6d  s_nop %5d  wait states %5d (%.2f per VALU)" % (name[:70], valu, nops, states,
                                                                             states / max(valu, 1)))
        if "-v" in sys.argv[0:1] or len(pats) == 1:
            for k, v in ctx.most_common(8):
                print("      %5d  %s -> %s" % (v, k[0], k[1]))
