"""Round-6 experiment record (not part of the build): generates fe128_asm.inc, the NTT butterfly's
128-bit field arithmetic as gfx950 inline-asm blocks whose carry chains are interleaved so that no
wait state is needed.  Measured and removed from kernels.hip: the
k_ntt_pass_rr<11> listing lost 78 % of its wait states and C2 did not move
(profiles/r06_ab_asm_c2.log), and the variant faulted in kernels where hipcc's own scalar code
follows an asm block that left a VALU-written carry SGPR (profiles/r06_ab_asm_prove_fault.log,
r06_pytest_gpu_asm_fault_ntt2p12.log): hipcc does not see the hazards inside inline asm.

Why (VERDICT r05 "Next round" 1): every 32-bit carry link is a VALU that writes an SGPR carry and a
VALU that reads it; gfx950 needs two wait states between the two.  hipcc allocates every chain's
carry to VCC, which serializes independent chains, and pads each link with `s_nop 1`: the shipped
k_ntt_pass_rr<11> carried 5 361 wait states against 11 136 VALU instructions.  Here the carries are
virtual SGPR pairs, a list scheduler interleaves the chains of one Montgomery product (its product
columns, both reduction steps and the final conditional subtraction) with the previous butterfly's
lazy add / sub chains, and inserts `s_nop` only where nothing is ready.  Pairs are allocated
even-aligned (gfx950 requires aligned 64-bit VGPR operands) in a fixed VGPR window that the asm
declares clobbered, because inline asm cannot name the halves of a 64-bit operand.

Every generated block is executed by the instruction simulator below on random and edge-case
inputs and compared with the field arithmetic (`python tools/gen_fe_asm.py --check` runs it; the
build does not need it).  The arithmetic is the one of csrc/fe128.hpp (mont_mul, fe_add_lazy,
fe_sub_lazy): p = 1 + 407 * 2^119 (field/field.rs:10), R = 2^128, two 64-bit Montgomery steps.

  python tools/gen_fe_asm.py [out.inc]  # write the .inc (default /tmp/fe128_asm.inc) and check it
"""
import os
import random
import re
import sys

P = 1 + 407 * (1 << 119)
P3 = 0xCB800000
NEG_P3 = 0x347FFFFF
M32 = 0xFFFFFFFF
R = 1 << 128
RINV = pow(R, -1, P)

# ----------------------------------------------------------------------------- program builder


class Op:
    __slots__ = ("fmt", "vdst", "vsrc", "sdst", "ssrc", "kind", "idx", "salu")

    def __init__(self, fmt, vdst=(), vsrc=(), sdst=(), ssrc=(), kind="valu"):
        self.fmt, self.vdst, self.vsrc, self.sdst, self.ssrc, self.kind = fmt, list(vdst), list(vsrc), list(sdst), list(ssrc), kind
        self.salu = kind == "salu"


class Prog:
    """Ops over named registers.  V registers: 'tN' virtual 32-bit temps, 'pN' virtual 64-bit pairs
    (halves 'pN.lo' / 'pN.hi'), or operand names ('a0', ...).  S registers: 'cN' virtual SGPR pairs,
    'junk' (an unread carry-out), or operand names.  Constants are written inline."""

    def __init__(self):
        self.ops = []
        self.n = 0

    def t(self):
        self.n += 1
        return "t%d" % self.n

    def p(self):
        self.n += 1
        return "p%d" % self.n

    def c(self):
        self.n += 1
        return "c%d" % self.n

    @staticmethod
    def halves(r):
        return [r + ".lo", r + ".hi"] if r.startswith("p") and "." not in r else [r]

    def emit(self, fmt, vdst=(), vsrc=(), sdst=(), ssrc=(), kind="valu"):
        vd = [h for r in vdst for h in self.halves(r)]
        vs = [h for r in vsrc for h in self.halves(r)]
        self.ops.append(Op(fmt, vd, vs, sdst, ssrc, kind))
        return self.ops[-1]

    # instruction helpers (gfx950 VOP3 forms, explicit carry SGPR pairs)
    def mad(self, dst, s0, s1, s2, cout="junk"):
        vs = [x for x in (s0, s1) if not isinstance(x, int) and not x.startswith("P3s")]
        ss = [x for x in (s0, s1) if isinstance(x, str) and x.startswith("P3s")]
        if isinstance(s2, str):
            vs.append(s2)
        self.emit("v_mad_u64_u32 {%s}, {%s}, %s, %s, %s" % (dst, cout, self.o(s0), self.o(s1), self.o(s2)),
                  [dst], vs, [cout], ss)

    @staticmethod
    def o(x):
        return str(x) if isinstance(x, int) else "{%s}" % x

    def _vs(self, *xs):
        return [x for x in xs if isinstance(x, str)]

    def add(self, d, a, b, cout="junk"):
        self.emit("v_add_co_u32_e64 {%s}, {%s}, %s, %s" % (d, cout, self.o(a), self.o(b)), [d], self._vs(a, b), [cout])

    def addc(self, d, a, b, cin, cout="junk"):
        self.emit("v_addc_co_u32_e64 {%s}, {%s}, %s, %s, {%s}" % (d, cout, self.o(a), self.o(b), cin),
                  [d], self._vs(a, b), [cout], [cin])

    def sub(self, d, a, b, cout="junk"):
        self.emit("v_sub_co_u32_e64 {%s}, {%s}, %s, %s" % (d, cout, self.o(a), self.o(b)), [d], self._vs(a, b), [cout])

    def subb(self, d, a, b, cin, cout="junk"):
        self.emit("v_subb_co_u32_e64 {%s}, {%s}, %s, %s, {%s}" % (d, cout, self.o(a), self.o(b), cin),
                  [d], self._vs(a, b), [cout], [cin])

    def cnd(self, d, a, b, mask):
        """d = mask ? b : a"""
        self.emit("v_cndmask_b32_e64 {%s}, %s, %s, {%s}" % (d, self.o(a), self.o(b), mask), [d], self._vs(a, b), [], [mask])

    def mov(self, d, a):
        self.emit("v_mov_b32 {%s}, %s" % (d, self.o(a)), [d], self._vs(a))

    def sor(self, d, a, b):
        self.emit("s_or_b64 {%s}, {%s}, {%s}" % (d, a, b), [], [], [d], [a, b], kind="salu")


# ----------------------------------------------------------------------------- arithmetic


def mont(g, a, b, out):
    """out = a * b * 2^-128 mod p (canonical) for a < 2^128, b < p: fe128.hpp mont_mul's algorithm
    (product scanning, two sparse 64-bit Montgomery steps, one conditional subtraction)."""
    # product columns: column k accumulates in pair A[k] = {lo, hi}; the column's carry count is
    # written straight into the next column's pair hi (A[k+1].hi), its hi is moved into A[k+1].lo
    prods = {k: [(i, k - i) for i in range(4) if 0 <= k - i < 4] for k in range(7)}
    A = [g.p() for _ in range(7)]
    g.mad(A[0], a[0], b[0], 0)
    g.mov(A[1] + ".lo", A[0] + ".hi")
    g.mov(A[1] + ".hi", 0)
    for k in range(1, 7):
        if k >= 2:
            g.mov(A[k] + ".lo", A[k - 1] + ".hi")
        cs = []
        for n, (i, j) in enumerate(prods[k]):
            if k == 1 and n == 0:
                g.mad(A[k], a[i], b[j], A[k])  # < 2^32 + (2^32 - 1)^2: no carry
            elif k == 6:
                g.mad(A[k], a[i], b[j], A[k])  # the top column cannot overflow (T < 2^256)
            else:
                c = g.c()
                g.mad(A[k], a[i], b[j], A[k], c)
                cs.append(c)
        if k < 6:
            nxt = A[k + 1] + ".hi"
            for n, c in enumerate(cs):
                if n == 0:
                    g.cnd(nxt, 0, 1, c)
                else:
                    g.addc(nxt, nxt, 0, c)
    t = [A[0] + ".lo", A[1] + ".lo", A[2] + ".lo", A[3] + ".lo", A[4] + ".lo", A[5] + ".lo", A[6] + ".lo", A[6] + ".hi"]

    def step(x0, x1, rest, last):
        # m = -(x1:x0) mod 2^64; (x1:x0) + m carries exactly when (x1:x0) != 0 (borrow br);
        # m * (p - 1) = (m * P3) << 96 = {q0.lo, q1.lo, q1.hi} at limbs 3..5
        m0, m1, b0, br = g.t(), g.t(), g.c(), g.c()
        g.sub(m0, 0, x0, b0)
        g.subb(m1, 0, x1, b0, br)
        q0, q1 = g.p(), g.p()
        g.mad(q0, m0, "P3s", 0)
        g.mov(q1 + ".lo", q0 + ".hi")
        g.mov(q1 + ".hi", 0)
        g.mad(q1, m1, "P3s", q1)
        addend = [None, q0 + ".lo", q1 + ".lo", q1 + ".hi"] + [None] * (len(rest) - 4)
        u = [g.t() for _ in rest]
        cy = br
        for i, x in enumerate(rest):
            last_link = i == len(rest) - 1
            nc = (last if last_link else g.c())
            g.addc(u[i], x, addend[i] if addend[i] else 0, cy, nc if nc else "junk")
            cy = nc
        return u

    u = step(t[0], t[1], t[2:8], None)       # U = (T + m p) / 2^64 < 2^192: u5 has no carry out
    cf = g.c()
    r = step(u[0], u[1], u[2:6], cf)          # r + cf 2^128 < 2p
    d = [g.t() for _ in range(4)]
    gc = [g.c() for _ in range(4)]
    g.add(d[0], r[0], -1, gc[0])
    g.addc(d[1], r[1], -1, gc[0], gc[1])
    g.addc(d[2], r[2], -1, gc[1], gc[2])
    g.addc(d[3], r[3], "NEGP3v", gc[2], gc[3])
    take = g.c()
    g.sor(take, cf, gc[3])
    for i in range(4):
        g.cnd(out[i], r[i], d[i], take)


def addsub(g, e, o, sum_out, diff_out):
    """sum_out = fe_add_lazy(e, o), diff_out = fe_sub_lazy(e, o) (fe128.hpp): e < 2^128, o < p."""
    s = [g.t() for _ in range(4)]
    d = [g.t() for _ in range(4)]
    ca = [g.c() for _ in range(4)]
    cb = [g.c() for _ in range(4)]
    g.add(s[0], e[0], o[0], ca[0])
    g.sub(d[0], e[0], o[0], cb[0])
    for i in range(1, 4):
        g.addc(s[i], e[i], o[i], ca[i - 1], ca[i])
        g.subb(d[i], e[i], o[i], cb[i - 1], cb[i])
    # add: on carry add 2^128 - p = [m, m, m, NEG_P3] under the carry mask
    m, m3 = g.t(), g.t()
    g.cnd(m, 0, -1, ca[3])
    g.cnd(m3, 0, "NEGP3v", ca[3])
    cc = [g.c() for _ in range(3)]
    g.add(sum_out[0], s[0], m, cc[0])
    g.addc(sum_out[1], s[1], m, cc[0], cc[1])
    g.addc(sum_out[2], s[2], m, cc[1], cc[2])
    g.addc(sum_out[3], s[3], m3, cc[2])
    # sub: on borrow add p = 1 + (P3 << 96)
    n3 = g.t()
    g.cnd(n3, 0, "P3v", cb[3])
    cd = [g.c() for _ in range(3)]
    g.addc(diff_out[0], d[0], 0, cb[3], cd[0])
    g.addc(diff_out[1], d[1], 0, cd[0], cd[1])
    g.addc(diff_out[2], d[2], 0, cd[1], cd[2])
    g.addc(diff_out[3], d[3], n3, cd[2])


# ----------------------------------------------------------------------------- scheduler

HAZ = 2  # wait states between a VALU write of an SGPR and a VALU read of it
# wait states between a VALU write of an SGPR and a scalar (SALU / SMEM / VMEM-address) access that
# may write or read it: the VALU's SGPR write-back can land after a scalar write issued too soon
# (a late carry overwrote a kernel-argument pointer that hipcc's s_load put in the same SGPR
# right after a block: an illegal address).  Inside a block this orders the s_or; at the end of a
# block the generator pads the last VALU-written SGPR to this distance, since hipcc cannot see it.
VALU_SGPR_SCALAR = 5


def deps(ops):
    """Predecessor lists: (pred, min distance in issue slots)."""
    last_w, reads_since = {}, {}
    preds = [[] for _ in ops]
    for i, op in enumerate(ops):
        for r in op.vsrc:
            if r in last_w:
                preds[i].append((last_w[r], 1))
        for r in op.ssrc:
            if r in last_w:
                w = last_w[r]
                dist = 1 + HAZ if not ops[w].salu and not op.salu else 1
                preds[i].append((w, dist))
        for r in op.vdst + [s for s in op.sdst if s != "junk"]:
            if r in last_w:
                w = last_w[r]
                # WAW: a scalar write after a VALU write of the same SGPR waits for its write-back
                dist = 1 + VALU_SGPR_SCALAR if r in op.sdst and op.salu and not ops[w].salu else 1
                preds[i].append((w, dist))
            for rd in reads_since.get(r, []):
                if rd != i:
                    preds[i].append((rd, 1))  # WAR
        for r in op.vsrc + op.ssrc:
            reads_since.setdefault(r, []).append(i)
        for r in op.vdst + [s for s in op.sdst if s != "junk"]:
            last_w[r] = i
            reads_since[r] = []
    return preds


def schedule(ops):
    n = len(ops)
    preds = deps(ops)
    succs = [[] for _ in ops]
    for i, ps in enumerate(preds):
        for p, d in ps:
            succs[p].append((i, d))
    # priority: longest path (in slots, mads weighted) to the end
    w = [2 if o.fmt.startswith("v_mad") else 1 for o in ops]
    prio = [0] * n
    for i in reversed(range(n)):
        prio[i] = w[i] + max([prio[s] + d - 1 for s, d in succs[i]] or [0])
    slot_of = [None] * n
    npred = [len(p) for p in preds]
    earliest = [0] * n
    ready = {i for i in range(n) if npred[i] == 0}
    out, slot, done = [], 0, 0
    while done < n:
        cand = [i for i in ready if earliest[i] <= slot]
        if not cand:
            out.append(None)  # one wait state
            slot += 1
            continue
        i = max(cand, key=lambda k: (prio[k], -k))
        ready.discard(i)
        slot_of[i] = slot
        out.append(i)
        done += 1
        for s, d in succs[i]:
            earliest[s] = max(earliest[s], slot + d)
            npred[s] -= 1
            if npred[s] == 0:
                ready.add(s)
        slot += 1
    return out


# ----------------------------------------------------------------------------- allocation


def allocate(ops, order, fixed_v, nsgpr_max=12):
    """Linear-scan allocation of virtual temps / pairs (window registers, pairs even-aligned) and
    virtual carries (SGPR operand pairs) over the scheduled order."""
    seq = [ops[i] for i in order if i is not None]
    first, last = {}, {}
    for k, op in enumerate(seq):
        for r in op.vdst + op.vsrc + op.sdst + op.ssrc:
            base = r.split(".")[0]
            first.setdefault(base, k)
            last[base] = k
    vmap, smap = {}, {}
    free_v, free_s = set(), []
    vbusy, sbusy = {}, {}
    nwin, nsg = 0, 0
    events = sorted(first, key=lambda b: first[b])
    for k, op in enumerate(seq):
        # free what died before k
        for b in list(vbusy):
            if last[b] < k:
                for reg in vbusy.pop(b):
                    free_v.add(reg)
        for b in list(sbusy):
            if last[b] < k:
                free_s.append(sbusy.pop(b))
        for r in op.vdst + op.sdst:
            b = r.split(".")[0]
            if b in vmap or b in smap or b in fixed_v or b == "junk":
                continue
            if b.startswith("t"):
                if free_v:
                    reg = min(free_v)
                    free_v.discard(reg)
                else:
                    reg, nwin = nwin, nwin + 1
                vmap[b] = [reg]
                vbusy[b] = [reg]
            elif b.startswith("p"):
                pairs = sorted(x for x in free_v if x % 2 == 0 and x + 1 in free_v)
                if pairs:
                    reg = pairs[0]
                    free_v -= {reg, reg + 1}
                else:
                    if nwin % 2:
                        free_v.add(nwin)
                        nwin += 1
                    reg, nwin = nwin, nwin + 2
                vmap[b] = [reg, reg + 1]
                vbusy[b] = [reg, reg + 1]
            elif b.startswith("c"):
                if op.salu:
                    # a scalar write never lands on a pair a VALU of this block wrote (its late
                    # write-back could overwrite it): SALU-written carries get pairs of their own
                    s = "salu%d" % len([k for k in smap.values() if str(k).startswith("salu")])
                elif free_s:
                    s = free_s.pop()
                else:
                    s, nsg = nsg, nsg + 1
                smap[b] = s
                if not op.salu:
                    sbusy[b] = s
        # a register read but never written (cannot happen for temps)
    assert nsg <= nsgpr_max, nsg
    return vmap, smap, nwin, nsg


# ----------------------------------------------------------------------------- emission


def render(ops, order, vmap, smap, win_base, opnames):
    """Asm text lines with GCC operand references for operands, physical window registers for temps."""
    def vname(r):
        b, _, half = r.partition(".")
        if b in vmap:
            regs = vmap[b]
            if half == "lo":
                return "v%d" % (win_base + regs[0])
            if half == "hi":
                return "v%d" % (win_base + regs[1])
            if len(regs) == 2:
                return "v[%d:%d]" % (win_base + regs[0], win_base + regs[1])
            return "v%d" % (win_base + regs[0])
        return "%%[%s]" % opnames.get(b, b)

    def sname(r):
        if r == "junk":
            return "%[sj]"
        if r in smap:
            return "%%[s%s]" % smap[r]
        return "%%[%s]" % opnames.get(r, r)

    lines, nops = [], 0
    for i in order:
        if i is None:
            nops += 1
            lines.append(None)
            continue
        op = ops[i]

        def sub(m):
            r = m.group(1)
            if r in op.sdst or r in op.ssrc or r == "junk":
                return sname(r)
            return vname(r)
        lines.append(re.sub(r"\{([^}]+)\}", sub, op.fmt))
    # the block's end: pad so that its last VALU-written SGPR is VALU_SGPR_SCALAR wait states old
    # (hipcc's next instruction may be a scalar write or read of that register)
    since = 0
    for l, i in zip(reversed(lines), reversed(order)):
        if l is None or ops[i].salu or not ops[i].sdst:
            since += 1
            continue
        break
    lines = lines + [None] * max(0, VALU_SGPR_SCALAR - since)
    nops += max(0, VALU_SGPR_SCALAR - since)
    # merge consecutive nops into s_nop N
    out, run = [], 0
    for l in lines + ["END"]:
        if l is None:
            run += 1
            continue
        while run:
            k = min(run, 8)
            out.append("s_nop %d" % (k - 1))
            run -= k
        if l != "END":
            out.append(l)
    return out, nops


# ----------------------------------------------------------------------------- simulator


def simulate(lines, env):
    """Executes the rendered lines on one lane.  env: operand name -> int (32-bit values, SGPR
    pairs as 0/1 carry bits), window registers 'vN'."""
    def val(tok):
        tok = tok.strip()
        if tok.startswith("%["):
            return env[tok[2:-1]]
        if tok.startswith("v["):
            lo, hi = map(int, tok[2:-1].split(":"))
            return env.get("v%d" % lo, 0) | (env.get("v%d" % hi, 0) << 32)
        if tok.startswith("v"):
            return env["v" + tok[1:]] if ("v" + tok[1:]) in env else env.setdefault("v" + tok[1:], 0)
        return int(tok, 0) & M32

    def put(tok, v):
        tok = tok.strip()
        if tok.startswith("%["):
            env[tok[2:-1]] = v
        elif tok.startswith("v["):
            lo, hi = map(int, tok[2:-1].split(":"))
            env["v%d" % lo] = v & M32
            env["v%d" % hi] = (v >> 32) & M32
        else:
            env[tok] = v

    for l in lines:
        if l.startswith("s_nop"):
            continue
        opc, rest = l.split(None, 1)
        a = [x.strip() for x in rest.split(",")]
        if opc == "v_mad_u64_u32":
            s2 = val(a[4]) if not a[4].strip().lstrip("-").isdigit() else int(a[4])
            r = val(a[2]) * val(a[3]) + s2
            put(a[0], r & ((1 << 64) - 1))
            put(a[1], r >> 64)
        elif opc == "v_add_co_u32_e64":
            r = val(a[2]) + val(a[3])
            put(a[0], r & M32)
            put(a[1], r >> 32)
        elif opc == "v_addc_co_u32_e64":
            r = val(a[2]) + val(a[3]) + val(a[4])
            put(a[0], r & M32)
            put(a[1], r >> 32)
        elif opc == "v_sub_co_u32_e64":
            r = val(a[2]) - val(a[3])
            put(a[0], r & M32)
            put(a[1], 1 if r < 0 else 0)
        elif opc == "v_subb_co_u32_e64":
            r = val(a[2]) - val(a[3]) - val(a[4])
            put(a[0], r & M32)
            put(a[1], 1 if r < 0 else 0)
        elif opc == "v_cndmask_b32_e64":
            put(a[0], val(a[2]) if val(a[3]) else val(a[1]))
        elif opc == "v_mov_b32":
            put(a[0], val(a[1]))
        elif opc == "s_or_b64":
            put(a[0], 1 if (val(a[1]) or val(a[2])) else 0)
        else:
            raise ValueError(l)
    return env


def limbs(x):
    return [(x >> (32 * i)) & M32 for i in range(4)]


def unlimbs(v):
    return sum(x << (32 * i) for i, x in enumerate(v))


# ----------------------------------------------------------------------------- blocks

OPS_IN = {}


def block_mont():
    g = Prog()
    a, b, o = ["a0", "a1", "a2", "a3"], ["b0", "b1", "b2", "b3"], ["o0", "o1", "o2", "o3"]
    mont(g, a, b, o)
    return g, dict(outs=o, ins=a + b, inout=[])


def block_bfly():
    """One radix-2 butterfly: o = mont(x, w); e <- e + o (lazy); x <- e - o (lazy)."""
    g = Prog()
    e, x, w = ["e0", "e1", "e2", "e3"], ["x0", "x1", "x2", "x3"], ["w0", "w1", "w2", "w3"]
    o = [g.t() for _ in range(4)]
    mont(g, x, w, o)
    addsub(g, e, o, e, x)
    return g, dict(outs=[], ins=w, inout=e + x)


def block_bfly_pipe():
    """Software-pipelined butterfly: o = mont(x, w) for this butterfly (out o*), and the lazy add /
    sub of the previous butterfly (pe <- pe + po, po <- pe - po)."""
    g = Prog()
    x, w, o = ["x0", "x1", "x2", "x3"], ["w0", "w1", "w2", "w3"], ["o0", "o1", "o2", "o3"]
    pe, po = ["pe0", "pe1", "pe2", "pe3"], ["po0", "po1", "po2", "po3"]
    addsub(g, pe, po, pe, po)
    mont(g, x, w, o)
    return g, dict(outs=o, ins=x + w, inout=pe + po)


def block_addsub():
    g = Prog()
    pe, po = ["pe0", "pe1", "pe2", "pe3"], ["po0", "po1", "po2", "po3"]
    addsub(g, pe, po, pe, po)
    return g, dict(outs=[], ins=[], inout=pe + po)


def block_addsub2():
    g = Prog()
    pe, po = ["pe0", "pe1", "pe2", "pe3"], ["po0", "po1", "po2", "po3"]
    qe, qo = ["qe0", "qe1", "qe2", "qe3"], ["qo0", "qo1", "qo2", "qo3"]
    addsub(g, pe, po, pe, po)
    addsub(g, qe, qo, qe, qo)
    return g, dict(outs=[], ins=[], inout=pe + po + qe + qo)


def build_block(maker, win_base):
    g, io = maker()
    fixed = set(io["outs"]) | set(io["ins"]) | set(io["inout"]) | {"P3s", "NEGP3v", "P3v"}
    order = schedule(g.ops)
    vmap, smap, nwin, nsg = allocate(g.ops, order, fixed)
    lines, nops = render(g.ops, order, vmap, smap, win_base, {})
    # an output operand ("=v") may share a register with an input: no input read after the first
    # output write
    seq = [g.ops[i] for i in order if i is not None]
    outs = set(io["outs"])
    first_out = min([k for k, op in enumerate(seq) if set(op.vdst) & outs] or [len(seq)])
    last_in = max([k for k, op in enumerate(seq) if set(op.vsrc) & set(io["ins"])] or [-1])
    assert last_in < first_out, "an output is written before the last input read"
    return dict(g=g, io=io, lines=lines, nops=nops, nwin=nwin, nsg=nsg, nvalu=sum(1 for o in seq if not o.salu),
                nsalu=sum(1 for o in seq if o.salu))


# ----------------------------------------------------------------------------- checks

EDGE = [0, 1, 2, P - 1, P - 2, (1 << 128) - 1, 1 << 127, (1 << 96) - 1, P3 << 96, (1 << 64) - 1, 1 << 64]


def check(blk, name, trials=3000, seed=1):
    rnd = random.Random(seed)
    io = blk["io"]

    def rand_lazy():
        return rnd.choice(EDGE) if rnd.random() < 0.2 else rnd.randrange(1 << 128)

    def rand_canon():
        return rnd.choice([v for v in EDGE if v < P]) if rnd.random() < 0.2 else rnd.randrange(P)

    const = {"P3s": P3, "NEGP3v": NEG_P3, "P3v": P3}
    for _ in range(trials):
        env = dict(const)
        if name == "mont":
            a, b = rand_lazy(), rand_canon()
            for i in range(4):
                env["a%d" % i], env["b%d" % i] = limbs(a)[i], limbs(b)[i]
            simulate(blk["lines"], env)
            got = unlimbs([env["o%d" % i] for i in range(4)])
            assert got == a * b * RINV % P, (name, a, b)
        elif name in ("bfly", "bfly_pipe", "addsub", "addsub2"):
            vals = {}
            groups = {"bfly": ["e", "x", "w"], "bfly_pipe": ["x", "w", "pe", "po"], "addsub": ["pe", "po"],
                      "addsub2": ["pe", "po", "qe", "qo"]}[name]
            for gname in groups:
                v = rand_canon() if gname in ("w", "po", "qo") else rand_lazy()
                vals[gname] = v
                for i in range(4):
                    env["%s%d" % (gname, i)] = limbs(v)[i]
            simulate(blk["lines"], env)
            res = {gname: unlimbs([env["%s%d" % (gname, i)] for i in range(4)]) for gname in groups}

            def lazy_add(e, o):
                s = e + o
                return s - P if s >= 1 << 128 else s

            def lazy_sub(e, o):
                s = e - o
                return s + P if s < 0 else s

            if name == "bfly":
                o = vals["x"] * vals["w"] * RINV % P
                assert res["e"] == lazy_add(vals["e"], o) and res["x"] == lazy_sub(vals["e"], o), name
                assert res["e"] % P == (vals["e"] + o) % P
            if name == "bfly_pipe":
                o = unlimbs([env["o%d" % i] for i in range(4)])
                assert o == vals["x"] * vals["w"] * RINV % P, name
            if name in ("bfly_pipe", "addsub", "addsub2"):
                assert res["pe"] == lazy_add(vals["pe"], vals["po"]) and res["po"] == lazy_sub(vals["pe"], vals["po"]), name
            if name == "addsub2":
                assert res["qe"] == lazy_add(vals["qe"], vals["qo"]) and res["qo"] == lazy_sub(vals["qe"], vals["qo"]), name
    return True


# ----------------------------------------------------------------------------- C++ emission

WIN_BASE = int(os.environ.get("SG_ASM_WIN_BASE", "2"))


def snames(blk):
    """The block's SGPR-pair operands: VALU carries s0.., SALU-only pairs ssalu0.., the junk pair."""
    text = "\n".join(blk["lines"])
    salu = sorted(set(re.findall(r"%\[(ssalu\d+)\]", text)))
    return ["s%d" % k for k in range(blk["nsg"])] + salu + ["sj"]


def cxx(name, blk, win_base):
    io = blk["io"]
    nwin = blk["nwin"]
    outs = ['[%s] "=v"(%s)' % (o, o) for o in io["outs"]]
    inouts = ['[%s] "+v"(%s)' % (o, o) for o in io["inout"]]
    souts = ['[%s] "=&s"(%s)' % (k, k) for k in snames(blk)]
    ins = ['[%s] "v"(%s)' % (i, i) for i in io["ins"]]
    used_consts = set(re.findall(r"%\[(P3s|NEGP3v|P3v)\]", "\n".join(blk["lines"])))
    cins = []
    if "P3s" in used_consts:
        cins.append('[P3s] "s"(0xCB800000u)')
    if "NEGP3v" in used_consts:
        cins.append('[NEGP3v] "v"(neg_p3)')
    if "P3v" in used_consts:
        cins.append('[P3v] "v"(p3)')
    clob = ", ".join('"v%d"' % (win_base + k) for k in range(nwin))
    body = "\n".join('      "%s\\n"' % l for l in blk["lines"])
    return body, ", ".join(outs + inouts + souts), ", ".join(ins + cins), clob


HEADER = """// GENERATED by tools/gen_fe_asm.py -- do not edit.  The NTT butterfly's field arithmetic
// (fe128.hpp mont_mul / fe_add_lazy / fe_sub_lazy, same results) as gfx950 inline asm whose carry
// chains are interleaved so that every VALU-written carry SGPR is read >= 2 instructions later:
// no wait states inside a block.  Temporaries live in the clobbered window v%d..v%d (64-bit pairs
// even-aligned); carries in compiler-allocated SGPR pairs.  Each block was executed by the
// generator's instruction simulator on random and edge-case inputs against the field arithmetic.
// Block statistics (VALU / SALU instructions, wait states padded by s_nop):
%s
#pragma once
#if defined(__HIP_DEVICE_COMPILE__)
namespace sg {
"""


def gen(win_base=WIN_BASE):
    blocks = {"mont": block_mont, "bfly": block_bfly, "bfly_pipe": block_bfly_pipe, "addsub": block_addsub,
              "addsub2": block_addsub2}
    built = {}
    for name, mk in blocks.items():
        blk = build_block(mk, win_base)
        check(blk, name)
        built[name] = blk
    nwin = max(b["nwin"] for b in built.values())
    stats = "\n".join("//   %-10s %3d VALU + %d SALU, %2d wait states, %2d window VGPRs, %d carry pairs"
                      % (n, b["nvalu"], b["nsalu"], b["nops"], b["nwin"], b["nsg"]) for n, b in built.items())
    src = [HEADER % (win_base, win_base + nwin - 1, stats)]
    # mont: fe mont_mul_asm(const fe& a, const fe& b)
    b = built["mont"]
    body, outs, ins, clob = cxx("mont", b, win_base)
    src.append("""__device__ __forceinline__ fe mont_mul_asm(const fe& a, const fe& b) {
  uint32_t a0 = a.w[0], a1 = a.w[1], a2 = a.w[2], a3 = a.w[3], b0 = b.w[0], b1 = b.w[1], b2 = b.w[2], b3 = b.w[3];
  uint32_t o0, o1, o2, o3;
  const uint32_t neg_p3 = 0x347FFFFFu;
  uint64_t %s;
  asm(
%s
      : %s
      : %s
      : %s);
  fe r = {{o0, o1, o2, o3}};
  return r;
}
""" % (", ".join(snames(b)), body, outs, ins, clob))
    for name, sig, pre, post in (
        ("bfly", "fe& e, fe& x, const fe& w",
         "uint32_t e0 = e.w[0], e1 = e.w[1], e2 = e.w[2], e3 = e.w[3], x0 = x.w[0], x1 = x.w[1], x2 = x.w[2], x3 = x.w[3];\n"
         "  const uint32_t w0 = w.w[0], w1 = w.w[1], w2 = w.w[2], w3 = w.w[3];",
         "e.w[0] = e0; e.w[1] = e1; e.w[2] = e2; e.w[3] = e3; x.w[0] = x0; x.w[1] = x1; x.w[2] = x2; x.w[3] = x3;"),
        ("bfly_pipe", "fe& pe, fe& po, const fe& x, const fe& w, fe& o",
         "uint32_t pe0 = pe.w[0], pe1 = pe.w[1], pe2 = pe.w[2], pe3 = pe.w[3], po0 = po.w[0], po1 = po.w[1], po2 = po.w[2], po3 = po.w[3];\n"
         "  const uint32_t x0 = x.w[0], x1 = x.w[1], x2 = x.w[2], x3 = x.w[3], w0 = w.w[0], w1 = w.w[1], w2 = w.w[2], w3 = w.w[3];\n"
         "  uint32_t o0, o1, o2, o3;",
         "pe.w[0] = pe0; pe.w[1] = pe1; pe.w[2] = pe2; pe.w[3] = pe3; po.w[0] = po0; po.w[1] = po1; po.w[2] = po2; po.w[3] = po3;\n"
         "  o.w[0] = o0; o.w[1] = o1; o.w[2] = o2; o.w[3] = o3;"),
        ("addsub", "fe& pe, fe& po",
         "uint32_t pe0 = pe.w[0], pe1 = pe.w[1], pe2 = pe.w[2], pe3 = pe.w[3], po0 = po.w[0], po1 = po.w[1], po2 = po.w[2], po3 = po.w[3];",
         "pe.w[0] = pe0; pe.w[1] = pe1; pe.w[2] = pe2; pe.w[3] = pe3; po.w[0] = po0; po.w[1] = po1; po.w[2] = po2; po.w[3] = po3;"),
        ("addsub2", "fe& pe, fe& po, fe& qe, fe& qo",
         "uint32_t pe0 = pe.w[0], pe1 = pe.w[1], pe2 = pe.w[2], pe3 = pe.w[3], po0 = po.w[0], po1 = po.w[1], po2 = po.w[2], po3 = po.w[3];\n"
         "  uint32_t qe0 = qe.w[0], qe1 = qe.w[1], qe2 = qe.w[2], qe3 = qe.w[3], qo0 = qo.w[0], qo1 = qo.w[1], qo2 = qo.w[2], qo3 = qo.w[3];",
         "pe.w[0] = pe0; pe.w[1] = pe1; pe.w[2] = pe2; pe.w[3] = pe3; po.w[0] = po0; po.w[1] = po1; po.w[2] = po2; po.w[3] = po3;\n"
         "  qe.w[0] = qe0; qe.w[1] = qe1; qe.w[2] = qe2; qe.w[3] = qe3; qo.w[0] = qo0; qo.w[1] = qo1; qo.w[2] = qo2; qo.w[3] = qo3;"),
    ):
        b = built[name]
        body, outs, ins, clob = cxx(name, b, win_base)
        fname = {"bfly": "bfly_asm", "bfly_pipe": "bfly_pipe_asm", "addsub": "addsub_asm", "addsub2": "addsub2_asm"}[name]
        src.append("""__device__ __forceinline__ void %s(%s) {
  %s
  const uint32_t neg_p3 = 0x347FFFFFu, p3 = 0xCB800000u;
  uint64_t %s;
  asm(
%s
      : %s
      : %s
      : %s);
  %s
}
""" % (fname, sig, pre, ", ".join(snames(b)), body, outs,
       ins if ins else "", clob if clob else "", post))
    src.append("}  // namespace sg\n#endif\n")
    return "".join(src), built


if __name__ == "__main__":
    text, built = gen()
    for n, b in built.items():
        print("%-10s VALU %3d SALU %d  wait states %2d  window %2d  carries %d" % (n, b["nvalu"], b["nsalu"], b["nops"], b["nwin"], b["nsg"]))
    if "--check" not in sys.argv:
        args = [a for a in sys.argv[1:] if not a.startswith("--")]
        out = args[0] if args else "/tmp/fe128_asm.inc"
        with open(out, "w") as f:
            f.write(text)
        print("wrote", out)
