"""CPU oracle, part 2: the reference's polynomial algebra, multivariate AIR, Rescue-Prime
and the end-to-end `Stark::prove` / `Stark::verify` (BASELINE config C4).

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the
checker.  The product path (`zk-stark-tutor_amd/`) never imports it.

Every function restates the reference crate (SpekalsG3/zk-stark-tutor, Rust)
at the cited `file:line` under `/root/reference/src/`, keeping the data
conventions that influence proof bytes:

* `Polynomial` (field/polynomial.rs) is a coefficient list that is never
  trimmed: `degree()` skips trailing zeros, `Add` of a zero polynomial returns
  the other operand, `Mul` has length len_a + len_b - 1.
* `MPolynomial` (m_polynomial.rs) is a dict {exponent tuple: coefficient}
  that keeps zero coefficients (Add/Mul never delete keys); the STARK's degree
  bounds are computed from the KEYS (stark.rs:117-160), so the key set is
  restated exactly.
* `thread_rng` randomness (stark.rs:283-298, 425-433) is unpinnable (crate
  `rand 0.8.5`, unseeded): `Stark.prove` takes the randomizer field elements as
  explicit arguments, in the order the reference draws them.

Parity of this restatement is pinned by the reference's own known-answer tests
(rescue_prime.rs:297-342: alpha, alpha_inv, MDS, MDS^-1, the 108 round
constants, hash(1), trace/constraint checks; matrix.rs tests) transcribed in
`tests/golden/reference_kats_e2e.json`, and by the reference's randomized
property tests (ntt_arithmetics.rs:354-560, stark.rs:810-881) restated in
`tests/test_oracle_e2e.py`.
"""
from __future__ import annotations

from math import gcd
from typing import Dict, List, Optional, Sequence, Tuple

from stark_oracle import (CODEWORD, FRI, GENERATOR, P, PATH, PROOF_BYTES, ROOT, VALUE,  # noqa: F401
                          IndependentProofStream, add_mod, div, fpow, intt, inv, merkle_commit,
                          merkle_levels, merkle_open_levels, merkle_verify, mul_mod, neg_mod, ntt,
                          primitive_nth_root, sample, shake256, sub_mod)

Poly = List[int]


# ------------------------------------------------------------ Polynomial (polynomial.rs)

def degree(p: Sequence[int]) -> Optional[int]:
    """polynomial.rs:41-58: index of the last non-zero coefficient, None if there is none."""
    d = None
    for i, c in enumerate(p):
        if c != 0:
            d = i
    return d


def is_zero(p: Sequence[int]) -> bool:
    """polynomial.rs:60-62."""
    return degree(p) is None


def p_add(a: Sequence[int], b: Sequence[int]) -> Poly:
    """polynomial.rs:251-276: a zero operand returns the other one unchanged (length kept)."""
    if degree(a) is None:
        return list(b)
    if degree(b) is None:
        return list(a)
    out = [0] * max(len(a), len(b))
    for i, c in enumerate(a):
        out[i] = add_mod(out[i], c)
    for i, c in enumerate(b):
        out[i] = add_mod(out[i], c)
    return out


def p_neg(a: Sequence[int]) -> Poly:
    """polynomial.rs:238-249."""
    return [neg_mod(c) for c in a]


def p_sub(a: Sequence[int], b: Sequence[int]) -> Poly:
    """polynomial.rs:278-283: a + (-b)."""
    return p_add(a, p_neg(b))


def p_mul(a: Sequence[int], b: Sequence[int]) -> Poly:
    """polynomial.rs:285-308: schoolbook, length len_a + len_b - 1, empty if either is empty."""
    if len(a) == 0 or len(b) == 0:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x == 0:
            continue
        for j, y in enumerate(b):
            out[i + j] = (out[i + j] + x * y) % P
    return out


def p_pow(a: Sequence[int], e: int) -> Poly:
    """polynomial.rs:328-356: zero -> zero; e == 0 -> [1]; MSB-first square-and-multiply."""
    if is_zero(a):
        return []
    acc = [1]
    if e == 0:
        return acc
    for i in range(e.bit_length() - 1, -1, -1):
        acc = p_mul(acc, acc)
        if (e >> i) & 1:
            acc = p_mul(acc, a)
    return acc


def p_scale(a: Sequence[int], factor: int) -> Poly:
    """polynomial.rs:109-121: c_i <- factor^i c_i."""
    out, pw = [], 1
    for c in a:
        out.append(mul_mod(pw, c))
        pw = mul_mod(pw, factor)
    return out


def p_evaluate(a: Sequence[int], x: int) -> int:
    """polynomial.rs:72-97 (sum of c_i x^i)."""
    acc, xi = 0, 1
    for c in a:
        acc = add_mod(acc, mul_mod(c, xi))
        xi = mul_mod(xi, x)
    return acc


def divide_with_rem(num: Sequence[int], den: Sequence[int]) -> Tuple[Poly, Poly]:
    """polynomial.rs:179-224 (long division; raises like the reference's Err on a zero denominator)."""
    dd = degree(den)
    if dd is None:
        raise ZeroDivisionError("Denominator is zero or empty")
    nd = degree(num)
    if nd is None or nd < dd:
        return [], list(num)
    rem = list(num)
    steps = nd - dd + 1
    q = [0] * steps
    lead = den[dd]
    for _ in range(steps):
        rd = degree(rem)
        if rd is None or rd < dd:
            break
        coef = div(rem[rd], lead)
        shift = rd - dd
        sub = p_mul([0] * shift + [coef], den)
        rem = p_sub(rem, sub)
        q[shift] = coef
    return q, rem


def p_rem(a: Sequence[int], b: Sequence[int]) -> Poly:
    """polynomial.rs:310-317."""
    return divide_with_rem(a, b)[1]


# ------------------------------------------------------- NTT arithmetic (ntt_arithmetics.rs)

def _check_root(root: int, root_order: int) -> None:
    """ntt_arithmetics.rs:11-24 (the assertions every fast_* function starts with)."""
    assert fpow(root, root_order) == 1, "supplied root does not have supplied root_order"
    assert fpow(root, root_order // 2) != 1, "supplied root is not a primitive of root_order"


def fast_multiply(root: int, root_order: int, lhs: Sequence[int], rhs: Sequence[int]) -> Poly:
    """ntt_arithmetics.rs:5-64: shrink the order while degree < order/2, NTT, Hadamard, INTT,
    truncate to deg+1."""
    _check_root(root, root_order)
    if is_zero(lhs) or is_zero(rhs):
        return []
    deg = degree(lhs) + degree(rhs)
    result_len = deg + 1
    order = root_order
    while deg < order // 2:
        root = mul_mod(root, root)
        order //= 2

    def inner(p):
        p = list(p) + [0] * max(0, order - len(p))
        return ntt(root, p)

    lv, rv = inner(lhs), inner(rhs)
    coeffs = intt(root, [mul_mod(x, y) for x, y in zip(lv, rv)])
    return coeffs[:result_len] if result_len < len(coeffs) else coeffs


def fast_zerofier(root: int, root_order: int, domain: Sequence[int]) -> Poly:
    """ntt_arithmetics.rs:66-113: product tree of (x - d) with fast_multiply."""
    _check_root(root, root_order)

    def inner(dom):
        if len(dom) == 0:
            return []
        if len(dom) == 1:
            return [neg_mod(dom[0]), 1]
        half = len(dom) // 2
        return fast_multiply(root, root_order, inner(dom[:half]), inner(dom[half:]))

    return inner(list(domain))


def fast_evaluate_domain(root: int, root_order: int, poly: Sequence[int], domain: Sequence[int]) -> List[int]:
    """ntt_arithmetics.rs:115-159: remainder tree."""
    _check_root(root, root_order)

    def inner(p, dom):
        if len(dom) == 0:
            return []
        if len(dom) == 1:
            return [p_evaluate(p, dom[0])]
        half = len(dom) // 2
        left = fast_zerofier(root, root_order, dom[:half])
        right = fast_zerofier(root, root_order, dom[half:])
        return inner(p_rem(p, left), dom[:half]) + inner(p_rem(p, right), dom[half:])

    return inner(list(poly), list(domain))


def fast_interpolate_domain(root: int, root_order: int, domain: Sequence[int], values: Sequence[int]) -> Poly:
    """ntt_arithmetics.rs:172-237: recursive halves, left*Z_right + right*Z_left."""
    _check_root(root, root_order)
    assert len(domain) == len(values)

    def inner(dom, vals):
        if len(dom) == 0:
            return []
        if len(dom) == 1:
            return [vals[0]]
        half = len(dom) // 2
        lz = fast_zerofier(root, root_order, dom[:half])
        rz = fast_zerofier(root, root_order, dom[half:])
        lo = fast_evaluate_domain(root, root_order, rz, dom[:half])
        ro = fast_evaluate_domain(root, root_order, lz, dom[half:])
        lt = [div(vals[i], d) for i, d in enumerate(lo)]
        rt = [div(vals[i + half], d) for i, d in enumerate(ro)]
        li = inner(dom[:half], lt)
        ri = inner(dom[half:], rt)
        return p_add(p_mul(li, rz), p_mul(ri, lz))

    return inner(list(domain), list(values))


def fast_coset_divide(root: int, root_order: int, offset: int, lhs: Sequence[int], rhs: Sequence[int]) -> Poly:
    """ntt_arithmetics.rs:239-310: scale both by offset, NTT at the shrunk order, pointwise
    division (panics on a zero divisor value), INTT, truncate to deg_l - deg_r + 1, unscale."""
    _check_root(root, root_order)
    assert not is_zero(rhs), "cannot divide by zero polynomial"
    if is_zero(lhs):
        return []
    dl, dr = degree(lhs), degree(rhs)
    assert dl >= dr, "cannot divide by polynomial of larger degree"
    deg = max(dl, dr)
    result_len = dl - dr + 1
    order = root_order
    while deg < order // 2:
        root = mul_mod(root, root)
        order //= 2

    def inner(p):
        p = p_scale(p, offset)
        p = p + [0] * max(0, order - len(p))
        return ntt(root, p)

    lv, rv = inner(lhs), inner(rhs)
    coeffs = intt(root, [div(x, y) for x, y in zip(lv, rv)])
    if result_len < len(coeffs):
        coeffs = coeffs[:result_len]
    return p_scale(coeffs, inv(offset))


# ------------------------------------------------------------ MPolynomial (m_polynomial.rs)

class MPolynomial:
    """m_polynomial.rs:11-300: {exponent tuple: coefficient}; zero coefficients are kept."""

    def __init__(self, d: Optional[Dict[Tuple[int, ...], int]] = None):
        self.d: Dict[Tuple[int, ...], int] = dict(d or {})

    @staticmethod
    def zero() -> "MPolynomial":
        return MPolynomial()

    @staticmethod
    def constant(c: int) -> "MPolynomial":
        """m_polynomial.rs:37-44: key [0] (one variable)."""
        return MPolynomial({(0,): c})

    @staticmethod
    def variables(n: int) -> List["MPolynomial"]:
        """m_polynomial.rs:49-64."""
        out = []
        for i in range(n):
            e = [0] * n
            e[i] = 1
            out.append(MPolynomial({tuple(e): 1}))
        return out

    @staticmethod
    def lift(poly: Sequence[int], variable_index: int) -> "MPolynomial":
        """m_polynomial.rs:66-81: sum of constant(c_i) * x_v^i over ALL coefficients (zeros too)."""
        acc = MPolynomial.zero()
        if is_zero(poly):
            return acc
        x = MPolynomial.variables(variable_index + 1)[-1]
        for i, c in enumerate(poly):
            acc = acc + MPolynomial.constant(c) * (x ** i)
        return acc

    def is_zero(self) -> bool:
        """m_polynomial.rs:83-93."""
        return all(v == 0 for v in self.d.values())

    def __neg__(self) -> "MPolynomial":
        return MPolynomial({k: neg_mod(v) for k, v in self.d.items()})

    def __add__(self, o: "MPolynomial") -> "MPolynomial":
        """m_polynomial.rs:183-222: pad keys to the longest, accumulate (keys never removed)."""
        if not self.d:
            return MPolynomial(o.d)
        if not o.d:
            return MPolynomial(self.d)
        nv = max(max(len(k) for k in self.d), max(len(k) for k in o.d))
        out: Dict[Tuple[int, ...], int] = {}
        for k, v in self.d.items():
            out[k + (0,) * (nv - len(k))] = v
        for k, v in o.d.items():
            k = k + (0,) * (nv - len(k))
            out[k] = add_mod(out[k], v) if k in out else v
        return MPolynomial(out)

    def __sub__(self, o: "MPolynomial") -> "MPolynomial":
        return self + (-o)

    def __mul__(self, o: "MPolynomial") -> "MPolynomial":
        """m_polynomial.rs:231-262: every pair of keys, summed exponents."""
        nv = max(max(len(k) for k in self.d), max(len(k) for k in o.d))
        out: Dict[Tuple[int, ...], int] = {}
        for k0, v0 in self.d.items():
            for k1, v1 in o.d.items():
                e = [0] * nv
                for i, x in enumerate(k0):
                    e[i] += x
                for i, x in enumerate(k1):
                    e[i] += x
                e = tuple(e)
                pr = mul_mod(v0, v1)
                out[e] = add_mod(out[e], pr) if e in out else pr
        return MPolynomial(out)

    def __pow__(self, e: int) -> "MPolynomial":
        """m_polynomial.rs:265-298: zero -> zero; acc = {0^nv: 1}; per bit (BitIter, at least
        one bit): acc = acc*acc, then * self on a set bit."""
        if self.is_zero():
            return MPolynomial.zero()
        nv = len(next(iter(self.d)))
        acc = MPolynomial({(0,) * nv: 1})
        nbits = max(e.bit_length(), 1)
        for i in range(nbits - 1, -1, -1):
            acc = acc * acc
            if (e >> i) & 1:
                acc = acc * self
        return acc

    def evaluate(self, point: Sequence[int]) -> int:
        """m_polynomial.rs:95-122."""
        acc = 0
        for k, c in self.d.items():
            prod = c
            for i, e in enumerate(k):
                prod = mul_mod(prod, fpow(point[i], e))
            acc = add_mod(acc, prod)
        return acc

    def evaluate_symbolic(self, point: Sequence[Sequence[int]]) -> Poly:
        """m_polynomial.rs:124-139: sum over keys of [c] * prod point_i ^ e_i.

        Powers point_i ^ e are memoised (the reference recomputes them per key; the
        polynomial computed is the same)."""
        cache: Dict[Tuple[int, int], Poly] = {}

        def pw(i, e):
            if (i, e) not in cache:
                cache[(i, e)] = p_pow(point[i], e)
            return cache[(i, e)]

        acc: Poly = []
        for k, c in self.d.items():
            prod = [c]
            for i, e in enumerate(k):
                prod = p_mul(prod, pw(i, e))
            acc = p_add(acc, prod)
        return acc


# ------------------------------------------------------------------- matrix (utils/matrix.rs)

def rref(m: List[List[int]]) -> None:
    """utils/matrix.rs:5-49 (in place)."""
    lead = 0
    rows, cols = len(m), len(m[0])
    for r in range(rows):
        if cols <= lead:
            break
        i = r
        stop = False
        while m[i][lead] == 0:
            i += 1
            if rows == i:
                i = r
                lead += 1
                if cols == lead:
                    stop = True
                    break
        if stop:
            break
        m[i], m[r] = m[r], m[i]
        if m[r][lead] != 0:
            piv = m[r][lead]
            m[r] = [div(el, piv) for el in m[r]]
        for i in range(rows):
            if i != r:
                hold = m[i][lead]
                for k in range(cols):
                    m[i][k] = sub_mod(m[i][k], mul_mod(hold, m[r][k]))
        lead += 1


def transpose(m: List[List[int]]) -> List[List[int]]:
    """utils/matrix.rs:52-66."""
    return [[m[r][c] for r in range(len(m))] for c in range(len(m[0]))]


def inverse(m: List[List[int]]) -> List[List[int]]:
    """utils/matrix.rs:68-110: rref of [M | I], check the left block is I."""
    n = len(m)
    aug = []
    for i, row in enumerate(m):
        assert len(row) == n, "Inverse exists only for square matrices"
        e = [0] * n
        e[i] = 1
        aug.append(list(row) + e)
    rref(aug)
    for i, row in enumerate(aug):
        if any(row[j] != (1 if j == i else 0) for j in range(n)):
            raise ValueError("Couldnt construct identity matrix to find inverse")
    return [row[n:] for row in aug]


# ------------------------------------------------------------- Rescue-Prime (rescue_prime.rs)

def smallest_generator() -> int:
    """field/field.rs:46-56: smallest k >= 3 with gcd(k, p - 1) == 1."""
    k = 3
    while gcd(k, P - 1) != 1:
        k += 1
    return k


class RescuePrime:
    """rescue_prime/rescue_prime.rs:10-272."""

    def __init__(self, m: int, capacity: int, security_level: int, N: int):
        g = smallest_generator()
        self.m, self.capacity, self.security_level, self.N = m, capacity, security_level, N
        self.alpha = g
        self.alpha_inv = inv(neg_mod(g))  # rescue_prime.rs:123 (field.inv(field.neg_mod(g)))
        self.MDS = self.get_mds(g, m)
        self.MDS_inv = inverse(self.MDS)
        self.round_constants = self.get_round_constants(m, capacity, security_level, N)

    @staticmethod
    def get_mds(g: int, m: int) -> List[List[int]]:
        """rescue_prime.rs:130-148: rref of [g^(i j)] (m x 2m), right half, transposed."""
        mat = [[fpow(g, i * j) for j in range(2 * m)] for i in range(m)]
        rref(mat)
        return transpose([row[m:] for row in mat])

    @staticmethod
    def get_round_constants(m: int, capacity: int, security_level: int, N: int) -> List[int]:
        """rescue_prime.rs:150-180: SHAKE256("Rescue-XLIX(p,m,cap,sec)"), 17-byte chunks,
        sum_j 256^j * b_j."""
        bytes_per_int = (P.bit_length() + 7) // 8 + 1
        num = 2 * m * N
        seed = "Rescue-XLIX({},{},{},{})".format(P, m, capacity, security_level).encode()
        raw = shake256(seed, bytes_per_int * num)
        # sum_j (256^j mod p) * b_j mod p == (little-endian integer of the chunk) mod p
        return [int.from_bytes(raw[bytes_per_int * i: bytes_per_int * (i + 1)], "little") % P for i in range(num)]

    def _round(self, state: List[int], r: int) -> List[int]:
        """rescue_prime.rs:52-106 (one round: S-box, MDS, constants, inverse S-box, MDS, constants)."""
        m, rc = self.m, self.round_constants
        s = [fpow(x, self.alpha) for x in state]
        s = [add_mod(sum_mod(mul_mod(self.MDS[j][i], s[i]) for i in range(m)), rc[2 * r * m + j]) for j in range(m)]
        s = [fpow(x, self.alpha_inv) for x in s]
        s = [add_mod(sum_mod(mul_mod(self.MDS[j][i], s[i]) for i in range(m)), rc[2 * r * m + m + j])
             for j in range(m)]
        return s

    def hash(self, x: int) -> int:
        """rescue_prime.rs:183-190."""
        state = [x] + [0] * (self.m - self.capacity)
        for r in range(self.N):
            state = self._round(state, r)
        return state[0]

    def trace(self, x: int) -> List[List[int]]:
        """rescue_prime.rs:192-204: N + 1 states."""
        state = [x] + [0] * (self.m - self.capacity)
        out = [list(state)]
        for r in range(self.N):
            state = self._round(state, r)
            out.append(list(state))
        return out

    def round_constants_polynomials(self, omicron: int, omicron_domain_length: int):
        """rescue_prime.rs:206-244."""
        domain = [fpow(omicron, r) for r in range(self.N)]
        m, rc = self.m, self.round_constants
        first = [MPolynomial.lift(fast_interpolate_domain(omicron, omicron_domain_length, domain,
                                                          [rc[2 * r * m + i] for r in range(self.N)]), 0)
                 for i in range(m)]
        second = [MPolynomial.lift(fast_interpolate_domain(omicron, omicron_domain_length, domain,
                                                           [rc[2 * r * m + m + i] for r in range(self.N)]), 0)
                  for i in range(m)]
        return first, second

    def transition_constraints(self, omicron: int, omicron_domain_length: int) -> List[MPolynomial]:
        """rescue_prime.rs:246-283."""
        first, second = self.round_constants_polynomials(omicron, omicron_domain_length)
        m = self.m
        var = MPolynomial.variables(1 + 2 * m)
        prev, nxt = var[1:1 + m], var[1 + m:1 + 2 * m]
        out = []
        for i in range(m):
            lhs = None
            for k in range(m):
                t = MPolynomial.constant(self.MDS[i][k]) * (prev[k] ** self.alpha)
                lhs = t if lhs is None else lhs + t
            lhs = lhs + first[i]
            rhs = None
            for k in range(m):
                t = MPolynomial.constant(self.MDS_inv[i][k]) * (nxt[k] - second[k])
                rhs = t if rhs is None else rhs + t
            rhs = rhs ** self.alpha
            out.append(lhs - rhs)
        return out

    def boundary_constraints(self, output_element: int) -> List[Tuple[int, int, int]]:
        """rescue_prime.rs:285-290."""
        return [(0, 1, 0), (self.N, 0, output_element)]


def sum_mod(it) -> int:
    acc = 0
    for v in it:
        acc = add_mod(acc, v)
    return acc


# ------------------------------------------------------------------------ STARK (stark.rs)

def bitlen_count(x: int) -> int:
    """utils/bit_iter.rs: BitIter::from(x).count() (1 for x == 0)."""
    return max(x.bit_length(), 1)


def randomness_from_seed(seed: bytes, count: int) -> List[int]:
    """Deterministic stand-in for thread_rng: field.sample of 17-byte chunks of SHAKE256(seed)
    (stark.rs:290-294 samples 17 random bytes per element the same way)."""
    raw = shake256(b"sg-stark-randomness" + seed, 17 * count)
    return [sample(raw[17 * i:17 * i + 17]) for i in range(count)]


class Stark:
    """stark/stark.rs:17-562 (prover) and :564-807 (verifier)."""

    def __init__(self, expansion_factor: int, num_colinearity_checks: int, security_level: int,
                 num_registers: int, num_cycles: int, transition_constraints_degree: int = 2):
        """stark.rs:71-114."""
        assert P.bit_length() >= security_level
        assert expansion_factor & (expansion_factor - 1) == 0, "expansion_factor must be a power of 2"
        assert expansion_factor >= 4, "expansion_factor must be at least 4"
        assert num_colinearity_checks * 2 >= security_level
        self.expansion_factor = expansion_factor
        self.num_registers = num_registers
        self.original_trace_length = num_cycles
        self.num_randomizers = 4 * num_colinearity_checks
        randomized = num_cycles + self.num_randomizers
        self.omicron_domain_length = 1 << bitlen_count(randomized * transition_constraints_degree)
        fri_len = self.omicron_domain_length * expansion_factor
        self.generator = GENERATOR
        self.omega = primitive_nth_root(fri_len)
        self.omicron = primitive_nth_root(self.omicron_domain_length)
        self.fri = FRI(GENERATOR, self.omega, fri_len, expansion_factor, num_colinearity_checks)

    # -- degree bookkeeping (stark.rs:117-196) --
    def transition_degree_bounds(self, tcs: Sequence[MPolynomial]) -> List[int]:
        pd = [1] + [self.original_trace_length + self.num_randomizers - 1] * (2 * self.num_registers)
        out = []
        for a in tcs:
            if len(a.d) == 0:
                raise ValueError("cannot calculate max on empty vec a")
            mx = 0
            for k in a.d:
                s = sum(r * l for r, l in zip(pd, k))
                mx = max(mx, s)
            out.append(mx)
        return out

    def transition_quotient_degree_bounds(self, tcs) -> List[int]:
        return [d - (self.original_trace_length - 1) for d in self.transition_degree_bounds(tcs)]

    def max_degree(self, tcs) -> int:
        md = max(self.transition_degree_bounds(tcs))
        return (1 << bitlen_count(md)) - 1

    def omicron_pow(self, i: int) -> int:
        return fpow(self.omicron, i)

    def transition_zerofier(self) -> Poly:
        """stark.rs:198-206."""
        dom = [self.omicron_pow(i) for i in range(self.original_trace_length - 1)]
        return fast_zerofier(self.omicron, self.omicron_domain_length, dom)

    def transition_zerofier_at(self, xs: Sequence[int]) -> List[int]:
        """transition_zerofier() (stark.rs:198-206) evaluated at each x: prod_{i < T-1} (x - omicron^i)."""
        tdom = [self.omicron_pow(i) for i in range(self.original_trace_length - 1)]
        out = []
        for x in xs:
            zx = 1
            for d in tdom:
                zx = zx * (x - d) % P
            out.append(zx)
        return out

    def boundary_zerofiers(self, boundary) -> List[Poly]:
        """stark.rs:208-226."""
        return [fast_zerofier(self.omicron, self.omicron_domain_length,
                              [self.omicron_pow(c) for (c, r, _) in boundary if r == s])
                for s in range(self.num_registers)]

    def boundary_interpolants(self, boundary) -> List[Poly]:
        """stark.rs:228-252."""
        out = []
        for s in range(self.num_registers):
            dom = [self.omicron_pow(c) for (c, r, _) in boundary if r == s]
            vals = [v for (c, r, v) in boundary if r == s]
            out.append(fast_interpolate_domain(self.omicron, self.omicron_domain_length, dom, vals))
        return out

    def boundary_quotient_degree_bounds(self, randomized_trace_length: int, boundary) -> List[int]:
        """stark.rs:254-266."""
        return [randomized_trace_length - 1 - degree(bz) for bz in self.boundary_zerofiers(boundary)]

    @staticmethod
    def sample_weights(number: int, randomness: bytes) -> List[int]:
        """stark.rs:268-274: sample(0^i || randomness) (only the last 16 bytes survive the fold)."""
        return [sample(bytes(i) + randomness) for i in range(number)]

    def num_randomizer_coefficients(self, tcs) -> int:
        """stark.rs:424-433: max_degree(tcs) + 1 random coefficients."""
        return self.max_degree(tcs) + 1

    # -- prover (stark.rs:276-562) --
    def prove(self, trace: Sequence[Sequence[int]], tcs: Sequence[MPolynomial], boundary,
              proof_stream: IndependentProofStream, trace_randomizers: Sequence[Sequence[int]],
              randomizer_coefficients: Sequence[int]) -> bytes:
        """Returns proof_stream.digest(); raises ValueError where the reference returns Err."""
        m = self.num_registers
        assert len(trace_randomizers) == self.num_randomizers
        trace = [list(r) for r in trace] + [list(r) for r in trace_randomizers]
        T = len(trace)
        tdom = [self.omicron_pow(i) for i in range(T)]
        trace_polys = [fast_interpolate_domain(self.omicron, self.omicron_domain_length, tdom,
                                               [row[s] for row in trace]) for s in range(m)]
        bi = self.boundary_interpolants(boundary)
        bz = self.boundary_zerofiers(boundary)
        bqs = [fast_coset_divide(self.omicron, self.omicron_domain_length, self.generator,
                                 p_sub(trace_polys[s], bi[s]), bz[s]) for s in range(m)]
        N = self.fri.domain_length
        bq_codewords = []
        for s in range(m):
            cw = fast_coset_evaluate_ref(self.omega, N, self.generator, bqs[s])
            proof_stream.push((ROOT, merkle_commit(cw)))
            bq_codewords.append(cw)
        point = [[0, 1]] + [list(tp) for tp in trace_polys] + [p_scale(tp, self.omicron) for tp in trace_polys]
        tz = self.transition_zerofier()
        tqs = []
        for tc in tcs:
            tpoly = tc.evaluate_symbolic(point)
            tqs.append(fast_coset_divide(self.omicron, self.omicron_domain_length, self.generator, tpoly, tz))
        tcd = self.max_degree(tcs)
        assert len(randomizer_coefficients) == tcd + 1
        rpoly = list(randomizer_coefficients)
        r_cw = fast_coset_evaluate_ref(self.omega, N, self.generator, rpoly)
        proof_stream.push((ROOT, merkle_commit(r_cw)))
        weights = self.sample_weights(1 + 2 * len(tqs) + 2 * len(bqs), proof_stream.fiat_shamir_prover(PROOF_BYTES))
        if [degree(tq) for tq in tqs] != self.transition_quotient_degree_bounds(tcs):
            raise ValueError("transition quotient degrees do not match with expectation")
        terms = [rpoly]
        tqdb = self.transition_quotient_degree_bounds(tcs)
        for i, tq in enumerate(tqs):
            terms.append(tq)
            shift = tcd - tqdb[i]
            terms.append(fast_multiply(self.omicron, self.omicron_domain_length, p_pow([0, 1], shift), tq))
        bqdb = self.boundary_quotient_degree_bounds(T, boundary)
        for i, bq in enumerate(bqs):
            terms.append(bq)
            shift = tcd - bqdb[i]
            terms.append(fast_multiply(self.omicron, self.omicron_domain_length, p_pow([0, 1], shift), bq))
        comb = None
        for w, t in zip(weights, terms):
            wt = p_mul([w], t)
            comb = wt if comb is None else p_add(comb, wt)
        comb_cw = fast_coset_evaluate_ref(self.omega, N, self.generator, comb)
        indices = self.fri.prove(comb_cw, proof_stream)
        dup = list(indices) + [(i + self.expansion_factor) % N for i in indices]
        quad = sorted(dup + [(i + N // 2) % N for i in dup])
        for cw in bq_codewords:
            lv = merkle_levels(cw)
            for i in quad:
                proof_stream.push((VALUE, cw[i]))
                proof_stream.push((PATH, merkle_open_levels(i, lv)))
        lv = merkle_levels(r_cw)
        for i in quad:
            proof_stream.push((VALUE, r_cw[i]))
            proof_stream.push((PATH, merkle_open_levels(i, lv)))
        return proof_stream.digest()

    # -- verifier (stark.rs:564-807) --
    def verify(self, tcs: Sequence[MPolynomial], boundary, proof_stream: IndependentProofStream) -> Tuple[bool, str]:
        otl = 1 + max(c for (c, _, _) in boundary)
        rtl = otl + self.num_randomizers
        bq_roots = [proof_stream.pull()[1] for _ in range(self.num_registers)]
        r_root = proof_stream.pull()[1]
        bi = self.boundary_interpolants(boundary)
        weights = self.sample_weights(1 + 2 * len(tcs) + 2 * len(bi), proof_stream.fiat_shamir_verifier(PROOF_BYTES))
        ok, err, points = self.fri.verify(proof_stream)
        if not ok:
            return False, "FRI verification failed: " + err
        points.sort(key=lambda p: p[0])
        indices = [p[0] for p in points]
        values = [p[1] for p in points]
        N = self.fri.domain_length
        dup = sorted(indices + [(i + self.expansion_factor) % N for i in indices])
        leafs = []
        for root in bq_roots:
            d = {}
            for i in dup:
                code, leaf = proof_stream.pull()
                assert code == VALUE
                code, path = proof_stream.pull()
                if not merkle_verify(root, i, path, leaf):
                    return False, "Boundary quotient root {} is not verified".format(i)
                d[i] = leaf
            leafs.append(d)
        rnd = {}
        for i in dup:
            code, leaf = proof_stream.pull()
            code, path = proof_stream.pull()
            if not merkle_verify(r_root, i, path, leaf):
                return False, "Randomizer leaf {} not verified".format(i)
            rnd[i] = leaf
        bz = self.boundary_zerofiers(boundary)
        tcd = self.max_degree(tcs)
        tqdb = self.transition_quotient_degree_bounds(tcs)
        bqdb = self.boundary_quotient_degree_bounds(rtl, boundary)
        # transition_zerofier().evaluate(x) == prod_{i < T-1} (x - omicron^i), evaluated directly
        zxs = self.transition_zerofier_at([mul_mod(self.fri.offset, fpow(self.fri.omega, ic)) for ic in indices])
        for ii, ic in enumerate(indices):
            x = mul_mod(self.fri.offset, fpow(self.fri.omega, ic))
            inx = (ic + self.expansion_factor) % N
            xn = mul_mod(self.fri.offset, fpow(self.fri.omega, inx))
            cur = [add_mod(mul_mod(leafs[s][ic], p_evaluate(bz[s], x)), p_evaluate(bi[s], x))
                   for s in range(self.num_registers)]
            nxt = [add_mod(mul_mod(leafs[s][inx], p_evaluate(bz[s], xn)), p_evaluate(bi[s], xn))
                   for s in range(self.num_registers)]
            point = [x] + cur + nxt
            tvals = [tc.evaluate(point) for tc in tcs]
            terms = [rnd[ic]]
            zx = zxs[ii]
            for s, tv in enumerate(tvals):
                q = div(tv, zx)
                terms.append(q)
                terms.append(mul_mod(q, fpow(x, tcd - tqdb[s])))
            for s in range(self.num_registers):
                b = leafs[s][ic]
                terms.append(b)
                terms.append(mul_mod(b, fpow(x, tcd - bqdb[s])))
            comb = sum_mod(mul_mod(t, w) for t, w in zip(terms, weights))
            if comb != values[ii]:
                return False, "Combination doesn't match with polynomial value"
        return True, ""


def fast_coset_evaluate_ref(generator: int, root_order: int, offset: int, coeffs: Sequence[int]) -> List[int]:
    """ntt_arithmetics.rs:161-170 (usize underflow -> panic when the polynomial is longer)."""
    if len(coeffs) > root_order:
        raise ValueError("polynomial longer than root_order")
    c = p_scale(coeffs, offset) + [0] * (root_order - len(coeffs))
    return ntt(generator, c)


# ------------------------------------------- Rescue AIR evaluated from its structure

class RescueAirAtPoint:
    """The value of RescuePrime.transition_constraints()[i] at a point, from the AIR's structure
    (rescue_prime.rs:246-283): sum_k MDS[i][k] prev_k^alpha + C1_i(x) - (sum_k MDS^-1[i][k]
    (next_k - C2_k(x)))^alpha, with the round-constant interpolants C1/C2 (degree < N over
    omicron^r, r < N) evaluated by the barycentric formula in O(N) per point.  Used to verify
    proofs at sizes where the expanded MPolynomial (O(N^2) to build) is out of reach; `d`
    holds keys whose maximum equals the full key set's in stark.rs:117-160 (which only takes a
    max): x^(3(N-1)), prev/next cubes and the mixed cubic terms."""

    def __init__(self, rp: RescuePrime, i: int, bary: "GeometricBarycentric"):
        self.rp, self.i, self.bary = rp, i, bary
        m, N = rp.m, rp.N
        nv = 1 + 2 * m
        keys = {(3 * (N - 1),) + (0,) * (2 * m), (N - 1,) + (0,) * (2 * m)}
        for k in range(m):
            e = [0] * nv
            e[1 + k] = 3
            keys.add(tuple(e))
            for a in range(4):
                e = [0] * nv
                e[1 + m + k] = a
                e[0] = (3 - a) * (N - 1)
                keys.add(tuple(e))
        self.d = {k: 0 for k in keys}

    @staticmethod
    def for_rescue(rp: RescuePrime, omicron: int) -> List["RescueAirAtPoint"]:
        m = rp.m
        cols = {}
        for i in range(m):
            cols[("c1", i)] = [rp.round_constants[2 * r * m + i] for r in range(rp.N)]
            cols[("c2", i)] = [rp.round_constants[2 * r * m + m + i] for r in range(rp.N)]
        bary = GeometricBarycentric(omicron, rp.N, cols)
        return [RescueAirAtPoint(rp, i, bary) for i in range(m)]

    def evaluate(self, point):
        rp, i, m = self.rp, self.i, self.rp.m
        x = point[0]
        prev, nxt = point[1:1 + m], point[1 + m:1 + 2 * m]
        lhs = self.bary.value(x, ("c1", i))
        for k in range(m):
            lhs = (lhs + rp.MDS[i][k] * fpow(prev[k], rp.alpha)) % P
        acc = 0
        for k in range(m):
            acc = (acc + rp.MDS_inv[i][k] * (nxt[k] - self.bary.value(x, ("c2", k)))) % P
        return (lhs - fpow(acc, rp.alpha)) % P


class GeometricBarycentric:
    """Barycentric evaluation of the interpolants through (q^r, v_r), r < n, q of order >= n,
    for a set of value columns: P(x) = Z(x) sum_r v_r w_r / (x - q^r),
    1/w_r = q^(r(r-1)/2 + r(n-1-r)) A_r B_(n-1-r), A_k = prod_{i<=k} (q^i - 1),
    B_k = prod_{i<=k} (1 - q^i).  Same values as the unique interpolant
    fast_interpolate_domain returns (ntt_arithmetics.rs:172-237)."""

    def __init__(self, q: int, n: int, columns):
        self.q, self.n = q, n
        self.dom = [1] * n
        for r in range(1, n):
            self.dom[r] = self.dom[r - 1] * q % P
        A, B = [1] * n, [1] * n
        for k in range(1, n):
            qk = self.dom[k]
            A[k] = A[k - 1] * (qk - 1) % P
            B[k] = B[k - 1] * (1 - qk) % P
        # q^(e_r), e_r = r(r-1)/2 + r(n-1-r); e_{r+1} - e_r = n - 2 - r
        qinv = inv(q)
        step = fpow(q, n - 2) if n >= 2 else 1
        pe, winv = 1, []
        for r in range(n):
            winv.append(pe * A[r] % P * B[n - 1 - r] % P)
            pe = pe * step % P
            step = step * qinv % P
        w = _batch_inv(winv)
        self.cols = {k: [v * wr % P for v, wr in zip(vals, w)] for k, vals in columns.items()}
        self.cache = {}

    def value(self, x: int, key) -> int:
        if x not in self.cache:
            diffs = [(x - d) % P for d in self.dom]
            z = 1
            for dd in diffs:
                z = z * dd % P
            iv = _batch_inv(diffs)
            self.cache[x] = {k: z * (sum(a * b for a, b in zip(col, iv)) % P) % P for k, col in self.cols.items()}
        return self.cache[x][key]


def _batch_inv(xs):
    pre, acc = [], 1
    for x in xs:
        pre.append(acc)
        acc = acc * x % P
    inv_acc = inv(acc)
    out = [0] * len(xs)
    for i in range(len(xs) - 1, -1, -1):
        out[i] = inv_acc * pre[i] % P
        inv_acc = inv_acc * xs[i] % P
    return out
