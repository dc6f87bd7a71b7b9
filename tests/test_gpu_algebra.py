"""GPU parity of the polynomial algebra (fft/ntt_arithmetics.rs):
libstarkgpu vs the CPU oracle (oracle/stark_prove_oracle.py), exact equality of the
coefficient vectors (same length, same values), plus size-independent properties at
sizes the oracle cannot reach."""
import random

import numpy as np
import pytest

import stark_oracle as o
import stark_prove_oracle as e
import starkgpu as sg

pytestmark = pytest.mark.gpu
P = o.P


def rpoly(rng, n, zeros_tail=0):
    return [rng.randrange(P) for _ in range(n)] + [0] * zeros_tail


def test_fast_multiply_vs_oracle():
    rng = random.Random(1)
    n = 1 << 6
    w = o.primitive_nth_root(n)
    cases = [(rpoly(rng, a), rpoly(rng, b)) for a, b in ((1, 1), (1, 5), (3, 7), (17, 15), (31, 32), (20, 12))]
    cases += [(rpoly(rng, 9, 3), rpoly(rng, 4, 2)), ([0, 0], rpoly(rng, 3)), ([], rpoly(rng, 3)),
              ([5], [7]), (rpoly(rng, 30), [0, 0, 0, 1])]
    for a, b in cases:
        got = sg.fast_multiply(w, n, a, b).coefficients
        assert got == e.fast_multiply(w, n, a, b), (len(a), len(b))
    # the reference test: fast_multiply == schoolbook (ntt_arithmetics.rs:354-371)
    for _ in range(10):
        a, b = rpoly(rng, rng.randrange(1, 32)), rpoly(rng, rng.randrange(1, 32))
        assert sg.fast_multiply(w, n, a, b).coefficients == e.p_mul(a, b)


def test_fast_multiply_large():
    rng = random.Random(2)
    n = 1 << 14
    w = o.primitive_nth_root(n)
    a, b = rpoly(rng, 3000), rpoly(rng, 5000)
    got = sg.fast_multiply(w, n, a, b).coefficients
    assert len(got) == 7999
    for x in (3, 12345, P - 7):
        assert e.p_evaluate(got, x) == o.mul_mod(e.p_evaluate(a, x), e.p_evaluate(b, x))


def test_fast_coset_divide_vs_oracle():
    rng = random.Random(3)
    n = 1 << 6
    w = o.primitive_nth_root(n)
    for la, lb in ((5, 3), (20, 11), (32, 1), (16, 16), (2, 2)):
        lhs, rhs = rpoly(rng, la), rpoly(rng, lb)
        prod = e.p_mul(lhs, rhs)
        # exact division (ntt_arithmetics.rs:525-560)
        assert sg.fast_coset_divide(w, n, 5, prod, rhs).coefficients == e.fast_coset_divide(w, n, 5, prod, rhs)
        # inexact: the reference's algorithm output, not a quotient
        noisy = list(prod)
        noisy[0] = (noisy[0] + 1) % P
        assert sg.fast_coset_divide(w, n, o.GENERATOR, noisy, rhs).coefficients == \
            e.fast_coset_divide(w, n, o.GENERATOR, noisy, rhs)
    assert sg.fast_coset_divide(w, n, 5, [0, 0], [1, 2]).coefficients == []
    with pytest.raises(sg.StarkGpuError):
        sg.fast_coset_divide(w, n, 5, [1, 2, 3], [0])
    with pytest.raises(sg.StarkGpuError):
        sg.fast_coset_divide(w, n, 5, [1, 2], [1, 2, 3])
    # a divisor vanishing on the coset: the reference panics "divide by zero"
    with pytest.raises(sg.StarkGpuError, match="divide by zero"):
        sg.fast_coset_divide(w, n, 1, [1, 2, 3, 4], [P - 1, 1])


@pytest.mark.parametrize("D,ns", [(1 << 6, [1, 2, 3, 17, 40, 63, 64]), (1 << 12, [1000, 4095, 4096])])
def test_zerofier_geometric_vs_oracle(D, ns):
    q = o.primitive_nth_root(D)
    for n in ns:
        dom = [o.fpow(q, i) for i in range(n)]
        got = sg.fast_zerofier(q, D, dom).coefficients
        if n <= 64:
            assert got == e.fast_zerofier(q, D, dom), n
        elif n == D:
            assert got == [0] * D  # the reference's wrapped last product
        else:
            assert len(got) == n + 1 and got[n] == 1
            for x in (dom[0], dom[n // 2], dom[-1]):
                assert e.p_evaluate(got, x) == 0
            z = 7
            ref = 1
            for d in dom:
                ref = o.mul_mod(ref, o.sub_mod(z, d))
            assert e.p_evaluate(got, z) == ref


def test_zerofier_and_interpolate_generic_domains():
    rng = random.Random(4)
    n = 1 << 6
    w = o.primitive_nth_root(n)
    for k in (0, 1, 2, 5, 30):
        dom = [rng.randrange(P) for _ in range(k)]
        vals = [rng.randrange(P) for _ in range(k)]
        assert sg.fast_zerofier(w, n, dom).coefficients == e.fast_zerofier(w, n, dom)
        assert sg.fast_interpolate_domain(w, n, dom, vals).coefficients == e.fast_interpolate_domain(w, n, dom, vals)


@pytest.mark.parametrize("D,ns", [(1 << 6, [1, 2, 3, 28, 36, 63, 64]), (1 << 8, [200, 255]),
                                  (1 << 8, [5, 33, 64, 65, 127, 128]), (1 << 10, [7, 60, 64, 65, 256])])
def test_interpolate_geometric_vs_oracle(D, ns):
    rng = random.Random(5)
    q = o.primitive_nth_root(D)
    for n in ns:
        dom = [o.fpow(q, i) for i in range(n)]
        vals = [rng.randrange(P) for _ in range(n)]
        got = sg.fast_interpolate_domain(q, D, dom, vals).coefficients
        assert got == e.fast_interpolate_domain(q, D, dom, vals), n


@pytest.mark.parametrize("logD,n", [(16, 65535 - 1000), (18, 65535), (20, 700001)])
def test_interpolate_geometric_large(logD, n):
    """At sizes the oracle cannot reach: the interpolant reproduces every value on the
    domain (LDE over the D-subgroup), has length n, and matches Horner at random points
    through the barycentric form on a small sample."""
    import torch
    D = 1 << logD
    q = o.primitive_nth_root(D)
    vals = o.synthetic_elements(9, b"interp", n)
    dev = torch.device("cuda", 0)
    y = torch.from_numpy(sg.fe_array(vals).view(np.int64)).to(dev)
    p = sg.fast_interpolate_geometric_dev(q, D, y.data_ptr(), n)
    assert len(p) == n
    cw = sg.fast_coset_evaluate(q, D, 1, p.array())
    assert sg.to_ints(cw[:n]) == vals


@pytest.mark.parametrize("logD", [14, 17])
def test_interpolate_geometric_decimated_vs_checker(logD, monkeypatch):
    """n <= D / f: the interpolant comes from its values on the subgroup of order D / f (f residue-class
    convolutions sharing one inverse transform) -- equal to the CPU checker (fast_cpu, pinned to the
    oracle) and to the full-group form (context option geo_decimate = 0), for f = 16, 4, 2 and none."""
    import torch
    import fast_cpu as fc
    D = 1 << logD
    q = o.primitive_nth_root(D)
    dev = torch.device("cuda", 0)
    for n in (D // 16 - 5, D // 4 - 1, D // 4, D // 4 + 1, D // 2, D - 3):
        vals = o.synthetic_elements(n, b"decimated", n)
        y = torch.from_numpy(sg.fe_array(vals).view(np.int64)).to(dev)
        want = fc.ints(fc.geo_interpolate(q, D, vals))
        got = sg.fast_interpolate_geometric_dev(q, D, y.data_ptr(), n)
        assert got.coefficients == want, n
        with sg.Context.default().option("geo_decimate", 0, 1):
            assert sg.fast_interpolate_geometric_dev(q, D, y.data_ptr(), n).coefficients == want, n


# ---- arbitrary (non-geometric) domains of any size (ntt_arithmetics.rs:66-113, 172-237) ----

def _fc():
    import fast_cpu as fc
    return fc


def test_zerofier_interpolate_arbitrary_2p10_vs_oracle():
    """2^10 random points: the coefficient vectors equal the oracle's recursion exactly."""
    rng = random.Random(10)
    n, D = 1 << 10, 1 << 12
    w = o.primitive_nth_root(D)
    dom = [rng.randrange(P) for _ in range(n)]
    vals = [rng.randrange(P) for _ in range(n)]
    assert sg.fast_zerofier(w, D, dom).coefficients == e.fast_zerofier(w, D, dom)
    assert sg.fast_interpolate_domain(w, D, dom, vals).coefficients == e.fast_interpolate_domain(w, D, dom, vals)


@pytest.mark.parametrize("logn", [11, 12, 13, 14])
def test_zerofier_arbitrary_large(logn):
    """Z = prod (x - d_i) of 2^logn random points + a ragged count: equal to the exact product
    (oracle/fast_cpu.cpp, O(n^2)), which is the reference's result below root_order."""
    fc = _fc()
    rng = random.Random(logn)
    for n in ((1 << logn), (1 << logn) - 3):
        D = 1 << (logn + 1)
        w = o.primitive_nth_root(D)
        dom = [rng.randrange(P) for _ in range(n)]
        got = sg.fast_zerofier(w, D, dom).coefficients
        assert len(got) == n + 1
        assert got == fc.ints(fc.poly_from_roots(dom))


@pytest.mark.parametrize("logn", [11, 12, 13, 14])
def test_interpolate_arbitrary_large(logn):
    """The interpolant through 2^logn (and a ragged count of) random points: length n, and it takes
    every value at its point -- the unique polynomial of degree < n, i.e. the reference's result."""
    fc = _fc()
    rng = random.Random(100 + logn)
    for n in ((1 << logn), (1 << logn) - 5):
        D = 1 << (logn + 1)
        w = o.primitive_nth_root(D)
        dom = [rng.randrange(P) for _ in range(n)]
        vals = [rng.randrange(P) for _ in range(n)]
        got = sg.fast_interpolate_domain(w, D, dom, vals).coefficients
        assert len(got) == n
        assert fc.ints(fc.eval_points(got, dom)) == vals


def test_zerofier_arbitrary_wraps_like_the_reference():
    """Domains at and above root_order: the reference's fast_multiply wraps its cyclic
    convolution; the recursion above the exact subtrees reproduces that output."""
    rng = random.Random(21)
    for D, n in ((16, 16), (16, 40), (64, 64), (64, 200)):
        w = o.primitive_nth_root(D)
        dom = [rng.randrange(P) for _ in range(n)]
        assert sg.fast_zerofier(w, D, dom).coefficients == e.fast_zerofier(w, D, dom), (D, n)


def test_interpolate_arbitrary_edge_cases():
    rng = random.Random(22)
    D = 1 << 8
    w = o.primitive_nth_root(D)
    # 0..9 points (below one leaf lane), and the largest domain whose half-zerofiers stay below
    # root_order (ceil(n/2) < D: n = 2D - 2)
    for n in list(range(10)) + [2 * D - 2]:
        dom = [rng.randrange(P) for _ in range(n)]
        vals = [rng.randrange(P) for _ in range(n)]
        assert sg.fast_interpolate_domain(w, D, dom, vals).coefficients == e.fast_interpolate_domain(w, D, dom, vals)
    # one more point and the reference's half-zerofier wraps: rejected, not silently different
    dom = [rng.randrange(P) for _ in range(2 * D - 1)]
    with pytest.raises(sg.StarkGpuError, match="wrap"):
        sg.fast_interpolate_domain(w, D, dom, dom)
    # a repeated point: the reference divides by zero (field_element.rs:82-90)
    dom = [rng.randrange(P) for _ in range(20)]
    dom[7] = dom[3]
    with pytest.raises(sg.StarkGpuError, match="divide by zero"):
        sg.fast_interpolate_domain(w, D, dom, [1] * 20)
    # zero values and a zero point
    dom = [0] + [rng.randrange(P) for _ in range(30)]
    vals = [0] * 31
    assert sg.fast_interpolate_domain(w, D, dom, vals).coefficients == [0] * 31


def test_degree_top_down_scan():
    """Polynomial::degree (polynomial.rs:41-58) on the device: the top-down chunked scan with
    early exit (k_last_nonzero) at every position class -- leading coefficient in the top
    chunk, at chunk edges, deep below the top, in the bottom chunk, and the zero polynomial
    (None) -- on buffers of 1 .. 2^20 + 7 elements."""
    chunk = 256 * 16
    for n in (1, 2, 17, chunk - 1, chunk, chunk + 1, 3 * chunk + 5, (1 << 20) + 7):
        cases = {None, 0, n - 1, n // 2, min(n - 1, chunk), max(0, n - chunk - 1), max(0, n - chunk)}
        for lead in sorted(cases, key=lambda x: -1 if x is None else x):
            a = np.zeros((n, 2), dtype=np.uint64)
            if lead is not None:
                a[lead, 0] = 1 + lead
                if lead > 0:
                    a[lead - 1, 1] = 9   # a nonzero below the leading one
                if lead >= 3:
                    a[lead // 3, 0] = 5
            p = sg.Polynomial.new(a)
            assert p.degree() == lead, (n, lead)
