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


@pytest.mark.parametrize("D,ns", [(1 << 6, [1, 2, 3, 28, 36, 63, 64]), (1 << 8, [200, 255])])
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
