"""GPU parity of MPolynomial, Rescue-Prime and the end-to-end Stark::prove (SURVEY.md 8(f)
f3/f4, BASELINE config C4): libstarkgpu vs the CPU oracle (oracle/stark_prove_oracle.py),
exact equality of group coefficient vectors and of the complete proof bytes."""
import json
import os
import random

import pytest

import stark_oracle as o
import stark_prove_oracle as e
import starkgpu as sg

pytestmark = pytest.mark.gpu
P = o.P
HERE = os.path.dirname(os.path.abspath(__file__))


def grouped(d):
    """oracle dict {(x, r1, ..): c} -> (nvars, {(r1, ..): dense x-coefficients})."""
    if not d:
        return 0, {}
    nv = len(next(iter(d)))
    out = {}
    for k, c in d.items():
        v = out.setdefault(tuple(k[1:]), [])
        if len(v) <= k[0]:
            v.extend([0] * (k[0] + 1 - len(v)))
        v[k[0]] = (v[k[0]] + c) % P
    return nv, out


def same(mp, od):
    assert mp.groups() == grouped(od.d)


def test_rescue_matches_reference_kats():
    with open(os.path.join(HERE, "golden", "reference_kats_e2e.json")) as f:
        k = json.load(f)
    r = k["rescue_new"]
    rp = sg.RescuePrime(2, 1, 128, 27)
    assert rp.alpha == r["alpha"] and rp.alpha_inv == int(r["alpha_inv"]), r["src"]
    assert rp.MDS == [[int(x) for x in row] for row in r["mds"]], r["src"]
    assert rp.MDS_inv == [[int(x) for x in row] for row in r["mds_inv"]], r["src"]
    assert rp.round_constants == [int(x) for x in r["round_constants"]], r["src"]
    h = k["rescue_hash"]
    assert rp.hash(int(h["input"])) == int(h["output"]), h["src"]
    t = k["rescue_trace"]
    tr = rp.trace(int(t["input"]))
    assert tr[0][0] == int(t["first_rate"]) and tr[-1][0] == int(t["last_rate"]), t["src"]
    orp = e.RescuePrime(2, 1, 128, 27)
    assert tr == orp.trace(int(t["input"]))
    # other shapes vs the oracle
    for (m, cap, sec, N) in ((3, 1, 2, 9), (2, 1, 2, 100)):
        a, b = sg.RescuePrime(m, cap, sec, N), e.RescuePrime(m, cap, sec, N)
        assert a.MDS == b.MDS and a.MDS_inv == b.MDS_inv and a.round_constants == b.round_constants
        assert a.trace(12345) == b.trace(12345)


def test_mpolynomial_ops_vs_oracle():
    with open(os.path.join(HERE, "golden", "reference_kats_e2e.json")) as f:
        k = json.load(f)
    for name, op in (("mpoly_mul", lambda a, b: a * b), ("mpoly_add", lambda a, b: a + b),
                     ("mpoly_sub", lambda a, b: a - b)):
        v = k[name]
        # the library needs keys of one length per polynomial; pad like the reference's Add/Mul
        na = max(len(x[0]) for x in v["a"])
        nb = max(len(x[0]) for x in v["b"])
        da = {tuple(x[0]) + (0,) * (na - len(x[0])): int(x[1]) for x in v["a"]}
        db = {tuple(x[0]) + (0,) * (nb - len(x[0])): int(x[1]) for x in v["b"]}
        got = op(sg.MPolynomial.new(da), sg.MPolynomial.new(db))
        want = op(e.MPolynomial(da), e.MPolynomial(db))
        same(got, want)
        assert grouped(want.d) == grouped({tuple(x[0]): int(x[1]) for x in v["out"]}), v["src"]
    rng = random.Random(3)
    for _ in range(5):
        nv = rng.randrange(1, 4)
        da = {tuple(rng.randrange(4) for _ in range(nv)): rng.choice([0, rng.randrange(P)]) for _ in range(6)}
        db = {tuple(rng.randrange(3) for _ in range(nv)): rng.randrange(P) for _ in range(4)}
        A, B = sg.MPolynomial.new(da), sg.MPolynomial.new(db)
        oa, ob = e.MPolynomial(da), e.MPolynomial(db)
        same(A * B, oa * ob)
        same(A + B, oa + ob)
        same(A - B, oa - ob)
        same(A ** 3, oa ** 3)
        same(A ** 0, oa ** 0)
        pt = [rng.randrange(P) for _ in range(nv)]
        assert A.evaluate(pt) == oa.evaluate(pt)
    same(sg.MPolynomial.lift([3, 0, 5, 0], 0), e.MPolynomial.lift([3, 0, 5, 0], 0))
    same(sg.MPolynomial.lift([3, 0, 5], 2), e.MPolynomial.lift([3, 0, 5], 2))
    for a, b in zip(sg.MPolynomial.variables(3), e.MPolynomial.variables(3)):
        same(a, b)


def test_rescue_transition_constraints_vs_oracle():
    st = e.Stark(4, 2, 2, 2, 28, 2)
    air_o = e.RescuePrime(2, 1, 2, 27).transition_constraints(st.omicron, st.omicron_domain_length)
    air_g = sg.RescuePrime(2, 1, 2, 27).transition_constraints(st.omicron, st.omicron_domain_length)
    for a, b in zip(air_g, air_o):
        same(a, b)


def _case(N, exp, c, sec, tcd, seed, m=2):
    rp_o, rp_g = e.RescuePrime(m, 1, sec, N), sg.RescuePrime(m, 1, sec, N)
    st_o = e.Stark(exp, c, sec, m, N + 1, tcd)
    st_g = sg.Stark(exp, c, sec, m, N + 1, tcd)
    assert st_g.omicron == st_o.omicron and st_g.omicron_domain_length == st_o.omicron_domain_length
    air_o = rp_o.transition_constraints(st_o.omicron, st_o.omicron_domain_length)
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    assert st_g.transition_degree_bounds(air_g) == st_o.transition_degree_bounds(air_o)
    assert st_g.max_degree(air_g) == st_o.max_degree(air_o)
    inp = o.sample(seed)
    out = rp_o.hash(inp)
    nrc = st_o.num_randomizer_coefficients(air_o)
    r = e.randomness_from_seed(seed, m * st_o.num_randomizers + nrc)
    tr = [r[m * i:m * i + m] for i in range(st_o.num_randomizers)]
    rc = r[m * st_o.num_randomizers:]
    return rp_o, st_o, st_g, air_o, air_g, rp_o.trace(inp), rp_o.boundary_constraints(out), tr, rc, out


@pytest.mark.parametrize("N,exp,c,sec,tcd", [(27, 4, 2, 2, 2), (27, 8, 4, 8, 3), (40, 4, 3, 4, 2), (9, 16, 2, 4, 4)])
def test_stark_prove_bytes_vs_oracle(N, exp, c, sec, tcd):
    """stark.rs:276-562 proof bytes == the oracle's (randomizers injected identically)."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(N, exp, c, sec, tcd, b"case-%d" % N)
    ops = o.IndependentProofStream()
    want = st_o.prove(trace, air_o, bnd, ops, tr, rc)
    gps = sg.IndependentProofStream()
    got = st_g.prove(trace, air_g, bnd, gps, tr, rc)
    assert got == want
    ok, err = st_o.verify(air_o, bnd, o.IndependentProofStream(ops.objects))
    # with transition_constraints_degree too small for alpha = 3 (max_degree >= omicron order)
    # the reference's NTT products wrap and its proof does not verify: same bytes, same verdict
    assert ok == (st_o.max_degree(air_o) < st_o.omicron_domain_length), err


def test_stark_prove_domain_tables_cached_and_recomputed(monkeypatch):
    """The public domain tables the context keeps (trace-domain zerofier transforms, the transition
    zerofier's coset values and inverse, the AIR x-polynomials' coset values, boundary-divisor
    inverses) give the same proof bytes as recomputing them: first proof (tables built), second
    proof (tables reused), and a proof with the tables recomputed (context option domain_cache = 0,
    what SG_NO_DOMAIN_CACHE=1 sets at creation) -- all equal to the oracle's."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(40, 4, 3, 4, 2, b"domain-cache")
    want = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    ctx = sg.Context(0)  # a fresh context: nothing cached yet
    st = sg.Stark(4, 3, 4, 2, 41, 2, ctx=ctx)
    air = sg.RescuePrime(2, 1, 4, 40, ctx=ctx).transition_constraints(st.omicron, st.omicron_domain_length)
    assert st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc) == want
    assert st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc) == want
    ctx.set_option("domain_cache", 0)
    assert st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc) == want


@pytest.mark.parametrize("generic", ["0", "1"])
def test_stark_prove_rebuilt_constraints_keep_tables_flat(monkeypatch, generic):
    """The reference rebuilds the transition constraints for every sign / verify (rpsss.rs:46,57).
    The AIR's coset tables are keyed by content (the Rescue parameters and domain, or a digest of
    each x-polynomial for the expanded groups), so rebuilding the constraints for each of 5 proofs
    leaves the context's table count where the first proof put it; every proof equals the oracle's."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(40, 4, 3, 4, 2, b"rebuilt-air")
    want = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    ctx = sg.Context(0)
    ctx.set_option("air_generic", int(generic))
    st = sg.Stark(4, 3, 4, 2, 41, 2, ctx=ctx)
    rpg = sg.RescuePrime(2, 1, 4, 40, ctx=ctx)
    counts = []
    for _ in range(5):
        air = rpg.transition_constraints(st.omicron, st.omicron_domain_length)
        assert st.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc) == want
        counts.append(ctx.cached_tables())
        del air
    # (with SG_NO_DOMAIN_CACHE=1 -- the alternate-paths suite -- nothing is cached: flat at zero)
    cached = os.environ.get("SG_NO_DOMAIN_CACHE") != "1"
    assert (counts[0][0] > 0 or not cached) and all(c == counts[0] for c in counts), counts


def test_stark_prove_constraints_shared_by_two_contexts():
    """Constraint objects built on one context and proved on two (the AIR's coset values live in
    each context's domain tables, not in the shared constraint), with sg_ctx_trim between proofs
    (it frees them): every proof equals the oracle's."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(40, 4, 3, 4, 2, b"two-contexts")
    want = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    c1, c2 = sg.Context(0), sg.Context(0)
    s1 = sg.Stark(4, 3, 4, 2, 41, 2, ctx=c1)
    s2 = sg.Stark(4, 3, 4, 2, 41, 2, ctx=c2)
    air = sg.RescuePrime(2, 1, 4, 40, ctx=c1).transition_constraints(s1.omicron, s1.omicron_domain_length)
    for ctx_stark in (s1, s2, s1, s2):
        assert ctx_stark.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc) == want
        ctx_stark.ctx.trim()
    assert s1.prove(trace, air, bnd, sg.IndependentProofStream(), tr, rc) == want


def test_stark_prove_contexts_in_concurrent_threads():
    """One context per host thread (the C ABI's rule), several proofs in flight on one GPU: three
    threads, each with its own context, prove C4-sized traces (trace 2^16, FRI domain 2^21) twice
    at the same time; every proof equals the same trace's proof run alone, and the small case equals
    the oracle's (tools/concurrent_provers.py times the headline this way)."""
    import threading
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(40, 4, 3, 4, 2, b"threads")
    want_small = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    N = 65278
    rp_o = e.RescuePrime(2, 1, 128, N)
    jobs = []
    for i in range(3):
        ctx = sg.Context(0)
        st = sg.Stark(8, 64, 128, 2, N + 1, 3, ctx=ctx)
        air = sg.RescuePrime(2, 1, 128, N, ctx=ctx).transition_constraints(st.omicron, st.omicron_domain_length)
        inp = o.sample(b"threads-%d" % i)
        r = e.randomness_from_seed(b"threads-%d" % i, 2 * st.num_randomizers + st.num_randomizer_coefficients(air))
        args = (sg.RescuePrime(2, 1, 128, N, ctx=ctx).trace_array(inp), air,
                rp_o.boundary_constraints(rp_o.hash(inp)))
        tr_i, rc_i = sg.fe_array(r[:2 * st.num_randomizers]), sg.fe_array(r[2 * st.num_randomizers:])
        alone = st.prove(*args, sg.IndependentProofStream(), tr_i, rc_i)
        jobs.append((st, args, tr_i, rc_i, alone))
    small_ctx = sg.Context(0)
    st_small = sg.Stark(4, 3, 4, 2, 41, 2, ctx=small_ctx)
    air_small = sg.RescuePrime(2, 1, 4, 40, ctx=small_ctx).transition_constraints(st_small.omicron,
                                                                                   st_small.omicron_domain_length)
    got, errs = {}, []
    start = threading.Barrier(len(jobs) + 1)

    def run(i):
        try:
            start.wait()
            if i == len(jobs):
                got[i] = [st_small.prove(trace, air_small, bnd, sg.IndependentProofStream(), tr, rc) for _ in range(4)]
                return
            st, args, tr_i, rc_i, _ = jobs[i]
            got[i] = [st.prove(*args, sg.IndependentProofStream(), tr_i, rc_i) for _ in range(2)]
        except Exception as ex:
            errs.append(repr(ex))

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(jobs) + 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for i, (_, _, _, _, alone) in enumerate(jobs):
        assert all(p == alone for p in got[i]), i
    assert all(p == want_small for p in got[len(jobs)])


@pytest.fixture(scope="module")
def c4_case():
    """C4 inputs (trace 2^16, FRI domain 2^21, c = 64) and the working-set peak of one proof."""
    N = 65278
    rp_o = e.RescuePrime(2, 1, 128, N)
    inp = o.sample(b"oom-c4")
    ctx = sg.Context(0)
    st = sg.Stark(8, 64, 128, 2, N + 1, 3, ctx=ctx)
    rp = sg.RescuePrime(2, 1, 128, N, ctx=ctx)
    air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
    r = e.randomness_from_seed(b"oom-c4", 2 * st.num_randomizers + st.num_randomizer_coefficients(air))
    case = {"N": N, "trace": rp.trace_array(inp), "bnd": rp_o.boundary_constraints(rp_o.hash(inp)),
            "tr": sg.fe_array(r[:2 * st.num_randomizers]), "rc": sg.fe_array(r[2 * st.num_randomizers:])}
    ctx.memory(reset_peak=True)
    case["proof"] = st.prove(case["trace"], air, case["bnd"], sg.IndependentProofStream(), case["tr"], case["rc"])
    case["peak"] = ctx.memory()["peak"]
    case["air"], case["ctx"] = air, ctx  # constraints built uncapped, proved on any context
    return case


@pytest.mark.parametrize("frac", [0.02, 0.15, 0.35, 0.55, 0.75, 0.95])
def test_stark_prove_out_of_memory_at_every_stage(monkeypatch, c4_case, frac):
    """A C4 prove whose buffer pool is capped below its working set (SG_POOL_LIMIT_BYTES, a test
    knob read at context creation) fails with SG_ERR_NOMEM wherever the cap bites -- early in the
    trace interpolation, amid the quotients and the side stream's trees, or in FRI -- hands every
    pool buffer back (live bytes as before the call), and leaves the context usable: a proof that
    fits under the cap then equals the oracle's, and the C4 proof equals the uncapped one once a
    context without the cap proves it.  (The constraints are built on an uncapped context.)"""
    from starkgpu._lib import SG_ERR_NOMEM
    limit = int(frac * c4_case["peak"])
    monkeypatch.setenv("SG_POOL_LIMIT_BYTES", str(limit))
    ctx = sg.Context(0)
    monkeypatch.delenv("SG_POOL_LIMIT_BYTES")
    N = c4_case["N"]
    st = sg.Stark(8, 64, 128, 2, N + 1, 3, ctx=ctx)
    live = ctx.memory()["live"]
    with pytest.raises(sg.StarkGpuError) as err:
        st.prove(c4_case["trace"], c4_case["air"], c4_case["bnd"], sg.IndependentProofStream(), c4_case["tr"],
                 c4_case["rc"])
    assert err.value.code == SG_ERR_NOMEM, err.value
    assert ctx.memory()["live"] == live
    # a small proof under the same cap, on the same context
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(40, 4, 3, 4, 2, b"after-oom")
    want = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    st_s = sg.Stark(4, 3, 4, 2, 41, 2, ctx=ctx)
    ctx.memory(reset_peak=True)
    assert st_s.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc) == want
    assert ctx.memory()["peak"] <= limit
    # the same C4 inputs on an uncapped context
    st2 = sg.Stark(8, 64, 128, 2, N + 1, 3, ctx=sg.Context(0))
    assert st2.prove(c4_case["trace"], c4_case["air"], c4_case["bnd"], sg.IndependentProofStream(), c4_case["tr"],
                     c4_case["rc"]) == c4_case["proof"]


def test_stark_prove_rescue_factored_air_equals_expanded(monkeypatch):
    """The native Rescue-Prime AIR is evaluated in its factored form (rescue_prime.rs:246-283:
    sum MDS prev^alpha + first(x) - (sum MDSinv (next - second(x)))^alpha); the context option
    air_generic = 1 evaluates its expanded monomial groups instead.  Same proof bytes either way, equal to the
    oracle's, for an honest and a false witness (the transition values differ from zero there)."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(40, 4, 3, 4, 2, b"factored-air")
    want = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    bad = [list(r) for r in trace]
    bad[17][0] = o.add_mod(bad[17][0], 5)
    want_bad = st_o.prove(bad, air_o, bnd, o.IndependentProofStream(), tr, rc)
    got = st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc)
    got_bad = st_g.prove(bad, air_g, bnd, sg.IndependentProofStream(), tr, rc)
    with st_g.ctx.option("air_generic", 1, 0):
        assert st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc) == want
        assert st_g.prove(bad, air_g, bnd, sg.IndependentProofStream(), tr, rc) == want_bad
    assert got == want and got_bad == want_bad


def test_stark_prove_c4_factored_air_equals_expanded(monkeypatch):
    """C4 size (trace 2^16, FRI domain 2^21): factored and expanded AIR evaluation give the same
    proof bytes (the oracle cannot rebuild the expanded AIR at this size; the factored proof is
    verified in test_stark_prove_c4_rescue_trace_2p16)."""
    N = 65278
    rp_g = sg.RescuePrime(2, 1, 128, N)
    st_g = sg.Stark(8, 64, 128, 2, N + 1, 3)
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    rp_o = e.RescuePrime(2, 1, 128, N)
    inp = o.sample(b"c4-factored")
    trace = rp_g.trace_array(inp)
    nrc = st_g.num_randomizer_coefficients(air_g)
    r = e.randomness_from_seed(b"c4-factored", 2 * st_g.num_randomizers + nrc)
    tr = sg.fe_array(r[:2 * st_g.num_randomizers])
    rc = sg.fe_array(r[2 * st_g.num_randomizers:])
    bnd = rp_o.boundary_constraints(rp_o.hash(inp))
    factored = st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc)
    with st_g.ctx.option("air_generic", 1, 0):
        assert st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc) == factored


@pytest.mark.parametrize("opts", [{"lean_drop": 1}, {"lean_drop": 2}, {"lean_trees": 0}])
def test_lean_tree_layouts_keep_proof_bytes(opts):
    """The prove's retained trees drop their low levels (three by default; an opening rehashes the
    8-leaf block around its leaf from the codeword): every layout -- one or two levels dropped, or
    every level kept -- writes the same proof bytes, equal to the oracle's at a small size and to
    each other at C4 (trace 2^16, FRI domain 2^21, c = 64: 13 FRI rounds, their paths rehashed)."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(40, 4, 3, 4, 2, b"lean-trees")
    want = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    N = 65278
    rp_g = sg.RescuePrime(2, 1, 128, N)
    st_c4 = sg.Stark(8, 64, 128, 2, N + 1, 3)
    air_c4 = rp_g.transition_constraints(st_c4.omicron, st_c4.omicron_domain_length)
    inp = o.sample(b"lean-trees-c4")
    trace_c4 = rp_g.trace_array(inp)
    r = e.randomness_from_seed(b"lean-trees-c4", 2 * st_c4.num_randomizers + st_c4.num_randomizer_coefficients(air_c4))
    tr_c4 = sg.fe_array(r[:2 * st_c4.num_randomizers])
    rc_c4 = sg.fe_array(r[2 * st_c4.num_randomizers:])
    rp_o = e.RescuePrime(2, 1, 128, N)
    bnd_c4 = rp_o.boundary_constraints(rp_o.hash(inp))
    default_small = st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc)
    default_c4 = st_c4.prove(trace_c4, air_c4, bnd_c4, sg.IndependentProofStream(), tr_c4, rc_c4)
    ctx = sg.Context.default()
    assert st_g.ctx is ctx and st_c4.ctx is ctx
    try:
        for k, v in opts.items():
            ctx.set_option(k, v)
        assert st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc) == want == default_small
        assert st_c4.prove(trace_c4, air_c4, bnd_c4, sg.IndependentProofStream(), tr_c4, rc_c4) == default_c4
    finally:
        ctx.set_option("lean_drop", 3)
        ctx.set_option("lean_trees", 1)


def test_stark_prove_negated_constraints():
    """A negated native Rescue-Prime constraint (-tc, and the empty MPolynomial minus tc: the
    reference's Add returns the other operand) is evaluated as -tc, not through the factored form of
    +tc; -(-tc) gives tc's proof (m_polynomial.rs:183-229)."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(27, 4, 2, 2, 2, b"neg")
    neg_o = [-a for a in air_o]
    want_neg = st_o.prove(trace, neg_o, bnd, o.IndependentProofStream(), tr, rc)
    want = st_o.prove(trace, air_o, bnd, o.IndependentProofStream(), tr, rc)
    zero = sg.MPolynomial.new({})
    assert st_g.prove(trace, [-a for a in air_g], bnd, sg.IndependentProofStream(), tr, rc) == want_neg
    assert st_g.prove(trace, [zero - a for a in air_g], bnd, sg.IndependentProofStream(), tr, rc) == want_neg
    assert st_g.prove(trace, [-(-a) for a in air_g], bnd, sg.IndependentProofStream(), tr, rc) == want


def test_stark_false_witness_and_claim():
    """stark.rs:845-880: a false witness gives the reference's (rejected) proof bytes; a false
    claim is rejected by the verifier."""
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(27, 4, 2, 2, 2, b"bad")
    bad = [list(r) for r in trace]
    bad[22][1] = o.add_mod(bad[22][1], 17274817952119230544216945715808633996)
    ops, gps = o.IndependentProofStream(), sg.IndependentProofStream()
    assert st_g.prove(bad, air_g, bnd, gps, tr, rc) == st_o.prove(bad, air_o, bnd, ops, tr, rc)
    ok, _ = st_o.verify(air_o, bnd, o.IndependentProofStream(ops.objects))
    assert not ok
    honest = sg.IndependentProofStream()
    st_g.prove(trace, air_g, bnd, honest, tr, rc)
    objs = honest.objects()
    ok, err = st_o.verify(air_o, bnd, o.IndependentProofStream(objs))
    assert ok, err
    ok, _ = st_o.verify(air_o, rp.boundary_constraints(o.add_mod(out, 1)), o.IndependentProofStream(objs))
    assert not ok


def test_stark_prove_callback_stream_and_errors():
    rp, st_o, st_g, air_o, air_g, trace, bnd, tr, rc, out = _case(27, 4, 2, 2, 2, b"cb")
    ops = o.IndependentProofStream()
    want = st_o.prove(trace, air_o, bnd, ops, tr, rc)
    # any ProofStream implementation through the callbacks
    pys = o.IndependentProofStream()
    st_g.prove(trace, air_g, bnd, pys, tr, rc)
    assert pys.digest() == want
    with pytest.raises(sg.StarkGpuError):
        st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc[:-1])


def test_stark_prove_c4_rescue_trace_2p16():
    """BASELINE config C4 at full size: Rescue-Prime (m=2, N=65278 -> trace 2^16 rows with the 256
    randomizer rows), expansion 8, 64 colinearity checks, security 128, transition degree 3
    (omicron domain 2^18, FRI domain 2^21).  The oracle cannot rebuild the expanded AIR at this
    size (O(N^2)), so the proof is checked by the oracle's verifier with the AIR evaluated from
    its structure (RescueAirAtPoint), and a false claim must be rejected."""
    import time
    N = 65278
    rp_g = sg.RescuePrime(2, 1, 128, N)
    st_g = sg.Stark(8, 64, 128, 2, N + 1, 3)
    assert st_g.omicron_domain_length == 1 << 18 and st_g.fri_domain_length == 1 << 21
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    rp_o = e.RescuePrime(2, 1, 128, N)
    assert rp_g.round_constants == rp_o.round_constants
    inp = o.sample(b"c4")
    out = rp_o.hash(inp)
    trace = rp_g.trace_array(inp)
    assert sg.to_ints(trace[-2:-1])[0] == out
    st_o = e.Stark(8, 64, 128, 2, N + 1, 3)
    sair = e.RescueAirAtPoint.for_rescue(rp_o, st_o.omicron)
    assert st_g.transition_degree_bounds(air_g) == st_o.transition_degree_bounds(sair)
    nrc = st_g.num_randomizer_coefficients(air_g)
    r = e.randomness_from_seed(b"c4", 2 * st_g.num_randomizers + nrc)
    tr = sg.fe_array(r[:2 * st_g.num_randomizers])
    rc = sg.fe_array(r[2 * st_g.num_randomizers:])
    bnd = rp_o.boundary_constraints(out)
    ps = sg.IndependentProofStream()
    t0 = time.perf_counter()
    st_g.prove(trace, air_g, bnd, ps, tr, rc)
    print("C4 prove: %.1f ms" % ((time.perf_counter() - t0) * 1e3))
    objs = ps.objects()
    ok, err = st_o.verify(sair, bnd, o.IndependentProofStream(objs))
    assert ok, err
    ok, _ = st_o.verify(sair, rp_o.boundary_constraints(o.add_mod(out, 1)), o.IndependentProofStream(objs))
    assert not ok


@pytest.fixture(scope="module")
def rpsss():
    """The reference's published RPSSS configuration (tests/rpsss_case.py) and the oracle's
    signature for it (Stark.prove through a SignatureProofStream, ~8 s)."""
    import rpsss_case as R
    c = R.Case()
    return R, c, c.oracle_sign()


def test_rpsss_published_configuration_bytes_length_verify(rpsss):
    """rpsss.rs:89,103,113-131: RPSSS::new(field, 4, 64, 128, 3) signs b"Hello, World!" --
    Rescue N = 27, Stark(4, 64, 128, 2, 28, 3), FRI domain 4096, c = 64, a SignatureProofStream,
    randomizers injected.  The GPU proof bytes equal the oracle's, the length is the reference's
    1 156 888, the oracle verifier accepts the signature for the document and rejects it for
    b"Malicious document"."""
    R, c, want = rpsss
    rp_g = sg.RescuePrime(*R.RESCUE)
    st_g = sg.Stark(R.EXPANSION, R.CHECKS, R.SECURITY, rp_g.m, R.RESCUE[3] + 1, R.TCD)
    assert (st_g.omicron_domain_length, st_g.fri_domain_length) == (1024, 4096)
    assert rp_g.hash(c.sk) == c.pk
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    assert st_g.transition_degree_bounds(air_g) == c.st.transition_degree_bounds(c.air)
    got = st_g.prove(rp_g.trace(c.sk), air_g, rp_g.boundary_constraints(c.pk), sg.SignatureProofStream(R.DOCUMENT),
                     c.trace_randomizers, c.randomizer_coefficients)
    assert len(got) == R.PROOF_LEN, "rpsss.rs:89"
    assert got == want
    assert c.oracle_verify(R.DOCUMENT, got) == (True, "")
    ok, err = c.oracle_verify(R.FORGED, got)
    assert not ok, "rpsss.rs:127-131: " + err
    # the same signature through a foreign (Python) proof stream driven by the callbacks
    ops = o.SignatureProofStream(R.DOCUMENT)
    assert st_g.prove(c.trace, air_g, c.boundary, ops, c.trace_randomizers, c.randomizer_coefficients) == want


def test_rpsss_published_configuration_signature_roundtrip(rpsss):
    """The signature deserializes (stark.rs:30-67, sg_stream_deserialize) into the objects the
    oracle's deserializer reads, and a second document signs to different bytes of the same length."""
    R, c, want = rpsss
    back = sg.IndependentProofStream.deserialize(want)
    assert back.digest() == want
    rp_g = sg.RescuePrime(*R.RESCUE)
    st_g = sg.Stark(R.EXPANSION, R.CHECKS, R.SECURITY, rp_g.m, R.RESCUE[3] + 1, R.TCD)
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    other = st_g.prove(c.trace, air_g, c.boundary, sg.SignatureProofStream(R.FORGED), c.trace_randomizers,
                       c.randomizer_coefficients)
    assert len(other) == R.PROOF_LEN and other != want
    assert c.oracle_verify(R.FORGED, other) == (True, "")


def test_midsize_proof_bytes_equal_oracle_digest():
    """A mid-size Stark::prove pinned to the Python oracle itself (tests/midsize_case.py): Rescue-Prime
    N = 1000 -> trace 1257 rows, omicron domain 4096, FRI domain 2^15, expansion 8, c = 64,
    transition degree 3 -- between the reference's published RPSSS configuration (FRI domain 4096)
    and the full-size cases, which only the CPU checker pins.  The GPU proof's length and SHA-256
    equal the oracle's (tests/golden/midsize_proof.json, written by tests/golden/make_midsize.py
    from stark_prove_oracle.Stark.prove, stark.rs:276-562); the oracle verifier accepts it and
    rejects a false claim."""
    import hashlib
    import midsize_case as M
    with open(os.path.join(os.path.dirname(__file__), "golden", "midsize_proof.json")) as f:
        g = json.load(f)
    rp_o, st_o, trace, bnd, tr, rc = M.light_inputs()
    rp_g = sg.RescuePrime(*M.RESCUE)
    st_g = sg.Stark(M.EXPANSION, M.CHECKS, M.SECURITY, rp_g.m, M.RESCUE[3] + 1, M.TCD)
    assert (st_g.omicron_domain_length, st_g.fri_domain_length) == (g["omicron_domain"], g["fri_domain"])
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    assert st_g.num_randomizer_coefficients(air_g) == len(rc)
    assert str(bnd[-1][2]) == g["output"]
    got = st_g.prove(trace, air_g, bnd, sg.IndependentProofStream(), tr, rc)
    assert len(got) == g["proof_len"]
    assert hashlib.sha256(got).hexdigest() == g["proof_sha256"], "GPU proof != oracle proof (digest)"
    sair = e.RescueAirAtPoint.for_rescue(rp_o, st_o.omicron)
    ok, err = st_o.verify(sair, bnd, o.IndependentProofStream(o.deserialize(got)))
    assert ok, err
    false_bnd = list(bnd[:-1]) + [(bnd[-1][0], bnd[-1][1], o.add_mod(bnd[-1][2], 1))]
    ok, _ = st_o.verify(sair, false_bnd, o.IndependentProofStream(o.deserialize(got)))
    assert not ok
