"""ctypes wrapper of oracle/fast_cpu.cpp (optimized C++ restatement: Montgomery, OpenMP).

TEST INFRASTRUCTURE ONLY (tests/ as the full-size checker, bench.py's all-cores
cpu_baseline leg).  Build with `make -C oracle` (done by __graft_entry__.build()).
Arrays are numpy uint64 of shape (n, 2): little-endian (lo, hi) limbs, canonical.
"""
import ctypes
import hashlib
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libfast_cpu.so")
P = 1 + 407 * (1 << 119)
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        l = ctypes.CDLL(LIB_PATH)
        vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
        l.fc_threads.restype = ctypes.c_int
        l.fc_set_threads.argtypes = [ctypes.c_int]
        for f in (l.fc_ntt, l.fc_intt):
            f.argtypes = [vp, vp, u64, vp]
            f.restype = ctypes.c_int
        l.fc_coset_evaluate.argtypes = [vp, u64, vp, vp, u64, vp]
        l.fc_coset_evaluate.restype = ctypes.c_int
        l.fc_merkle_commit.argtypes = [vp, u64, vp]
        l.fc_merkle_commit.restype = ctypes.c_int
        l.fc_blake2b512.argtypes = [vp, sz, vp]
        l.fc_shake256.argtypes = [vp, sz, vp, sz]
        l.fc_mul.argtypes = [vp, vp, vp]
        l.fc_inv.argtypes = [vp, vp]
        l.fc_fri_prove.argtypes = [vp, vp, vp, u64, u64, u64, vp, sz, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_size_t), vp]
        l.fc_fri_prove.restype = ctypes.c_long
        l.fc_free.argtypes = [vp]
        l.fc_geometric_prod.argtypes = [vp, u64, vp, u64, vp]
        l.fc_poly_from_roots.argtypes = [vp, u64, vp]
        l.fc_eval_points.argtypes = [vp, u64, vp, u64, vp]
        l.fc_geometric_bary.argtypes = [vp, u64, vp, u64, vp, u64, vp]
        l.fc_bary_create.argtypes = [vp, u64, vp, u64]
        l.fc_bary_create.restype = ctypes.c_void_p
        l.fc_bary_eval.argtypes = [vp, vp, vp]
        l.fc_bary_free.argtypes = [vp]
        l.fc_last_error.restype = ctypes.c_char_p
        l.fc_stark_prove_rescue.argtypes = [u64] * 7 + [vp, vp, vp, u64, vp, vp, vp, u64, vp, u64, vp, u64, vp, vp,
                                                        u64, vp, vp, vp, u64, ctypes.POINTER(ctypes.c_void_p),
                                                        ctypes.POINTER(ctypes.c_size_t), vp, ctypes.c_char_p,
                                                        ctypes.c_size_t]
        l.fc_stark_prove_rescue.restype = ctypes.c_long
        l.fc_geo_interpolate.argtypes = [vp, u64, vp, u64, vp]
        l.fc_geo_interpolate.restype = ctypes.c_long
        l.fc_geo_zerofier.argtypes = [vp, u64, vp]
        l.fc_geo_zerofier.restype = ctypes.c_long
        _lib = l
    return _lib


def threads() -> int:
    return lib().fc_threads()


def set_threads(n: int) -> None:
    """OpenMP threads of every later call (omp_set_num_threads)."""
    lib().fc_set_threads(n)


def _fe(v: int) -> np.ndarray:
    return np.array([v & ((1 << 64) - 1), v >> 64], dtype=np.uint64)


def arr(values) -> np.ndarray:
    """Python ints (or an (n, 2) array) -> contiguous (n, 2) uint64."""
    if isinstance(values, np.ndarray):
        return np.ascontiguousarray(values.reshape(-1, 2).view(np.uint64) if values.dtype != np.uint64
                                    else values.reshape(-1, 2))
    out = np.empty((len(values), 2), dtype=np.uint64)
    for i, v in enumerate(values):
        out[i, 0] = v & ((1 << 64) - 1)
        out[i, 1] = v >> 64
    return out


def ints(a: np.ndarray):
    a = np.ascontiguousarray(a).reshape(-1, 2).astype(np.uint64)
    return [int(lo) | (int(hi) << 64) for lo, hi in a]


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _next_pow2(n: int) -> int:
    return 1 << max(0, (n - 1).bit_length())


def ntt(root: int, x) -> np.ndarray:
    """fft/ntt.rs:7-49 (zero-padded to the next power of two)."""
    a = arr(x)
    out = np.empty((_next_pow2(len(a)), 2), dtype=np.uint64)
    r = _fe(root)
    if lib().fc_ntt(_p(r), _p(a), len(a), _p(out)) != 0:
        raise ValueError("ntt of an empty input")
    return out


def intt(root: int, x) -> np.ndarray:
    """fft/ntt.rs:51-68."""
    a = arr(x)
    out = np.empty((_next_pow2(len(a)) if len(a) >= 2 else len(a), 2), dtype=np.uint64)
    r = _fe(root)
    lib().fc_intt(_p(r), _p(a), len(a), _p(out))
    return out


def fast_coset_evaluate(generator: int, root_order: int, offset: int, coeffs) -> np.ndarray:
    """fft/ntt_arithmetics.rs:161-170."""
    a = arr(coeffs)
    out = np.empty((root_order, 2), dtype=np.uint64)
    g, o = _fe(generator), _fe(offset)
    if lib().fc_coset_evaluate(_p(g), root_order, _p(o), _p(a), len(a), _p(out)) != 0:
        raise ValueError("polynomial longer than root_order / root_order not a power of two")
    return out


def merkle_commit(leaves) -> bytes:
    """merkle_root.rs:21-32."""
    a = arr(leaves)
    root = np.zeros(64, dtype=np.uint8)
    if lib().fc_merkle_commit(_p(a), len(a), _p(root)) != 0:
        raise ValueError("Leafs len must be power of two")
    return root.tobytes()


def blake2b512(data: bytes) -> bytes:
    buf = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, dtype=np.uint8)
    out = np.zeros(64, dtype=np.uint8)
    lib().fc_blake2b512(_p(buf), len(data), _p(out))
    return out.tobytes()


def shake256(data: bytes, n: int) -> bytes:
    buf = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, dtype=np.uint8)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().fc_shake256(_p(buf), len(data), _p(out), n)
    return out.tobytes()[:n]


def fri_prove(offset: int, omega: int, codeword, expansion: int, colinearity: int, prefix: bytes = bytes(16)):
    """FRI::prove (fri.rs:210-248) on a proof stream whose serialized form is `prefix`.
    Returns (serialized stream after the call, top-level indices)."""
    a = arr(codeword)
    o, w = _fe(offset), _fe(omega)
    pre = np.frombuffer(prefix, dtype=np.uint8).copy()
    out = ctypes.c_void_p()
    out_len = ctypes.c_size_t()
    top = np.zeros(colinearity, dtype=np.uint64)
    r = lib().fc_fri_prove(_p(o), _p(w), _p(a), len(a), expansion, colinearity, _p(pre), len(prefix),
                           ctypes.byref(out), ctypes.byref(out_len), _p(top))
    if r < 0:
        raise ValueError(f"fc_fri_prove failed ({r})")
    try:
        data = ctypes.string_at(out.value, out_len.value)
    finally:
        lib().fc_free(out)
    return data, [int(t) for t in top]


def poly_from_roots(domain) -> np.ndarray:
    """prod (x - d) over an arbitrary domain, length n + 1 (fast_zerofier without wrap-around)."""
    d = arr(domain)
    out = np.zeros((len(d) + 1, 2), dtype=np.uint64)
    lib().fc_poly_from_roots(_p(d), len(d), _p(out))
    return out


def eval_points(coeffs, xs) -> np.ndarray:
    """Polynomial::evaluate at every x (Horner, points over threads)."""
    c, x = arr(coeffs), arr(xs)
    out = np.zeros((len(x), 2), dtype=np.uint64)
    lib().fc_eval_points(_p(c), len(c), _p(x), len(x), _p(out))
    return out


def geometric_prod(q: int, n: int, xs):
    """prod_{r<n} (x - q^r) for each x."""
    x = arr(xs)
    out = np.empty_like(x)
    lib().fc_geometric_prod(_p(_fe(q)), n, _p(x), len(x), _p(out))
    return ints(out)


def geometric_bary(q: int, cols, xs):
    """Interpolants through (q^r, col[r]), r < n, evaluated at each x: result[j][c]."""
    n = len(cols[0])
    c = np.ascontiguousarray(np.concatenate([arr(col) for col in cols]))
    x = arr(xs)
    out = np.empty((len(x) * len(cols), 2), dtype=np.uint64)
    lib().fc_geometric_bary(_p(_fe(q)), n, _p(c), len(cols), _p(x), len(x), _p(out))
    v = ints(out)
    return [v[j * len(cols):(j + 1) * len(cols)] for j in range(len(x))]


class Barycentric:
    """Interpolants through (q^r, col[r]), r < n, of several columns; value(x, key) in O(n)
    (same interface as stark_prove_oracle.GeometricBarycentric)."""

    def __init__(self, q: int, n: int, columns):
        self.keys = list(columns)
        c = np.ascontiguousarray(np.concatenate([arr(columns[k])[:n] for k in self.keys]))
        self.h = lib().fc_bary_create(_p(_fe(q)), n, _p(c), len(self.keys))
        self.cache = {}

    def value(self, x: int, key) -> int:
        if x not in self.cache:
            out = np.empty((len(self.keys), 2), dtype=np.uint64)
            lib().fc_bary_eval(ctypes.c_void_p(self.h), _p(_fe(x % P)), _p(out))
            self.cache[x] = dict(zip(self.keys, ints(out)))
        return self.cache[x][key]

    def __del__(self):
        if getattr(self, "h", None):
            lib().fc_bary_free(ctypes.c_void_p(self.h))
            self.h = None


def rescue_air_at_point(rp, omicron: int):
    """stark_prove_oracle.RescueAirAtPoint for every register, with the round-constant
    interpolants evaluated by this library (O(N) per point in C++ instead of Python)."""
    import stark_prove_oracle as e
    m = rp.m
    cols = {}
    for i in range(m):
        cols[("c1", i)] = np.array([rp.round_constants[2 * r * m + i] for r in range(rp.N)], dtype=object)
        cols[("c2", i)] = np.array([rp.round_constants[2 * r * m + m + i] for r in range(rp.N)], dtype=object)
    bary = Barycentric(omicron, rp.N, {k: _obj_to_arr(v) for k, v in cols.items()})
    return [e.RescueAirAtPoint(rp, i, bary) for i in range(m)]


def _obj_to_arr(v) -> np.ndarray:
    lo = np.array([int(x) & ((1 << 64) - 1) for x in v], dtype=np.uint64)
    hi = np.array([int(x) >> 64 for x in v], dtype=np.uint64)
    return np.ascontiguousarray(np.stack([lo, hi], axis=1))


def geo_interpolate(q: int, D: int, values):
    """Unique interpolant (degree < n, length n) through (q^i, v_i), i < n, q of order D."""
    y = arr(values)
    out = np.zeros((max(len(y), 1), 2), dtype=np.uint64)
    r = lib().fc_geo_interpolate(_p(_fe(q)), D, _p(y), len(y), _p(out))
    if r < 0:
        raise ValueError(lib().fc_last_error().decode())
    return out[:r]


def geo_zerofier(q: int, n: int):
    """prod_{i<n} (x - q^i), n + 1 coefficients."""
    out = np.zeros((n + 1, 2), dtype=np.uint64)
    r = lib().fc_geo_zerofier(_p(_fe(q)), n, _p(out))
    if r < 0:
        raise ValueError(lib().fc_last_error().decode())
    return out[:r]


def rescue_degree_bounds(rp, st):
    """(transition quotient degree bounds, max_degree) of RescuePrime.transition_constraints for the
    Stark `st` (stark.rs:117-196 over the AIR's key set; RescueAirAtPoint carries keys whose maximum
    equals the expanded AIR's)."""
    import stark_prove_oracle as e
    sair = [e.RescueAirAtPoint(rp, i, None) for i in range(rp.m)]
    return st.transition_quotient_degree_bounds(sair), st.max_degree(sair)


PHASES = ("trace_interpolation", "boundary_quotients", "bq_codewords_commit", "transition_quotients",
          "randomizer_commit", "combination_lde", "fri_prove", "openings")


def stark_prove_rescue(rp, st, trace, boundary, trace_randomizers, randomizer_coefficients, bounds=None,
                       phases=None, document=None) -> bytes:
    """Stark::prove (stark.rs:276-562) of a Rescue-Prime trace on the CPU (Montgomery + OpenMP):
    the serialized proof stream (IndependentProofStream, stark.rs:562; with `document`, a
    SignatureProofStream's: every Fiat-Shamir draw hashes [len u64 BE][blake2b512(document)]
    before the stream, rescue_prime/proof_stream.rs:22-39).  `rp` / `st` are the
    oracle's RescuePrime / Stark (or any objects with the same attributes); `trace` rows x m
    (list of lists or an (rows * m, 2) array); the two thread_rng draws are explicit like the
    oracle's prove.  Raises ValueError with the reference's message where it returns Err/panics."""
    m = rp.m
    t = arr(trace if isinstance(trace, np.ndarray) else [v for row in trace for v in row])
    rows = len(t) // m
    tr = arr(trace_randomizers if isinstance(trace_randomizers, np.ndarray)
             else [v for row in trace_randomizers for v in row])
    rc = arr(randomizer_coefficients)
    tqdb, tcd = bounds if bounds is not None else rescue_degree_bounds(rp, st)
    mds = arr([v for row in rp.MDS for v in row])
    mdsi = arr([v for row in rp.MDS_inv for v in row])
    rcs = _obj_to_arr(np.array(rp.round_constants, dtype=object)) if len(rp.round_constants) \
        else np.zeros((1, 2), dtype=np.uint64)
    tq = np.array(tqdb, dtype=np.uint64)
    bc = np.array([c for (c, _, _) in boundary] or [0], dtype=np.uint64)
    br = np.array([r for (_, r, _) in boundary] or [0], dtype=np.uint64)
    bv = arr([v for (_, _, v) in boundary] or [0])
    out = ctypes.c_void_p()
    out_len = ctypes.c_size_t()
    ph = np.zeros(8, dtype=np.float64)
    prefix = b""
    if document is not None:
        h = hashlib.blake2b(bytes(document), digest_size=64).digest()
        prefix = len(h).to_bytes(8, "big") + h
    r = lib().fc_stark_prove_rescue(m, st.original_trace_length, st.num_randomizers, st.omicron_domain_length,
                                    st.fri.domain_length, st.expansion_factor, st.fri.num_colinearity_tests,
                                    _p(_fe(st.omicron)), _p(_fe(st.omega)), _p(_fe(st.generator)), rp.alpha,
                                    _p(mds), _p(mdsi), _p(rcs), rp.N, _p(tq), tcd, _p(t), rows, _p(tr), _p(rc),
                                    len(rc), _p(bc), _p(br), _p(bv), len(boundary), ctypes.byref(out),
                                    ctypes.byref(out_len), _p(ph), prefix, len(prefix))
    if r < 0:
        raise ValueError(lib().fc_last_error().decode())
    try:
        data = ctypes.string_at(out.value, out_len.value)
    finally:
        lib().fc_free(out)
    if phases is not None:
        prev = 0.0
        for name, v in zip(PHASES, ph):
            phases[name] = float(v) - prev
            prev = float(v)
    return data


def verifier_stark(*args, **kwargs):
    """stark_prove_oracle.Stark whose verifier evaluates the transition zerofier
    prod_{i < T-1} (x - omicron^i) at the query points with this library."""
    import stark_prove_oracle as e

    class _Stark(e.Stark):
        def transition_zerofier_at(self, xs):
            return geometric_prod(self.omicron, self.original_trace_length - 1, xs)

    return _Stark(*args, **kwargs)
