"""ctypes wrapper of oracle/ref_cpu.c (reference-faithful C restatement).

TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline leg).  Build with
`make -C oracle` (done by __graft_entry__.build()).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libref_cpu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        l = ctypes.CDLL(LIB_PATH)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        l.ora_ntt.argtypes = [vp, vp, sz, vp]
        l.ora_intt.argtypes = [vp, vp, sz, vp]
        l.ora_coset_evaluate.argtypes = [vp, ctypes.c_uint64, vp, vp, sz, vp]
        l.ora_coset_evaluate.restype = ctypes.c_int
        l.ora_merkle_commit.argtypes = [vp, sz, vp]
        l.ora_merkle_commit.restype = ctypes.c_int
        l.ora_blake2b512.argtypes = [vp, sz, vp]
        l.ora_shake256.argtypes = [vp, sz, vp, sz]
        l.ora_fri_commit.argtypes = [vp, vp, vp, sz, sz, sz, vp, sz, vp, sz, vp, vp]
        l.ora_fri_commit.restype = ctypes.c_long
        l.ora_merkle_open.argtypes = [sz, vp, sz, vp]
        l.ora_merkle_open.restype = ctypes.c_long
        _lib = l
    return _lib


def _fe2(v: int) -> np.ndarray:
    return np.array([v & ((1 << 64) - 1), v >> 64], dtype=np.uint64)


def _arr(values) -> np.ndarray:
    if isinstance(values, np.ndarray):
        return np.ascontiguousarray(values, dtype=np.uint64)
    vals = list(values)
    a = np.empty((len(vals), 2), dtype=np.uint64)
    for i, v in enumerate(vals):
        a[i, 0] = v & ((1 << 64) - 1)
        a[i, 1] = v >> 64
    return a


def _p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def _next_pow2(n):
    return 1 if n <= 1 else 1 << (n - 1).bit_length()


def ntt(root, values) -> np.ndarray:
    x = _arr(values)
    out = np.empty((_next_pow2(len(x)), 2), dtype=np.uint64)
    r = _fe2(root)
    lib().ora_ntt(_p(r), _p(x), len(x), _p(out))
    return out


def intt(root, values) -> np.ndarray:
    x = _arr(values)
    out = np.empty((_next_pow2(len(x)) if len(x) > 1 else len(x), 2), dtype=np.uint64)
    r = _fe2(root)
    lib().ora_intt(_p(r), _p(x), len(x), _p(out))
    return out


def fast_coset_evaluate(generator, root_order, offset, coeffs) -> np.ndarray:
    c = _arr(coeffs) if len(coeffs) else np.zeros((1, 2), dtype=np.uint64)
    out = np.empty((_next_pow2(root_order), 2), dtype=np.uint64)
    g, o = _fe2(generator), _fe2(offset)
    if lib().ora_coset_evaluate(_p(g), root_order, _p(o), _p(c), len(coeffs), _p(out)) != 0:
        raise ValueError("polynomial longer than root_order")
    return out


def merkle_commit(values) -> bytes:
    x = _arr(values)
    root = (ctypes.c_uint8 * 64)()
    if lib().ora_merkle_commit(_p(x), len(x), root) != 0:
        raise ValueError("Leafs len must be power of two")
    return bytes(root)


def fri_commit(offset, omega, codeword, expansion, colinearity, prefix=bytes(16), want_codewords=False):
    """fri.rs:115-172 from a serialized stream prefix; returns (stream bytes, roots[, codewords])."""
    x = _arr(codeword)
    n = len(x)
    rounds, ln = 0, n
    while ln > expansion and ln > 4 * colinearity:
        ln //= 2
        rounds += 1
    cap = len(prefix) + 73 * rounds + 9 + 16 * n + 64
    out = (ctypes.c_uint8 * cap)()
    roots = (ctypes.c_uint8 * (64 * max(rounds, 1)))()
    pre = (ctypes.c_uint8 * len(prefix)).from_buffer_copy(prefix)
    o, w = _fe2(offset), _fe2(omega)
    cws = np.zeros((2 * n, 2), dtype=np.uint64) if want_codewords else None
    ln = lib().ora_fri_commit(_p(o), _p(w), _p(x), n, expansion, colinearity, pre, len(prefix), out, cap, roots,
                              _p(cws) if want_codewords else None)
    if ln < 0:
        raise ValueError("fri commit rejected its arguments")
    rb = bytes(roots)
    res = (bytes(out)[:ln], [rb[64 * i:64 * i + 64] for i in range(rounds)])
    if not want_codewords:
        return res
    parts, pos, ln2 = [], 0, n
    for _ in range(rounds):
        parts.append(cws[pos:pos + ln2])
        pos += ln2
        ln2 //= 2
    return res + (parts,)


def merkle_open(index, values):
    """merkle_root.rs:55-66 with the reference's O(n) recomputation per call."""
    x = _arr(values)
    depth = max(len(x).bit_length() - 1, 1)
    buf = (ctypes.c_uint8 * (64 * depth))()
    n = lib().ora_merkle_open(index, _p(x), len(x), buf)
    if n < 0:
        raise ValueError("invalid open")
    b = bytes(buf)
    return [b[64 * i:64 * i + 64] for i in range(n)]
