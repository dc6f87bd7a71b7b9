"""MPolynomial, RescuePrime and Stark over libstarkgpu (m_polynomial.rs,
rescue_prime/rescue_prime.rs, stark/stark.rs).

Same names and argument meaning as the reference; `Stark.prove` takes the two
thread_rng draws (trace randomizer rows, randomizer polynomial coefficients) as
explicit arguments and returns the proof stream's digest() like the reference's
`Ok(Bytes)`; where the reference returns `Err(String)` this raises
`StarkGpuError` with the same text.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ._lib import StarkGpuError, sg_fe, sg_fri
from .api import (CallbackProofStream, Context, IndependentProofStream, _ctx, _fe, _int, _ptr, fe_array, to_ints)


class sg_boundary(ctypes.Structure):
    _fields_ = [("cycle", ctypes.c_uint64), ("reg", ctypes.c_uint64), ("value", sg_fe)]


class MPolynomial:
    """m_polynomial.rs MPolynomial (grouped by register exponents in the library)."""

    def __init__(self, handle, ctx: Context):
        self.handle = handle
        self.ctx = ctx

    @classmethod
    def _make(cls, c: Context, fn, *args) -> "MPolynomial":
        h = ctypes.c_void_p()
        c.check(fn(c.handle, *args, ctypes.byref(h)))
        return cls(h, c)

    @classmethod
    def new(cls, dictionary: Dict[Tuple[int, ...], int], ctx: Optional[Context] = None) -> "MPolynomial":
        """MPolynomial::new({exponents: coefficient}) (all keys of one length)."""
        c = _ctx(ctx)
        keys = list(dictionary)
        nv = len(keys[0]) if keys else 0
        if any(len(k) != nv for k in keys):
            raise ValueError("all exponent vectors must have the same length")
        exps = (ctypes.c_uint32 * max(nv * len(keys), 1))(*[e for k in keys for e in k])
        coeffs = fe_array([dictionary[k] for k in keys])
        return cls._make(c, c._lib.sg_mpoly_create, nv, len(keys), exps, _ptr(coeffs))

    @classmethod
    def constant(cls, v: int, ctx: Optional[Context] = None) -> "MPolynomial":
        c = _ctx(ctx)
        return cls._make(c, c._lib.sg_mpoly_constant, _fe(v))

    @classmethod
    def variables(cls, n: int, ctx: Optional[Context] = None) -> List["MPolynomial"]:
        c = _ctx(ctx)
        return [cls._make(c, c._lib.sg_mpoly_variable, n, i) for i in range(n)]

    @classmethod
    def lift(cls, coeffs, variable_index: int, ctx: Optional[Context] = None) -> "MPolynomial":
        c = _ctx(ctx)
        x = fe_array(coeffs)
        return cls._make(c, c._lib.sg_mpoly_lift, _ptr(x), len(x), variable_index)

    def __neg__(self):
        return self._make(self.ctx, self.ctx._lib.sg_mpoly_neg, self.handle)

    def __add__(self, o):
        return self._make(self.ctx, self.ctx._lib.sg_mpoly_add, self.handle, o.handle)

    def __sub__(self, o):
        return self._make(self.ctx, self.ctx._lib.sg_mpoly_sub, self.handle, o.handle)

    def __mul__(self, o):
        return self._make(self.ctx, self.ctx._lib.sg_mpoly_mul, self.handle, o.handle)

    def __pow__(self, e: int):
        """m_polynomial.rs:265-298 (u128 exponent)."""
        return self._make(self.ctx, self.ctx._lib.sg_mpoly_pow, self.handle, _fe_u128(e))

    def is_zero(self) -> bool:
        return self.ctx._lib.sg_mpoly_is_zero(self.handle) == 1

    def evaluate(self, point: Sequence[int]) -> int:
        x = fe_array(point)
        out = sg_fe()
        self.ctx.check(self.ctx._lib.sg_mpoly_evaluate(self.ctx.handle, self.handle, _ptr(x), len(x),
                                                       ctypes.byref(out)))
        return _int(out)

    def groups(self) -> Tuple[int, Dict[Tuple[int, ...], List[int]]]:
        """(nvars, {register exponents: dense coefficients in variable 0})."""
        nv, ng, nc = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        self.ctx._lib.sg_mpoly_shape(self.handle, ctypes.byref(nv), ctypes.byref(ng), ctypes.byref(nc))
        k = max(nv.value - 1, 0)
        exps = (ctypes.c_uint32 * max(k * ng.value, 1))()
        lens = (ctypes.c_uint64 * max(ng.value, 1))()
        coeffs = np.empty((max(nc.value, 1), 2), dtype=np.uint64)
        self.ctx._lib.sg_mpoly_export(self.handle, exps, lens, _ptr(coeffs))
        vals = to_ints(coeffs[:nc.value])
        out, pos = {}, 0
        for g in range(ng.value):
            key = tuple(exps[g * k:(g + 1) * k])
            out[key] = vals[pos:pos + lens[g]]
            pos += lens[g]
        return nv.value, out

    def free(self) -> None:
        if self.handle:
            self.ctx._lib.sg_mpoly_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _fe_u128(e: int) -> sg_fe:
    if not 0 <= e < (1 << 128):
        raise ValueError("exponent must fit in 128 bits")
    return sg_fe(e & ((1 << 64) - 1), e >> 64)


class RescuePrime:
    """rescue_prime/rescue_prime.rs RescuePrime (native: constants, trace, AIR)."""

    def __init__(self, m: int, capacity: int, security_level: int, N: int, ctx: Optional[Context] = None):
        self.ctx = _ctx(ctx)
        self.m, self.capacity, self.security_level, self.N = m, capacity, security_level, N
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx._lib.sg_rescue_create(self.ctx.handle, m, capacity, security_level, N,
                                                      ctypes.byref(h)))
        self.handle = h
        a, ai = sg_fe(), sg_fe()
        mds = np.empty((m * m, 2), dtype=np.uint64)
        mdsi = np.empty((m * m, 2), dtype=np.uint64)
        rc = np.empty((max(2 * m * N, 1), 2), dtype=np.uint64)
        self.ctx._lib.sg_rescue_info(self.handle, ctypes.byref(a), ctypes.byref(ai), _ptr(mds), _ptr(mdsi), _ptr(rc))
        self.alpha, self.alpha_inv = _int(a), _int(ai)
        flat, flati = to_ints(mds), to_ints(mdsi)
        self.MDS = [flat[i * m:(i + 1) * m] for i in range(m)]
        self.MDS_inv = [flati[i * m:(i + 1) * m] for i in range(m)]
        self.round_constants = to_ints(rc[:2 * m * N])

    def hash(self, x: int) -> int:
        out = sg_fe()
        self.ctx.check(self.ctx._lib.sg_rescue_hash(self.ctx.handle, self.handle, _fe(x), ctypes.byref(out)))
        return _int(out)

    def trace(self, x: int) -> List[List[int]]:
        t = np.empty(((self.N + 1) * self.m, 2), dtype=np.uint64)
        self.ctx.check(self.ctx._lib.sg_rescue_trace(self.ctx.handle, self.handle, _fe(x), _ptr(t)))
        flat = to_ints(t)
        return [flat[i * self.m:(i + 1) * self.m] for i in range(self.N + 1)]

    def trace_array(self, x: int) -> np.ndarray:
        """The trace as an ((N+1) * m, 2) uint64 array (row-major), without Python ints."""
        t = np.empty(((self.N + 1) * self.m, 2), dtype=np.uint64)
        self.ctx.check(self.ctx._lib.sg_rescue_trace(self.ctx.handle, self.handle, _fe(x), _ptr(t)))
        return t

    def transition_constraints(self, omicron: int, omicron_domain_length: int) -> List[MPolynomial]:
        out = (ctypes.c_void_p * self.m)()
        self.ctx.check(self.ctx._lib.sg_rescue_transition_constraints(self.ctx.handle, self.handle, _fe(omicron),
                                                                      omicron_domain_length, out))
        return [MPolynomial(ctypes.c_void_p(out[i]), self.ctx) for i in range(self.m)]

    def boundary_constraints(self, output_element: int) -> List[Tuple[int, int, int]]:
        return [(0, 1, 0), (self.N, 0, output_element)]

    def __del__(self):
        try:
            if self.handle:
                self.ctx._lib.sg_rescue_free(self.handle)
                self.handle = None
        except Exception:
            pass


class Stark:
    """stark/stark.rs Stark (the prover on the GPU)."""

    def __init__(self, expansion_factor: int, num_colinearity_checks: int, security_level: int, num_registers: int,
                 num_cycles: int, transition_constraints_degree: int = 2, ctx: Optional[Context] = None):
        self.ctx = _ctx(ctx)
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx._lib.sg_stark_create(self.ctx.handle, expansion_factor, num_colinearity_checks,
                                                     security_level, num_registers, num_cycles,
                                                     transition_constraints_degree, ctypes.byref(h)))
        self.handle = h
        self.expansion_factor = expansion_factor
        self.num_registers = num_registers
        self.original_trace_length = num_cycles
        om, D, fri, nr = sg_fe(), ctypes.c_uint64(), sg_fri(), ctypes.c_size_t()
        self.ctx._lib.sg_stark_params(self.handle, ctypes.byref(om), ctypes.byref(D), ctypes.byref(fri),
                                      ctypes.byref(nr))
        self.omicron = _int(om)
        self.omicron_domain_length = D.value
        self.num_randomizers = nr.value
        self.fri_domain_length = fri.domain_length
        self.omega = _int(fri.omega)

    @staticmethod
    def _tcs(tcs: Sequence[MPolynomial]):
        return (ctypes.c_void_p * max(len(tcs), 1))(*[t.handle.value for t in tcs])

    def max_degree(self, tcs: Sequence[MPolynomial]) -> int:
        out = ctypes.c_uint64()
        self.ctx.check(self.ctx._lib.sg_stark_max_degree(self.ctx.handle, self.handle, self._tcs(tcs), len(tcs),
                                                         ctypes.byref(out)))
        return out.value

    def transition_degree_bounds(self, tcs: Sequence[MPolynomial]) -> List[int]:
        out = (ctypes.c_uint64 * max(len(tcs), 1))()
        self.ctx.check(self.ctx._lib.sg_stark_degree_bounds(self.ctx.handle, self.handle, self._tcs(tcs), len(tcs),
                                                            out))
        return list(out)[:len(tcs)]

    def num_randomizer_coefficients(self, tcs: Sequence[MPolynomial]) -> int:
        return self.max_degree(tcs) + 1

    def _stream(self, proof_stream):
        if isinstance(proof_stream, IndependentProofStream):
            return proof_stream.callbacks(), None
        adapter = CallbackProofStream(proof_stream)
        return adapter.callbacks(), adapter

    def _host_args(self, trace, boundary, trace_randomizers, randomizer_coefficients):
        m = self.num_registers
        if isinstance(trace, np.ndarray):
            t = fe_array(trace)
        else:
            t = fe_array([v for row in trace for v in row])
        tr = fe_array([v for row in trace_randomizers for v in row]) if not isinstance(trace_randomizers, np.ndarray) \
            else fe_array(trace_randomizers)
        rc = fe_array(randomizer_coefficients)
        bnd = (sg_boundary * max(len(boundary), 1))(*[sg_boundary(c, r, _fe(v)) for (c, r, v) in boundary])
        return t, len(t) // m, tr, rc, bnd

    def _finish(self, rcode, adapter):
        if adapter is not None and adapter.error is not None:
            raise adapter.error
        self.ctx.check(rcode)

    def prove(self, trace, transition_constraints: Sequence[MPolynomial], boundary: Sequence[Tuple[int, int, int]],
              proof_stream, trace_randomizers, randomizer_coefficients, dist=None) -> bytes:
        """stark.rs:276-562; `trace` is rows x registers (list of lists or an (rows*m, 2) array).

        With `dist` (a starkgpu.dist.NativeDist whose context this Stark and the constraints were
        created on) the codeword domain is sharded over the communicator (sg_dist_stark_prove):
        every rank calls with the same arguments and gets the single-GPU proof bytes."""
        t, rows, tr, rc, bnd = self._host_args(trace, boundary, trace_randomizers, randomizer_coefficients)
        cb, adapter = self._stream(proof_stream)
        tcs = self._tcs(transition_constraints)
        if dist is None:
            rcode = self.ctx._lib.sg_stark_prove(self.ctx.handle, self.handle, _ptr(t), rows, tcs,
                                                 len(transition_constraints), bnd, len(boundary), _ptr(tr),
                                                 _ptr(rc), len(rc), ctypes.byref(cb))
        else:
            if dist.ctx is not self.ctx:
                raise ValueError("the Stark must be created on the communicator's context")
            dist._torch_ready()
            rcode = self.ctx._lib.sg_dist_stark_prove(dist.handle, self.handle, _ptr(t), rows, tcs,
                                                      len(transition_constraints), bnd, len(boundary), _ptr(tr),
                                                      _ptr(rc), len(rc), ctypes.byref(cb))
        self._finish(rcode, adapter)
        return proof_stream.digest()

    def prove_dev(self, d_trace: int, rows: int, transition_constraints: Sequence[MPolynomial],
                  boundary: Sequence[Tuple[int, int, int]], proof_stream, d_trace_randomizers: int,
                  d_randomizer_coefficients: int, n_randomizer_coefficients: int, dist=None) -> None:
        """prove() with the trace (rows x registers, row-major), the trace randomizers and the
        randomizer coefficients already in device memory (e.g. torch tensor data_ptr())."""
        bnd = (sg_boundary * max(len(boundary), 1))(*[sg_boundary(c, r, _fe(v)) for (c, r, v) in boundary])
        cb, adapter = self._stream(proof_stream)
        args = (self.handle, ctypes.c_void_p(d_trace), rows, self._tcs(transition_constraints),
                len(transition_constraints), bnd, len(boundary), ctypes.c_void_p(d_trace_randomizers),
                ctypes.c_void_p(d_randomizer_coefficients), n_randomizer_coefficients, ctypes.byref(cb))
        if dist is None:
            rcode = self.ctx._lib.sg_stark_prove_dev(self.ctx.handle, *args)
        else:
            if dist.ctx is not self.ctx:
                raise ValueError("the Stark must be created on the communicator's context")
            dist._torch_ready()
            rcode = self.ctx._lib.sg_dist_stark_prove_dev(dist.handle, *args)
        self._finish(rcode, adapter)

    def __del__(self):
        try:
            if self.handle:
                self.ctx._lib.sg_stark_free(self.handle)
                self.handle = None
        except Exception:
            pass
