"""Polynomial algebra over libstarkgpu (fft/ntt_arithmetics.rs, field/polynomial.rs).

`Polynomial` is a device-resident coefficient vector owned by the library
(never trimmed, like the reference's `Polynomial`); the module functions mirror
`fast_multiply`, `fast_zerofier`, `fast_interpolate_domain` and
`fast_coset_divide` (same arguments, same outputs, `StarkGpuError` where the
reference panics).  Every call runs HIP kernels; there is no CPU path.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from .api import Context, _ctx, _fe, _ptr, fe_array, to_ints


class Polynomial:
    """field/polynomial.rs Polynomial held in device memory."""

    def __init__(self, handle, ctx: Context):
        self.handle = handle
        self.ctx = ctx

    @classmethod
    def new(cls, coeffs, ctx: Optional[Context] = None) -> "Polynomial":
        c = _ctx(ctx)
        x = fe_array(coeffs)
        h = ctypes.c_void_p()
        c.check(c._lib.sg_poly_create(c.handle, _ptr(x), len(x), ctypes.byref(h)))
        return cls(h, c)

    @classmethod
    def from_device(cls, d_ptr: int, n: int, ctx: Optional[Context] = None) -> "Polynomial":
        c = _ctx(ctx)
        h = ctypes.c_void_p()
        c.check(c._lib.sg_poly_create_dev(c.handle, ctypes.c_void_p(d_ptr), n, ctypes.byref(h)))
        return cls(h, c)

    def __len__(self) -> int:
        return int(self.ctx._lib.sg_poly_len(self.handle))

    @property
    def data_ptr(self) -> int:
        return int(self.ctx._lib.sg_poly_data_dev(self.handle) or 0)

    def array(self) -> np.ndarray:
        out = np.empty((len(self), 2), dtype=np.uint64)
        self.ctx.check(self.ctx._lib.sg_poly_read(self.ctx.handle, self.handle, _ptr(out)))
        return out

    @property
    def coefficients(self) -> List[int]:
        return to_ints(self.array())

    def degree(self) -> Optional[int]:
        """polynomial.rs:41-58 (None for the zero polynomial)."""
        d = ctypes.c_int64()
        self.ctx.check(self.ctx._lib.sg_poly_degree(self.ctx.handle, self.handle, ctypes.byref(d)))
        return None if d.value < 0 else int(d.value)

    def free(self) -> None:
        if self.handle:
            self.ctx._lib.sg_poly_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _poly_out(c: Context, rc: int, h) -> Polynomial:
    c.check(rc)
    return Polynomial(h, c)


def _as_poly(p, c: Context) -> Polynomial:
    return p if isinstance(p, Polynomial) else Polynomial.new(p, ctx=c)


def fast_multiply(root: int, root_order: int, lhs, rhs, ctx: Optional[Context] = None) -> Polynomial:
    """ntt_arithmetics.rs:5-64."""
    c = _ctx(ctx)
    a, b = _as_poly(lhs, c), _as_poly(rhs, c)
    h = ctypes.c_void_p()
    return _poly_out(c, c._lib.sg_fast_multiply(c.handle, _fe(root), root_order, a.handle, b.handle,
                                                ctypes.byref(h)), h)


def fast_coset_divide(root: int, root_order: int, offset: int, lhs, rhs, ctx: Optional[Context] = None) -> Polynomial:
    """ntt_arithmetics.rs:239-310."""
    c = _ctx(ctx)
    a, b = _as_poly(lhs, c), _as_poly(rhs, c)
    h = ctypes.c_void_p()
    return _poly_out(c, c._lib.sg_fast_coset_divide(c.handle, _fe(root), root_order, _fe(offset), a.handle, b.handle,
                                                    ctypes.byref(h)), h)


def fast_zerofier(root: int, root_order: int, domain: Sequence[int], ctx: Optional[Context] = None) -> Polynomial:
    """ntt_arithmetics.rs:66-113."""
    c = _ctx(ctx)
    d = fe_array(domain)
    h = ctypes.c_void_p()
    return _poly_out(c, c._lib.sg_fast_zerofier(c.handle, _fe(root), root_order, _ptr(d), len(d), ctypes.byref(h)), h)


def fast_interpolate_domain(root: int, root_order: int, domain: Sequence[int], values: Sequence[int],
                            ctx: Optional[Context] = None) -> Polynomial:
    """ntt_arithmetics.rs:172-237."""
    c = _ctx(ctx)
    d, v = fe_array(domain), fe_array(values)
    if len(d) != len(v):
        raise ValueError("number of elements in domain does not match number of values")
    h = ctypes.c_void_p()
    return _poly_out(c, c._lib.sg_fast_interpolate_domain(c.handle, _fe(root), root_order, _ptr(d), _ptr(v), len(d),
                                                          ctypes.byref(h)), h)


def fast_zerofier_geometric(root: int, root_order: int, n: int, ctx: Optional[Context] = None) -> Polynomial:
    """fast_zerofier on the domain root^0 .. root^(n-1)."""
    c = _ctx(ctx)
    h = ctypes.c_void_p()
    return _poly_out(c, c._lib.sg_fast_zerofier_geometric(c.handle, _fe(root), root_order, n, ctypes.byref(h)), h)


def fast_interpolate_geometric_dev(root: int, root_order: int, d_values: int, n: int,
                                   ctx: Optional[Context] = None) -> Polynomial:
    """fast_interpolate_domain on root^0 .. root^(n-1) with device-resident values."""
    c = _ctx(ctx)
    h = ctypes.c_void_p()
    return _poly_out(c, c._lib.sg_fast_interpolate_geometric_dev(c.handle, _fe(root), root_order,
                                                                 ctypes.c_void_p(d_values), n, ctypes.byref(h)), h)
