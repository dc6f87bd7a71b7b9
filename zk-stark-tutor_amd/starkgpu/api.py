"""Host-side mirror of the reference's hot-path API over libstarkgpu's C ABI.

Names, argument meaning and error behaviour follow the reference crate
(SpekalsG3/zk-stark-tutor, src/): `ntt`/`intt` (fft/ntt.rs:7-68),
`fast_coset_evaluate` (fft/ntt_arithmetics.rs:161-170), `MerkleRoot`
(merkle_root.rs:21-95), the proof streams (proof_stream.rs:15-78,
rescue_prime/proof_stream.rs:9-61, stark/proof_stream_enum.rs) and `FRI`
(fri.rs:13-248).  Where the reference panics, these raise `StarkGpuError`
(or `ValueError` for arguments rejected before the library is called).

Field elements cross the boundary as numpy uint64 arrays of shape (n, 2) =
(lo, hi) little-endian limbs of the canonical value; Python ints are accepted
and converted.  Every compute call runs the HIP kernels; there is no CPU path.
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from ._lib import (PUSH_CB, FS_CB, StarkGpuError, lib, sg_fe, sg_fri, sg_proof_stream)

FIELD_PRIME = 1 + 407 * (1 << 119)
MASK64 = (1 << 64) - 1
PROOF_BYTES = 32

ROOT, CODEWORD, PATH, LEAFS, VALUE = 0, 1, 2, 3, 4

FeArray = np.ndarray


# ------------------------------------------------------------------ conversions

def fe_array(values: Union[Sequence[int], np.ndarray]) -> np.ndarray:
    """Python ints (canonical) -> contiguous uint64 array of shape (n, 2)."""
    if isinstance(values, np.ndarray):
        arr = np.ascontiguousarray(values, dtype=np.uint64)
        if arr.ndim != 2 or arr.shape[1] != 2:
            raise ValueError("field-element arrays have shape (n, 2)")
        return arr
    vals = list(values)
    arr = np.empty((len(vals), 2), dtype=np.uint64)
    for i, v in enumerate(vals):
        v = int(v)
        arr[i, 0] = v & MASK64
        arr[i, 1] = v >> 64
    return arr


def to_ints(arr: np.ndarray) -> List[int]:
    """(n, 2) uint64 array -> list of Python ints."""
    lo = arr[:, 0].tolist()
    hi = arr[:, 1].tolist()
    return [(h << 64) | l for l, h in zip(lo, hi)]


def _fe(v: int) -> sg_fe:
    v = int(v)
    if not 0 <= v < FIELD_PRIME:
        raise ValueError("field element must be canonical (0 <= v < p)")
    return sg_fe(v & MASK64, v >> 64)


def _int(f: sg_fe) -> int:
    return (int(f.hi) << 64) | int(f.lo)


def _ptr(arr: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(arr.ctypes.data)


def _u8(data: bytes):
    buf = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data if data else b"\0")
    return buf


# ------------------------------------------------------------------ context

class Context:
    """One libstarkgpu context (device + stream + buffer pool + twiddle cache)."""

    _default = {}

    def __init__(self, device: int = 0):
        self._lib = lib()
        h = ctypes.c_void_p()
        rc = self._lib.sg_ctx_create(device, ctypes.byref(h))
        if rc != 0:
            raise StarkGpuError(rc, f"sg_ctx_create(device={device}) failed")
        self.handle = h
        self.device = device

    @classmethod
    def default(cls, device: int = 0) -> "Context":
        if device not in cls._default:
            cls._default[device] = Context(device)
        return cls._default[device]

    def check(self, rc: int) -> None:
        if rc != 0:
            raise StarkGpuError(rc, self._lib.sg_last_error(self.handle).decode(errors="replace"))

    @property
    def stream(self) -> int:
        return self._lib.sg_ctx_stream(self.handle) or 0

    def set_async(self, enable: bool) -> None:
        """_dev transforms return once enqueued (stream-ordered); call synchronize() before reading."""
        self.check(self._lib.sg_ctx_set_async(self.handle, int(enable)))

    def synchronize(self) -> None:
        self.check(self._lib.sg_ctx_synchronize(self.handle))

    def profile(self, enable: bool) -> None:
        """Start (resetting totals) or stop per-kernel HIP-event timing."""
        self.check(self._lib.sg_ctx_profile(self.handle, 1 if enable else 0))

    def profile_only(self, kernel: Optional[str]) -> None:
        """Time only launches of `kernel` (None = all)."""
        self.check(self._lib.sg_ctx_profile_only(self.handle, (kernel or "").encode()))

    def profile_report(self) -> dict:
        """{kernel: {"launches", "ms", "bytes"}} accumulated since profile(True)."""
        import json
        n = ctypes.c_size_t()
        self.check(self._lib.sg_ctx_profile_report(self.handle, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        self.check(self._lib.sg_ctx_profile_report(self.handle, buf, n.value, ctypes.byref(n)))
        return json.loads(buf.value.decode())

    def trim(self) -> None:
        self.check(self._lib.sg_ctx_trim(self.handle))

    def set_option(self, name: str, value) -> None:
        """sg_ctx_set_option: "domain_cache", "air_generic", "geo_decimate", "lean_trees", "stream_pin",
        "world1_sharded", "lean_drop" -- equivalent paths (same proof bytes) that the tests compare."""
        self.check(self._lib.sg_ctx_set_option(self.handle, name.encode(), int(value)))

    @contextlib.contextmanager
    def option(self, name: str, value, default):
        """set_option(name, value) for a `with` block, then back to `default`."""
        self.set_option(name, value)
        try:
            yield self
        finally:
            self.set_option(name, default)

    def cached_tables(self) -> Tuple[int, int]:
        """(public domain / AIR tables, twiddle tables) the context keeps (sg_ctx_cached_tables)."""
        d, t = ctypes.c_size_t(), ctypes.c_size_t()
        self.check(self._lib.sg_ctx_cached_tables(self.handle, ctypes.byref(d), ctypes.byref(t)))
        return d.value, t.value

    def memory(self, reset_peak: bool = False) -> dict:
        """Device memory (sg_ctx_memory): the buffer pool's bytes in use, their high-water mark since
        creation or the last reset, the pool's cached free bytes, and hipMemGetInfo's used / total."""
        v = [ctypes.c_uint64() for _ in range(5)]
        self.check(self._lib.sg_ctx_memory(self.handle, *[ctypes.byref(x) for x in v], int(reset_peak)))
        return dict(zip(("live", "peak", "pooled", "device_used", "device_total"), (x.value for x in v)))

    def hbm_copy_gbs(self, nbytes: int = 1 << 30, iters: int = 10, blocks: int = 0) -> float:
        """Read + write GB/s of the library's dwordx4 streaming copy kernel (best of `iters`)."""
        out = ctypes.c_double()
        self.check(self._lib.sg_hbm_copy_probe(self.handle, nbytes, iters, blocks, ctypes.byref(out)))
        return out.value

    def close(self) -> None:
        if self.handle:
            self._lib.sg_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostContext(Context):
    """No device: a NULL context for the host-only entry points (Rescue-Prime constants /
    hash / trace, MPolynomial arithmetic on small polynomials, Stark sizing and degree
    bounds).  Device entry points reject it with "a GPU context is required"."""

    def __init__(self):  # noqa: super().__init__ would open a device
        self._lib = lib()
        self.handle = None
        self.device = -1

    def close(self) -> None:
        pass


def _ctx(ctx: Optional[Context]) -> Context:
    return ctx if ctx is not None else Context.default()


# ------------------------------------------------------------------ field

def generator() -> int:
    """field/field.rs:41-44 Field::generator."""
    return _int(lib().sg_field_generator())


def primitive_nth_root(n: int) -> int:
    """field/field.rs:58-71 Field::primitive_nth_root."""
    if n <= 0 or n & (n - 1) or n > (1 << 119):
        raise ValueError("Field does not have any roots where n > 2^119 or not a power of two.")
    if n > (1 << 63):
        raise ValueError("n above 2^63 is not supported by the C ABI")
    out = sg_fe()
    rc = lib().sg_primitive_nth_root(n, ctypes.byref(out))
    if rc != 0:
        raise StarkGpuError(rc, "primitive_nth_root")
    return _int(out)


def sample(data: bytes) -> int:
    """field/field.rs:87-99 Field::sample."""
    return _int(lib().sg_field_sample(_u8(data), len(data)))


def fe_mul(a: int, b: int) -> int:
    return _int(lib().sg_fe_mul(_fe(a), _fe(b)))


def fe_inverse(a: int) -> int:
    return _int(lib().sg_fe_inverse(_fe(a)))


def fe_pow(a: int, e: int) -> int:
    return _int(lib().sg_fe_pow(_fe(a), e))


# ------------------------------------------------------------------ transforms

def _next_pow2(n: int) -> int:
    return 1 if n <= 1 else 1 << (n - 1).bit_length()


def ntt(root: int, inputs, ctx: Optional[Context] = None) -> np.ndarray:
    """fft/ntt.rs:7-49: NTT with `root`; zero-pads to the next power of two."""
    c = _ctx(ctx)
    x = fe_array(inputs)
    if len(x) == 0:
        raise ValueError("ntt of empty input (reference indexes inputs[0])")
    out = np.empty((_next_pow2(len(x)), 2), dtype=np.uint64)
    c.check(c._lib.sg_ntt(c.handle, _fe(root), _ptr(x), len(x), _ptr(out)))
    return out


def intt(root: int, inputs, ctx: Optional[Context] = None) -> np.ndarray:
    """fft/ntt.rs:51-68: inverse NTT (root^-1, then * n^-1); len < 2 returns the input."""
    c = _ctx(ctx)
    x = fe_array(inputs)
    n_out = len(x) if len(x) < 2 else _next_pow2(len(x))
    out = np.empty((n_out, 2), dtype=np.uint64)
    c.check(c._lib.sg_intt(c.handle, _fe(root), _ptr(x), len(x), _ptr(out)))
    return out


def fast_coset_evaluate(generator_: int, root_order: int, offset: int, coeffs,
                        ctx: Optional[Context] = None) -> np.ndarray:
    """fft/ntt_arithmetics.rs:161-170: the LDE P(offset * generator^k), k < root_order."""
    c = _ctx(ctx)
    x = fe_array(coeffs)
    if len(x) > root_order:
        raise ValueError("polynomial longer than root_order (reference panics)")
    out = np.empty((_next_pow2(root_order), 2), dtype=np.uint64)
    c.check(c._lib.sg_fast_coset_evaluate(c.handle, _fe(generator_), root_order, _fe(offset), _ptr(x), len(x),
                                          _ptr(out)))
    return out


# device-resident variants: pointers are device addresses (e.g. torch.Tensor.data_ptr())

def ntt_dev(root: int, d_in: int, n_in: int, d_out: int, ctx: Optional[Context] = None) -> None:
    c = _ctx(ctx)
    c.check(c._lib.sg_ntt_dev(c.handle, _fe(root), ctypes.c_void_p(d_in), n_in, ctypes.c_void_p(d_out)))


def intt_dev(root: int, d_in: int, n_in: int, d_out: int, ctx: Optional[Context] = None) -> None:
    c = _ctx(ctx)
    c.check(c._lib.sg_intt_dev(c.handle, _fe(root), ctypes.c_void_p(d_in), n_in, ctypes.c_void_p(d_out)))


def fast_coset_evaluate_dev(generator_: int, root_order: int, offset: int, d_coeffs: int, d: int, d_out: int,
                            ctx: Optional[Context] = None) -> None:
    c = _ctx(ctx)
    c.check(c._lib.sg_fast_coset_evaluate_dev(c.handle, _fe(generator_), root_order, _fe(offset),
                                              ctypes.c_void_p(d_coeffs), d, ctypes.c_void_p(d_out)))


def fast_coset_evaluate_batch_dev(generator_: int, root_order: int, offset: int, d_coeffs: Sequence[int], d: int,
                                  d_outs: Sequence[int], ctx: Optional[Context] = None) -> None:
    """Up to 4 LDEs with the same (generator, root_order, offset) in one launch sequence."""
    c = _ctx(ctx)
    k = len(d_coeffs)
    ins = (ctypes.c_void_p * k)(*d_coeffs)
    outs = (ctypes.c_void_p * k)(*d_outs)
    c.check(c._lib.sg_fast_coset_evaluate_batch_dev(c.handle, _fe(generator_), root_order, _fe(offset), ins, d,
                                                    outs, k))


# ------------------------------------------------------------------ Merkle

class MerkleRoot:
    """merkle_root.rs: leaf = blake2b512(decimal(v)), node = blake2b512(L || R)."""

    @staticmethod
    def commit(leafs, ctx: Optional[Context] = None) -> bytes:
        c = _ctx(ctx)
        x = fe_array(leafs)
        root = (ctypes.c_uint8 * 64)()
        c.check(c._lib.sg_merkle_commit(c.handle, _ptr(x), len(x), root))
        return bytes(root)

    @staticmethod
    def open(index: int, leafs, ctx: Optional[Context] = None) -> List[bytes]:
        c = _ctx(ctx)
        x = fe_array(leafs)
        depth = max(len(x).bit_length() - 1, 0)
        buf = (ctypes.c_uint8 * (64 * max(depth, 1)))()
        plen = ctypes.c_size_t()
        c.check(c._lib.sg_merkle_open(c.handle, index, _ptr(x), len(x), buf, ctypes.byref(plen)))
        raw = bytes(buf)
        return [raw[64 * i:64 * i + 64] for i in range(plen.value)]

    @staticmethod
    def verify(root: bytes, index: int, path: Sequence[bytes], leaf: int) -> bool:
        raw = b"".join(path)
        rc = lib().sg_merkle_verify(_u8(root), index, _u8(raw), len(path), _fe(leaf))
        if rc < 0:
            raise StarkGpuError(rc, "Cannot verify invalid index")
        return rc == 1


class DeviceTree:
    """A retained device Merkle tree (build once, open in O(log n))."""

    def __init__(self, d_leaves: int, n: int, ctx: Optional[Context] = None, _handle=None):
        self.ctx = _ctx(ctx)
        self.n = n
        if _handle is not None:
            self.handle = _handle
            return
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx._lib.sg_merkle_build_dev(self.ctx.handle, ctypes.c_void_p(d_leaves), n,
                                                         ctypes.byref(h)))
        self.handle = h

    @classmethod
    def build_batch(cls, d_leaves: Sequence[int], n: int, ctx: Optional[Context] = None) -> List["DeviceTree"]:
        """Up to 4 equal-size trees built in one launch sequence."""
        c = _ctx(ctx)
        k = len(d_leaves)
        ins = (ctypes.c_void_p * k)(*d_leaves)
        outs = (ctypes.c_void_p * k)()
        c.check(c._lib.sg_merkle_build_batch_dev(c.handle, ins, n, k, outs))
        return [cls(0, n, ctx=c, _handle=ctypes.c_void_p(outs[i])) for i in range(k)]

    def root(self) -> bytes:
        r = (ctypes.c_uint8 * 64)()
        self.ctx.check(self.ctx._lib.sg_tree_root(self.handle, r))
        return bytes(r)

    def open(self, index: int) -> List[bytes]:
        depth = max(self.n.bit_length() - 1, 1)
        buf = (ctypes.c_uint8 * (64 * depth))()
        plen = ctypes.c_size_t()
        self.ctx.check(self.ctx._lib.sg_tree_open(self.ctx.handle, self.handle, index, buf, ctypes.byref(plen)))
        raw = bytes(buf)
        return [raw[64 * i:64 * i + 64] for i in range(plen.value)]

    def free(self) -> None:
        if self.handle:
            self.ctx._lib.sg_tree_free(self.ctx.handle, self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ------------------------------------------------------------------ proof streams

def _u128be(v: int) -> bytes:
    return int(v).to_bytes(16, "big")


def encode_object(obj) -> Tuple[int, bytes]:
    """StarkProofStreamEnum::to_bytes (stark/proof_stream_enum.rs:67-127)."""
    code, val = obj
    if code == ROOT:
        return ROOT, bytes(val)
    if code == CODEWORD:
        return CODEWORD, b"".join(_u128be(v) for v in val)
    if code == PATH:
        return PATH, b"".join(len(b).to_bytes(8, "big") + bytes(b) for b in val)
    if code == LEAFS:
        return LEAFS, b"".join(_u128be(v) for v in val)
    if code == VALUE:
        return VALUE, _u128be(val)
    raise ValueError("Unknown code")


def decode_object(code: int, payload: bytes):
    """StarkProofStreamEnum::from_bytes (stark/proof_stream_enum.rs:18-65)."""
    if code == ROOT:
        return (ROOT, payload)
    if code == CODEWORD:
        return (CODEWORD, [int.from_bytes(payload[i:i + 16], "big") for i in range(0, len(payload), 16)])
    if code == PATH:
        out, pos = [], 0
        while pos + 8 <= len(payload):
            sz = int.from_bytes(payload[pos:pos + 8], "big")
            out.append(payload[pos + 8:pos + 8 + sz])
            pos += 8 + sz
        return (PATH, out)
    if code == LEAFS:
        vals = [int.from_bytes(payload[i:i + 16], "big") for i in range(0, 48, 16)]
        return (LEAFS, tuple(vals))
    if code == VALUE:
        return (VALUE, int.from_bytes(payload, "big"))
    raise ValueError("Unknown code")


_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]


class IndependentProofStream:
    """proof_stream.rs:15-78, held natively by the library (byte-exact digest)."""

    def __init__(self, _handle=None):
        self._lib = lib()
        self.handle = _handle if _handle is not None else self._lib.sg_stream_create()
        if not self.handle:
            raise StarkGpuError(-5, "sg_stream_create failed")

    @classmethod
    def deserialize(cls, data: bytes) -> "IndependentProofStream":
        """stark/stark.rs:30-67 deser_independent_proof_stream."""
        h = ctypes.c_void_p()
        rc = lib().sg_stream_deserialize(_u8(data), len(data), ctypes.byref(h))
        if rc != 0:
            raise StarkGpuError(rc, "malformed proof stream")
        return cls(h.value)

    def push(self, obj) -> None:
        code, payload = encode_object(obj)
        rc = self._lib.sg_stream_push(self.handle, code, _u8(payload), len(payload))
        if rc != 0:
            raise StarkGpuError(rc, "push")

    def pull(self):
        code = ctypes.c_uint8()
        p = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        rc = self._lib.sg_stream_pull(self.handle, ctypes.byref(code), ctypes.byref(p), ctypes.byref(n))
        if rc != 0:
            raise StarkGpuError(rc, "Cannot pull, queue is empty")
        return decode_object(code.value, ctypes.string_at(p, n.value) if n.value else b"")

    def __len__(self) -> int:
        return self._lib.sg_stream_count(self.handle)

    def digest(self) -> bytes:
        n = ctypes.c_size_t()
        rc = self._lib.sg_stream_digest(self.handle, None, 0, ctypes.byref(n))
        if rc != 0:
            raise StarkGpuError(rc, "digest")
        # serialize straight into a fresh bytes object (one allocation, one pass)
        out = _new_bytes(None, n.value)
        rc = self._lib.sg_stream_digest(self.handle, ctypes.cast(ctypes.c_char_p(out), ctypes.c_void_p), n.value,
                                        ctypes.byref(n))
        if rc != 0:
            raise StarkGpuError(rc, "digest")
        return out

    def fiat_shamir_prover(self, num_bytes: int) -> bytes:
        buf = (ctypes.c_uint8 * max(num_bytes, 1))()
        self._lib.sg_stream_fiat_shamir_prover(self.handle, num_bytes, buf)
        return bytes(buf)[:num_bytes]

    def fiat_shamir_verifier(self, num_bytes: int) -> bytes:
        buf = (ctypes.c_uint8 * max(num_bytes, 1))()
        self._lib.sg_stream_fiat_shamir_verifier(self.handle, num_bytes, buf)
        return bytes(buf)[:num_bytes]

    def objects(self) -> list:
        """All objects, decoded (does not move the read index)."""
        data = self.digest()
        pos, out = 16, []
        while pos < len(data):
            code = data[pos]
            sz = int.from_bytes(data[pos + 1:pos + 9], "big")
            out.append(decode_object(code, data[pos + 9:pos + 9 + sz]))
            pos += 9 + sz
        return out

    def callbacks(self) -> sg_proof_stream:
        return self._lib.sg_stream_callbacks(self.handle)

    def __del__(self):
        try:
            if self.handle:
                self._lib.sg_stream_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class SignatureProofStream(IndependentProofStream):
    """rescue_prime/proof_stream.rs:9-61: Fiat-Shamir prefixed by blake2b(document)."""

    def __init__(self, document: bytes):
        h = lib().sg_stream_create_signature(_u8(document), len(document))
        super().__init__(h)


class CallbackProofStream:
    """Adapter for any Python object with push(obj) / fiat_shamir_prover(n) (proof_stream.rs:6-12)."""

    def __init__(self, inner):
        self.inner = inner
        self.error = None

        def _push(user, code, payload, n):
            try:
                self.inner.push(decode_object(code, ctypes.string_at(payload, n) if n else b""))
                return 0
            except Exception as e:  # surfaces as SG_ERR_CALLBACK
                self.error = e
                return 1

        def _fs(user, n, out):
            try:
                b = self.inner.fiat_shamir_prover(n)
                ctypes.memmove(out, b, n)
                return 0
            except Exception as e:
                self.error = e
                return 1

        self._push = PUSH_CB(_push)
        self._fs = FS_CB(_fs)

    def callbacks(self) -> sg_proof_stream:
        return sg_proof_stream(None, self._push, self._fs)


# ------------------------------------------------------------------ FRI

class FRI:
    """fri.rs:13-248 on the GPU (commit, prove); the verifier side stays on the host."""

    def __init__(self, offset: int, omega: int, domain_length: int, expansion_factor: int,
                 num_colinearity_tests: int, ctx: Optional[Context] = None):
        self.offset = offset
        self.omega = omega
        self.domain_length = domain_length
        self.expansion_factor = expansion_factor
        self.num_colinearity_tests = num_colinearity_tests
        self.ctx = _ctx(ctx)
        self._p = sg_fri(_fe(offset), _fe(omega), domain_length, expansion_factor, num_colinearity_tests)

    def num_rounds(self) -> int:
        return lib().sg_fri_num_rounds(ctypes.byref(self._p))

    @staticmethod
    def sample_indices(seed: bytes, size: int, reduced_size: int, number: int) -> List[int]:
        out = (ctypes.c_size_t * max(number, 1))()
        rc = lib().sg_fri_sample_indices(_u8(seed), len(seed), size, reduced_size, number, out)
        if rc != 0:
            raise StarkGpuError(rc, "sample_indices: invalid arguments")
        return list(out)[:number]

    def _stream(self, proof_stream):
        if isinstance(proof_stream, IndependentProofStream):
            return proof_stream.callbacks(), None
        adapter = CallbackProofStream(proof_stream)
        return adapter.callbacks(), adapter

    def commit(self, codeword, proof_stream) -> None:
        """fri.rs:115-172 (pushes the roots and the last codeword)."""
        x = fe_array(codeword)
        cb, adapter = self._stream(proof_stream)
        rc = self.ctx._lib.sg_fri_commit(self.ctx.handle, ctypes.byref(self._p), _ptr(x), len(x),
                                         ctypes.byref(cb), None)
        if adapter is not None and adapter.error is not None:
            raise adapter.error
        self.ctx.check(rc)

    def prove(self, codeword, proof_stream) -> List[int]:
        """fri.rs:210-248: returns the top-level indices."""
        x = fe_array(codeword)
        cb, adapter = self._stream(proof_stream)
        out = (ctypes.c_size_t * max(self.num_colinearity_tests, 1))()
        rc = self.ctx._lib.sg_fri_prove(self.ctx.handle, ctypes.byref(self._p), _ptr(x), len(x),
                                        ctypes.byref(cb), out)
        if adapter is not None and adapter.error is not None:
            raise adapter.error
        self.ctx.check(rc)
        return list(out)[:self.num_colinearity_tests]

    def commit_dev(self, d_codeword: int, n: int, proof_stream) -> None:
        cb, adapter = self._stream(proof_stream)
        rc = self.ctx._lib.sg_fri_commit_dev(self.ctx.handle, ctypes.byref(self._p), ctypes.c_void_p(d_codeword), n,
                                             ctypes.byref(cb), None)
        if adapter is not None and adapter.error is not None:
            raise adapter.error
        self.ctx.check(rc)

    def prove_dev(self, d_codeword: int, n: int, proof_stream) -> List[int]:
        cb, adapter = self._stream(proof_stream)
        out = (ctypes.c_size_t * max(self.num_colinearity_tests, 1))()
        rc = self.ctx._lib.sg_fri_prove_dev(self.ctx.handle, ctypes.byref(self._p), ctypes.c_void_p(d_codeword), n,
                                            ctypes.byref(cb), out)
        if adapter is not None and adapter.error is not None:
            raise adapter.error
        self.ctx.check(rc)
        return list(out)[:self.num_colinearity_tests]
