"""Multi-GPU LDE / NTT / Merkle / FRI over one node: the Python mirror of the
C ABI's sharded path (``sg_dist_*``, csrc/dist.cpp) -- ``NativeDist`` -- plus the host helpers
that scatter / gather its shard layouts.

One process per GPU; the communicator is RCCL over xGMI (the library's own, from a unique id
broadcast over the torch.distributed group) or a host transport over a torch.distributed group
(gloo: several ranks on one GPU).  The reference is single-threaded; the library shards its path
the way the north star asks: the codeword is split across the ranks and the only data exchange of
a transform is ONE all-to-all at the four-step transpose.  (The round-1 composition of the same
algorithm over torch.distributed, ``DistStark``, is a test model now: tests/dist_model.py.)

Four-step decomposition (n = N1 * N2, G ranks, N1 % G == N2 % G == 0):

  input index  j = j1 + N1 * j2         output index  k = k2 + N2 * k1
  X[k2 + N2 k1] = sum_j1 w_N1^(j1 k1) * w^(j1 k2) * sum_j2 w_N2^(j2 k2) x[j1 + N1 j2]

with w_N2 = w^N1 and w_N1 = w^N2.  For a root of order exactly n the DFT is
unique, so the result is bit-identical to the reference's radix-2 DIT
(fft/ntt.rs:7-49); a root of smaller order is rejected (the reference's own
callers always pass primitive roots).

Shard layouts (rank g, R = N2 / G):

  column shard  [N1/G][row]  row r = x[(g N1/G + r) + N1 j2] for j2 < row length
  run shard     [N1][R]      element [k1][c] = X[k1 N2 + g R + c]

The run shard is what the Merkle commit and FRI need: every k1 holds a run of R
consecutive codeword positions, so each rank hashes N1 subtrees of R leaves,
the N1*G run roots are all-gathered (64 B each) and every rank finishes the
(small) top of the tree itself.  The FRI fold pairs i with i + n/2 = same k2,
k1 + N1/2: always on the same rank, so folds are local until one run per rank
is left, after which the (N2-element) codeword is all-gathered and the
remaining rounds run on each rank's GPU.  Every rank computes the same roots,
hence the same Fiat-Shamir challenges, with no broadcast.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import api
from ._lib import StarkGpuError, lib

P = api.FIELD_PRIME
ROOT, CODEWORD = api.ROOT, api.CODEWORD


# ---------------------------------------------------------------- helpers

def _log2(n: int) -> int:
    if n <= 0 or n & (n - 1):
        raise ValueError(f"{n} is not a power of two")
    return n.bit_length() - 1


def plan(n: int, world: int) -> Tuple[int, int]:
    """(N1, N2) for an n-point transform over `world` ranks: N1 = 2^floor(log n / 2) (sg_dist_plan's
    split, csrc/dist.cpp dist_split)."""
    logn = _log2(n)
    _log2(world)
    n1 = 1 << (logn // 2)
    n2 = n // n1
    if n1 % world or n2 % world:
        raise ValueError(f"n = {n} is too small for {world} ranks (needs n >= world^2)")
    return n1, n2


def _check_primitive(root: int, n: int) -> None:
    # order exactly n  <=>  root^(n/2) == -1 (n a power of two >= 2)
    if n >= 2 and api.fe_pow(root, n // 2) != P - 1:
        raise ValueError("distributed ntt needs a root of order exactly n")
    if n == 1 and root % P == 0:
        raise ValueError("root must be non-zero")


def scatter_columns(values: Sequence[int], n: int, world: int, rank: int) -> List[List[int]]:
    """Host helper: rank `rank`'s column shard of a length-<=n vector (zero padded).

    Row r is x[(rank N1/G + r) + N1 j2] for j2 < ceil(len / N1).  This is the
    host-controlled input scatter of the four-step (inputs arrive strided).
    """
    n1, _ = plan(n, world)
    d = len(values)
    row = max(1, -(-d // n1))
    rows = n1 // world
    out = []
    for r in range(rows):
        j1 = rank * rows + r
        out.append([int(values[j1 + n1 * j2]) if j1 + n1 * j2 < d else 0 for j2 in range(row)])
    return out


def scatter_columns_np(values, n: int, world: int, rank: int):
    """scatter_columns for a (d, 2) uint64 array: returns ((N1/G) * row, 2) and the row length."""
    import numpy as np
    n1, _ = plan(n, world)
    d = values.shape[0]
    row = max(1, -(-d // n1))
    pad = np.zeros((n1 * row, 2), dtype=np.uint64)
    pad[:d] = values
    rows = n1 // world
    cols = pad.reshape(row, n1, 2).transpose(1, 0, 2)[rank * rows:(rank + 1) * rows]
    return np.ascontiguousarray(cols).reshape(-1, 2), row


def gather_runs_np(shards, n: int, world: int):
    """gather_runs for (N1 * R, 2) uint64 arrays -> (n, 2) natural order."""
    import numpy as np
    n1, n2 = plan(n, world)
    r = n2 // world
    parts = [np.asarray(sh).reshape(n1, r, 2) for sh in shards]
    return np.ascontiguousarray(np.stack(parts, axis=1)).reshape(n, 2)


def gather_runs(shards: Sequence[Sequence[int]], n: int, world: int) -> List[int]:
    """Host helper: natural-order vector from every rank's flattened run shard."""
    n1, n2 = plan(n, world)
    r = n2 // world
    out = [0] * n
    for g, sh in enumerate(shards):
        for k1 in range(n1):
            base = k1 * n2 + g * r
            out[base:base + r] = sh[k1 * r:(k1 + 1) * r]
    return out


# ---------------------------------------------------------------- the C-ABI communicator

class NativeDist:
    """The sharded pipeline inside libstarkgpu (csrc/dist.cpp, include/stark_gpu.h sg_dist_*):
    what a Rust caller binds.  ``transport="rccl"`` creates an RCCL communicator from a unique id
    broadcast over the torch.distributed group (RCCL over xGMI, collectives on the library's
    stream); ``transport="host"`` hands the library all-to-all / all-gather callbacks over host
    buffers that run on the torch.distributed group (gloo), e.g. several ranks on one GPU.

    Shards are int64 device tensors (2 words per element) in the layouts of the module docstring:
    column shard in, run shard out (ntt / coset_evaluate), the reverse for intt."""

    def __init__(self, ctx: Optional[api.Context] = None, transport: str = "rccl", group=None, abort=None):
        """``abort`` (host transport, optional): called with no arguments when a call fails on this
        rank and the library poisons the communicator, e.g. to tear the group down so the peers'
        pending exchanges fail instead of waiting (sg_dist_transport.abort)."""
        from ._lib import A2A_CB, ABORT_CB, sg_dist_transport
        self.ctx = api._ctx(ctx)
        self._lib = lib()
        self.group = group
        init = dist.is_available() and dist.is_initialized()
        self.G = dist.get_world_size(group) if init else 1
        self.g = dist.get_rank(group) if init else 0
        self.device = torch.device("cuda", self.ctx.device)
        h = ctypes.c_void_p()
        if transport == "rccl":
            uid = (ctypes.c_uint8 * 128)()
            if self.g == 0:
                self.ctx.check(self._lib.sg_dist_unique_id(uid))
            if self.G > 1:
                box = [bytes(uid)]
                dist.broadcast_object_list(box, src=0, group=group)
                uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
            self.ctx.check(self._lib.sg_dist_create(self.ctx.handle, uid, self.G, self.g, ctypes.byref(h)))
        elif transport == "host":
            def _view(ptr, nbytes):  # host buffer as int64 words (elements are 16 B, digests 64 B)
                return torch.from_numpy(np.ctypeslib.as_array((ctypes.c_int64 * (nbytes // 8)).from_address(ptr)))

            def a2a(_user, send, recv, nbytes):
                try:
                    dist.all_to_all_single(_view(recv, nbytes * self.G), _view(send, nbytes * self.G),
                                           group=self.group)
                    return 0
                except Exception:  # noqa: BLE001 - reported to the library as a callback failure
                    return 1

            def ag(_user, send, recv, nbytes):
                try:
                    parts = list(_view(recv, nbytes * self.G).chunk(self.G))
                    dist.all_gather(parts, _view(send, nbytes).clone(), group=self.group)
                    return 0
                except Exception:  # noqa: BLE001
                    return 1

            def on_abort(_user):
                if abort is not None:
                    try:
                        abort()
                    except Exception:  # noqa: BLE001 - the library is already returning an error
                        pass

            self._cbs = (A2A_CB(a2a), A2A_CB(ag), ABORT_CB(on_abort))  # keep the thunks alive
            self._tr = sg_dist_transport(None, self._cbs[0], self._cbs[1], self._cbs[2])
            self.ctx.check(self._lib.sg_dist_create_transport(self.ctx.handle, self.G, self.g, ctypes.byref(self._tr),
                                                              ctypes.byref(h)))
        else:
            raise ValueError(f"unknown transport {transport!r}")
        self.handle = h

    def set_fri_tail(self, log2_elements: int) -> None:
        """Collective (every rank, same value): the codeword size at which a sharded FRI commit
        hands over to the single-GPU rounds (sg_dist_set_fri_tail)."""
        self.ctx.check(self._lib.sg_dist_set_fri_tail(self.handle, int(log2_elements)))

    def set_timeout(self, seconds: float) -> None:
        """Deadline of one host wait inside a communicator call (sg_dist_set_timeout)."""
        self.ctx.check(self._lib.sg_dist_set_timeout(self.handle, float(seconds)))

    def counters(self) -> Tuple[int, int, int]:
        """(collectives issued, transition quotients and trace columns whose coset work /
        interpolation ran on run shards) (sg_dist_counters)."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self.ctx.check(self._lib.sg_dist_counters(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    @property
    def poisoned(self) -> bool:
        """True once a call failed on this rank: every later call fails (sg_dist_poisoned)."""
        return bool(self._lib.sg_dist_poisoned(self.handle))

    def close(self) -> None:
        if self.handle:
            self._lib.sg_dist_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()

    @staticmethod
    def plan(n: int, world: int) -> Tuple[int, int]:
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        rc = lib().sg_dist_plan(n, world, ctypes.byref(a), ctypes.byref(b))
        if rc != 0:
            raise StarkGpuError(rc, f"no plan for n = {n} over {world} ranks")
        return a.value, b.value

    def _alloc(self, count: int) -> torch.Tensor:
        return torch.empty(2 * count, dtype=torch.int64, device=self.device)

    def _torch_ready(self) -> None:
        """The library works on its own stream: drain torch's current stream first, so an input
        still being written by queued torch work is complete and an output block torch.empty
        handed out is no longer used by pending torch work (the library call itself returns
        after its stream is drained)."""
        torch.cuda.current_stream(self.device).synchronize()

    def ntt(self, root: int, cols: torch.Tensor, row_len: int, n: int) -> torch.Tensor:
        """fft/ntt.rs:7-49: column shard -> run shard."""
        n1, n2 = self.plan(n, self.G)
        out = self._alloc(n1 * (n2 // self.G))
        self._torch_ready()
        self.ctx.check(self._lib.sg_dist_ntt(self.handle, api._fe(root), ctypes.c_void_p(cols.data_ptr()), row_len,
                                             n, ctypes.c_void_p(out.data_ptr())))
        return out

    def intt(self, root: int, runs: torch.Tensor, n: int) -> torch.Tensor:
        """fft/ntt.rs:51-68: run shard -> column shard (rows of N2)."""
        n1, n2 = self.plan(n, self.G)
        out = self._alloc((n1 // self.G) * n2)
        self._torch_ready()
        self.ctx.check(self._lib.sg_dist_intt(self.handle, api._fe(root), ctypes.c_void_p(runs.data_ptr()), n,
                                              ctypes.c_void_p(out.data_ptr())))
        return out

    def coset_evaluate(self, generator: int, root_order: int, offset: int, cols: torch.Tensor,
                       row_len: int) -> torch.Tensor:
        """fft/ntt_arithmetics.rs:161-170: coefficient column shard -> codeword run shard."""
        n1, n2 = self.plan(root_order, self.G)
        out = self._alloc(n1 * (n2 // self.G))
        self._torch_ready()
        self.ctx.check(self._lib.sg_dist_coset_evaluate(self.handle, api._fe(generator), root_order, api._fe(offset),
                                                        ctypes.c_void_p(cols.data_ptr()), row_len,
                                                        ctypes.c_void_p(out.data_ptr())))
        return out

    def merkle_root(self, runs: torch.Tensor, n: int) -> bytes:
        root = (ctypes.c_uint8 * 64)()
        self._torch_ready()
        self.ctx.check(self._lib.sg_dist_merkle_root(self.handle, ctypes.c_void_p(runs.data_ptr()), n, root))
        return bytes(root)

    def fri_commit(self, offset: int, omega: int, runs: torch.Tensor, n: int, expansion: int, c: int,
                   proof_stream) -> None:
        fri = api.FRI(offset, omega, n, expansion, c, ctx=self.ctx)
        cb, adapter = fri._stream(proof_stream)
        self._torch_ready()
        rc = self._lib.sg_dist_fri_commit(self.handle, ctypes.byref(fri._p), ctypes.c_void_p(runs.data_ptr()), n,
                                          ctypes.byref(cb))
        if adapter is not None and adapter.error is not None:
            raise adapter.error
        self.ctx.check(rc)

    def fri_prove(self, offset: int, omega: int, runs: torch.Tensor, n: int, expansion: int, c: int,
                  proof_stream) -> List[int]:
        """fri.rs:210-248 on a run-sharded codeword: the same proof-stream bytes and top-level indices
        as the single-GPU FRI::prove on every rank."""
        fri = api.FRI(offset, omega, n, expansion, c, ctx=self.ctx)
        cb, adapter = fri._stream(proof_stream)
        top = (ctypes.c_size_t * max(c, 1))()
        self._torch_ready()
        rc = self._lib.sg_dist_fri_prove(self.handle, ctypes.byref(fri._p), ctypes.c_void_p(runs.data_ptr()), n,
                                         ctypes.byref(cb), top)
        if adapter is not None and adapter.error is not None:
            raise adapter.error
        self.ctx.check(rc)
        return [int(t) for t in top[:c]]


def gather_runs_sized(shards: Sequence[Sequence[int]], n1: int, n2: int, world: int) -> List[int]:
    """Natural order of a codeword of n1 * n2 held as run shards [n1][n2 / world]."""
    r = n2 // world
    out = [0] * (n1 * n2)
    for g, sh in enumerate(shards):
        for k1 in range(n1):
            out[k1 * n2 + g * r:k1 * n2 + (g + 1) * r] = sh[k1 * r:(k1 + 1) * r]
    return out


__all__ = ["NativeDist", "plan", "scatter_columns", "scatter_columns_np", "gather_runs", "gather_runs_np",
           "gather_runs_sized", "StarkGpuError"]
