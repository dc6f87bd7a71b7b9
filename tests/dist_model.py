"""TEST MODEL of the sharded path (tests/ only; never imported by the product).

The round-1 composition of the four-step NTT / LDE, the run-sharded Merkle root and the sharded
FRI commit over ``torch.distributed``, one local row step at a time.  The product is the C ABI's
``sg_dist_*`` (csrc/dist.cpp, mirrored by ``starkgpu.dist.NativeDist``); this model stays because
it runs the same distribution logic -- the four-step index maps and its one all-to-all, the
inverse with swapped factors, the coset scale on column shards, run-root gathering, run-sharded
folds, the gathered tail -- on CPU over gloo at world 2 and 4 with the oracle's row steps
(tests/dist_cpu_backend.py, tests/test_dist_cpu.py), where no GPU and hence no library call is
available, and on the GPU with the row-sharded entry points of the C ABI (``GpuRows``:
``sg_ntt_rows_dev``, ``sg_mul_pow_dev``, ``sg_transpose_dev``, ``sg_merkle_forest_dev``,
``sg_merkle_top_dev``, ``sg_fri_fold_runs_dev``) in tests/test_gpu_dist.py.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from starkgpu import api
from starkgpu._lib import lib
from starkgpu.dist import _check_primitive, _log2, gather_runs_sized, plan

P = api.FIELD_PRIME
ROOT, CODEWORD = api.ROOT, api.CODEWORD


# ---------------------------------------------------------------- communicator

class Comm:
    """Equal-split all-to-all / all-gather over a torch.distributed group.

    With the "nccl" (RCCL) backend device tensors go straight over xGMI; with
    another backend (gloo) device tensors are staged through host memory.
    """

    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            self.backend = dist.get_backend(group)
        else:
            self.world, self.rank, self.backend = 1, 0, "none"

    def _staged(self, t: torch.Tensor) -> bool:
        return t.is_cuda and self.backend != "nccl"

    @staticmethod
    def _sync(t: torch.Tensor) -> None:
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.world == 1:
            out.copy_(inp)
        elif self._staged(inp):
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, group=self.group)
        self._sync(out)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.world == 1:
            out.copy_(inp)
        elif self._staged(inp):
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather_into_tensor(o, inp.cpu(), group=self.group)
            out.copy_(o)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.group)
        self._sync(out)


# ---------------------------------------------------------------- GPU row backend

class GpuRows:
    """Local steps on this rank's GPU through libstarkgpu (the product backend).

    Field buffers are int64 device tensors of 2 * count words (lo, hi limbs);
    digest buffers are uint8 device tensors of 64 bytes per digest.
    """

    def __init__(self, ctx: Optional[api.Context] = None):
        self.ctx = api._ctx(ctx)
        self.device = torch.device("cuda", self.ctx.device)
        self._lib = lib()

    # buffers
    def alloc(self, count: int) -> torch.Tensor:
        return torch.empty(2 * count, dtype=torch.int64, device=self.device)

    def alloc_digests(self, count: int) -> torch.Tensor:
        return torch.empty(64 * count, dtype=torch.uint8, device=self.device)

    def from_ints(self, values: Sequence[int]) -> torch.Tensor:
        a = api.fe_array(values)
        return torch.from_numpy(a.view("int64").reshape(-1).copy()).to(self.device)

    def to_ints(self, buf: torch.Tensor, count: Optional[int] = None) -> List[int]:
        t = buf.cpu().numpy().view("uint64")
        if count is not None:
            t = t[:2 * count]
        return api.to_ints(t.reshape(-1, 2))

    @staticmethod
    def _p(t: torch.Tensor) -> ctypes.c_void_p:
        return ctypes.c_void_p(t.data_ptr())

    # local steps
    def ntt_rows(self, root: int, src, n_in: int, rows: int, dst, n: int) -> None:
        self.ctx.check(self._lib.sg_ntt_rows_dev(self.ctx.handle, api._fe(root), self._p(src), n_in, rows,
                                                 self._p(dst), n))

    def mul_pow(self, base: int, buf, rows: int, cols: int, a0: int, a1: int, b0: int, b1: int) -> None:
        self.ctx.check(self._lib.sg_mul_pow_dev(self.ctx.handle, api._fe(base), self._p(buf), rows, cols,
                                                a0, a1, b0, b1))

    def scale(self, buf, count: int, c: int) -> None:
        self.ctx.check(self._lib.sg_scale_dev(self.ctx.handle, self._p(buf), count, api._fe(c)))

    def transpose(self, src, dst, A: int, B: int, C: int) -> None:
        self.ctx.check(self._lib.sg_transpose_dev(self.ctx.handle, self._p(src), self._p(dst), A, B, C))

    def forest_roots(self, buf, run: int, runs: int) -> torch.Tensor:
        h = ctypes.c_void_p()
        self.ctx.check(self._lib.sg_merkle_forest_dev(self.ctx.handle, self._p(buf), run, runs, ctypes.byref(h)))
        try:
            roots = self.alloc_digests(runs)
            self.ctx.check(self._lib.sg_forest_roots_dev(self.ctx.handle, h, self._p(roots)))
        finally:
            self._lib.sg_forest_free(self.ctx.handle, h)
        return roots

    def digest_transpose(self, src, dst, A: int, B: int) -> None:
        # a digest is 4 field-element slots (64 bytes)
        self.ctx.check(self._lib.sg_transpose_dev(self.ctx.handle, self._p(src), self._p(dst), A, B, 4))

    def top_root(self, digests, count: int) -> bytes:
        h = ctypes.c_void_p()
        self.ctx.check(self._lib.sg_merkle_top_dev(self.ctx.handle, self._p(digests), count, ctypes.byref(h)))
        root = (ctypes.c_uint8 * 64)()
        self._lib.sg_tree_root(h, root)
        self._lib.sg_tree_free(self.ctx.handle, h)
        return bytes(root)

    def fold_runs(self, omega: int, offset: int, alpha: int, src, n_local: int, run: int, run_stride: int,
                  run_off: int, n_global: int, dst) -> None:
        self.ctx.check(self._lib.sg_fri_fold_runs_dev(self.ctx.handle, api._fe(omega), api._fe(offset),
                                                      api._fe(alpha), self._p(src), n_local, run, run_stride,
                                                      run_off, n_global, self._p(dst)))

    def fri_commit(self, offset: int, omega: int, n: int, expansion: int, c: int, buf, proof_stream) -> None:
        fri = api.FRI(offset, omega, n, expansion, c, ctx=self.ctx)
        fri.commit_dev(buf.data_ptr(), n, proof_stream)

    @staticmethod
    def sample(data: bytes) -> int:
        return api.sample(data)

    @staticmethod
    def num_rounds(n: int, expansion: int, c: int) -> int:
        return api.FRI(1, 1, n, expansion, c).num_rounds()


# ---------------------------------------------------------------- the distributed path

class DistStark:
    """The sharded LDE -> Merkle -> FRI-commit pipeline for one rank.

    ``rows`` is the local backend (GpuRows in production); ``comm`` the group.
    """

    def __init__(self, rows=None, comm: Optional[Comm] = None):
        self.rows = rows if rows is not None else GpuRows()
        self.comm = comm if comm is not None else Comm()
        self.G, self.g = self.comm.world, self.comm.rank

    # ---- four-step NTT: column shard -> run shard (one all-to-all)
    def _four_step(self, root: int, shard, row_len: int, n1: int, n2: int):
        """X = DFT_root(x) for n = n1 n2: column shard of (n1, n2) in, run shard [n1][n2/G] out."""
        G, g, be = self.G, self.g, self.rows
        rows, R = n1 // G, n2 // G
        if not 1 <= row_len <= n2:
            raise ValueError("row length must be in [1, N2]")
        z = be.alloc(rows * n2)
        be.ntt_rows(api.fe_pow(root, n1), shard, row_len, rows, z, n2)        # size-N2 DFTs over j2
        be.mul_pow(root, z, rows, n2, g * rows, 1, 0, 0)                       # * w^(j1 k2)
        send = be.alloc(rows * n2)
        be.transpose(z, send, rows, G, R)                                      # [j1][h][c] -> [h][j1][c]
        del z
        recv = be.alloc(n1 * R)
        self.comm.all_to_all(recv, send)                                       # [j1 (all)][c]
        del send
        t = be.alloc(n1 * R)
        be.transpose(recv, t, n1, R, 1)                                        # [c][j1]
        del recv
        u = be.alloc(n1 * R)
        be.ntt_rows(api.fe_pow(root, n2), t, n1, R, u, n1)                     # size-N1 DFTs over j1
        del t
        out = be.alloc(n1 * R)
        be.transpose(u, out, R, n1, 1)                                         # [k1][c]: run shard
        return out

    def ntt(self, root: int, shard, row_len: int, n: int):
        """fft/ntt.rs:7-49 on a column shard (row_len <= N2 entries per row, zero padded)."""
        _check_primitive(root, n)
        n1, n2 = plan(n, self.G)
        return self._four_step(root, shard, row_len, n1, n2)

    def intt(self, root: int, run_shard, n: int):
        """fft/ntt.rs:51-68 on a run shard; returns the column shard (rows of length N2).

        The run shard of (N1, N2) is, transposed, the column shard of (N2, N1):
        index k1 N2 + (g R + c) = j1' + N2 j2' with j1' = g R + c, j2' = k1.
        So the inverse is the four-step with the factors swapped and root^-1,
        whose run shard [N2][N1/G] transposes back to the column shard of x.
        """
        G, be = self.G, self.rows
        if n < 2:
            raise ValueError("distributed intt needs n >= 2")
        inv_root = api.fe_inverse(root)
        _check_primitive(inv_root, n)
        n1, n2 = plan(n, G)
        R = n2 // G
        col = be.alloc(n1 * R)
        be.transpose(run_shard, col, n1, R, 1)                     # [c][k1]: column shard of (N2, N1)
        y = self._four_step(inv_root, col, n1, n2, n1)             # run shard [N2][N1/G]
        be.scale(y, n1 * R, api.fe_inverse(n % P))
        out = be.alloc(n1 * R)
        be.transpose(y, out, n2, n1 // G, 1)                       # [N1/G][N2]
        return out

    # ---- LDE: scale by offset^j then the four-step (fft/ntt_arithmetics.rs:161-170)
    def coset_evaluate(self, generator: int, root_order: int, offset: int, shard, row_len: int):
        """fast_coset_evaluate on a column shard of the coefficients; returns a run shard."""
        n = root_order
        _log2(n)
        n1, _ = plan(n, self.G)
        rows = n1 // self.G
        scaled = self.rows.alloc(rows * row_len)
        scaled.copy_(shard.reshape(-1)[:2 * rows * row_len])
        # coefficient j = (g rows + r) + N1 c gets offset^j
        self.rows.mul_pow(offset, scaled, rows, row_len, n1, 0, self.g * rows, 1)
        return self.ntt(generator, scaled, row_len, n)

    # ---- Merkle root of a run shard (merkle_root.rs:21-32)
    def merkle_root(self, run_shard, n1: int, run: int) -> bytes:
        """Root of the natural-order codeword whose runs [k1][run] are held per rank."""
        be, G = self.rows, self.G
        roots = be.forest_roots(run_shard, run, n1)                # [k1] local run roots
        allr = be.alloc_digests(G * n1)
        self.comm.all_gather(allr, roots)                          # [g][k1]
        ordered = be.alloc_digests(G * n1)
        be.digest_transpose(allr, ordered, G, n1)                  # [k1][g]: global run order
        return be.top_root(ordered, G * n1)

    # ---- FRI commit on a run shard (fri.rs:115-172)
    def fri_commit(self, offset: int, omega: int, run_shard, n: int, expansion: int, c: int, proof_stream) -> None:
        G, g, be = self.G, self.g, self.rows
        n1, n2 = plan(n, G)
        R = n2 // G
        rounds = be.num_rounds(n, expansion, c)
        if rounds < 1:
            raise ValueError("FRI: zero rounds for this domain")
        cur, k1s, length = run_shard, n1, n
        r = 0
        while k1s > 1 and r < rounds:
            if api.fe_pow(omega, length - 1) != api.fe_inverse(omega):
                raise ValueError("error in commit: omega does not have the right order!")
            proof_stream.push((ROOT, self.merkle_root(cur, k1s, R)))
            if r == rounds - 1:
                break
            alpha = be.sample(proof_stream.fiat_shamir_prover(api.PROOF_BYTES))
            nxt = be.alloc(k1s * R // 2)
            be.fold_runs(omega, offset, alpha, cur, k1s * R, R, n2, g * R, length, nxt)
            cur, k1s, length = nxt, k1s // 2, length // 2
            omega = api.fe_pow(omega, 2)
            offset = api.fe_pow(offset, 2)
            r += 1
        if r == rounds - 1 and k1s > 1:
            # every round done while still sharded: gather the last codeword (fri.rs:166)
            full = be.alloc(G * k1s * R)
            self.comm.all_gather(full, cur)
            shards = [be.to_ints(full[2 * q * k1s * R:2 * (q + 1) * k1s * R]) for q in range(G)]
            proof_stream.push((CODEWORD, gather_runs_sized(shards, k1s, n2, G)))
            return
        # one run per rank left: the codeword (length N2) is block-distributed; gather it
        full = be.alloc(G * R)
        self.comm.all_gather(full, cur)
        left = rounds - r
        if be.num_rounds(length, expansion, c) != left:
            raise AssertionError("FRI tail round count mismatch")
        be.fri_commit(offset, omega, length, expansion, c, full, proof_stream)
