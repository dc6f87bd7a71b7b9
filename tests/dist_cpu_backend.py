"""Oracle-backed local backend for the multi-GPU driver (test infrastructure only).

`dist_model.DistStark` (the test model of the sharded path) composes local row steps with
collectives; these CPU
versions of the row steps (built from the oracle, oracle/stark_oracle.py) let
the distribution logic -- index maps, the all-to-all, run-root gathering,
run-sharded folds, the FRI tail -- run over gloo on CPU with world_size > 1.
Its GPU backend is `dist_model.GpuRows` (HIP kernels through the C ABI's row entry points); the
product's sharded path is the C ABI's `sg_dist_*` (`starkgpu.dist.NativeDist`).
"""
from typing import List, Optional, Sequence

import torch

import stark_oracle as O

MASK64 = (1 << 64) - 1


def _pack(values: Sequence[int]) -> List[int]:
    out = []
    for v in values:
        lo, hi = v & MASK64, v >> 64
        out.append(lo - (1 << 64) if lo >> 63 else lo)
        out.append(hi - (1 << 64) if hi >> 63 else hi)
    return out


class CpuRows:
    def __init__(self):
        self.device = torch.device("cpu")

    # buffers: int64 tensors of (lo, hi) words; digests: uint8 tensors
    def alloc(self, count: int) -> torch.Tensor:
        return torch.zeros(2 * count, dtype=torch.int64)

    def alloc_digests(self, count: int) -> torch.Tensor:
        return torch.zeros(64 * count, dtype=torch.uint8)

    def from_ints(self, values: Sequence[int]) -> torch.Tensor:
        return torch.tensor(_pack(values), dtype=torch.int64)

    def to_ints(self, buf: torch.Tensor, count: Optional[int] = None) -> List[int]:
        w = [x & MASK64 for x in buf.tolist()]
        vals = [(w[2 * i + 1] << 64) | w[2 * i] for i in range(len(w) // 2)]
        return vals if count is None else vals[:count]

    def _set(self, buf: torch.Tensor, values: Sequence[int]) -> None:
        buf[:2 * len(values)] = torch.tensor(_pack(values), dtype=torch.int64)

    @staticmethod
    def _digests(buf: torch.Tensor) -> List[bytes]:
        b = bytes(buf.tolist())
        return [b[i:i + 64] for i in range(0, len(b), 64)]

    # local steps (same contracts as dist_model.GpuRows)
    def ntt_rows(self, root, src, n_in, rows, dst, n):
        x = self.to_ints(src, rows * n_in)
        out = []
        for r in range(rows):
            row = x[r * n_in:(r + 1) * n_in] + [0] * (n - n_in)
            out += O.ntt(root, row)
        self._set(dst, out)

    def mul_pow(self, base, buf, rows, cols, a0, a1, b0, b1):
        x = self.to_ints(buf, rows * cols)
        for r in range(rows):
            for c in range(cols):
                e = (a0 + a1 * r) * c + b0 + b1 * r
                x[r * cols + c] = O.mul_mod(x[r * cols + c], O.fpow(base, e))
        self._set(buf, x)

    def scale(self, buf, count, c):
        self._set(buf, [O.mul_mod(v, c) for v in self.to_ints(buf, count)])

    def transpose(self, src, dst, A, B, C):
        x = self.to_ints(src, A * B * C)
        out = [0] * (A * B * C)
        for a in range(A):
            for b in range(B):
                out[(b * A + a) * C:(b * A + a + 1) * C] = x[(a * B + b) * C:(a * B + b + 1) * C]
        self._set(dst, out)

    def forest_roots(self, buf, run, runs):
        x = self.to_ints(buf, run * runs)
        roots = b"".join(O.merkle_commit(x[k * run:(k + 1) * run]) for k in range(runs))
        return torch.tensor(list(roots), dtype=torch.uint8)

    def digest_transpose(self, src, dst, A, B):
        d = self._digests(src)
        out = [b""] * (A * B)
        for a in range(A):
            for b in range(B):
                out[b * A + a] = d[a * B + b]
        dst[:] = torch.tensor(list(b"".join(out)), dtype=torch.uint8)

    def top_root(self, digests, count):
        level = self._digests(digests)[:count]
        while len(level) > 1:
            level = [O.blake2b512(level[2 * i] + level[2 * i + 1]) for i in range(len(level) // 2)]
        return level[0]

    def fold_runs(self, omega, offset, alpha, src, n_local, run, run_stride, run_off, n_global, dst):
        x = self.to_ints(src, n_local)
        half = n_local // 2
        assert (half // run) * run_stride == n_global // 2
        two_inv = O.inv(2)
        out = []
        for l in range(half):
            i = (l // run) * run_stride + run_off + l % run
            abo = O.div(alpha, O.mul_mod(offset, O.fpow(omega, i)))
            first = O.mul_mod(O.add_mod(1, abo), x[l])
            second = O.mul_mod(O.sub_mod(1, abo), x[l + half])
            out.append(O.mul_mod(two_inv, O.add_mod(first, second)))
        self._set(dst, out)

    def fri_commit(self, offset, omega, n, expansion, c, buf, proof_stream):
        O.FRI(offset, omega, n, expansion, c).commit(self.to_ints(buf, n), proof_stream)

    @staticmethod
    def sample(data: bytes) -> int:
        return O.sample(data)

    @staticmethod
    def num_rounds(n, expansion, c) -> int:
        return O.FRI(1, 1, n, expansion, c).num_rounds()
