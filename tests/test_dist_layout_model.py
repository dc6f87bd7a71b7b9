"""CPU model of the sharded trace interpolation's data flow (csrc/stark.cpp
interpolate_geometric_batch_dist), at toy sizes with the oracle's arithmetic.

Every distributed step is modelled by its contract, not its kernels: a distributed NTT maps a
column shard to the run shard of the whole transform, the distributed INTT the reverse (csrc/dist.cpp
header), and the new column-shard assembly uses the index map k = row0 + r + N1 j of
k_interp_assemble_cols.  The model must reproduce the reference's interpolant
(fast_interpolate_domain, ntt_arithmetics.rs:172-237) on q^0..q^(n-1) for every rank count the
sharded path accepts -- it pins the layout algebra the GPU code follows; the GPU code itself is
checked byte for byte by tests/test_gpu_dist.py (counters assert the sharded branch ran).
"""
import stark_oracle as o
import stark_prove_oracle as e

P = o.P


def plan(n, G):
    logn = n.bit_length() - 1
    n1 = 1 << (logn // 2)  # dist.cpp dist_split
    return n1, n // n1


def can_shard(n, G):  # dist.cpp dist_can_shard
    n1, n2 = plan(n, G)
    return n1 % G == 0 and n2 % (4 * G) == 0 and n2 % G == 0 and n1 // G >= 4 and (n1 // G) % 4 == 0


def col_shard(x, n, G, g):
    """column shard [N1/G][N2]: row r = x[(g rows + r) + N1 j] (zero past len(x))."""
    n1, n2 = plan(n, G)
    rows = n1 // G
    return [[x[g * rows + r + n1 * j] if g * rows + r + n1 * j < len(x) else 0 for j in range(n2)]
            for r in range(rows)]


def from_cols(shards, n, G):
    n1, n2 = plan(n, G)
    rows = n1 // G
    out = [0] * n
    for g, sh in enumerate(shards):
        for r in range(rows):
            for j in range(n2):
                out[g * rows + r + n1 * j] = sh[r][j]
    return out


def run_shard(X, n, G, g):
    """run shard [N1][N2/G]: element [k1][c] = X[k1 N2 + g R + c]."""
    n1, n2 = plan(n, G)
    R = n2 // G
    return [[X[k1 * n2 + g * R + c] for c in range(R)] for k1 in range(n1)]


def from_runs(shards, n, G):
    n1, n2 = plan(n, G)
    R = n2 // G
    out = [0] * n
    for g, sh in enumerate(shards):
        for k1 in range(n1):
            for c in range(R):
                out[k1 * n2 + g * R + c] = sh[k1][c]
    return out


def dist_ntt(root, shards, n, G):  # column shards in, run shards out
    X = o.ntt(root, from_cols(shards, n, G))
    return [run_shard(X, n, G, g) for g in range(G)]


def dist_intt(root, shards, n, G):  # run shards in, column shards out
    x = o.intt(root, from_runs(shards, n, G))
    return [col_shard(x, n, G, g) for g in range(G)]


def sharded_interpolate(q, D, y, G):
    """interpolate_geometric_batch_dist for one column, step by step."""
    n = len(y)
    logf = 0
    logD = D.bit_length() - 1
    while logf < 4 and (D >> (logf + 1)) >= n and logD - (logf + 1) >= 6 and logD >= 2 * (logf + 1):
        logf += 1
    assert logf >= 1
    f, M = 1 << logf, D >> logf
    Mf = M >> logf
    qf = o.fpow(q, f)
    assert can_shard(M, G)
    dom = [o.fpow(q, i) for i in range(n)]
    Z = e.fast_zerofier(q, D, dom)                       # prod (x - q^i)
    Zv = [e.p_evaluate(Z, o.fpow(q, f * k)) for k in range(M)]
    dZ = [(i * c) % P for i, c in enumerate(Z)][1:]
    a = [y[i] * o.inv(e.p_evaluate(dZ, dom[i])) % P for i in range(n)]   # y_i / Z'(q^i)
    b = [0] + [o.inv((1 - o.fpow(o.inv(q), j)) % P) for j in range(1, D)]
    # geo_rows: row r of the residue class i = f j + r (Mf entries), replicated
    rows = [[a[f * j + r] if f * j + r < n else 0 for j in range(Mf)] for r in range(f)]
    # K rows: K_r[j] = b[(f j - r) mod D], transformed with qf
    Khat = [o.ntt(qf, [b[(f * j - r) % D] for j in range(M)]) for r in range(f)]
    # per rank: gather the column shard of each row, distributed NTT -> run shards
    A = [dist_ntt(qf, [col_shard(rows[r], M, G, g) for g in range(G)], M, G) for r in range(f)]
    # pointwise sum over r on the run shards with the sliced K rows
    Shat = []
    for g in range(G):
        Kg = [run_shard(Khat[r], M, G, g) for r in range(f)]
        n1, n2 = plan(M, G)
        Shat.append([[sum(A[r][g][k1][c] * Kg[r][k1][c] for r in range(f)) % P for c in range(n2 // G)]
                     for k1 in range(n1)])
    Scol = dist_intt(qf, Shat, M, G)
    # column-shard assembly (k_interp_assemble_cols): k = row0 + r + n1 j, values / M
    n1, n2 = plan(M, G)
    rows_g = n1 // G
    minv = o.inv(M)
    V = []
    for g in range(G):
        sh = []
        for r in range(rows_g):
            row = []
            for j in range(n2):
                k = g * rows_g + r + n1 * j
                m = k << logf
                if m < n:
                    v = y[m]
                else:
                    v = Zv[k] * o.fpow(o.inv(q), m) % P * Scol[g][r][j] % P
                row.append(v * minv % P)
            sh.append(row)
        V.append(sh)
    coeffs = from_runs(dist_ntt(o.inv(qf), V, M, G), M, G)
    return coeffs[:n], coeffs[n:]


def test_sharded_interpolation_model_equals_reference():
    for (D, n, G) in ((256, 44, 2), (256, 60, 2), (1024, 200, 4), (1024, 284, 2), (1024, 284, 4)):
        q = o.primitive_nth_root(D)
        y = o.synthetic_elements(n, b"model", n)
        got, above = sharded_interpolate(q, D, y, G)
        want = e.fast_interpolate_domain(q, D, [o.fpow(q, i) for i in range(n)], y)
        assert got == want, (D, n, G)
        assert not any(above), (D, n, G)
