"""Writes tests/golden/fullsize_digests.json: the Python oracle's own outputs at BASELINE.json's
full sizes, as SHA-256 digests and lengths, so the GPU suite pins C2 and C3 to the oracle itself
(not only to the optimized CPU checker oracle/fast_cpu.cpp):

* C2 (fft/ntt.rs:7-68): the 2^22-point NTT of synthetic(0, b"c2"), its INTT (== the input), and the
  NTT of the ragged input x[:n - 5] (zero-padded to 2^22, utils/bit_reverse_copy.rs:3-34);
* C3 (fft/ntt_arithmetics.rs:161-170, fri.rs:210-248): the LDE 2^21 -> 2^24 of synthetic(0, b"c3")
  on the coset GENERATOR * <w>, and FRI::prove (expansion 8, 64 colinearity tests) of that codeword
  into an IndependentProofStream: proof bytes, round roots, top-level query indices.

Element arrays are digested as the GPU returns them: each element as 16 little-endian bytes
(lo u64, hi u64), in order.  The two cases run in two processes; C3 takes ~30-60 min of Python.

Run from the repo root: python tests/golden/make_fullsize.py
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "..", "oracle")]
import stark_oracle as o  # noqa: E402


def elem_digest(values) -> dict:
    h = hashlib.sha256()
    for v in values:
        h.update(v.to_bytes(16, "little"))
    return {"len": len(values), "sha256": h.hexdigest()}


def log(msg):
    print("[%s] %s" % (time.strftime("%H:%M:%S"), msg), flush=True)


def case_c2():
    n = 1 << 22
    root = o.primitive_nth_root(n)
    x = o.synthetic_elements(0, b"c2", n)
    t0 = time.time()
    X = o.ntt(root, x)
    log("c2 ntt done %.0f s" % (time.time() - t0))
    Y = o.intt(root, X)
    log("c2 intt done %.0f s" % (time.time() - t0))
    assert Y == x, "oracle intt(ntt(x)) != x"
    R = o.ntt(root, x[: n - 5])
    log("c2 ragged ntt done %.0f s" % (time.time() - t0))
    return "c2", {
        "src": "fft/ntt.rs:7-68; x = synthetic(0, b'c2', 2^22), root = primitive_nth_root(2^22)",
        "n": n,
        "input": elem_digest(x),
        "ntt": elem_digest(X),
        "intt_of_ntt_equals_input": True,
        "ragged_ntt_n_minus_5": elem_digest(R),
        "oracle_seconds": round(time.time() - t0, 1),
    }


def case_c3():
    N, exp, c = 1 << 24, 8, 64
    d = N // exp
    w = o.primitive_nth_root(N)
    coeffs = o.synthetic_elements(0, b"c3", d)
    t0 = time.time()
    cw = o.fast_coset_evaluate(w, N, o.GENERATOR, coeffs)
    log("c3 LDE done %.0f s" % (time.time() - t0))
    lde = elem_digest(cw)
    fri = o.FRI(o.GENERATOR, w, N, exp, c)
    ps = o.IndependentProofStream()
    top = fri.prove(cw, ps)
    log("c3 FRI::prove done %.0f s" % (time.time() - t0))
    proof = ps.digest()
    roots = [obj[1].hex() for obj in ps.objects if obj[0] == o.ROOT]
    return "c3", {
        "src": "fft/ntt_arithmetics.rs:161-170 + fri.rs:210-248; coeffs = synthetic(0, b'c3', 2^21), "
               "w = primitive_nth_root(2^24), offset GENERATOR, expansion 8, 64 colinearity tests",
        "N": N, "expansion": exp, "colinearity_tests": c,
        "coeffs": elem_digest(coeffs),
        "lde": lde,
        "num_rounds": fri.num_rounds(),
        "roots": roots,
        "top_indices": top,
        "proof_len": len(proof),
        "proof_sha256": hashlib.sha256(proof).hexdigest(),
        "oracle_seconds": round(time.time() - t0, 1),
    }


def run(name):
    return {"c2": case_c2, "c3": case_c3}[name]()


if __name__ == "__main__":
    t0 = time.time()
    with mp.Pool(2) as pool:
        results = dict(pool.map(run, ["c3", "c2"]))
    out = {"generator": "tests/golden/make_fullsize.py (Python oracle, oracle/stark_oracle.py)",
           "element_encoding": "16 bytes per element, little-endian (lo u64, hi u64)",
           **results, "total_seconds": round(time.time() - t0, 1)}
    with open(os.path.join(HERE, "fullsize_digests.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
