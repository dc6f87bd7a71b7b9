"""The drop-in boundary from a compiled host: examples/prove_rescue.c calls libstarkgpu through
include/stark_gpu.h only (no Python, no torch in that process) and writes Stark::prove's bytes
(stark/stark.rs:276-562) for a Rescue-Prime statement; they must equal the oracle's proof for the
same injected randomness, and at C4 the Python binding's (itself byte-equal to the CPU checker,
test_gpu_fullsize.py)."""
import os
import subprocess

import numpy as np
import pytest

import stark_oracle as o
import stark_prove_oracle as e

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "build", "prove_rescue")


def _run(tmp_path, N, exp, c, sec, tcd, seed, dist=False):
    assert os.path.exists(BIN), "examples/build/prove_rescue missing: run __graft_entry__.build()"
    st = e.Stark(exp, c, sec, 2, N + 1, tcd)
    inp = o.sample(seed)
    rp = e.RescuePrime(2, 1, sec, N)
    if N < 1000:
        air = rp.transition_constraints(st.omicron, st.omicron_domain_length)
        nrc = st.num_randomizer_coefficients(air)
    else:
        air, nrc = None, None
    if nrc is None:  # the C host reports how many draws it needs
        probe = subprocess.run([BIN, str(N), str(exp), str(c), str(sec), str(tcd), str(inp & (2**64 - 1)),
                                str(inp >> 64), os.devnull, os.devnull], capture_output=True, text=True,
                               timeout=120)
        assert probe.returncode == 2, probe.stderr
        nrc = int(probe.stdout.split()[1]) - 2 * st.num_randomizers
    r = e.randomness_from_seed(seed, 2 * st.num_randomizers + nrc)
    rnd = np.array([[v & (2**64 - 1), v >> 64] for v in r], dtype=np.uint64)
    rfile, pfile = tmp_path / "randomness.bin", tmp_path / "proof.bin"
    rnd.tofile(rfile)
    # a fresh id path per run and a per-run nonce: a stale id file is never read as this run's
    extra = ["--dist", str(tmp_path / "rccl.id"), "0", "1", str(int.from_bytes(os.urandom(7), "big"))] if dist else []
    res = subprocess.run([BIN, str(N), str(exp), str(c), str(sec), str(tcd), str(inp & (2**64 - 1)), str(inp >> 64),
                          str(rfile), str(pfile)] + extra, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    return pfile.read_bytes(), st, rp, air, inp, r


@pytest.mark.parametrize("dist", [False, True])
@pytest.mark.parametrize("N,exp,c,sec,tcd", [(27, 4, 2, 2, 2), (40, 4, 3, 4, 2), (27, 8, 4, 8, 3)])
def test_c_host_proof_equals_oracle(tmp_path, N, exp, c, sec, tcd, dist):
    """dist: the same through sg_dist_stark_prove on a one-rank RCCL communicator created from a
    unique id passed through a file (what a multi-process Rust / C caller does)."""
    got, st, rp, air, inp, r = _run(tmp_path, N, exp, c, sec, tcd, b"c-host-%d-%d" % (N, exp), dist)
    m = 2
    trace = rp.trace(inp)
    bnd = rp.boundary_constraints(rp.hash(inp))
    tr = [r[m * i:m * i + m] for i in range(st.num_randomizers)]
    want = st.prove(trace, air, bnd, o.IndependentProofStream(), tr, r[m * st.num_randomizers:])
    assert got == want


@pytest.mark.timeout(600)
def test_c_host_c4_equals_python_binding(tmp_path):
    """C4 (trace 2^16, FRI domain 2^21): the compiled host's bytes == the ctypes binding's."""
    import starkgpu as sg
    N, exp, c, sec, tcd = 65278, 8, 64, 128, 3
    got, st, rp, _, inp, r = _run(tmp_path, N, exp, c, sec, tcd, b"c-host-c4")
    rp_g = sg.RescuePrime(2, 1, sec, N)
    st_g = sg.Stark(exp, c, sec, 2, N + 1, tcd)
    air_g = rp_g.transition_constraints(st_g.omicron, st_g.omicron_domain_length)
    nr = st_g.num_randomizers
    want = st_g.prove(rp_g.trace_array(inp), air_g, rp.boundary_constraints(rp.hash(inp)),
                      sg.IndependentProofStream(), sg.fe_array(r[:2 * nr]), sg.fe_array(r[2 * nr:]))
    assert got == want


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dist", [False, True])
def test_c_host_rpsss_signature_equals_oracle(tmp_path, dist):
    """RPSSS::sign at the reference's published configuration (rpsss.rs:103-108; tests/rpsss_case.py)
    from the compiled host: `--document "Hello, World!"` puts the proof through a
    SignatureProofStream; the bytes equal the oracle's signature and its length is the reference's
    1 156 888 (rpsss.rs:89).  dist: the same through sg_dist_stark_prove (one-rank RCCL)."""
    import rpsss_case as R
    c = R.Case()
    want = c.oracle_sign()
    r = [v for row in c.trace_randomizers for v in row] + list(c.randomizer_coefficients)
    rnd = np.array([[v & (2**64 - 1), v >> 64] for v in r], dtype=np.uint64)
    rfile, pfile = tmp_path / "randomness.bin", tmp_path / "sig.bin"
    rnd.tofile(rfile)
    extra = ["--dist", str(tmp_path / "rccl.id"), "0", "1", str(int.from_bytes(os.urandom(7), "big"))] if dist else []
    res = subprocess.run([BIN, str(R.RESCUE[3]), str(R.EXPANSION), str(R.CHECKS), str(R.SECURITY), str(R.TCD),
                          str(c.sk & (2**64 - 1)), str(c.sk >> 64), str(rfile), str(pfile), "--document",
                          R.DOCUMENT.decode()] + extra, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    got = pfile.read_bytes()
    assert len(got) == R.PROOF_LEN and got == want
