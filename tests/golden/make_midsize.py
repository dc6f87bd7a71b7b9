"""Writes tests/golden/midsize_proof.json: the Python oracle's `Stark::prove` bytes (length and
SHA-256) for the mid-size Rescue-Prime statement of tests/midsize_case.py (trace 1257 rows, FRI
domain 2^15, c = 64), plus the oracle verifier's verdict on them and on a false claim.  The oracle
prove takes minutes in Python, so the suites compare against this digest instead of re-running it.

Run from the repo root: python tests/golden/make_midsize.py
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "..", "oracle")]
import midsize_case as M  # noqa: E402
import stark_oracle as o  # noqa: E402

t0 = time.time()
rp, st, air, trace, bnd, tr, rc = M.inputs()
t1 = time.time()
proof = st.prove(trace, air, bnd, o.IndependentProofStream(), tr, rc)
t2 = time.time()
ok, err = st.verify(air, bnd, o.IndependentProofStream(o.deserialize(proof)))
assert ok, err
false_bnd = [(c, r, o.add_mod(v, 1)) if i == len(bnd) - 1 else (c, r, v) for i, (c, r, v) in enumerate(bnd)]
bad, why = st.verify(air, false_bnd, o.IndependentProofStream(o.deserialize(proof)))
assert not bad
t3 = time.time()
out = {
    "src": "tests/midsize_case.py: RescuePrime::new(2, 1, 128, 1000) (rescue_prime.rs:107-114), "
           "Stark::new(8, 64, 128, 2, 1001, 3) (stark.rs:71-114), IndependentProofStream, seed b'midsize'",
    "trace_rows": len(trace) + st.num_randomizers,
    "omicron_domain": st.omicron_domain_length,
    "fri_domain": st.omicron_domain_length * st.expansion_factor,
    "output": str(bnd[-1][2]),
    "proof_len": len(proof),
    "proof_sha256": hashlib.sha256(proof).hexdigest(),
    "oracle_verify": ok,
    "false_claim_rejected": not bad,
    "false_claim_error": why,
    "oracle_seconds": {"setup": round(t1 - t0, 1), "prove": round(t2 - t1, 1), "verify": round(t3 - t2, 1)},
}
with open(os.path.join(HERE, "midsize_proof.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
