"""Writes tests/golden/rpsss_published.json: the oracle's signature at the reference's published
RPSSS configuration (rpsss.rs:103; tests/rpsss_case.py) -- its length (the reference pins
1 156 888 bytes, rpsss.rs:89), SHA-256, and the seeded key pair -- so the CPU suite can hold the
checkers to it without re-running the 8 s Python prove in every test.

Run from the repo root: python tests/golden/make_rpsss.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "..", "oracle")]
import rpsss_case as R  # noqa: E402

c = R.Case()
sig = c.oracle_sign()
ok, err = c.oracle_verify(R.DOCUMENT, sig)
bad, why = c.oracle_verify(R.FORGED, sig)
assert ok and not bad and len(sig) == R.PROOF_LEN, (ok, err, bad, len(sig))
out = {
    "src": "rpsss.rs:89,103,113-131 via tests/rpsss_case.py (seed b'rpsss')",
    "seed": "rpsss",
    "sk": str(c.sk),
    "pk": str(c.pk),
    "document": R.DOCUMENT.decode(),
    "proof_len": len(sig),
    "proof_sha256": hashlib.sha256(sig).hexdigest(),
    "forged_document": R.FORGED.decode(),
    "forged_error": why,
}
with open(os.path.join(HERE, "rpsss_published.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
