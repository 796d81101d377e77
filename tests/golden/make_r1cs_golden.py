"""Generates tests/golden/r1cs_proofs.json: for each reference R1CS fixture
(copied by tests/golden/r1cs/copy_fixtures.py), the trace dimensions, the three
roots and the SHA-256 of the StarkProof JSON produced by the CPU oracle's
restatement of mk_r1cs_proof (oracle/r1cs.c), after checking that the
restated verifier (oracle/stark_verify.py) accepts the proof.

Run from the repo root:  python tests/golden/make_r1cs_golden.py
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import Oracle  # noqa: E402
from r1cs import build_trace, load_fixture, mk_r1cs_proof_json, verifier_inputs  # noqa: E402
from stark_verify import verify_r1cs_proof  # noqa: E402

FIXTURES = ["compute", "poseidon3_test", "pedersen_test", "bits"]


def main():
    orc = Oracle()
    out = {}
    d = os.path.join(ROOT, "tests", "golden", "r1cs")
    for name in FIXTURES:
        r1cs, wit = load_fixture(d, name)
        tr = build_trace(r1cs, wit)
        s = mk_r1cs_proof_json(orc, tr)
        vi = verifier_inputs(r1cs, tr.public_wires)
        assert verify_r1cs_proof(orc, s, tr.public_wires, vi["public_first_indices"], vi["permuted_indices"],
                                 vi["coefficients"], vi["flag0"], vi["flag1"], vi["flag2"], vi["n_constraints"],
                                 vi["n_wires"])
        p = json.loads(s)
        out[name] = {
            "original_steps": len(tr.coefficients),
            "n_public_first": len(tr.public_first_indices),
            "m_root": bytes(p["m_root"]).hex(),
            "l_root": bytes(p["l_root"]).hex(),
            "a_root": bytes(p["a_root"]).hex(),
            "fri_layers": len(p["fri_proof"]),
            "json_len": len(s),
            "json_sha256": hashlib.sha256(s.encode()).hexdigest(),
        }
        print(name, out[name])
    with open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
