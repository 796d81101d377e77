"""R1CS front end and the CPU oracle's mk_r1cs_proof (no GPU).

- The Python readers are pinned by the reference's own reader tests
  (r1cs-stark/src/reader.rs:44-89: compute.r1cs == compute.r1cs.json, and the
  compute.wtns wire values).
- libstark_hip's host trace builder (stark_r1cs_trace_build, run.rs:310-437)
  must equal the Python restatement on every fixture (host code: runs here).
- Oracle proofs are accepted by the restated verifier (verify.rs:13-258) and
  match the committed digests in tests/golden/r1cs_proofs.json; tampering is
  rejected.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import from_limbs, to_limbs
import r1cs as R
from stark_verify import verify_r1cs_proof

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "r1cs")
GOLDEN = json.load(open(os.path.join(HERE, "golden", "r1cs_proofs.json")))


def _read(name, ext):
    with open(os.path.join(FIX, f"{name}.{ext}"), "rb") as f:
        return f.read()


def test_read_r1cs_matches_reference_json():
    """reader.rs:44-62: read_r1cs(compute.r1cs) == compute.r1cs.json."""
    got = R.read_r1cs(_read("compute", "r1cs"))
    want = json.load(open(os.path.join(FIX, "compute.r1cs.json")))
    h = want["header"]
    assert got.version == want["version"]
    assert got.header.field_size == h["field_size"]
    assert list(got.header.prime_number) == h["prime_number"]
    for k in ("n_wires", "n_public_outputs", "n_public_inputs", "n_private_inputs", "n_labels", "n_constraints"):
        assert getattr(got.header, k) == h[k], k
    assert len(got.constraints) == len(want["constraints"])
    for gc, wc in zip(got.constraints, want["constraints"]):
        for gf, wf in zip(gc, wc["factors"]):
            assert len(gf) == wf["n_coefficient"]
            assert [(wid, list(v)) for wid, v in gf] == [(c["wire_id"], c["value"]) for c in wf["coefficients"]]


def test_read_witness_matches_reference():
    """reader.rs:64-89."""
    w = R.read_witness(_read("compute", "wtns"))
    assert w == [bytes([1]),
                 bytes([135, 136, 135, 103, 17, 74, 207, 218, 212, 163, 232, 164, 38, 238, 216, 34, 56, 221, 180,
                        135, 36, 249, 144, 247, 19, 79, 126, 26, 164, 114, 177, 5]),
                 bytes([17]), bytes([33, 1]), bytes([49, 19])]


@pytest.fixture(scope="module")
def traces():
    return {n: R.build_trace(*R.load_fixture(FIX, n)) for n in GOLDEN}


def test_trace_dims(traces):
    for name, tr in traces.items():
        assert len(tr.coefficients) == GOLDEN[name]["original_steps"]
        assert len(tr.public_first_indices) == GOLDEN[name]["n_public_first"]
        assert sorted(tr.permuted_indices) == list(range(len(tr.coefficients)))  # a permutation


@pytest.mark.parametrize("name", list(GOLDEN))
def test_library_trace_builder_matches_restatement(name, traces):
    """stark_r1cs_trace_build (host C++) == oracle/r1cs.py build_trace, field by field."""
    from stark_amd.r1cs import R1csTrace
    tr = traces[name]
    lib_tr = R1csTrace(_read(name, "r1cs"), _read(name, "wtns")).export()
    for k in ("witness_trace", "computational_trace", "coefficients", "flag0", "flag1", "flag2", "public_wires"):
        assert from_limbs(lib_tr[k]) == list(getattr(tr, k)), k
    assert lib_tr["permuted_indices"] == tr.permuted_indices
    assert lib_tr["public_first_indices"] == [tuple(x) for x in tr.public_first_indices]
    assert (lib_tr["n_constraints"], lib_tr["n_wires"]) == (tr.n_constraints, tr.n_wires)


def test_library_trace_builder_rejects_malformed():
    from stark_amd import StarkError
    from stark_amd.r1cs import R1csTrace
    r1, wt = _read("compute", "r1cs"), _read("compute", "wtns")
    with pytest.raises(StarkError):
        R1csTrace(r1[:100], wt)           # truncated constraints (reader.rs get_u32_le underflow)
    with pytest.raises(StarkError):
        R1csTrace(b"xxxx" + r1[4:], wt)   # bad magic (reader.rs:6-7)
    bad_prime = bytearray(r1)
    bad_prime[12 + 12 + 4] ^= 1           # header prime (run.rs:344-350)
    with pytest.raises(StarkError):
        R1csTrace(bytes(bad_prime), wt)
    bad_w = bytearray(wt)
    bad_w[4 * 7 + 32 + 16] = 2            # witness[0] = 2 (run.rs:358)
    with pytest.raises(StarkError):
        R1csTrace(r1, bytes(bad_w))


def _verify(oracle, tr, proof):
    return verify_r1cs_proof(oracle, proof, tr.public_wires, tr.public_first_indices, tr.permuted_indices,
                             tr.coefficients, tr.flag0, tr.flag1, tr.flag2, tr.n_constraints, tr.n_wires)


@pytest.mark.parametrize("name", ["compute", "poseidon3_test"])
def test_oracle_proof_golden_and_verifies(name, oracle, traces):
    tr = traces[name]
    s = R.mk_r1cs_proof_json(oracle, tr)
    g = GOLDEN[name]
    assert hashlib.sha256(s.encode()).hexdigest() == g["json_sha256"]
    p = json.loads(s)
    assert bytes(p["a_root"]).hex() == g["a_root"]
    assert len(p["main_branches"]) == 320 and len(p["linear_comb_branches"]) == 80
    assert all(len(b["leaf"]) == 256 for b in p["main_branches"])
    assert _verify(oracle, tr, p)


def test_verifier_rejects_tampering(oracle, traces):
    tr = traces["compute"]
    p = json.loads(R.mk_r1cs_proof_json(oracle, tr))
    cases = []
    q = json.loads(json.dumps(p)); q["main_branches"][5]["leaf"][40] ^= 1; cases.append(q)      # opened value
    q = json.loads(json.dumps(p)); q["fri_proof"][-1]["Last"]["last"][3][0] ^= 1; cases.append(q)  # FRI last layer
    q = json.loads(json.dumps(p)); q["a_root"][0] ^= 1; cases.append(q)                        # transcript root
    for q in cases:
        with pytest.raises(AssertionError):
            _verify(oracle, tr, q)


def test_unsatisfied_witness_fails_divisibility(oracle, traces):
    """A wrong computational-trace value breaks Q1's divisibility by Z (utils.rs:379-390)."""
    tr = traces["compute"]
    bad = R.Trace(**{**tr.__dict__, "computational_trace": list(tr.computational_trace)})
    bad.computational_trace[3] = (bad.computational_trace[3] + 1) % R.P
    with pytest.raises(AssertionError, match="err 2"):
        R.mk_r1cs_proof_json(oracle, bad)
