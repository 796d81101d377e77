"""mk_r1cs_proof on the GPU (stark_mk_r1cs_proof / stark_prove_r1cs_trace)
against the CPU oracle, byte for byte, on the reference's own R1CS fixtures.

Bar: the StarkProof JSON is identical to oracle/r1cs.c's (the restatement of
prove.rs:14-378), its digest equals the committed golden digest, and the
restated verifier (verify.rs:13-258) accepts it.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import r1cs as R
from oracle import to_limbs
from stark_verify import verify_r1cs_proof

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "r1cs")
GOLDEN = json.load(open(os.path.join(HERE, "golden", "r1cs_proofs.json")))

pytestmark = pytest.mark.gpu


def _read(name, ext):
    with open(os.path.join(FIX, f"{name}.{ext}"), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name", list(GOLDEN))
def test_prove_with_witness_matches_oracle(ctx, oracle, name):
    from stark_amd.r1cs import prove_with_witness
    proof = prove_with_witness(ctx, _read(name, "r1cs"), _read(name, "wtns"))
    s = proof.to_json()
    assert hashlib.sha256(s.encode()).hexdigest() == GOLDEN[name]["json_sha256"]
    tr = R.build_trace(*R.load_fixture(FIX, name))
    if name in ("compute", "poseidon3_test"):
        assert s == R.mk_r1cs_proof_json(oracle, tr)
    roots = proof.roots()
    assert roots["m_root"].hex() == GOLDEN[name]["m_root"]
    assert roots["a_root"].hex() == GOLDEN[name]["a_root"]
    assert verify_r1cs_proof(oracle, s, tr.public_wires, tr.public_first_indices, tr.permuted_indices,
                             tr.coefficients, tr.flag0, tr.flag1, tr.flag2, tr.n_constraints, tr.n_wires)


def test_mk_r1cs_proof_from_python_trace(ctx, oracle):
    """The prove.rs-level entry point fed with the Python-built trace."""
    from stark_amd.r1cs import mk_r1cs_proof
    tr = R.build_trace(*R.load_fixture(FIX, "poseidon3_test"))
    p = mk_r1cs_proof(ctx, to_limbs(tr.witness_trace), to_limbs(tr.computational_trace), to_limbs(tr.public_wires),
                      tr.public_first_indices, tr.permuted_indices, to_limbs(tr.coefficients), to_limbs(tr.flag0),
                      to_limbs(tr.flag1), to_limbs(tr.flag2), tr.n_constraints, tr.n_wires)
    assert hashlib.sha256(p.to_json().encode()).hexdigest() == GOLDEN["poseidon3_test"]["json_sha256"]


def test_unsatisfied_witness_is_rejected(ctx):
    """The reference panics in calc_d1_polynomial (utils.rs:379-390); the library returns STARK_ERR_CHECK."""
    from stark_amd import StarkError
    from stark_amd.r1cs import mk_r1cs_proof
    tr = R.build_trace(*R.load_fixture(FIX, "compute"))
    ct = list(tr.computational_trace)
    ct[3] = (ct[3] + 1) % R.P
    with pytest.raises(StarkError) as e:
        mk_r1cs_proof(ctx, to_limbs(tr.witness_trace), to_limbs(ct), to_limbs(tr.public_wires),
                      tr.public_first_indices, tr.permuted_indices, to_limbs(tr.coefficients), to_limbs(tr.flag0),
                      to_limbs(tr.flag1), to_limbs(tr.flag2), tr.n_constraints, tr.n_wires)
    assert e.value.code == 8


def test_bad_public_wire_is_rejected(ctx):
    """A public wire that disagrees with the trace breaks B2 (utils.rs:477-499)."""
    from stark_amd import StarkError
    from stark_amd.r1cs import mk_r1cs_proof
    tr = R.build_trace(*R.load_fixture(FIX, "compute"))
    pw = list(tr.public_wires)
    pw[1] = (pw[1] + 1) % R.P
    with pytest.raises(StarkError) as e:
        mk_r1cs_proof(ctx, to_limbs(tr.witness_trace), to_limbs(tr.computational_trace), to_limbs(pw),
                      tr.public_first_indices, tr.permuted_indices, to_limbs(tr.coefficients), to_limbs(tr.flag0),
                      to_limbs(tr.flag1), to_limbs(tr.flag2), tr.n_constraints, tr.n_wires)
    assert e.value.code == 8


def test_repeated_proofs_identical(ctx):
    """No state leaks between proofs on one context (cached twiddles, scratch buffers)."""
    from stark_amd.r1cs import prove_with_witness
    a = prove_with_witness(ctx, _read("compute", "r1cs"), _read("compute", "wtns")).to_json()
    b = prove_with_witness(ctx, _read("pedersen_test", "r1cs"), _read("pedersen_test", "wtns")).to_json()
    c = prove_with_witness(ctx, _read("compute", "r1cs"), _read("compute", "wtns")).to_json()
    assert a == c
    assert hashlib.sha256(b.encode()).hexdigest() == GOLDEN["pedersen_test"]["json_sha256"]


def _synth(log_steps):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import synth_r1cs
    return synth_r1cs.for_steps(log_steps)


def test_synthetic_circuit_matches_oracle(ctx, oracle):
    """A larger circuit than the fixtures (2^13 steps, precision 2^16), byte-identical to the oracle."""
    from stark_amd.r1cs import prove_with_witness
    r1, wt = _synth(13)
    got = prove_with_witness(ctx, r1, wt).to_json()
    tr = R.build_trace(R.read_r1cs(r1), R.read_witness(wt))
    assert got == R.mk_r1cs_proof_json(oracle, tr)


def test_synthetic_2_17_steps_matches_oracle_and_verifies(ctx, oracle):
    """precision 2^20 (7 FRI layers): byte-identical to the oracle, and accepted by the restated
    verifier (verify.rs:13-258)."""
    from stark_amd.r1cs import prove_with_witness
    r1, wt = _synth(17)
    proof = prove_with_witness(ctx, r1, wt).to_json()
    tr = R.build_trace(R.read_r1cs(r1), R.read_witness(wt))
    assert proof == R.mk_r1cs_proof_json(oracle, tr, cpus=16)
    assert verify_r1cs_proof(oracle, proof, tr.public_wires, tr.public_first_indices, tr.permuted_indices,
                             tr.coefficients, tr.flag0, tr.flag1, tr.flag2, tr.n_constraints, tr.n_wires)


@pytest.mark.parametrize("name", list(GOLDEN))
def test_device_trace_equals_host_trace(ctx, name):
    """stark_prove_r1cs_bytes (trace built on the GPU) and the host trace builder give the same proof."""
    from stark_amd.r1cs import prove_with_witness, prove_with_witness_host_trace
    r1, wt = _read(name, "r1cs"), _read(name, "wtns")
    assert prove_with_witness(ctx, r1, wt).to_json() == prove_with_witness_host_trace(ctx, r1, wt).to_json()


def test_device_trace_synthetic_equals_host_trace(ctx):
    from stark_amd.r1cs import prove_with_witness, prove_with_witness_host_trace
    r1, wt = _synth(15)
    assert prove_with_witness(ctx, r1, wt).to_json() == prove_with_witness_host_trace(ctx, r1, wt).to_json()


def test_device_trace_rejects_bad_inputs(ctx):
    """A wire id beyond n_wires inside a record (found on the device) and a witness whose first value
    is not 1 (run.rs:358) are rejected like the host builder rejects them."""
    import struct
    from stark_amd import StarkError
    from stark_amd.r1cs import prove_with_witness
    r1, wt = bytearray(_read("compute", "r1cs")), bytearray(_read("compute", "wtns"))
    n_wires = struct.unpack_from("<I", r1, 4 * 4 + 8 + 4 + 32)[0]
    cons = 4 * 4 + 8 + 4 + 32 + 4 * 4 + 8 + 4 + 4 + 8   # header section, then the constraint section header
    bad = bytearray(r1)
    first_nc = struct.unpack_from("<I", bad, cons)[0]
    assert first_nc > 0
    struct.pack_into("<I", bad, cons + 4, n_wires + 5)   # first record's wire id
    with pytest.raises(StarkError):
        prove_with_witness(ctx, bytes(bad), bytes(wt))
    badw = bytearray(wt)
    n_wit = struct.unpack_from("<I", badw, 4 + 5 * 4 + 4 + 32)[0]  # wtns v2: header section, 32-B prime
    wval = len(badw) - 32 * n_wit                        # witness value 0
    assert wval == 4 + 5 * 4 + 4 + 32 + 4 + 3 * 4
    badw[wval] ^= 2
    with pytest.raises(StarkError):
        prove_with_witness(ctx, bytes(r1), bytes(badw))


def _record_offsets(r1: bytes):
    """Byte offsets of every constraint record (36 B: wire id + 32-B coefficient) of a .r1cs v1 file, in
    push order (constraint, factor, record), from its header and constraint section."""
    import struct
    n_c = struct.unpack_from("<I", r1, 4 * 4 + 8 + 4 + 32 + 4 * 4 + 8)[0]
    pos = 4 * 4 + 8 + 4 + 32 + 4 * 4 + 8 + 4 + 4 + 8
    offs = []
    for _ in range(n_c):
        for _f in range(3):
            nc = struct.unpack_from("<I", r1, pos)[0]
            pos += 4
            offs += [pos + 36 * i for i in range(nc)]
            pos += 36 * nc
    return offs


@pytest.mark.parametrize("name", ["compute", "pedersen_test", "poseidon3_test"])
def test_device_trace_late_bad_wire_is_rejected(ctx, name):
    """A wire id >= n_wires in the LAST record.  compute and pedersen_test use every public wire before it,
    so the host scan finds their first uses, the device trace builder does not read back, and the prover
    reports the device's flag at its first synchronisation; poseidon3_test first uses public wire 1 in that
    very record, so the scan meets the bad id and the builder reads back as before.  Both: STARK_ERR_BAD_ARG
    (3), and the context proves correctly afterwards."""
    import hashlib
    import struct
    from stark_amd import StarkError
    from stark_amd.r1cs import prove_with_witness
    r1, wt = _read(name, "r1cs"), _read(name, "wtns")
    n_wires = struct.unpack_from("<I", r1, 4 * 4 + 8 + 4 + 32)[0]
    offs = _record_offsets(r1)
    assert struct.unpack_from("<I", r1, offs[0])[0] < n_wires
    bad = bytearray(r1)
    struct.pack_into("<I", bad, offs[-1], n_wires + 5)
    with pytest.raises(StarkError) as e:
        prove_with_witness(ctx, bytes(bad), wt)
    assert e.value.code == 3
    js = prove_with_witness(ctx, r1, wt).to_json()
    assert hashlib.sha256(js.encode()).hexdigest() == GOLDEN[name]["json_sha256"]


@pytest.mark.parametrize("name", list(GOLDEN))
def test_prepared_circuit_matches_golden(ctx, name):
    """R1csCircuit (circuit-only work and LDE columns prepared once) gives the golden proof, twice."""
    from stark_amd.r1cs import R1csCircuit
    c = R1csCircuit(ctx, _read(name, "r1cs"))
    wt = _read(name, "wtns")
    for _ in range(2):
        assert hashlib.sha256(c.prove(wt).to_json().encode()).hexdigest() == GOLDEN[name]["json_sha256"]


def test_prepared_circuit_new_witnesses(ctx):
    """One prepared synthetic circuit, three witnesses: each proof equals prove_with_witness's."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import synth_r1cs
    from stark_amd.r1cs import R1csCircuit, prove_with_witness
    r1, _ = synth_r1cs.for_steps(14)
    c = R1csCircuit(ctx, r1)
    for inputs in [(11, 22), (3, 5), (R.P - 1, 7)]:
        r1b, wt = synth_r1cs.for_steps(14, inputs=inputs)
        assert r1b == r1
        assert c.prove(wt).to_json() == prove_with_witness(ctx, r1, wt).to_json()


def test_prepared_circuit_rejects_bad_inputs(ctx):
    """A witness for a different circuit size, a first value other than 1 and an unsatisfying witness."""
    from stark_amd import StarkError
    from stark_amd.r1cs import R1csCircuit
    c = R1csCircuit(ctx, _read("pedersen_test", "r1cs"))
    with pytest.raises(StarkError):
        c.prove(_read("compute", "wtns"))          # fewer witness values than the circuit's wires
    wt = bytearray(_read("pedersen_test", "wtns"))
    bad = bytearray(wt)
    bad[-32 * 1997] ^= 1                                # witness[0] != 1 (n_wit = 1997 for pedersen_test)
    with pytest.raises(StarkError):
        c.prove(bytes(bad))
    bad = bytearray(wt)
    bad[-32 * 100] ^= 1                                 # some wire value: constraints fail
    with pytest.raises(StarkError) as e:
        c.prove(bytes(bad))
    assert e.value.code == 8


def test_shared_f0_extension_under_cache_caps():
    """F0 is 1 on every trace row (calc_flags, run.rs:283-308) and Zb3 = x - x_last depends on the size
    alone, so the cold prover shares F0's extension and 1 / Zb3 per size like IDX's extension
    (csrc/r1cs.hip ext_const_column).  Bit-exact under the default cap (all three cached), under a cap of 0
    (F0 extended with the other columns, Zb3 inverted with Zb2, IDX in a per-proof buffer) and under a cap
    of one column (each reservation evicts the previous column: the prover falls back for F0 and 1 / Zb3).
    compute's precision is below the full-twiddle-table sizes, so the cache holds only these columns."""
    import stark_amd as S
    from stark_amd.r1cs import prove_with_witness
    r1, wt = _read("compute", "r1cs"), _read("compute", "wtns")
    want = GOLDEN["compute"]["json_sha256"]
    digest = lambda c: hashlib.sha256(prove_with_witness(c, r1, wt).to_json().encode()).hexdigest()  # noqa: E731
    col = 128 * 32  # one extension: os = 15 -> 16 steps -> precision 128
    c = S.Context(0)
    try:
        assert digest(c) == want
        assert c.memory()["cached"] >= 3 * col  # IDX's and F0's extensions, 1 / Zb3
        assert digest(c) == want  # from the cached extensions
    finally:
        c.close()
    for cap in (0, col):
        c = S.Context(0)
        try:
            c.set_cache_limit(cap)
            assert digest(c) == want, cap
            assert digest(c) == want, cap
            assert c.memory()["cached"] <= cap
        finally:
            c.close()
