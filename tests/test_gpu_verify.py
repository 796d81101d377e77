"""The product verifier (stark_verify_r1cs_* in libstark_hip.so, stark_amd/verify.py):
verify_with_witness / verify_with_file_path (run.rs:454-592) -> verify_r1cs_proof
(verify.rs:13-258) with the circuit's extensions from a prepared circuit on the GPU.

It must accept every golden proof (each equal to the oracle's, test_gpu_r1cs.py) and
a synthetic one, and reject what the restated verifier (oracle/stark_verify.py)
rejects: tampered leaves, paths, roots, public wires and FRI layers."""
import copy
import hashlib
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "r1cs")
GOLDEN = json.load(open(os.path.join(HERE, "golden", "r1cs_proofs.json")))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))

pytestmark = pytest.mark.gpu


def _read(name, ext):
    with open(os.path.join(FIX, f"{name}.{ext}"), "rb") as f:
        return f.read()


@pytest.fixture(scope="module")
def proofs(ctx):
    from stark_amd.r1cs import prove_with_witness
    out = {}
    for name in GOLDEN:
        r1, wt = _read(name, "r1cs"), _read(name, "wtns")
        js = prove_with_witness(ctx, r1, wt).to_json()
        assert hashlib.sha256(js.encode()).hexdigest() == GOLDEN[name]["json_sha256"]
        out[name] = (r1, wt, js)
    return out


@pytest.mark.parametrize("name", list(GOLDEN))
def test_accepts_golden_proofs(ctx, proofs, name):
    from stark_amd.verify import verify_with_wtns
    r1, wt, js = proofs[name]
    assert verify_with_wtns(ctx, r1, wt, js)


def test_verify_with_file_path(ctx, proofs, tmp_path):
    from stark_amd.verify import verify_with_file_path
    r1, wt, js = proofs["pedersen_test"]
    (tmp_path / "p.json").write_text(js)
    verify_with_file_path(ctx, os.path.join(FIX, "pedersen_test.r1cs"), os.path.join(FIX, "pedersen_test.wtns"),
                          str(tmp_path / "p.json"))


def _tampered(js):
    """(what, proof dict) pairs: each must be rejected with AssertionError."""
    p = json.loads(js)
    out = []
    def t(what, f):
        q = copy.deepcopy(p)
        f(q)
        out.append((what, q))
    t("main leaf", lambda q: q["main_branches"][0]["leaf"].__setitem__(40, q["main_branches"][0]["leaf"][40] ^ 1))
    t("main node", lambda q: q["main_branches"][7]["nodes"][2].__setitem__(0, q["main_branches"][7]["nodes"][2][0] ^ 1))
    t("lcomb leaf", lambda q: q["linear_comb_branches"][3]["leaf"].__setitem__(0, q["linear_comb_branches"][3]["leaf"][0] ^ 4))
    t("m_root", lambda q: q["m_root"].__setitem__(5, q["m_root"][5] ^ 1))
    t("a_root", lambda q: q["a_root"].__setitem__(0, q["a_root"][0] ^ 1))
    t("l_root", lambda q: q["l_root"].__setitem__(31, q["l_root"][31] ^ 1))
    t("fri column", lambda q: q["fri_proof"][0]["Middle"]["column_branches"][1]["leaf"].__setitem__(
        3, q["fri_proof"][0]["Middle"]["column_branches"][1]["leaf"][3] ^ 1))
    t("fri last", lambda q: q["fri_proof"][-1]["Last"]["last"][2].__setitem__(
        0, q["fri_proof"][-1]["Last"]["last"][2][0] ^ 1))
    return out


@pytest.mark.parametrize("name", ["compute", "pedersen_test"])
def test_rejects_tampered_proofs(ctx, oracle, proofs, name):
    import r1cs as R
    from stark_amd.verify import verify_with_wtns
    from stark_verify import verify_r1cs_proof
    r1, wt, js = proofs[name]
    tr = R.build_trace(*R.load_fixture(FIX, name))
    for what, q in _tampered(js):
        with pytest.raises(AssertionError):
            verify_with_wtns(ctx, r1, wt, q)
        with pytest.raises(AssertionError):  # the restated verifier agrees
            verify_r1cs_proof(oracle, q, tr.public_wires, tr.public_first_indices, tr.permuted_indices,
                              tr.coefficients, tr.flag0, tr.flag1, tr.flag2, tr.n_constraints, tr.n_wires)


def test_rejects_wrong_public_wires(ctx, proofs):
    import r1cs as R
    from stark_amd.verify import verify_with_witness
    r1, wt, js = proofs["pedersen_test"]
    tr = R.build_trace(*R.load_fixture(FIX, "pedersen_test"))
    pub = list(tr.public_wires)
    assert verify_with_witness(ctx, r1, pub, js)
    bad = pub[:]
    bad[1] = (bad[1] + 1)
    with pytest.raises(AssertionError):
        verify_with_witness(ctx, r1, bad, js)
    with pytest.raises(AssertionError):          # public_wires[0] must be one (run.rs:480)
        verify_with_witness(ctx, r1, [2] + pub[1:], js)
    # The reference takes boundary points from every supplied wire (run.rs:503-509): a count other
    # than the header's 1 + n_pub_in + n_pub_out is refused (STARK_ERR_BAD_ARG), never truncated.
    from stark_amd import StarkError
    for wrong in (pub + [5], pub[:-1]):
        with pytest.raises(StarkError) as e:
            verify_with_witness(ctx, r1, wrong, js)
        assert e.value.code == 3


def test_rejects_proof_of_other_circuit(ctx, proofs):
    from stark_amd.verify import verify_with_wtns
    r1, wt, _ = proofs["compute"]
    with pytest.raises(AssertionError):
        verify_with_wtns(ctx, r1, wt, proofs["poseidon3_test"][2])


def test_malformed_json_raises(ctx, proofs):
    from stark_amd import StarkError
    from stark_amd.verify import verify_with_wtns
    r1, wt, js = proofs["compute"]
    for bad in [js[:-1], js.replace('"m_root"', '"x_root"'), "{}", js + "x", js.replace("[", "[300,", 1)]:
        with pytest.raises(StarkError):
            verify_with_wtns(ctx, r1, wt, bad)


def test_json_reader_arena_edges(ctx, proofs):
    """The proof reader writes every opening's bytes into one arena sized from the text (a number takes
    two characters at least).  Whitespace anywhere serde_json allows it still verifies (the reader
    accepts it as serde_json does); adversarial texts -- truncations at many points, short and long
    digests, over-long leaves of one-digit numbers, 4-digit numbers -- are refused (StarkError or
    AssertionError), never a crash or an acceptance."""
    from stark_amd import StarkError
    from stark_amd.verify import verify_with_wtns
    r1, wt, js = proofs["pedersen_test"]
    spaced = js.replace(",", ", ").replace(":", " : ").replace("[", "[ ")
    assert verify_with_wtns(ctx, r1, wt, spaced)
    q = json.loads(js)
    bad = []
    for cut in range(7, len(js), max(1, len(js) // 23)):
        bad.append(js[:cut])
    b = json.loads(js)
    b["main_branches"][3]["nodes"][2] = [1]  # a short digest
    bad.append(json.dumps(b, separators=(",", ":")))
    b = json.loads(js)
    b["main_branches"][5]["nodes"][0] = list(range(33))  # a long digest
    bad.append(json.dumps(b, separators=(",", ":")))
    b = json.loads(js)
    b["linear_comb_branches"][1]["leaf"] = [1] * 5000  # a long leaf of one-digit numbers
    bad.append(json.dumps(b, separators=(",", ":")))
    b = json.loads(js)
    b["fri_proof"][0]["Middle"]["poly_branches"][7]["nodes"] = [[1] * 32] * 4000  # many nodes
    bad.append(json.dumps(b, separators=(",", ":")))
    bad.append(js.replace("[", "[0255,", 1))
    bad.append(js.replace("]]", "],[]]", 3))
    # a leading zero on a leaf value, the array otherwise intact: serde_json refuses "07" (no value changes,
    # so only the reader can reject it)
    at = js.index('"leaf":[') + len('"leaf":[')
    bad.append(js[:at] + "0" + js[at:])
    assert q["main_branches"]  # (the fixture is a full proof)
    for t in bad:
        with pytest.raises((StarkError, AssertionError)):
            verify_with_wtns(ctx, r1, wt, t)
    assert verify_with_wtns(ctx, r1, wt, js)  # the context is still good


def test_prepared_circuit_verifies_many(ctx):
    """R1csCircuit + verify_circuit on a synthetic 2^13-step circuit, two witnesses."""
    import synth_r1cs
    from stark_amd.r1cs import R1csCircuit
    from stark_amd.verify import verify_circuit
    r1, _ = synth_r1cs.for_steps(13)
    c = R1csCircuit(ctx, r1)
    import r1cs as R
    for inputs in [(5, 6), (7, 8)]:
        _, wt = synth_r1cs.for_steps(13, inputs=inputs)
        js = c.prove(wt).to_json()
        h = R.read_r1cs(r1).header
        n_pub = 1 + h.n_public_inputs + h.n_public_outputs
        pub = R.read_witness(wt)[:n_pub]
        assert verify_circuit(ctx, c, pub, js)
        q = json.loads(js)
        q["linear_comb_branches"][0]["leaf"][1] ^= 1
        with pytest.raises(AssertionError):
            verify_circuit(ctx, c, pub, q)


def test_cold_verify_under_cache_caps(proofs):
    """The cold verifier makes no extension: it evaluates K, F0-F2, IDX and PIDX at its spot positions from
    their first forward passes (csrc/r1cs.hip circuit_spot_values), F0's and IDX's from the context's
    capped cache when it holds them (default cap), else computed with the others (cap 0; a cap of one
    column, where IDX's reservation evicts F0's).  Each case accepts the golden proof and rejects a
    tampered one, twice per context, and the prover beside it (whose shared F0 / IDX / 1/Zb3 columns use
    the same cache) still gives the golden digest."""
    import stark_amd as S
    from stark_amd.r1cs import prove_with_witness
    from stark_amd.verify import verify_with_wtns
    r1, wt, js = proofs["compute"]
    col = 128 * 32  # one extension: os = 15 -> 16 steps -> precision 128
    bad = json.loads(js)
    bad["linear_comb_branches"][0]["leaf"][1] ^= 1
    for cap in (None, 0, col):
        c = S.Context(0)
        try:
            if cap is not None:
                c.set_cache_limit(cap)
            for _ in range(2):  # the second call finds whatever the first one cached
                assert verify_with_wtns(c, r1, wt, js), cap
                with pytest.raises(AssertionError):
                    verify_with_wtns(c, r1, wt, bad)
            if cap is not None:
                assert c.memory()["cached"] <= cap
            js2 = prove_with_witness(c, r1, wt).to_json()
            assert hashlib.sha256(js2.encode()).hexdigest() == GOLDEN["compute"]["json_sha256"], cap
        finally:
            c.close()


@pytest.mark.parametrize("log_steps", [16, 17, 20])
def test_cold_verify_synthetic_spot_sizes(ctx, log_steps):
    """Cold verify_with_wtns of synthetic 2^16-, 2^17- and 2^20-step proofs: first passes of radix 2^6, 2^8
    (the 16 x 16 kernel, sparse, of 2^20's (8, 4, 8) plan) and 2^7, with runs of A = 2^13, 2^12 and 2^16
    values per column and position split over 8, 4 and 16 workgroups per position (circuit_spot_values).
    Accepts the prover's proof; a flipped main-branch leaf byte (P at a spot position) and a flipped L
    leaf are rejected."""
    import synth_r1cs
    from stark_amd.r1cs import prove_with_witness
    from stark_amd.verify import verify_with_wtns
    r1, wt = synth_r1cs.for_steps(log_steps)
    js = prove_with_witness(ctx, r1, wt).to_json()
    assert verify_with_wtns(ctx, r1, wt, js)
    p = json.loads(js)
    for path in (("main_branches", 1, 5), ("linear_comb_branches", 7, 30)):
        q = copy.deepcopy(p)
        q[path[0]][path[1]]["leaf"][path[2]] ^= 1
        with pytest.raises(AssertionError):
            verify_with_wtns(ctx, r1, wt, q)



def test_json_reader_follows_serde_on_fields(ctx, proofs):
    """serde_json (run.rs:579, no deny_unknown_fields on StarkProof / Proof / FriProof) ignores members it
    does not know -- any JSON value, escapes and nesting included -- matches member names after
    unescaping, and refuses a duplicate field.  The reader does the same: extra members at every level
    and reordered, escaped names still verify; duplicates, a bad escape and a leading zero inside an
    ignored member are refused (StarkError)."""
    from stark_amd import StarkError
    from stark_amd.verify import verify_with_wtns
    r1, wt, js = proofs["compute"]
    p = json.loads(js)
    junk = {"a": [1, -2.5e3, {"b": None, "c": [True, False, [], {}]}], "s": 'q"é\U0001F600 \x00/'}
    q = {"extra": junk}
    q.update(p)
    q["zzz"] = 0
    m0 = q["main_branches"][0]
    q["main_branches"][0] = {"nodes": m0["nodes"], "x": junk, "leaf": m0["leaf"]}
    q["linear_comb_branches"][1]["y"] = "z"
    q["fri_proof"][0]["Middle"]["extra"] = [junk, 7]
    q["fri_proof"][-1]["Last"]["e"] = {"k": junk}
    text = json.dumps(q, separators=(",", ":"))
    assert "\\u00e9" in text and "\\ud83d\\ude00" in text
    text = text.replace('"root2"', '"root\\u0032"', 1)
    assert verify_with_wtns(ctx, r1, wt, text)
    dup_top = js[:-1] + ',"a_root":' + json.dumps(p["a_root"], separators=(",", ":")) + "}"
    leaf = json.dumps(p["main_branches"][2]["leaf"], separators=(",", ":"))
    dup_leaf = js.replace('{"leaf":' + leaf, '{"leaf":' + leaf + ',"leaf":' + leaf, 1)
    assert dup_leaf != js
    bad_escape = text.replace("\\u00e9", "\\x00e9", 1)
    lead_zero = js.replace("{", '{"u":01,', 1)
    for t in (dup_top, dup_leaf, bad_escape, lead_zero):
        with pytest.raises(StarkError):
            verify_with_wtns(ctx, r1, wt, t)


@pytest.mark.parametrize("name", ["compute", "pedersen_test"])
def test_json_reader_nested_branch_objects(ctx, proofs, name):
    """An unknown member whose value is itself Branch-shaped ({"leaf":..,"nodes":..}) inside an opening is
    skipped by serde_json, so the proof still verifies; the reader's parallel pre-parse starts a parse at
    the nested key too, and must neither let it overwrite the opening's bytes nor take it for the opening
    (ADVICE r5).  pedersen's text is large enough for the parallel parse to run on several threads.  The
    same nesting with the real bytes inside and wrong ones outside is refused."""
    from stark_amd import StarkError
    from stark_amd.verify import verify_with_wtns
    r1, wt, js = proofs[name]
    p = json.loads(js)
    mb = p["main_branches"]
    for i in range(0, len(mb), 7):            # every 7th main opening gets a decoy with other bytes
        other = mb[(i + 1) % len(mb)]
        decoy = {"leaf": other["leaf"] + other["leaf"], "nodes": other["nodes"] + other["nodes"]}
        mb[i] = {"leaf": mb[i]["leaf"], "x": decoy, "nodes": mb[i]["nodes"]}
    lb = p["linear_comb_branches"]
    lb[0] = {"x": {"leaf": [9] * 300, "nodes": [[1] * 32] * 40}, "leaf": lb[0]["leaf"], "nodes": lb[0]["nodes"]}
    text = json.dumps(p, separators=(",", ":"))
    assert verify_with_wtns(ctx, r1, wt, text)
    # the real opening inside, a wrong one outside: the outer is what serde reads, so it fails
    q = json.loads(js)
    b = q["main_branches"][3]
    wrong = {"leaf": [(v + 1) % 256 for v in b["leaf"]], "nodes": b["nodes"]}
    q["main_branches"][3] = {"leaf": wrong["leaf"], "x": b, "nodes": wrong["nodes"]}
    with pytest.raises((StarkError, AssertionError)):
        verify_with_wtns(ctx, r1, wt, json.dumps(q, separators=(",", ":")))
