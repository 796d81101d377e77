"""CPU: the C-ABI library loads, exports every symbol include/stark_hip.h
declares, and its host-only helpers (Blake2s, index sampler, proof
verification) match the oracle.  No GPU compute is called here."""
import ctypes
import json
import os

import pytest

import oracle as O
import stark_amd as S

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))


def test_library_exports_header_symbols():
    lib = S.load_library()
    syms = S.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # every declared symbol has a Python signature, and vice versa
    assert sorted(S._SIGNATURES) == syms


def test_status_strings():
    lib = S.load_library()
    for code in range(8):
        assert lib.stark_status_str(code)


def test_blake_host_kats():
    for v in KATS["blake"]["vectors"]:
        assert S.blake(bytes.fromhex(v["msg_hex"])).hex() == v["digest_hex"]
    for length in (0, 1, 64, 65, 200):
        msg = bytes(range(256))[:length]
        assert S.blake(msg) == O.py_blake(msg)


def test_pseudorandom_indices_host():
    for v in KATS["pseudorandom_indices"]["vectors"]:
        seed = O.py_blake(v["seed_msg"].encode())
        assert S.get_pseudorandom_indices(seed, v["modulus"], v["count"], v["exclude"]) == v["out"]
    seed = O.py_blake(b"x")
    assert S.get_pseudorandom_indices(seed, 1 << 20, 80, 8) == O.py_get_pseudorandom_indices(seed, 1 << 20, 80, 8)


def test_pseudorandom_indices_errors():
    seed = O.py_blake(b"x")
    with pytest.raises(S.StarkError):  # modulus >= 2^24 (utils.rs:88 assert)
        S.get_pseudorandom_indices(seed, 1 << 24, 4, 0)
    with pytest.raises(S.StarkError):  # real modulus 0 -> % 0 panics in the reference
        S.get_pseudorandom_indices(seed, 1, 4, 8)


def test_merkle_verify_host():
    k = KATS["merkle_16"]
    root = bytes.fromhex(k["root_hex"])
    proof = S.Proof(bytes.fromhex(k["leaf_hex"]), [bytes.fromhex(h) for h in k["nodes_hex"]])
    assert proof.validate(root, k["index"]) == bytes.fromhex(k["leaf_hex"])
    with pytest.raises(AssertionError):
        proof.validate(root, k["index"] + 1)


def test_no_gpu_fails_loudly():
    # In this container there is no GPU: the product must refuse, not fall back.
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import stark_amd as S\n"
            "try:\n    S.Context(0)\nexcept S.StarkError as e:\n    print('refused', e.code)\n"
            "else:\n    print('gpu')\n") % os.path.join(os.path.dirname(HERE), "stark-pure-rust_amd")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120).stdout
    assert out.strip() in ("refused 6", "gpu")


def test_json_view_decode():
    """StarkProof.to_json decodes the library's JSON text in place (stark_r1cs_proof_json_view)."""
    import ctypes
    from stark_amd.r1cs import ascii_at
    text = '{"m_root":[1,2,3],"x":[255,0]}' * 1000
    buf = ctypes.create_string_buffer(text.encode())
    assert ascii_at(ctypes.addressof(buf), len(text)) == text
    assert ascii_at(ctypes.addressof(buf), 0) == ""
    bad = ctypes.create_string_buffer(b"[1,\xff]")
    with pytest.raises(UnicodeDecodeError):
        ascii_at(ctypes.addressof(bad), 5)
