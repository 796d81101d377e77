"""Verifier over libstark_hip.so: verify_low_degree_proof (packages/fri/src/fri.rs:226-404),
verify_with_witness / verify_r1cs_proof (packages/r1cs-stark/src/run.rs:454-526,
verify.rs:13-258) and verify_with_file_path (run.rs:556-592).

Like the reference, a proof that fails a check raises AssertionError; malformed input
(including JSON that is not a StarkProof) raises StarkError.  The circuit-only
extensions (K, F0-F2, IDX, PIDX) come from a prepared circuit on the GPU; the FRI
verifier alone is host code (stark_verify_low_degree_proof needs no device).
"""
from __future__ import annotations

import ctypes
import json

from . import Context, StarkError, _limbs, load_library

STARK_ERR_CHECK = 8


class _Branches(ctypes.Structure):
    """stark_branches: k proofs with leaf_len-byte leaves and depth 32-byte nodes each."""
    _fields_ = [("leaves", ctypes.c_char_p), ("nodes", ctypes.c_char_p), ("k", ctypes.c_size_t),
                ("leaf_len", ctypes.c_size_t), ("depth", ctypes.c_size_t)]


class _FriLayer(ctypes.Structure):
    _fields_ = [("root2", ctypes.c_char_p), ("column", _Branches), ("poly", _Branches)]


def _uniform_branches(proofs: list, keep: list) -> _Branches:
    """serde Proof dicts ({"leaf": [...], "nodes": [[...], ...]}) as one stark_branches."""
    leaf_len = len(proofs[0]["leaf"]) if proofs else 0
    depth = len(proofs[0]["nodes"]) if proofs else 0
    if any(len(p["leaf"]) != leaf_len or len(p["nodes"]) != depth for p in proofs):
        raise StarkError(3, "verify_low_degree_proof", "branches of unequal shape")
    leaves = b"".join(bytes(p["leaf"]) for p in proofs)
    nodes = b"".join(bytes(n) for p in proofs for n in p["nodes"])
    keep += [leaves, nodes]
    return _Branches(leaves, nodes, len(proofs), leaf_len, depth)


def _result(rc: int, where: str) -> bool:
    if rc == STARK_ERR_CHECK:
        raise AssertionError(f"{where}: the proof does not verify")
    if rc != 0:
        raise StarkError(rc, where)
    return True


def verify_low_degree_proof(merkle_root: bytes, root_of_unity: int, proof, max_deg_plus_1: int,
                            exclude_multiples_of: int) -> bool:
    """fri.rs:226-242.  `proof` = Vec<FriProof> as parsed serde JSON (list) or its text."""
    if isinstance(proof, (str, bytes)):
        proof = json.loads(proof)
    lib = load_library()
    keep = []
    if not proof or "Last" not in proof[-1] or any("Middle" not in x for x in proof[:-1]):
        raise StarkError(3, "verify_low_degree_proof", "Middle layers then one Last layer expected")
    mids = [x["Middle"] for x in proof[:-1]]
    arr = (_FriLayer * max(len(mids), 1))()
    for i, m in enumerate(mids):
        root2 = bytes(m["root2"])
        keep.append(root2)
        arr[i] = _FriLayer(root2, _uniform_branches(m["column_branches"], keep),
                           _uniform_branches(m["poly_branches"], keep))
    last = [bytes(v) for v in proof[-1]["Last"]["last"]]
    ptrs = (ctypes.c_char_p * max(len(last), 1))(*last)
    lens = (ctypes.c_size_t * max(len(last), 1))(*[len(v) for v in last])
    root = _limbs(root_of_unity)
    rc = lib.stark_verify_low_degree_proof(bytes(merkle_root), root.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                           ctypes.cast(arr, ctypes.c_void_p), len(mids), ctypes.cast(ptrs, ctypes.c_void_p),
                                           lens, len(last), max_deg_plus_1, exclude_multiples_of)
    return _result(rc, "verify_low_degree_proof")


def _json_bytes(proof) -> bytes:
    if isinstance(proof, bytes):
        return proof
    if isinstance(proof, str):
        return proof.encode()
    return json.dumps(proof, separators=(",", ":")).encode()


def _wire_bytes(public_wires) -> bytes:
    """Public wires as 32-byte little-endian integers (ints, or byte strings as read_witness gives)."""
    out = []
    for w in public_wires:
        b = w.to_bytes(32, "little") if isinstance(w, int) else bytes(w)
        if len(b) > 32:
            raise StarkError(3, "verify_with_witness", "public wire wider than 32 bytes")
        out.append(b.ljust(32, b"\0"))
    return b"".join(out)


def verify_with_witness(ctx: Context, r1cs: bytes, public_wires, proof) -> bool:
    """run.rs:454-526: `public_wires` = witness[..1 + n_public_inputs + n_public_outputs]."""
    js = _json_bytes(proof)
    pub = _wire_bytes(public_wires)
    rc = ctx.lib.stark_verify_r1cs_bytes(ctx.h, r1cs, len(r1cs), pub, len(pub) // 32, js, len(js))
    return _result(rc, "verify_with_witness")


def verify_circuit(ctx: Context, circuit, public_wires, proof) -> bool:
    """verify_with_witness on an R1csCircuit (the circuit's extensions already in HBM)."""
    js = _json_bytes(proof)
    pub = _wire_bytes(public_wires)
    rc = ctx.lib.stark_verify_r1cs_circuit(ctx.h, circuit.h, pub, len(pub) // 32, js, len(js))
    return _result(rc, "verify_with_witness")


def verify_with_wtns(ctx: Context, r1cs: bytes, wtns: bytes, proof) -> bool:
    """verify_with_file_path (run.rs:556-592) on file contents."""
    js = _json_bytes(proof)
    rc = ctx.lib.stark_verify_with_witness(ctx.h, r1cs, len(r1cs), wtns, len(wtns), js, len(js))
    return _result(rc, "verify_with_file_path")


def verify_with_file_path(ctx: Context, r1cs_file_path: str, witness_file_path: str, proof_json_path: str) -> None:
    """run.rs:556-592."""
    with open(r1cs_file_path, "rb") as f:
        r1cs = f.read()
    with open(witness_file_path, "rb") as f:
        wtns = f.read()
    with open(proof_json_path, "rb") as f:
        js = f.read()
    verify_with_wtns(ctx, r1cs, wtns, js)
