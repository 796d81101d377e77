"""Python mirror of packages/r1cs-stark over libstark_hip.so.

    mk_r1cs_proof(ctx, ...)            prove.rs:14-378 (GPU-resident)
    R1csTrace.build(r1cs, wtns)        read_r1cs + read_witness + run.rs:310-437
    prove_with_witness(ctx, r1cs, wtns)   run.rs:310-452
    prove_with_file_path(ctx, ...)     run.rs:528-554 (writes the proof JSON)
    R1csCircuit(ctx, r1cs).prove(wtns) the same proofs, circuit-only work done once
    StarkProof                         utils.rs:122-130 (serde_json text + roots)

Everything runs in libstark_hip.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import sys

import numpy as np

from . import Context, StarkError, _elems, _p64, _szp, _vp, load_library

# PyUnicode_DecodeASCII(const char*, Py_ssize_t, errors): one pass from the library's buffer to a str.
_decode_ascii = ctypes.pythonapi.PyUnicode_DecodeASCII
_decode_ascii.restype = ctypes.py_object
_decode_ascii.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_char_p]


def ascii_at(ptr: int, n: int) -> str:
    """The n ASCII bytes at address ptr as a str (UnicodeDecodeError on a non-ASCII byte)."""
    return _decode_ascii(ptr, n, None) if n else ""


# PyUnicode_New(n, 127): a compact ASCII str whose n + 1 data bytes follow the object header, filled by
# the library in place (stark_r1cs_proof_json copies a multi-MB text on its host workers) instead of
# one decode pass on this thread.  The header size is checked once against a known string; when the
# layout is not the expected one, to_json decodes instead.
_unicode_new = ctypes.pythonapi.PyUnicode_New
_unicode_new.restype = ctypes.py_object
_unicode_new.argtypes = [ctypes.c_ssize_t, ctypes.c_uint32]


def _ascii_header():
    try:
        h = sys.getsizeof("") - 1
        probe = "".join(["stark", "-ascii-", "probe"])
        if ctypes.string_at(id(probe) + h, len(probe) + 1) == probe.encode() + b"\0":
            return h
    except Exception:
        pass
    return None


_ASCII_HEADER = _ascii_header()


class StarkProof:
    """StarkProof<BlakeDigest> held by the library (r1cs-stark/src/utils.rs:122-130)."""

    def __init__(self, lib, h):
        self.lib = lib
        self.h = h

    def __del__(self):
        try:
            if self.h:
                self.lib.stark_r1cs_proof_free(self.h)
        except Exception:
            pass

    def to_json(self) -> str:
        """serde_json::to_string(&proof) (run.rs:549), decoded straight from the proof's own
        text (stark_r1cs_proof_json_view: no intermediate buffers for a multi-MB proof)."""
        p = ctypes.c_void_p()
        n = ctypes.c_size_t(0)
        self.lib.stark_r1cs_proof_json_view(self.h, ctypes.byref(p), ctypes.byref(n))
        if _ASCII_HEADER is None or n.value < (1 << 20):
            return ascii_at(p.value, n.value)
        s = _unicode_new(n.value, 127)
        got = ctypes.c_size_t(0)
        dst = ctypes.cast(id(s) + _ASCII_HEADER, ctypes.c_char_p)
        rc = self.lib.stark_r1cs_proof_json(self.h, dst, n.value + 1, ctypes.byref(got))
        if rc != 0 or got.value != n.value:
            raise StarkError(rc, "stark_r1cs_proof_json", f"{got.value} of {n.value} bytes")
        return s

    def roots(self) -> dict:
        m, l, a = (ctypes.create_string_buffer(32) for _ in range(3))
        self.lib.stark_r1cs_proof_roots(self.h, m, l, a)
        return {"m_root": m.raw, "l_root": l.raw, "a_root": a.raw}


def _sz(v) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(v, dtype=np.uint64).reshape(-1))
    return a if a.size else np.zeros(1, dtype=np.uint64)


def mk_r1cs_proof(ctx: Context, witness_trace, computational_trace, public_wires, public_first_indices,
                  permuted_indices, coefficients, flag0, flag1, flag2, n_constraints: int,
                  n_wires: int) -> StarkProof:
    """prove.rs:14-26 argument order; field vectors as (n, 4) canonical limbs or int lists."""
    def el(x):
        if isinstance(x, np.ndarray):
            return _elems(x)
        from . import _limbs
        return _elems(np.array([_limbs(int(v)) for v in x], dtype=np.uint64).reshape(-1, 4)) if len(x) else \
            np.zeros((0, 4), dtype=np.uint64)
    w, ct, co = el(witness_trace), el(computational_trace), el(coefficients)
    f0, f1, f2, pw = el(flag0), el(flag1), el(flag2), el(public_wires)
    os_ = len(co)
    pfi = _sz([x for pair in public_first_indices for x in pair])
    perm = _sz(permuted_indices)
    szp = lambda a: a.ctypes.data_as(_szp)
    h = _vp()
    ctx.check(ctx.lib.stark_mk_r1cs_proof(ctx.h, _p64(w), _p64(ct), os_, _p64(pw), len(pw), szp(pfi),
                                          len(public_first_indices), szp(perm), _p64(co), _p64(f0), _p64(f1),
                                          _p64(f2), n_constraints, n_wires, ctypes.byref(h)), "mk_r1cs_proof")
    return StarkProof(ctx.lib, h)


class R1csTrace:
    """The mk_r1cs_proof arguments built by the library from .r1cs/.wtns bytes."""

    def __init__(self, r1cs: bytes, wtns: bytes):
        self.lib = load_library()
        self.h = _vp()
        rc = self.lib.stark_r1cs_trace_build(r1cs, len(r1cs), wtns, len(wtns), ctypes.byref(self.h))
        if rc != 0:
            self.h = None
            raise StarkError(rc, "r1cs_trace_build")

    def __del__(self):
        try:
            if self.h:
                self.lib.stark_r1cs_trace_free(self.h)
        except Exception:
            pass

    def dims(self) -> dict:
        v = [ctypes.c_size_t(0) for _ in range(5)]
        self.lib.stark_r1cs_trace_dims(self.h, *[ctypes.byref(x) for x in v])
        keys = ("original_steps", "n_public", "n_public_first", "n_constraints", "n_wires")
        return dict(zip(keys, (x.value for x in v)))

    def export(self) -> dict:
        d = self.dims()
        n = d["original_steps"]
        arrs = {k: np.zeros((n, 4), dtype=np.uint64) for k in ("witness_trace", "computational_trace",
                                                               "coefficients", "flag0", "flag1", "flag2")}
        perm = np.zeros(max(n, 1), dtype=np.uint64)
        pw = np.zeros((max(d["n_public"], 1), 4), dtype=np.uint64)
        pfi = np.zeros(max(2 * d["n_public_first"], 1), dtype=np.uint64)
        szp = lambda a: a.ctypes.data_as(_szp)
        self.lib.stark_r1cs_trace_export(self.h, *[_p64(arrs[k]) for k in ("witness_trace", "computational_trace",
                                                                           "coefficients", "flag0", "flag1",
                                                                           "flag2")],
                                         szp(perm), _p64(pw), szp(pfi))
        arrs["permuted_indices"] = [int(x) for x in perm[:n]]
        arrs["public_wires"] = pw[:d["n_public"]]
        arrs["public_first_indices"] = [(int(pfi[2 * i]), int(pfi[2 * i + 1])) for i in range(d["n_public_first"])]
        arrs.update(n_constraints=d["n_constraints"], n_wires=d["n_wires"])
        return arrs


def prove_with_witness(ctx: Context, r1cs: bytes, wtns: bytes) -> StarkProof:
    """run.rs:310-452, the trace built on the GPU (stark_prove_r1cs_bytes)."""
    h = _vp()
    ctx.check(ctx.lib.stark_prove_r1cs_bytes(ctx.h, r1cs, len(r1cs), wtns, len(wtns), ctypes.byref(h)),
              "prove_with_witness")
    return StarkProof(ctx.lib, h)


def prove_with_witness_host_trace(ctx: Context, r1cs: bytes, wtns: bytes) -> StarkProof:
    """run.rs:310-452 with the host trace builder (R1csTrace) feeding the same prover."""
    tr = R1csTrace(r1cs, wtns)
    h = _vp()
    ctx.check(ctx.lib.stark_prove_r1cs_trace(ctx.h, tr.h, ctypes.byref(h)), "prove_with_witness")
    return StarkProof(ctx.lib, h)


class R1csCircuit:
    """A circuit prepared once for many proofs (stark_r1cs_circuit_new): everything of
    prove_with_witness (run.rs:310-452) that depends on the .r1cs alone, including the
    LDEs of K, F0-F2, IDX and PIDX, stays in HBM; prove(wtns) extends only S, P and A.
    The proofs equal prove_with_witness(ctx, r1cs, wtns)."""

    def __init__(self, ctx: Context, r1cs: bytes):
        self.ctx = ctx
        self.h = _vp()
        ctx.check(ctx.lib.stark_r1cs_circuit_new(ctx.h, r1cs, len(r1cs), ctypes.byref(self.h)), "r1cs_circuit_new")

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.stark_r1cs_circuit_free(self.h)
        except Exception:
            pass

    def prove(self, wtns: bytes) -> StarkProof:
        h = _vp()
        self.ctx.check(self.ctx.lib.stark_prove_r1cs_circuit(self.ctx.h, self.h, wtns, len(wtns), ctypes.byref(h)),
                       "prove_r1cs_circuit")
        return StarkProof(self.ctx.lib, h)


def prove_with_file_path(ctx: Context, r1cs_file_path: str, witness_file_path: str, proof_json_path: str) -> None:
    """run.rs:528-554."""
    with open(r1cs_file_path, "rb") as f:
        r1cs = f.read()
    with open(witness_file_path, "rb") as f:
        wtns = f.read()
    proof = prove_with_witness(ctx, r1cs, wtns)
    with open(proof_json_path, "w") as f:
        f.write(proof.to_json())
