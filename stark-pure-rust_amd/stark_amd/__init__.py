"""Python mirror of the reference's hot-path API over libstark_hip.so.

Names, argument meaning and error behaviour follow the Rust items the C ABI
replaces (see include/stark_hip.h for file:line citations):

    fri::fft::{best_fft, inv_best_fft, expand_root_of_unity, serial_fft}
    fri::poly_utils::{multi_inv, eval_poly_at}
    fri::utils::{blake, get_pseudorandom_indices}
    commitment::merkle_proof_in_place::MerkleProofInPlace (MerkleTree trait)
    commitment::merkle_tree::{Proof, verify_multi_branch}
    fri::fri::prove_low_degree -> list of FriProof (serde-JSON identical)

Field elements are numpy (n, 4) uint64 arrays of canonical little-endian limbs
(the to_bytes_le image).  Every computation runs in libstark_hip.so on a
gfx950 GPU; there is no CPU fallback: a missing library or GPU raises.
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libstark_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "stark_hip.h")

P = 21888242871839275222246405745257275088548364400416034343698204186575808495617

STATUS = {0: "ok", 1: "bad length", 2: "bad root", 3: "bad argument", 4: "out of memory", 5: "HIP error",
          6: "no gfx950 device", 7: "bad call order", 8: "constraint check failed"}


class StarkError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = code
        super().__init__(f"{where}: {STATUS.get(code, code)}" + (f" ({detail})" if detail else ""))


_u64p = ctypes.POINTER(ctypes.c_uint64)
_u8p = ctypes.c_char_p
_szp = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p

_SIGNATURES = {
    "stark_abi_version": ([], ctypes.c_uint32),
    "stark_verify_simd_width": ([], ctypes.c_uint32),
    "stark_json_simd_width": ([], ctypes.c_uint32),
    "stark_ctx_create": ([ctypes.c_int, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_ctx_destroy": ([_vp], None),
    "stark_status_str": ([ctypes.c_int], ctypes.c_char_p),
    "stark_ctx_last_error": ([_vp], ctypes.c_char_p),
    "stark_ctx_stream": ([_vp], _vp),
    "stark_ctx_set_cache_limit": ([_vp, ctypes.c_size_t], ctypes.c_int),
    "stark_ctx_memory": ([_vp, _szp, _szp, _szp], ctypes.c_int),
    "stark_best_fft": ([_vp, _u64p, ctypes.c_size_t, _u64p, ctypes.c_uint32, _u64p], ctypes.c_int),
    "stark_inv_best_fft": ([_vp, _u64p, ctypes.c_size_t, _u64p, ctypes.c_uint32, _u64p], ctypes.c_int),
    "stark_fft_in_place": ([_vp, _u64p, _u64p, ctypes.c_uint32, ctypes.c_int], ctypes.c_int),
    "stark_ntt_dev": ([_vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _u64p, ctypes.c_int, _vp], ctypes.c_int),
    "stark_ntt_plan": ([ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32], ctypes.c_uint32),
    "stark_expand_root_of_unity": ([_vp, _u64p, _u64p, ctypes.c_size_t, _szp], ctypes.c_int),
    "stark_multi_inv": ([_vp, _u64p, ctypes.c_size_t, _u64p], ctypes.c_int),
    "stark_eval_poly_at_multi": ([_vp, _u64p, ctypes.c_size_t, _u64p, ctypes.c_size_t, _u64p], ctypes.c_int),
    "stark_blake": ([_u8p, ctypes.c_size_t, _u8p], None),
    "stark_get_pseudorandom_indices": ([_u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "stark_merkle_new": ([_vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_merkle_free": ([_vp], None),
    "stark_merkle_update": ([_vp, _u8p, ctypes.c_size_t, ctypes.c_size_t], ctypes.c_int),
    "stark_merkle_update_dev": ([_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, _vp], ctypes.c_int),
    "stark_merkle_width": ([_vp], ctypes.c_size_t),
    "stark_merkle_leaf_len": ([_vp], ctypes.c_size_t),
    "stark_merkle_get_root": ([_vp, _u8p, _szp], ctypes.c_int),
    "stark_merkle_gen_proofs": ([_vp, _szp, ctypes.c_size_t, _u8p, _u8p], ctypes.c_int),
    "stark_merkle_verify": ([_u8p, _szp, ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t],
                            ctypes.c_int),
    "stark_prove_low_degree": ([_vp, _u64p, ctypes.c_size_t, _u64p, ctypes.c_size_t, ctypes.c_uint32,
                                ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_prove_low_degree_dev": ([_vp, _vp, ctypes.c_size_t, _u64p, ctypes.c_size_t, ctypes.c_uint32,
                                    ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_fri_proof_free": ([_vp], None),
    "stark_fri_proof_json": ([_vp, ctypes.c_char_p, ctypes.c_size_t, _szp], ctypes.c_int),
    "stark_fri_proof_num_layers": ([_vp], ctypes.c_size_t),
    "stark_fri_proof_layer_info": ([_vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), _u8p, _szp, _szp, _szp,
                                    _szp, _szp], ctypes.c_int),
    "stark_fri_proof_layer_data": ([_vp, ctypes.c_size_t] + [_u8p, ctypes.c_size_t] * 5, ctypes.c_int),
    "stark_mk_r1cs_proof": ([_vp, _u64p, _u64p, ctypes.c_size_t, _u64p, ctypes.c_size_t, _szp, ctypes.c_size_t,
                             _szp, _u64p, _u64p, _u64p, _u64p, ctypes.c_size_t, ctypes.c_size_t,
                             ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_r1cs_proof_json": ([_vp, ctypes.c_char_p, ctypes.c_size_t, _szp], ctypes.c_int),
    "stark_r1cs_proof_json_view": ([_vp, ctypes.POINTER(ctypes.c_void_p), _szp], ctypes.c_int),
    "stark_r1cs_proof_roots": ([_vp, _u8p, _u8p, _u8p], ctypes.c_int),
    "stark_r1cs_proof_branches": ([_vp, ctypes.c_int, _szp, _szp, _szp, _u8p, ctypes.c_size_t, _u8p,
                                   ctypes.c_size_t], ctypes.c_int),
    "stark_r1cs_proof_fri": ([_vp], _vp),
    "stark_r1cs_proof_free": ([_vp], None),
    "stark_r1cs_trace_build": ([_u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_r1cs_trace_dims": ([_vp, _szp, _szp, _szp, _szp, _szp], ctypes.c_int),
    "stark_r1cs_trace_export": ([_vp, _u64p, _u64p, _u64p, _u64p, _u64p, _u64p, _szp, _u64p, _szp], ctypes.c_int),
    "stark_r1cs_trace_free": ([_vp], None),
    "stark_prove_r1cs_trace": ([_vp, _vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_prove_r1cs_bytes": ([_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_lde": ([_vp, _u64p, ctypes.c_size_t, _u64p, ctypes.c_uint32, _u64p, _u64p], ctypes.c_int),
    "stark_lde_dev": ([_vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u64p, _vp],
                      ctypes.c_int),
    "stark_multi_interp_4": ([_vp, _u64p, _u64p, ctypes.c_size_t, _u64p], ctypes.c_int),
    "stark_eval_quartic_multi": ([_vp, _u64p, _u64p, ctypes.c_size_t, _u64p], ctypes.c_int),
    "stark_lincomb": ([_vp, _u64p, ctypes.c_uint32, ctypes.c_size_t, _u64p, _u64p], ctypes.c_int),
    "stark_lincomb_dev": ([_vp, _vp, ctypes.c_uint32, ctypes.c_size_t, _u64p, _vp, _vp], ctypes.c_int),
    "stark_ntt_strided_dev": ([_vp, _vp, ctypes.c_uint32, ctypes.c_size_t, _u64p, ctypes.c_int, _vp], ctypes.c_int),
    "stark_ntt_strided_tw_dev": ([_vp, _vp, ctypes.c_uint32, ctypes.c_size_t, _u64p, ctypes.c_int, _u64p,
                                  ctypes.c_uint32, ctypes.c_uint64, _vp], ctypes.c_int),
    "stark_transpose_dev": ([_vp, _vp, _vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32, _vp], ctypes.c_int),
    "stark_twiddle2d_dev": ([_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64, _u64p,
                             ctypes.c_uint32, _vp], ctypes.c_int),
    "stark_dev_alloc": ([_vp, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_dev_free": ([_vp, _vp], ctypes.c_int),
    "stark_memcpy_h2d": ([_vp, _vp, _vp, ctypes.c_size_t], ctypes.c_int),
    "stark_memcpy_d2h": ([_vp, _vp, _vp, ctypes.c_size_t], ctypes.c_int),
    "stark_ctx_synchronize": ([_vp], ctypes.c_int),
    "stark_merkle_leaf_digests_dev": ([_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, _vp, _vp], ctypes.c_int),
    "stark_merkle_update_digests_dev": ([_vp, _vp, ctypes.c_size_t, ctypes.c_uint32, _vp], ctypes.c_int),
    "stark_open_batch": ([_vp, _vp, ctypes.c_size_t, _vp], ctypes.c_int),
    "stark_r1cs_circuit_new": ([_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_r1cs_circuit_free": ([_vp], None),
    "stark_prove_r1cs_circuit": ([_vp, _vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_dprove_circuit_new": ([_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t,
                                  ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_dprove_begin_circuit": ([_vp, _vp, ctypes.c_char_p, ctypes.c_size_t, _vp, ctypes.POINTER(_vp)],
                                   ctypes.c_int),
    "stark_fri_fold_dev": ([_vp, _vp, _vp, ctypes.c_size_t, _u64p, _u8p, ctypes.c_uint32, ctypes.c_uint32, _vp],
                           ctypes.c_int),
    "stark_fri_fold_dev_root": ([_vp, _vp, _vp, ctypes.c_size_t, _u64p, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp],
                                ctypes.c_int),
    "stark_merkle_root_dev": ([_vp, _vp, _vp], ctypes.c_int),
    "stark_cyclic_ntt_local_dev": ([_vp, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u64p, ctypes.c_int,
                                    _vp], ctypes.c_int),
    "stark_merkle_top_dev": ([_vp, _vp, ctypes.c_size_t, _vp, _vp], ctypes.c_int),
    "stark_dprove_lincomb_dev": ([_vp, _vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_r1cs_proof_json_from_parts": ([_u8p, _u8p, _u8p, _vp, _vp, _vp, ctypes.c_size_t, _u8p, ctypes.c_size_t,
                                          ctypes.c_char_p, ctypes.c_size_t, _szp], ctypes.c_int),
    "stark_dprove_begin": ([_vp, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u64p, ctypes.c_size_t, _u64p,
                            ctypes.c_size_t, _szp, ctypes.c_size_t, _szp, _u64p, _u64p, _u64p, _u64p, ctypes.c_size_t,
                            ctypes.c_size_t, _vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_dprove_begin_bytes": ([_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t,
                                  ctypes.c_char_p, ctypes.c_size_t, _vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_dprove_info": ([_vp, _szp, _szp, _szp, _u64p, _u8p], ctypes.c_int),
    "stark_dprove_rows": ([_vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_dprove_lincomb": ([_vp, _u8p, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_dprove_free": ([_vp], None),
    "stark_verify_low_degree_proof": ([_u8p, _u64p, _vp, ctypes.c_size_t, _vp, _szp, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.c_uint32], ctypes.c_int),
    "stark_verify_r1cs_circuit": ([_vp, _vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t],
                                  ctypes.c_int),
    "stark_verify_r1cs_bytes": ([_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                 ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "stark_group_create": ([ctypes.POINTER(ctypes.c_int), ctypes.c_uint32, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_group_destroy": ([_vp], None),
    "stark_group_size": ([_vp], ctypes.c_uint32),
    "stark_group_ctx": ([_vp, ctypes.c_uint32], _vp),
    "stark_group_last_error": ([_vp], ctypes.c_char_p),
    "stark_group_synchronize": ([_vp], ctypes.c_int),
    "stark_group_best_fft": ([_vp, _u64p, ctypes.c_size_t, _u64p, ctypes.c_uint32, _u64p], ctypes.c_int),
    "stark_group_inv_best_fft": ([_vp, _u64p, ctypes.c_size_t, _u64p, ctypes.c_uint32, _u64p], ctypes.c_int),
    "stark_group_ntt_dev": ([_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.c_uint32, _u64p, ctypes.c_int],
                            ctypes.c_int),
    "stark_group_merkle_new": ([_vp, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_group_merkle_free": ([_vp], None),
    "stark_group_merkle_update": ([_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t], ctypes.c_int),
    "stark_group_merkle_update_dev": ([_vp, ctypes.POINTER(_vp), ctypes.c_size_t, ctypes.c_size_t], ctypes.c_int),
    "stark_group_merkle_width": ([_vp], ctypes.c_size_t),
    "stark_group_merkle_get_root": ([_vp, ctypes.c_char_p, _szp], ctypes.c_int),
    "stark_group_merkle_gen_proofs": ([_vp, _szp, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p], ctypes.c_int),
    "stark_group_prove_r1cs_bytes": ([_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                      ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_group_circuit_new": ([_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_group_prove_r1cs_circuit": ([_vp, ctypes.POINTER(_vp), ctypes.c_char_p, ctypes.c_size_t,
                                        ctypes.POINTER(_vp)], ctypes.c_int),
    "stark_verify_with_witness": ([_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                   ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
}

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Loads libstark_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libstark_hip.so not built at {path}: run `make -C stark-pure-rust_amd` "
                           "or __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (args, res) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    want = header_abi_version()
    if lib.stark_abi_version() != want:
        raise RuntimeError(f"{path} implements ABI {lib.stark_abi_version()}, include/stark_hip.h declares {want}: "
                           "rebuild the library")
    _lib = lib
    return lib


def header_abi_version(path: str = HEADER_PATH) -> int:
    """STARK_ABI_VERSION of include/stark_hip.h."""
    import re
    m = re.search(r"#define\s+STARK_ABI_VERSION\s+(\d+)u?", open(path).read())
    return int(m.group(1))


HIP_STREAM_LEGACY = 1  # hipStreamLegacy (hip_runtime_api.h): the legacy default stream as a handle


def torch_stream() -> int:
    """torch's current stream as the handle the library's _dev calls take.  torch's default stream
    has handle 0, which the library reads as "the context's own stream" (a non-blocking stream the
    default stream does not order against): it is passed as hipStreamLegacy instead, so the library's
    kernels and torch's copies and collectives run in one stream order either way."""
    import torch
    s = torch.cuda.current_stream().cuda_stream
    return s if s else HIP_STREAM_LEGACY


def header_symbols(path: str = HEADER_PATH) -> list:
    """Function names declared in include/stark_hip.h."""
    import re
    text = open(path).read()
    return sorted(set(re.findall(r"\b(stark_[a-z0-9_]+)\s*\(", text)))


def _p64(a: np.ndarray):
    return a.ctypes.data_as(_u64p)


def _limbs(x) -> np.ndarray:
    if isinstance(x, (int, np.integer)):
        x = int(x) % P
        return np.array([(x >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)], dtype=np.uint64)
    a = np.ascontiguousarray(x, dtype=np.uint64).reshape(4)
    return a


def _elems(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, 4)


def _out_array(out, log_n: int) -> np.ndarray:
    if out is None:
        return np.empty((1 << log_n, 4), dtype=np.uint64)
    if not (isinstance(out, np.ndarray) and out.dtype == np.uint64 and out.flags["C_CONTIGUOUS"]
            and out.shape == (1 << log_n, 4)):
        raise ValueError("out must be a C-contiguous (2^log_n, 4) uint64 array")
    return out


class Context:
    """One GPU (replaces commitment::multicore::Worker, multicore.rs:43-45)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _vp()
        rc = self.lib.stark_ctx_create(device, ctypes.byref(h))
        if rc != 0:
            raise StarkError(rc, "stark_ctx_create")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            self.lib.stark_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, where: str):
        if rc != 0:
            detail = self.lib.stark_ctx_last_error(self.h).decode() if rc in (5, 8) else ""
            raise StarkError(rc, where, detail)

    @property
    def stream(self) -> int:
        return self.lib.stark_ctx_stream(self.h)

    def synchronize(self):
        self.check(self.lib.stark_ctx_synchronize(self.h), "synchronize")

    def set_cache_limit(self, nbytes: int):
        """Cap on the context's cached tables (full last-pass twiddle tables, IDX extensions)."""
        self.check(self.lib.stark_ctx_set_cache_limit(self.h, int(nbytes)), "set_cache_limit")

    def memory(self) -> dict:
        """{'cached': bytes of cached tables, 'cache_limit': their cap, 'resident': all device bytes held}."""
        c, l, r = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        self.check(self.lib.stark_ctx_memory(self.h, ctypes.byref(c), ctypes.byref(l), ctypes.byref(r)), "memory")
        return {"cached": c.value, "cache_limit": l.value, "resident": r.value}

    # ---- fri::fft ----------------------------------------------------------
    def best_fft(self, coefficients, root_of_unity, log_order_of_root: int, out=None) -> np.ndarray:
        """fft.rs:327-357.  `out` (optional): a C-contiguous (2^log, 4) uint64 array to write into, as the
        reference's best_fft writes into the caller's Vec; a fresh array costs its page faults on every call."""
        c = _elems(coefficients)
        out = _out_array(out, log_order_of_root)
        r = _limbs(root_of_unity)
        self.check(self.lib.stark_best_fft(self.h, _p64(c), len(c), _p64(r), log_order_of_root, _p64(out)),
                   "best_fft")
        return out

    def inv_best_fft(self, evaluations, root_of_unity, log_order_of_root: int, out=None) -> np.ndarray:
        """fft.rs:359-379 (`out` as in best_fft)."""
        c = _elems(evaluations)
        out = _out_array(out, log_order_of_root)
        r = _limbs(root_of_unity)
        self.check(self.lib.stark_inv_best_fft(self.h, _p64(c), len(c), _p64(r), log_order_of_root, _p64(out)),
                   "inv_best_fft")
        return out

    def serial_fft(self, values: np.ndarray, root_of_unity, log_order_of_root: int) -> None:
        """fft.rs:150-193 (in place on exactly 2^log values)."""
        v = values
        assert v.dtype == np.uint64 and v.flags["C_CONTIGUOUS"]
        r = _limbs(root_of_unity)
        self.check(self.lib.stark_fft_in_place(self.h, _p64(v), _p64(r), log_order_of_root, 0), "serial_fft")

    def inv_serial_fft(self, values: np.ndarray, root_of_unity, log_order_of_root: int) -> None:
        """fft.rs:284-293 (in place on exactly 2^log values, root^-1 then n^-1)."""
        v = values
        assert v.dtype == np.uint64 and v.flags["C_CONTIGUOUS"]
        r = _limbs(root_of_unity)
        self.check(self.lib.stark_fft_in_place(self.h, _p64(v), _p64(r), log_order_of_root, 1), "inv_serial_fft")

    def ntt_dev(self, d_ptr: int, log_n: int, batch: int, root, inverse: bool = False, stream: int = 0) -> None:
        r = _limbs(root)
        self.check(self.lib.stark_ntt_dev(self.h, d_ptr, log_n, batch, _p64(r), 1 if inverse else 0, stream or None),
                   "ntt_dev")

    def ntt_strided_dev(self, d_ptr: int, log_g: int, stride: int, root, inverse: bool = False,
                        stream: int = 0) -> None:
        """For each i < stride: DFT over d[i + stride*j], j < 2^log_g (in place)."""
        r = _limbs(root)
        self.check(self.lib.stark_ntt_strided_dev(self.h, d_ptr, log_g, stride, _p64(r), 1 if inverse else 0,
                                                  stream or None), "ntt_strided")

    def cyclic_ntt_local_dev(self, d_ptr: int, log_n: int, log_g: int, rank: int, root, inverse: bool = False,
                             stream: int = 0) -> None:
        """The rank's local M-point NTT of the one-exchange distributed NTT with its twiddle w^(rank k)
        applied in the last pass (stark_cyclic_ntt_local_dev)."""
        r = _limbs(root)
        self.check(self.lib.stark_cyclic_ntt_local_dev(self.h, d_ptr, log_n, log_g, rank, _p64(r), 1 if inverse else 0,
                                                       stream or None), "cyclic_ntt_local")

    def ntt_strided_tw_dev(self, d_ptr: int, log_g: int, stride: int, root, tw_root, log_order: int, tw_base: int,
                           inverse: bool = False, stream: int = 0) -> None:
        """ntt_strided_dev after d[i + stride*j] *= tw_root^(j*(tw_base + i))."""
        r, t = _limbs(root), _limbs(tw_root)
        self.check(self.lib.stark_ntt_strided_tw_dev(self.h, d_ptr, log_g, stride, _p64(r), 1 if inverse else 0,
                                                     _p64(t), log_order, tw_base, stream or None), "ntt_strided_tw")

    def transpose_dev(self, d_src: int, d_dst: int, rows: int, cols: int, batch: int = 1, stream: int = 0) -> None:
        self.check(self.lib.stark_transpose_dev(self.h, d_src, d_dst, rows, cols, batch, stream or None), "transpose")

    def twiddle2d_dev(self, d_ptr: int, rows: int, cols: int, row_base: int, col_base: int, root, log_order: int,
                      stream: int = 0) -> None:
        r = _limbs(root)
        self.check(self.lib.stark_twiddle2d_dev(self.h, d_ptr, rows, cols, row_base, col_base, _p64(r), log_order,
                                                stream or None), "twiddle2d")

    def expand_root_of_unity(self, root_of_unity) -> np.ndarray:
        """fft.rs:5-14."""
        r = _limbs(root_of_unity)
        cnt = ctypes.c_size_t(0)
        self.check(self.lib.stark_expand_root_of_unity(self.h, _p64(r), None, 0, ctypes.byref(cnt)),
                   "expand_root_of_unity")
        out = np.empty((cnt.value, 4), dtype=np.uint64)
        self.check(self.lib.stark_expand_root_of_unity(self.h, _p64(r), _p64(out), cnt.value, ctypes.byref(cnt)),
                   "expand_root_of_unity")
        return out

    # ---- fri::poly_utils ----------------------------------------------------
    def multi_inv(self, values) -> np.ndarray:
        """poly_utils.rs:38-70."""
        v = _elems(values)
        out = np.empty_like(v)
        self.check(self.lib.stark_multi_inv(self.h, _p64(v), len(v), _p64(out)), "multi_inv")
        return out

    def eval_poly_at_multi(self, poly, xs) -> np.ndarray:
        """[eval_poly_at(poly, x) for x in xs] (poly_utils.rs:93-102)."""
        p = _elems(poly)
        x = _elems(xs)
        out = np.empty_like(x)
        self.check(self.lib.stark_eval_poly_at_multi(self.h, _p64(p), len(p), _p64(x), len(x), _p64(out)),
                   "eval_poly_at")
        return out

    def multi_interp_4(self, xsets, ysets) -> np.ndarray:
        """multi_interp_4 (poly_utils.rs:449-511): rows x 4 points -> rows x 4 coefficients
        (element arrays of 4 * rows elements, row-major)."""
        x, y = _elems(xsets), _elems(ysets)
        if len(x) != len(y) or len(x) % 4:
            raise ValueError("multi_interp_4: xsets and ysets need 4 elements per row, same row count")
        out = np.empty_like(x)
        self.check(self.lib.stark_multi_interp_4(self.h, _p64(x), _p64(y), len(x) // 4, _p64(out)), "multi_interp_4")
        return out

    def eval_quartic_multi(self, polys, xs) -> np.ndarray:
        """[eval_quartic(p_i, x_i)] (poly_utils.rs:442-446); polys holds 4 coefficients per x."""
        p, x = _elems(polys), _elems(xs)
        if len(p) != 4 * len(x):
            raise ValueError("eval_quartic_multi: 4 coefficients per point")
        out = np.empty_like(x)
        self.check(self.lib.stark_eval_quartic_multi(self.h, _p64(p), _p64(x), len(x), _p64(out)), "eval_quartic")
        return out

    def lincomb(self, cols, coeffs) -> np.ndarray:
        """out[i] = sum_c coeffs[c] * cols[c][i]; cols is n_cols x n elements (row-major)."""
        c = _elems(coeffs)
        v = _elems(cols)
        n_cols = len(c)
        if n_cols == 0 or len(v) % n_cols:
            raise ValueError("lincomb: cols must hold n_cols equal columns")
        n = len(v) // n_cols
        out = np.empty((n, 4), dtype=np.uint64)
        self.check(self.lib.stark_lincomb(self.h, _p64(v), n_cols, n, _p64(c), _p64(out)), "lincomb")
        return out

    def lde(self, values, g1, log_blowup: int, g2) -> np.ndarray:
        """inv_best_fft(values, g1) then best_fft(padded, g2) (prove.rs:100-101)."""
        v = _elems(values)
        out = np.empty((len(v) << log_blowup, 4), dtype=np.uint64)
        self.check(self.lib.stark_lde(self.h, _p64(v), len(v), _p64(_limbs(g1)), log_blowup, _p64(_limbs(g2)),
                                      _p64(out)), "lde")
        return out

    def lde_dev(self, d_values: int, d_out: int, log_steps: int, log_blowup: int, batch: int, g1, g2,
                stream: int = 0) -> None:
        self.check(self.lib.stark_lde_dev(self.h, d_values, d_out, log_steps, log_blowup, batch, _p64(_limbs(g1)),
                                          _p64(_limbs(g2)), stream or None), "lde_dev")

    # ---- device memory (plumbing) -------------------------------------------
    def alloc(self, nbytes: int) -> int:
        p = _vp()
        self.check(self.lib.stark_dev_alloc(self.h, nbytes, ctypes.byref(p)), "dev_alloc")
        return p.value

    def free(self, ptr: int):
        self.check(self.lib.stark_dev_free(self.h, ptr), "dev_free")

    def h2d(self, ptr: int, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        self.check(self.lib.stark_memcpy_h2d(self.h, ptr, a.ctypes.data, a.nbytes), "h2d")

    def d2h(self, arr: np.ndarray, ptr: int):
        assert arr.flags["C_CONTIGUOUS"]
        self.check(self.lib.stark_memcpy_d2h(self.h, arr.ctypes.data, ptr, arr.nbytes), "d2h")

    # ---- fri::fri -------------------------------------------------------------
    def prove_low_degree(self, values, root_of_unity, max_deg_plus_1: int, exclude_multiples_of: int):
        """fri.rs:46-62.  Returns a FriProofList."""
        v = _elems(values)
        r = _limbs(root_of_unity)
        h = _vp()
        self.check(self.lib.stark_prove_low_degree(self.h, _p64(v), len(v), _p64(r), max_deg_plus_1,
                                                   exclude_multiples_of, ctypes.byref(h)), "prove_low_degree")
        return FriProofList(self.lib, h)

    def prove_low_degree_dev(self, d_ptr: int, n: int, root_of_unity, max_deg_plus_1: int,
                             exclude_multiples_of: int):
        r = _limbs(root_of_unity)
        h = _vp()
        self.check(self.lib.stark_prove_low_degree_dev(self.h, d_ptr, n, _p64(r), max_deg_plus_1,
                                                       exclude_multiples_of, ctypes.byref(h)), "prove_low_degree")
        return FriProofList(self.lib, h)


class FriProofList:
    """Vec<FriProof<BlakeDigest>> (fri.rs:16-26) held by the library."""

    def __init__(self, lib, h):
        self.lib = lib
        self.h = h

    def __del__(self):
        try:
            if self.h:
                self.lib.stark_fri_proof_free(self.h)
        except Exception:
            pass

    def __len__(self):
        return self.lib.stark_fri_proof_num_layers(self.h)

    def to_json(self) -> str:
        """serde_json::to_string(&Vec<FriProof<BlakeDigest>>)."""
        n = ctypes.c_size_t(0)
        self.lib.stark_fri_proof_json(self.h, None, 0, ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        self.lib.stark_fri_proof_json(self.h, buf, n.value + 1, ctypes.byref(n))
        return buf.value.decode()

    def layers(self) -> list:
        return json.loads(self.to_json())


# ---- host-side helpers with the reference names ------------------------------
def ntt_plan(log_n: int) -> list:
    """log2 radices of the Stockham passes of a 2^log_n transform (stark_ntt_plan; host-only)."""
    lib = load_library()
    out = (ctypes.c_uint32 * 8)()
    k = lib.stark_ntt_plan(log_n, out, 8)
    return list(out)[:k]


def blake(message: bytes) -> bytes:
    """fri/src/utils.rs:5-10 (computed by libstark_hip's host Blake2s)."""
    lib = load_library()
    out = ctypes.create_string_buffer(32)
    lib.stark_blake(message, len(message), out)
    return out.raw


def get_pseudorandom_indices(seed: bytes, modulus: int, count: int, exclude_multiples_of: int) -> list:
    """fri/src/utils.rs:82-109.  Raises StarkError where the reference panics."""
    lib = load_library()
    out = (ctypes.c_uint32 * max(count, 1))()
    rc = lib.stark_get_pseudorandom_indices(seed, len(seed), modulus, count, exclude_multiples_of, out)
    if rc != 0:
        raise StarkError(rc, "get_pseudorandom_indices")
    return list(out)[:count]


@dataclass
class Proof:
    """commitment::merkle_tree::Proof (merkle_tree.rs:14-43)."""
    leaf: bytes
    nodes: list = field(default_factory=list)

    def validate(self, root: bytes, index: int) -> bytes:
        lib = load_library()
        idx = (ctypes.c_size_t * 1)(index)
        rc = lib.stark_merkle_verify(root, idx, 1, self.leaf, len(self.leaf), b"".join(self.nodes), len(self.nodes))
        if rc != 0:
            raise AssertionError("Merkle proof does not hash to root")
        return self.leaf


def verify_multi_branch(root: bytes, indices, proofs) -> list:
    """merkle_tree.rs:46-58."""
    return [p.validate(root, i) for i, p in zip(indices, proofs)]


class MerkleProofInPlace:
    """MerkleTree<Vec<u8>, BlakeDigest> for MerkleProofInPlace
    (merkle_tree.rs:60-73, merkle_proof_in_place.rs:9-50)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = _vp()
        ctx.check(ctx.lib.stark_merkle_new(ctx.h, ctypes.byref(h)), "MerkleProofInPlace::new")
        self.h = h
        self.leaf_len = 0

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.stark_merkle_free(self.h)
        except Exception:
            pass

    def width(self) -> int:
        return self.ctx.lib.stark_merkle_width(self.h)

    def get_root(self) -> bytes:
        """Empty bytes before the first gen_proofs (H::default())."""
        out = ctypes.create_string_buffer(32)
        n = ctypes.c_size_t(0)
        self.ctx.check(self.ctx.lib.stark_merkle_get_root(self.h, out, ctypes.byref(n)), "get_root")
        return out.raw[:n.value]

    def update(self, leaves) -> None:
        leaves = list(leaves)
        if not leaves:
            raise StarkError(1, "update", "empty leaf set")
        ln = len(leaves[0])
        if any(len(x) != ln for x in leaves):
            raise StarkError(3, "update", "leaves must have equal length")
        self.leaf_len = ln
        blob = b"".join(leaves)
        self.ctx.check(self.ctx.lib.stark_merkle_update(self.h, blob, len(leaves), ln), "update")

    def update_bytes(self, blob: bytes, n: int, leaf_len: int) -> None:
        self.leaf_len = leaf_len
        self.ctx.check(self.ctx.lib.stark_merkle_update(self.h, blob, n, leaf_len), "update")

    def update_dev(self, d_ptr: int, n: int, leaf_len: int, stream: int = 0) -> None:
        self.leaf_len = leaf_len
        self.ctx.check(self.ctx.lib.stark_merkle_update_dev(self.h, d_ptr, n, leaf_len, stream or None), "update")

    def update_digests_dev(self, d_ptr: int, n: int, interleave: int = 1, stream: int = 0) -> None:
        """Tree over n given leaf digests (device), stored as `interleave` residue-class chunks
        (stark_merkle_update_digests_dev); proofs return the leaf digest as the leaf."""
        self.leaf_len = 32
        self.ctx.check(self.ctx.lib.stark_merkle_update_digests_dev(self.h, d_ptr, n, interleave, stream or None),
                       "update_digests")

    def gen_proofs(self, indices) -> list:
        idx = list(indices)
        k = len(idx)
        depth = max(self.width().bit_length() - 1, 0)
        arr = (ctypes.c_size_t * max(k, 1))(*idx)
        leaves = ctypes.create_string_buffer(max(k * self.leaf_len, 1))
        nodes = ctypes.create_string_buffer(max(k * depth * 32, 1))
        self.ctx.check(self.ctx.lib.stark_merkle_gen_proofs(self.h, arr, k, leaves, nodes), "gen_proofs")
        lr, nr = leaves.raw, nodes.raw
        return [Proof(lr[i * self.leaf_len:(i + 1) * self.leaf_len],
                      [nr[(i * depth + d) * 32:(i * depth + d + 1) * 32] for d in range(depth)]) for i in range(k)]
