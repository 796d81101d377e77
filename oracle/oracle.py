"""CPU oracle for the FRI-prover hot path -- TEST INFRASTRUCTURE ONLY.

Two independent restatements of the reference algorithms:

* ``Oracle`` -- ctypes binding of ``liboracle.so`` (oracle.c), the C
  restatement that follows the reference loops as written (serial_fft,
  bellman parallel_fft, gen_multi_proofs_multi_core, prove_low_degree).  It is
  the large-n checker and the timed ``cpu_baseline`` in bench.py.
* ``py_*`` functions -- pure-Python exact-integer restatements used only at
  small sizes to cross-check the C oracle (naive DFT by definition, hashlib
  blake2s, Merkle, index sampler, FRI).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import
this module.  The product library never does.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

# BN254 scalar field r (packages/ff_utils/src/fp.rs:9), generator 7 (fp.rs:10).
P = 21888242871839275222246405745257275088548364400416034343698204186575808495617
GENERATOR = 7
TWO_ADICITY = 28


def build() -> str:
    """Compile liboracle.so from oracle.c (gcc only; no reference sources)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


# ---------------------------------------------------------------- codecs
def to_limbs(values) -> np.ndarray:
    """ints -> (n, 4) uint64 canonical little-endian limbs (= to_bytes_le)."""
    vals = list(values)
    out = np.zeros((len(vals), 4), dtype=np.uint64)
    for i, v in enumerate(vals):
        for k in range(4):
            out[i, k] = (v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    return out


def from_limbs(arr) -> list:
    a = np.asarray(arr, dtype=np.uint64).reshape(-1, 4)
    return [int(r[0]) | (int(r[1]) << 64) | (int(r[2]) << 128) | (int(r[3]) << 192) for r in a]


def to_bytes_le(x: int) -> bytes:
    """ToBytes::to_bytes_le (ff_utils/src/fp.rs:39-43): 32-byte canonical LE."""
    return (x % P).to_bytes(32, "little")


def from_bytes_le(b: bytes) -> int:
    """FromBytes::from_bytes_le (fp.rs:74-76): LE integer reduced mod p."""
    return int.from_bytes(b, "little") % P


def root_of_unity(log_n: int) -> int:
    """7^((p-1)/2^log_n), as r1cs-stark/src/prove.rs:71-82 builds g2."""
    return pow(GENERATOR, (P - 1) >> log_n, P)


def random_elements(n: int, seed: int) -> np.ndarray:
    """Synthetic input of BASELINE.md: splitmix64 -> 4 limbs masked to 254
    bits, rejected if >= p.  Vectorised with numpy."""
    out = np.empty((n, 4), dtype=np.uint64)
    state = np.uint64(seed)
    filled = 0
    mask254 = np.uint64((1 << 62) - 1)
    p_limbs = to_limbs([P])[0]
    with np.errstate(over="ignore"):
        while filled < n:
            m = (n - filled) * 4 + 64
            idx = np.arange(1, m + 1, dtype=np.uint64)
            z = state + idx * np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            state = state + np.uint64(m) * np.uint64(0x9E3779B97F4A7C15)
            cand = z[: (m // 4) * 4].reshape(-1, 4).copy()
            cand[:, 3] &= mask254
            # lexicographic compare against p (limb 3 most significant)
            lt = np.zeros(len(cand), dtype=bool)
            eq = np.ones(len(cand), dtype=bool)
            for k in (3, 2, 1, 0):
                lt |= eq & (cand[:, k] < p_limbs[k])
                eq &= cand[:, k] == p_limbs[k]
            good = cand[lt]
            take = min(len(good), n - filled)
            out[filled:filled + take] = good[:take]
            filled += take
    return out


# ---------------------------------------------------------------- ctypes
class Oracle:
    """ctypes binding of liboracle.so (C restatement, oracle.c)."""

    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            build()
        self.lib = ctypes.CDLL(path)
        L = self.lib
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.oracle_best_fft.argtypes = [u64p, ctypes.c_size_t, u64p, ctypes.c_uint32, ctypes.c_uint32, u64p]
        L.oracle_inv_best_fft.argtypes = L.oracle_best_fft.argtypes
        L.oracle_expand_root_of_unity.argtypes = [u64p, u64p, ctypes.c_size_t]
        L.oracle_expand_root_of_unity.restype = ctypes.c_size_t
        L.oracle_root_of_unity.argtypes = [ctypes.c_uint32, u64p]
        L.oracle_multi_inv.argtypes = [u64p, ctypes.c_size_t, u64p]
        L.oracle_eval_poly_multi.argtypes = [u64p, ctypes.c_size_t, u64p, ctypes.c_size_t, u64p]
        L.oracle_multi_interp_4.argtypes = [u64p, u64p, ctypes.c_size_t, u64p]
        L.oracle_eval_quartic_multi.argtypes = [u64p, u64p, ctypes.c_size_t, u64p]
        L.oracle_blake2s.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_get_pseudorandom_indices.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32,
                                                      ctypes.c_size_t, ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_merkle_proofs.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_prove_low_degree_json.argtypes = [u64p, ctypes.c_size_t, u64p, ctypes.c_size_t,
                                                   ctypes.c_uint32, ctypes.c_size_t]
        L.oracle_prove_low_degree_json.restype = ctypes.c_void_p
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_from_bytes_le.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64p]

    @staticmethod
    def _p(a: np.ndarray):
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))

    def best_fft(self, coeffs: np.ndarray, root: int, log_n: int, cpus: int = 1) -> np.ndarray:
        c = np.ascontiguousarray(coeffs, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros((1 << log_n, 4), dtype=np.uint64)
        r = to_limbs([root])
        rc = self.lib.oracle_best_fft(self._p(c), len(c), self._p(r), log_n, cpus, self._p(out))
        if rc != 0:
            raise ValueError("oracle_best_fft: length exceeds 2^log_n")
        return out

    def inv_best_fft(self, evals: np.ndarray, root: int, log_n: int, cpus: int = 1) -> np.ndarray:
        c = np.ascontiguousarray(evals, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros((1 << log_n, 4), dtype=np.uint64)
        r = to_limbs([root])
        rc = self.lib.oracle_inv_best_fft(self._p(c), len(c), self._p(r), log_n, cpus, self._p(out))
        if rc != 0:
            raise ValueError("oracle_inv_best_fft: length exceeds 2^log_n")
        return out

    def expand_root_of_unity(self, root: int) -> np.ndarray:
        r = to_limbs([root])
        n = self.lib.oracle_expand_root_of_unity(self._p(r), None, 0)
        out = np.zeros((n, 4), dtype=np.uint64)
        self.lib.oracle_expand_root_of_unity(self._p(r), self._p(out), n)
        return out

    def multi_inv(self, values: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros_like(v)
        self.lib.oracle_multi_inv(self._p(v), len(v), self._p(out))
        return out

    def eval_poly_multi(self, poly: np.ndarray, xs: np.ndarray) -> np.ndarray:
        p = np.ascontiguousarray(poly, dtype=np.uint64).reshape(-1, 4)
        x = np.ascontiguousarray(xs, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros_like(x)
        self.lib.oracle_eval_poly_multi(self._p(p), len(p), self._p(x), len(x), self._p(out))
        return out

    def multi_interp_4(self, xsets: np.ndarray, ysets: np.ndarray) -> np.ndarray:
        """poly_utils.rs:449-511: rows x 4 points -> rows x 4 coefficients."""
        x = np.ascontiguousarray(xsets, dtype=np.uint64).reshape(-1, 4)
        y = np.ascontiguousarray(ysets, dtype=np.uint64).reshape(-1, 4)
        rows = len(x) // 4
        out = np.zeros((4 * rows, 4), dtype=np.uint64)
        self.lib.oracle_multi_interp_4(self._p(x), self._p(y), rows, self._p(out))
        return out

    def eval_quartic_multi(self, polys: np.ndarray, xs: np.ndarray) -> np.ndarray:
        """eval_quartic (poly_utils.rs:442-446) of polys[i] (4 coefficients) at xs[i]."""
        p = np.ascontiguousarray(polys, dtype=np.uint64).reshape(-1, 4)
        x = np.ascontiguousarray(xs, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros_like(x)
        self.lib.oracle_eval_quartic_multi(self._p(p), self._p(x), len(x), self._p(out))
        return out

    def blake2s(self, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.oracle_blake2s(msg, len(msg), out)
        return out.raw

    def get_pseudorandom_indices(self, seed: bytes, modulus: int, count: int, exclude: int) -> list:
        out = (ctypes.c_uint32 * count)()
        rc = self.lib.oracle_get_pseudorandom_indices(seed, len(seed), modulus, count, exclude, out)
        if rc != 0:
            raise ValueError(f"get_pseudorandom_indices: rc={rc}")
        return list(out)

    def merkle(self, leaves: bytes, n: int, leaf_len: int, indices=(), chunks: int = 1):
        """Returns (root, [[sibling digests leaf->root] per index])."""
        k = len(indices)
        idx = (ctypes.c_size_t * max(k, 1))(*indices)
        logn = max(n.bit_length() - 1, 0)
        root = ctypes.create_string_buffer(32)
        nodes = ctypes.create_string_buffer(max(k * logn * 32, 1))
        rc = self.lib.oracle_merkle_proofs(leaves, n, leaf_len, idx, k, chunks, root, nodes)
        if rc != 0:
            raise ValueError("merkle: leaf count is not a power of two")
        raw = nodes.raw
        paths = [[raw[(i * logn + d) * 32:(i * logn + d + 1) * 32] for d in range(logn)] for i in range(k)]
        return root.raw, paths

    def prove_low_degree_json(self, values: np.ndarray, root: int, max_deg_plus_1: int, exclude: int,
                              chunks: int = 1) -> str:
        v = np.ascontiguousarray(values, dtype=np.uint64).reshape(-1, 4)
        r = to_limbs([root])
        ptr = self.lib.oracle_prove_low_degree_json(self._p(v), len(v), self._p(r), max_deg_plus_1, exclude,
                                                    chunks)
        s = ctypes.string_at(ptr).decode()
        self.lib.oracle_free(ptr)
        return s

    def from_bytes_le(self, b: bytes) -> int:
        out = np.zeros(4, dtype=np.uint64)
        self.lib.oracle_from_bytes_le(b, len(b), self._p(out))
        return from_limbs(out)[0]


# ------------------------------------------------------- pure-Python (small)
def py_blake(msg: bytes) -> bytes:
    """fri/src/utils.rs:5-10 (Blake2s-256, unkeyed)."""
    return hashlib.blake2s(msg, digest_size=32).digest()


def py_dft(coeffs, root: int, n: int, p: int = P) -> list:
    """The DFT by definition: out[i] = sum_j c_j root^(i j) (zero-padded)."""
    c = list(coeffs) + [0] * (n - len(coeffs))
    w = [pow(root, k, p) for k in range(n)]
    return [sum(c[j] * w[(i * j) % n] for j in range(n)) % p for i in range(n)]


def py_serial_fft(values, root: int, log_n: int, p: int = P) -> list:
    """fri/src/fft.rs:150-193 over any prime p."""
    n = 1 << log_n
    v = list(values)
    assert len(v) == n
    for k in range(n):
        rk = int(format(k, f"0{log_n}b")[::-1], 2) if log_n else 0
        if k < rk:
            v[k], v[rk] = v[rk], v[k]
    m = 1
    for _ in range(log_n):
        w_m = pow(root, n // (2 * m), p)
        for k in range(0, n, 2 * m):
            w = 1
            for j in range(m):
                t = v[k + j + m] * w % p
                v[k + j + m] = (v[k + j] - t) % p
                v[k + j] = (v[k + j] + t) % p
                w = w * w_m % p
        m *= 2
    return v


def py_multi_inv(values, p: int = P) -> list:
    """fri/src/poly_utils.rs:38-70 (zero maps to zero), over any prime p."""
    partials = [1]
    for x in values:
        partials.append(partials[-1] * (x if x else 1) % p)
    inv = pow(partials[-1], p - 2, p)
    out = [0] * len(values)
    for i in range(len(values) - 1, -1, -1):
        out[i] = partials[i] * inv % p if values[i] else 0
        inv = inv * (values[i] if values[i] else 1) % p
    return out


def py_expand_root_of_unity(root: int, p: int = P) -> list:
    """fri/src/fft.rs:5-14."""
    out = [1]
    cur = root % p
    while cur != 1:
        out.append(cur)
        cur = cur * root % p
    return out


def py_get_pseudorandom_indices(seed: bytes, modulus: int, count: int, exclude: int) -> list:
    """fri/src/utils.rs:82-109."""
    assert modulus < 2 ** 24
    data = bytearray(seed)
    while len(data) < 4 * count:
        data += py_blake(bytes(data[-32:]))
    words = [int.from_bytes(data[i:i + 4], "big") for i in range(0, 4 * count, 4)]
    if exclude == 0:
        return [w % modulus for w in words]
    real = modulus * (exclude - 1) // exclude
    return [(w % real) + 1 + (w % real) // (exclude - 1) for w in words]


def py_merkle(leaves: list, indices=()):
    """Standard tree of commitment/src/merkle_proof_in_place.rs:106-206:
    leaf node = H(leaf), parent = H(left || right); proofs leaf->root in the
    caller's index order.  Returns (root, paths)."""
    n = len(leaves)
    assert n and n & (n - 1) == 0
    layers = [[py_blake(x) for x in leaves]]
    while len(layers[-1]) > 1:
        prev = layers[-1]
        layers.append([py_blake(prev[2 * i] + prev[2 * i + 1]) for i in range(len(prev) // 2)])
    paths = []
    for idx in indices:
        path, i = [], idx
        for layer in layers[:-1]:
            path.append(layer[i ^ 1])
            i >>= 1
        paths.append(path)
    return layers[-1][0], paths


def py_fri_fold_column(values: list, xs: list, special_x: int) -> list:
    """fri.rs:141-164 restated via Lagrange interpolation of each 4-point row
    (multi_interp_4 poly_utils.rs:449-511 yields the same unique cubic)."""
    q = len(xs) // 4
    out = []
    for i in range(q):
        px = [xs[i + q * j] for j in range(4)]
        py = [values[i + q * j] for j in range(4)]
        acc = 0
        for j in range(4):
            num, den = 1, 1
            for k in range(4):
                if k != j:
                    num = num * (special_x - px[k]) % P
                    den = den * (px[j] - px[k]) % P
            acc = (acc + py[j] * num * pow(den, P - 2, P)) % P
        out.append(acc)
    return out


def _json_bytes(b: bytes) -> str:
    return "[" + ",".join(str(x) for x in b) + "]"


def _json_proofs(leaves: list, idx: list, paths: list) -> str:
    return "[" + ",".join(
        '{"leaf":' + _json_bytes(leaves[i]) + ',"nodes":[' + ",".join(_json_bytes(d) for d in path) + "]}"
        for i, path in zip(idx, paths)) + "]"


def py_prove_low_degree_json(values: list, root: int, max_deg_plus_1: int, exclude: int) -> str:
    """fri/src/fri.rs:46-224, serialised as serde_json compact
    Vec<FriProof<BlakeDigest>>."""
    parts = []
    vals = [v % P for v in values]
    while True:
        xs = py_expand_root_of_unity(root)
        if max_deg_plus_1 <= 16:
            parts.append('{"Last":{"last":[' + ",".join(_json_bytes(to_bytes_le(v)) for v in vals) + "]}}")
            break
        enc = [to_bytes_le(v) for v in vals]
        m_root, _ = py_merkle(enc)
        special_x = from_bytes_le(m_root)
        column = py_fri_fold_column(vals, xs, special_x)
        enc_col = [to_bytes_le(v) for v in column]
        m2_root, _ = py_merkle(enc_col)
        ys = py_get_pseudorandom_indices(m2_root, len(column), 40, exclude)
        _, col_paths = py_merkle(enc_col, ys)
        pos = [y + (len(xs) // 4) * j for y in ys for j in range(4)]
        _, poly_paths = py_merkle(enc, pos)
        parts.append('{"Middle":{"root2":' + _json_bytes(m2_root) + ',"column_branches":'
                     + _json_proofs(enc_col, ys, col_paths) + ',"poly_branches":'
                     + _json_proofs(enc, pos, poly_paths) + "}}")
        vals = column
        root = pow(root, 4, P)
        max_deg_plus_1 //= 4
    return "[" + ",".join(parts) + "]"
