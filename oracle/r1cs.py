"""Python restatement of the R1CS front end of the reference prover.

TEST INFRASTRUCTURE ONLY (see oracle.c): the checker for libstark_hip's
R1CS/witness readers and trace builder (stark_r1cs_trace_*), and the source
of the inputs handed to oracle_mk_r1cs_proof_json.

Follows, line by line:
  - read_r1cs      packages/circom2bellman_core/src/reader.rs:4-89
  - read_witness   packages/r1cs-stark/src/reader.rs:7-42
  - calc_coefficients_and_witness  packages/r1cs-stark/src/run.rs:109-281
  - calc_coefficients              run.rs:21-107 (verifier side)
  - calc_flags                     run.rs:283-308
  - prove_with_witness             run.rs:310-452 (permuted indices :388-401,
                                   public_first_indices :411-419)
Pinned by the reference's own tests: reader.rs:44-62 (compute.r1cs equals
compute.r1cs.json) and reader.rs:64-89 (compute.wtns values).
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass, field

import numpy as np

from oracle import P, Oracle, to_limbs

BN254_R_LE = bytes([1, 0, 0, 240, 147, 245, 225, 67, 145, 112, 185, 121, 72, 232, 51, 40, 93, 88, 129, 129,
                    182, 69, 80, 184, 41, 160, 49, 225, 114, 78, 100, 48])  # run.rs:344-350


@dataclass
class Header:
    field_size: int
    prime_number: bytes
    n_wires: int
    n_public_outputs: int
    n_public_inputs: int
    n_private_inputs: int
    n_labels: int
    n_constraints: int


@dataclass
class R1cs:
    version: int
    header: Header
    # constraints[c] = [A, B, C], each a list of (wire_id, value bytes (32, LE))
    constraints: list = field(default_factory=list)


class _Reader:
    def __init__(self, b: bytes):
        self.b = b
        self.o = 0

    def u32(self) -> int:
        v = struct.unpack_from("<I", self.b, self.o)[0]
        self.o += 4
        return v

    def u64(self) -> int:
        v = struct.unpack_from("<Q", self.b, self.o)[0]
        self.o += 8
        return v

    def raw(self, n: int) -> bytes:
        v = self.b[self.o:self.o + n]
        if len(v) != n:
            raise ValueError("truncated")
        self.o += n
        return v


def read_r1cs(data: bytes) -> R1cs:
    """circom2bellman_core/src/reader.rs:4-89 (header section then constraint section, fixed order)."""
    p = _Reader(data)
    assert p.u32() == int.from_bytes(b"r1cs", "little")
    version = p.u32()
    assert version == 1
    assert p.u32() == 3                       # n_section
    assert p.u32() == 1                       # HeaderSection
    p.u64()
    field_size = p.u32()
    prime = p.raw(32)
    n_wires = p.u32()
    n_pub_out = p.u32()
    n_pub_in = p.u32()
    n_prv_in = p.u32()
    n_labels = p.u64()
    n_constraints = p.u32()
    hdr = Header(field_size, prime, n_wires, n_pub_out, n_pub_in, n_prv_in, n_labels, n_constraints)
    assert p.u32() == 2                       # ConstraintSection
    p.u64()
    cons = []
    for _ in range(n_constraints):
        factors = []
        for _ in range(3):
            nc = p.u32()
            factors.append([(p.u32(), p.raw(32)) for _ in range(nc)])
        cons.append(factors)
    return R1cs(version, hdr, cons)


def read_witness(data: bytes) -> list:
    """r1cs-stark/src/reader.rs:7-42: returns BigUint::to_bytes_le of every wire value."""
    p = _Reader(data)
    assert p.u32() == 1936618615              # "wtns"
    for _ in range(5):
        p.u32()
    field_size = p.u32()
    for _ in range(field_size // 4):
        p.u32()
    n_wires = p.u32()
    p.u32(); p.u32(); p.u32()
    out = []
    for _ in range(n_wires):
        v = 0
        for k in range(field_size // 4):
            v += p.u32() << (32 * k)
        b = v.to_bytes(max(1, (v.bit_length() + 7) // 8), "little")  # BigUint::to_bytes_le ([0] for zero)
        out.append(b)
    return out


def fe(b: bytes) -> int:
    """T::from_bytes_le (ff_utils/src/fp.rs:70-77): LE integer mod p."""
    return int.from_bytes(b, "little") % P


@dataclass
class Trace:
    """The arguments of mk_r1cs_proof (prove.rs:14-26) as run.rs builds them."""
    witness_trace: list
    computational_trace: list
    public_wires: list
    public_first_indices: list   # [(wire k, trace position w)]
    permuted_indices: list
    coefficients: list
    flag0: list
    flag1: list
    flag2: list
    n_constraints: int
    n_wires: int


def _factor_walk(constraints, n_wires, witness=None):
    """The per-constraint loops of run.rs:127-253 (witness given) / run.rs:33-97 (verifier)."""
    lists = {0: ([], [], []), 1: ([], [], []), 2: ([], [], [])}   # (wit, trace, coeff) per factor
    wire_using = [[] for _ in range(n_wires)]
    last_coeff = []
    acc = 0
    for con in constraints:
        n_coeff = max(len(con[0]), len(con[1]), len(con[2]))
        for f in range(3):
            wit_l, tr_l, co_l = lists[f]
            t = 0
            for i in range(n_coeff):
                if i < len(con[f]):
                    wire_id, value = con[f][i]
                    c = fe(value)
                else:
                    wire_id, c = n_wires - 1, 0
                if witness is not None:
                    w = witness[wire_id]
                    if i < len(con[f]):
                        t = (t + c * w) % P
                    wit_l.append(w)
                    tr_l.append(t)
                wire_using[wire_id].append((f, len(co_l)))
                co_l.append(c)
        acc += n_coeff
        last_coeff.append(acc - 1)
    return lists, wire_using, last_coeff


def calc_flags(last_coeff_list, coefficients_len):
    """run.rs:283-308"""
    assert coefficients_len % 3 == 0
    a_len = coefficients_len // 3
    flag0 = [1] * coefficients_len
    flag1 = [1] * coefficients_len
    for v in last_coeff_list:
        k = (v + 1) % a_len
        flag1[k] = flag1[k + a_len] = flag1[k + 2 * a_len] = 0
    flag2 = [0] * coefficients_len
    for k in last_coeff_list:
        flag2[k] = 1
    return flag0, flag1, flag2


def _permutation(wire_using, length, a_len):
    """run.rs:388-401"""
    perm = [0] * length
    for vs in wire_using:
        if not vs:
            continue
        old = a_len * vs[-1][0] + vs[-1][1]
        for k, v in vs:
            w = a_len * k + v
            perm[w] = old
            old = w
    return perm


def build_trace(r1cs: R1cs, witness_bytes: list) -> Trace:
    """prove_with_witness, run.rs:310-452 (up to the mk_r1cs_proof call)."""
    h = r1cs.header
    assert h.prime_number == BN254_R_LE
    witness = [fe(x) for x in witness_bytes]
    assert witness[0] == 1
    public_wires = witness[:1 + h.n_public_inputs + h.n_public_outputs]
    lists, wire_using, last_coeff = _factor_walk(r1cs.constraints, h.n_wires, witness)
    witness_trace = lists[0][0] + lists[1][0] + lists[2][0]
    computational_trace = lists[0][1] + lists[1][1] + lists[2][1]
    coefficients = lists[0][2] + lists[1][2] + lists[2][2]
    flag0, flag1, flag2 = calc_flags(last_coeff, len(coefficients))
    a_len = len(coefficients) // 3
    perm = _permutation(wire_using, len(computational_trace), a_len)
    pfi = []
    for w in range(len(public_wires)):
        if wire_using[w]:
            k, v = wire_using[w][0]
            pfi.append((w, a_len * k + v))
    return Trace(witness_trace, computational_trace, public_wires, pfi, perm, coefficients, flag0, flag1, flag2,
                 h.n_constraints, h.n_wires)


def verifier_inputs(r1cs: R1cs, public_wires: list):
    """verify_with_witness, run.rs:454-526: the verifier-side trace metadata."""
    h = r1cs.header
    lists, wire_using, last_coeff = _factor_walk(r1cs.constraints, h.n_wires, None)
    coefficients = lists[0][2] + lists[1][2] + lists[2][2]
    flag0, flag1, flag2 = calc_flags(last_coeff, len(coefficients))
    a_len = len(coefficients) // 3
    perm = _permutation(wire_using, len(coefficients), a_len)
    pfi = []
    for w in range(len(public_wires)):
        if wire_using[w]:
            k, v = wire_using[w][0]
            pfi.append((w, a_len * k + v))
    return dict(coefficients=coefficients, flag0=flag0, flag1=flag1, flag2=flag2, permuted_indices=perm,
                public_first_indices=pfi, n_constraints=h.n_constraints, n_wires=h.n_wires)


def load_fixture(directory: str, name: str):
    with open(f"{directory}/{name}.r1cs", "rb") as f:
        r1cs = read_r1cs(f.read())
    with open(f"{directory}/{name}.wtns", "rb") as f:
        wit = read_witness(f.read())
    return r1cs, wit



def mk_r1cs_proof_json(orc: Oracle, tr: Trace, cpus: int = 8) -> str:
    """oracle_mk_r1cs_proof_json (oracle/r1cs.c): prove.rs:14-378 on the CPU."""
    lib = orc.lib
    fn = lib.oracle_mk_r1cs_proof_json
    fn.restype = ctypes.c_void_p
    n = len(tr.coefficients)
    arrs = [to_limbs(v) for v in (tr.witness_trace, tr.computational_trace, tr.public_wires, tr.coefficients,
                                  tr.flag0, tr.flag1, tr.flag2)]
    pfi = np.array([x for pair in tr.public_first_indices for x in pair] or [0], dtype=np.uint64)
    perm = np.array(tr.permuted_indices or [0], dtype=np.uint64)
    err = ctypes.c_int(0)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    res = fn(ptr(arrs[0]), ptr(arrs[1]), ctypes.c_size_t(n), ptr(arrs[2]), ctypes.c_size_t(len(tr.public_wires)),
             ptr(pfi), ctypes.c_size_t(len(tr.public_first_indices)), ptr(perm), ptr(arrs[3]), ptr(arrs[4]),
             ptr(arrs[5]), ptr(arrs[6]), ctypes.c_size_t(tr.n_constraints), ctypes.c_size_t(tr.n_wires),
             ctypes.c_uint32(cpus), ctypes.byref(err))
    if not res:
        raise AssertionError(f"oracle mk_r1cs_proof failed (err {err.value})")
    s = ctypes.string_at(res).decode()
    lib.oracle_free(ctypes.c_void_p(res))
    return s


def r1cs_rows(orc: Oracle, tr: Trace, cpus: int = 8):
    """oracle_r1cs_rows (oracle/r1cs.c): the main-tree rows of every precision point
    (prove.rs:235-258) and a_root, for checking the distributed prover's per-rank slices."""
    lib = orc.lib
    fn = lib.oracle_r1cs_rows
    fn.restype = ctypes.c_void_p
    n = len(tr.coefficients)
    arrs = [to_limbs(v) for v in (tr.witness_trace, tr.computational_trace, tr.public_wires, tr.coefficients,
                                  tr.flag0, tr.flag1, tr.flag2)]
    pfi = np.array([x for pair in tr.public_first_indices for x in pair] or [0], dtype=np.uint64)
    perm = np.array(tr.permuted_indices or [0], dtype=np.uint64)
    err = ctypes.c_int(0)
    a_root = ctypes.create_string_buffer(32)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    res = fn(ptr(arrs[0]), ptr(arrs[1]), ctypes.c_size_t(n), ptr(arrs[2]), ctypes.c_size_t(len(tr.public_wires)),
             ptr(pfi), ctypes.c_size_t(len(tr.public_first_indices)), ptr(perm), ptr(arrs[3]), ptr(arrs[4]),
             ptr(arrs[5]), ptr(arrs[6]), ctypes.c_size_t(tr.n_constraints), ctypes.c_size_t(tr.n_wires),
             ctypes.c_uint32(cpus), ctypes.byref(err), a_root)
    if not res:
        raise AssertionError(f"oracle r1cs_rows failed (err {err.value})")
    log_steps = max((n - 1).bit_length(), 3)
    prec = 8 << log_steps
    rows = ctypes.string_at(res, 256 * prec)
    lib.oracle_free(ctypes.c_void_p(res))
    return rows, a_root.raw
