"""Synthetic, satisfiable R1CS + witness in the circom binary formats the
reference reads (circom2bellman_core/src/reader.rs:4-89, r1cs-stark/src/reader.rs:7-42).

Stand-in for sha256_2_test, whose .r1cs the reference does not ship
(SURVEY.md 0.6): a chain of constraints with 3 terms per factor,

    (w[i] + a_i w[i-1] + 1) * (w[i] + b_i w[i-2] + 2) = w[i+1] + c_i w[1] + 3 w[0]

so that every constraint has n_coeff = 3 (9 trace slots).  original_steps =
9 * n_constraints; n_constraints = ceil(target / 9) gives steps = the next
power of two >= target.  Wire 0 is the constant 1; wire 1 is the public
output (the last chain value is copied into it by a final constraint) and
wire 2 the public input.
"""
from __future__ import annotations

import struct

P = 21888242871839275222246405745257275088548364400416034343698204186575808495617
P_LE = P.to_bytes(32, "little")


def _fe(x: int) -> bytes:
    return (x % P).to_bytes(32, "little")


def synth(n_constraints: int, seed: int = 1, inputs=None):
    """Returns (r1cs_bytes, wtns_bytes).  inputs = (public output, public input) overrides
    the seeded ones: the same circuit (identical .r1cs) with another witness."""
    import random
    rnd = random.Random(seed)
    n_chain = n_constraints - 1
    # wires: 0 = 1, 1 = public output, 2 = public input, 3.. chain values
    n_wires = 3 + n_chain + 1
    w = [0] * n_wires
    w[0] = 1
    w[2] = rnd.randrange(P)
    w[3] = w[2]
    cons = []
    for i in range(n_chain):
        cur = 3 + i
        p1 = cur - 1 if cur - 1 >= 2 else 2
        p2 = cur - 2 if cur - 2 >= 2 else 2
        a, b, c = rnd.randrange(1, P), rnd.randrange(1, P), rnd.randrange(1, P)
        av = (w[cur] + a * w[p1] + 1) % P
        bv = (w[cur] + b * w[p2] + 2) % P
        # w[cur+1] = av * bv - c * w[1] - 3, with w[1] fixed below -> use w[1] = 0 for now, patched after
        cons.append(((cur, a, p1), (cur, b, p2), (cur + 1, c), av, bv))
    # choose the public output as the final chain value; constraints reference it, so compute forward
    # with w[1] unknown: solve sequentially treating w[1] as fixed random public output.
    w[1] = rnd.randrange(P)
    if inputs is not None:
        w[1], w[2] = inputs[0] % P, inputs[1] % P
        w[3] = w[2]
    out = []
    for (cur, a, p1), (_, b, p2), (nxt, c), _, _ in cons:
        av = (w[cur] + a * w[p1] + 1) % P
        bv = (w[cur] + b * w[p2] + 2) % P
        w[nxt] = (av * bv - c * w[1] - 3) % P
        A = [(cur, 1), (p1, a), (0, 1)]
        B = [(cur, 1), (p2, b), (0, 2)]
        C = [(nxt, 1), (1, c), (0, 3)]
        out.append((A, B, C))
    # final constraint: w[last] * 1 = w[1] + 0 ... keep it non-trivial but satisfied: (w[last]) * (1) = (w[last])
    last = 3 + n_chain
    out.append(([(last, 1), (0, 0), (2, 0)], [(0, 1), (1, 0), (2, 0)], [(last, 1), (0, 0), (1, 0)]))
    body = bytearray()
    for A, B, C in out:
        for fac in (A, B, C):
            body += struct.pack("<I", len(fac))
            for wid, v in fac:
                body += struct.pack("<I", wid) + _fe(v)
    hdr = struct.pack("<I", 32) + P_LE + struct.pack("<IIIIQI", n_wires, 1, 1, 0, n_wires, len(out))
    r1cs = bytearray()
    r1cs += b"r1cs" + struct.pack("<II", 1, 3)
    r1cs += struct.pack("<IQ", 1, len(hdr)) + hdr
    r1cs += struct.pack("<IQ", 2, len(body)) + body
    wt = bytearray()
    wt += struct.pack("<I", 1936618615) + struct.pack("<IIIII", 2, 2, 1, 0, 0)
    wt += struct.pack("<I", 32) + P_LE
    wt += struct.pack("<IIII", n_wires, 0, 0, 0)
    for x in w:
        wt += _fe(x)
    return bytes(r1cs), bytes(wt)


def for_steps(log_steps: int, seed: int = 1, inputs=None):
    """A circuit whose padded trace length is 2^log_steps (original_steps = 9 n_constraints)."""
    target = 1 << log_steps
    n = (target // 2) // 9 + 1            # original_steps in (2^(k-1), 2^k]
    return synth(n, seed, inputs)
