"""Restated verifier: verify_r1cs_proof (packages/r1cs-stark/src/verify.rs:13-258)
and verify_low_degree_proof (packages/fri/src/fri.rs:226-404).

TEST INFRASTRUCTURE ONLY (see oracle.c).  Accepting a proof is the pin for
full proofs that the reference's tests do not hold:
the GPU proofs and the oracle's proofs must both verify.  Every check
raises AssertionError with the reference's assertion, never a bool.

Exact integers mod p; the O(steps log steps) interpolations use the C
oracle's inv_best_fft/best_fft/eval_poly_multi.
"""
from __future__ import annotations

import hashlib
import json

from oracle import P, Oracle, to_limbs, from_limbs, root_of_unity

MIN_DEG_DIRECT_CHECKING = 16          # fri.rs:14
EXTENSION_FACTOR = 8                  # r1cs-stark/src/utils.rs:135
LOG_EXTENSION_FACTOR = 3
SPOT_CHECK_SECURITY_FACTOR = 80


def blake(m: bytes) -> bytes:
    return hashlib.blake2s(m).digest()


def fe(b) -> int:
    return int.from_bytes(bytes(b), "little") % P


def inv(x: int) -> int:
    return pow(x, P - 2, P)


def get_pseudorandom_indices(seed: bytes, modulus: int, count: int, exclude: int) -> list:
    """fri/src/utils.rs:82-109"""
    assert modulus < 2 ** 24
    data = bytearray(seed)
    while len(data) < 4 * count:
        data += blake(bytes(data[-32:]))
    words = [int.from_bytes(data[4 * i:4 * i + 4], "big") for i in range(count)]
    if exclude == 0:
        return [w % modulus for w in words]
    real = modulus * (exclude - 1) // exclude
    return [(w % real) + 1 + (w % real) // (exclude - 1) for w in words]


def verify_multi_branch(root, indices, proofs) -> list:
    """commitment/src/merkle_tree.rs:25-58"""
    out = []
    for index, prf in zip(indices, proofs):
        cur = blake(bytes(prf["leaf"]))
        tmp = index
        for node in prf["nodes"]:
            cur = blake(cur + bytes(node)) if tmp % 2 == 0 else blake(bytes(node) + cur)
            tmp //= 2
        assert cur == bytes(root), "merkle branch does not reach the root"
        out.append(bytes(prf["leaf"]))
    return out


def merkle_root(leaves: list) -> bytes:
    layer = [blake(bytes(x)) for x in leaves]
    while len(layer) > 1:
        layer = [blake(layer[2 * i] + layer[2 * i + 1]) for i in range(len(layer) // 2)]
    return layer[0]


def eval_poly_at(poly, x) -> int:
    y = 0
    for c in reversed(poly):
        y = (y * x + c) % P
    return y


def lagrange_interp(xs, ys) -> list:
    """poly_utils.rs:409-439 (the unique interpolant, len(xs) coefficients)."""
    n = len(xs)
    root = [1]
    for x in xs:  # prod (X - x), low degree first
        nxt = [0] * (len(root) + 1)
        for i, c in enumerate(root):
            nxt[i + 1] = (nxt[i + 1] + c) % P
            nxt[i] = (nxt[i] - c * x) % P
        root = nxt
    b = [0] * n
    for i, x in enumerate(xs):
        # root / (X - x) by synthetic division
        num = [0] * n
        carry = 0
        for d in range(n, 0, -1):
            carry = (root[d] + carry * x) % P if d < n else root[d]
            num[d - 1] = carry
        den = eval_poly_at(num, x)
        s = ys[i] * inv(den) % P
        for j in range(n):
            b[j] = (b[j] + num[j] * s) % P
    return b


def _interp4_at(xs4, ys4, x) -> int:
    """multi_interp_4 + eval_quartic (poly_utils.rs:442-511) at one point: the cubic through 4 points."""
    acc = 0
    for i in range(4):
        num, den = 1, 1
        for j in range(4):
            if j != i:
                num = num * (x - xs4[j]) % P
                den = den * (xs4[i] - xs4[j]) % P
        acc = (acc + ys4[i] * num * inv(den)) % P
    return acc


def verify_low_degree_proof(merkle_root_b: bytes, root_of_unity_v: int, proof: list, max_deg_plus_1: int,
                            exclude: int) -> bool:
    """fri.rs:244-404"""
    rou_deg = 1
    t = root_of_unity_v
    while t != 1:
        rou_deg *= 2
        t = t * t % P
    w = root_of_unity_v
    quartic = [1, pow(w, rou_deg // 4, P), pow(w, rou_deg // 2, P), pow(w, rou_deg * 3 // 4, P)]
    for prf in proof[:-1]:
        assert "Middle" in prf, "FRI proofs must consist of FriProof::Middle except the last element."
        m = prf["Middle"]
        root2 = bytes(m["root2"])
        special_x = fe(merkle_root_b)
        ys = get_pseudorandom_indices(root2, rou_deg // 4, 40, exclude)
        poly_positions = [j * (rou_deg // 4) + y for y in ys for j in range(4)]
        column_values = verify_multi_branch(root2, ys, m["column_branches"])
        poly_values = verify_multi_branch(merkle_root_b, poly_positions, m["poly_branches"])
        for i, y in enumerate(ys):
            x1 = pow(w, y, P)
            xc = [q * x1 % P for q in quartic]
            row = [fe(poly_values[i * 4 + j]) for j in range(4)]
            assert _interp4_at(xc, row, special_x) == fe(column_values[i]), "FRI column check failed"
        merkle_root_b = root2
        w = pow(w, 4, P)
        max_deg_plus_1 //= 4
        rou_deg //= 4
    assert max_deg_plus_1 >= MIN_DEG_DIRECT_CHECKING // 2, "the degree of direct checking is too low"
    assert "Last" in proof[-1], "The last element of FRI proofs must be FriProof::Last."
    last = [bytes(v) for v in proof[-1]["Last"]["last"]]
    assert len(last) > max_deg_plus_1
    dec = [fe(v) for v in last]
    assert merkle_root(last) == merkle_root_b, "FRI last-layer root mismatch"
    xs = [pow(w, i, P) for i in range(rou_deg)]
    pts = [p for p in range(len(last)) if exclude == 0 or p % exclude != 0]
    rest = pts[max_deg_plus_1:]
    pts = pts[:max_deg_plus_1]
    poly = lagrange_interp([xs[p] for p in pts], [dec[p] for p in pts])
    for p in rest:
        assert eval_poly_at(poly, xs[p]) == dec[p], "FRI last-layer degree check failed"
    return True


def _log2_ceil(v: int) -> int:
    """r1cs-stark/src/utils.rs:14-23"""
    lv, t = 1, v
    while t > 1:
        t //= 2
        lv += 1
    return lv


def verify_r1cs_proof(orc: Oracle, proof, public_wires, public_first_indices, permuted_indices, coefficients,
                      flag0, flag1, flag2, n_constraints, n_wires) -> bool:
    """verify.rs:13-258.  `proof` is the parsed StarkProof JSON (dict) or its text."""
    if isinstance(proof, (str, bytes)):
        proof = json.loads(proof)
    original_steps = len(coefficients)
    assert original_steps <= 3 * n_constraints * n_wires
    assert original_steps % 3 == 0
    log_steps = _log2_ceil(original_steps - 1)
    steps = max(2 ** log_steps, 8)
    precision = steps * EXTENSION_FACTOR
    log_precision = log_steps + LOG_EXTENSION_FACTOR
    assert precision <= 2 ** 28
    permuted = list(permuted_indices) + list(range(original_steps, steps))
    coeffs = list(coefficients) + [0] * (steps - original_steps)
    m_root, l_root, a_root = (bytes(proof[k]) for k in ("m_root", "l_root", "a_root"))
    g2 = root_of_unity(log_precision)
    xs = [1] * precision
    for i in range(1, precision):
        xs[i] = xs[i - 1] * g2 % P
    skips = precision // steps
    g1 = xs[skips]

    def ifft(v):
        return orc.inv_best_fft(to_limbs(v), g1, log_steps)

    k_poly, f0_poly, f1_poly, f2_poly = ifft(coeffs), ifft(flag0), ifft(flag1), ifft(flag2)
    assert verify_low_degree_proof(l_root, g2, proof["fri_proof"], precision // 4, skips)
    positions = get_pseudorandom_indices(l_root, precision, SPOT_CHECK_SECURITY_FACTOR, skips)
    aug = []
    for j in positions:
        aug += [j, (j + precision - skips) % precision, (j + original_steps // 3 * skips) % precision,
                (j + 2 * original_steps // 3 * skips) % precision]
    main_leaves = verify_multi_branch(m_root, aug, proof["main_branches"])
    l_leaves = verify_multi_branch(l_root, positions, proof["linear_comb_branches"])
    # Z(x) = x^steps - 1 evaluated at the spot-check points (verify.rs:121-122)
    ext_idx = from_limbs(orc.best_fft(orc.inv_best_fft(to_limbs(range(steps)), g1, log_steps), g2, log_precision))
    ext_pidx = from_limbs(orc.best_fft(orc.inv_best_fft(to_limbs(permuted), g1, log_steps), g2, log_precision))
    pxs = to_limbs([xs[p] for p in positions])
    k_at, f0_at, f1_at, f2_at = (from_limbs(orc.eval_poly_multi(pl, pxs)) for pl in (k_poly, f0_poly, f1_poly,
                                                                                      f2_poly))
    x_vals = [xs[skips * w] for (_, w) in public_first_indices]
    y_vals = [public_wires[k] for (k, _) in public_first_indices]
    interp2 = lagrange_interp(x_vals, y_vals)
    x_last = xs[(steps - 1) * skips]
    interp3 = lagrange_interp([xs[precision - skips]], [1])
    # r and k (verify.rs:159-175)
    rnd = get_pseudorandom_indices(a_root, precision, 24, 0)
    r = [int.from_bytes(b"".join(v.to_bytes(4, "big") for v in rnd[8 * c:8 * c + 8]), "little") % P
         for c in range(3)]
    kk = [1] + [int.from_bytes(blake(m_root + bytes([i])), "big") % P for i in range(1, 11)]
    for i, pos in enumerate(positions):
        x = xs[pos]
        b = [[fe(main_leaves[i * 4 + q][32 * c:32 * c + 32]) for c in range(8)] for q in range(4)]
        p_x, a_x, s_x, d1, d2, d3, b2, b3 = b[0]
        p_prev, a_prev = b[1][0], b[1][1]
        p_w, p_2w = b[2][0], b[3][0]
        z = (pow(x, steps, P) - 1) % P
        k_x, f0, f1, f2 = k_at[i], f0_at[i], f1_at[i], f2_at[i]
        assert f0 * (p_x - f1 * p_prev - k_x * s_x) % P == z * d1 % P, "Q1 = Z * D1"
        assert f2 * (p_2w - p_x * p_w) % P == z * d2 % P, "Q2 = Z * D2"
        nmr = (r[0] + r[1] * ext_idx[pos] + r[2] * s_x) % P
        dnm = (r[0] + r[1] * ext_pidx[pos] + r[2] * s_x) % P
        assert (a_x * dnm - a_prev * nmr) % P == z * d3 % P, "Q3 = Z * D3"
        zb2 = 1
        for (_, w) in public_first_indices:
            zb2 = zb2 * (x - xs[w * skips]) % P
        assert (s_x - eval_poly_at(interp2, x)) % P == zb2 * b2 % P, "S - I2 = Zb2 * B2"
        assert (a_x - eval_poly_at(interp3, x)) % P == (x - x_last) * b3 % P, "A - I3 = Zb3 * B3"
        xst = pow(x, steps, P)
        l_x = fe(l_leaves[i])
        want = (kk[0] * d1 + kk[1] * d2 + kk[2] * d3 + kk[3] * p_x + kk[4] * p_x * xst + kk[5] * b2
                + kk[6] * b2 * xst + kk[7] * b3 + kk[8] * b3 * xst + kk[9] * a_x + kk[10] * s_x) % P
        assert l_x == want, "linear combination"
    return True
