"""Digit-basis constant product (csrc/fe_db.h): CPU emulation, tables and the GPU check.

    python tools/db_check.py make  N db_in.bin     # N random (a, W) records (+ edge cases)
    python tools/db_check.py check db_in.bin db_out.bin

`db_emulate` restates fe_mul_db step by step with exact integers and IEEE doubles (Python floats;
fma by exact rational arithmetic rounded once), so the CPU test can check the quotient bound on
inputs built to sit next to the margin.
"""
import math
import random
import struct
import sys
from fractions import Fraction

P = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
M29 = (1 << 29) - 1
N261 = (1 << 261) - P
N_LIMBS = [(N261 >> (29 * j)) & M29 for j in range(9)]
C8 = float(Fraction(1 << 232, P))
C7 = float(Fraction(1 << 235, P))
MARGIN = 2.0 ** -12


def db_table(w):
    """72 u32: limb j (29 bits) of W_i = w 2^(32 i) mod p at 9 i + j."""
    out = []
    for i in range(8):
        wi = (w << (32 * i)) % P
        out += [(wi >> (29 * j)) & M29 for j in range(9)]
    return out


def _fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _trunc_u32(x):
    # v_cvt_u32_f64: truncate toward zero, saturate to [0, 2^32 - 1]
    if x != x or x <= 0:
        return 0
    return min(int(x), (1 << 32) - 1)


def db_emulate(a, table):
    """fe_mul_db (csrc/fe_db.h) step by step; a < 4p + 2^224."""
    assert 0 <= a < 4 * P + (1 << 224)
    aw = [(a >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
    acc = [sum(aw[i] * table[9 * i + j] for i in range(8)) for j in range(9)]
    d8 = _fma(float(acc[8] >> 32), 2.0 ** 32, float(acc[8] & 0xFFFFFFFF))
    d7 = float(acc[7] >> 32)
    f = max(_fma(d8, C8, _fma(d7, C7, -MARGIN)), 0.0)
    qh = _trunc_u32(f * 2.0 ** -29)
    ql = _trunc_u32(_fma(float(qh), -(2.0 ** 29), f))
    for j in range(9):
        acc[j] += ql * N_LIMBS[j] + (qh * N_LIMBS[j - 1] if j else 0)
    r = [0] * 9
    c = 0
    for j in range(9):
        t = acc[j] + c
        assert t < (1 << 64), "column overflow"
        r[j] = t & M29
        c = t >> 29
    val = sum(r[j] << (29 * j) for j in range(9))
    words = [
        (r[0] | (r[1] << 29)) & 0xFFFFFFFF,
        ((r[1] >> 3) | (r[2] << 26)) & 0xFFFFFFFF,
        ((r[2] >> 6) | (r[3] << 23)) & 0xFFFFFFFF,
        ((r[3] >> 9) | (r[4] << 20)) & 0xFFFFFFFF,
        ((r[4] >> 12) | (r[5] << 17)) & 0xFFFFFFFF,
        ((r[5] >> 15) | (r[6] << 14)) & 0xFFFFFFFF,
        ((r[6] >> 18) | (r[7] << 11)) & 0xFFFFFFFF,
        ((r[7] >> 21) | (r[8] << 8)) & 0xFFFFFFFF,
    ]
    out = sum(x << (32 * k) for k, x in enumerate(words))
    assert out == val, "repack lost bits (value >= 2^256)"
    return out


def make(n, path, seed=1):
    rng = random.Random(seed)
    recs = []
    edge_a = [0, 1, P - 1, P, 2 * P - 1, 4 * P - 1, 3 * P, (1 << 255)]
    edge_w = [0, 1, P - 1, 2, (P + 1) // 2]
    for k in range(n):
        if k < len(edge_a) * len(edge_w):
            a, w = edge_a[k % len(edge_a)], edge_w[k // len(edge_a)]
        else:
            a = rng.randrange(4 * P)
            w = rng.randrange(P)
        recs.append((a, w))
    with open(path, "wb") as fh:
        for a, w in recs:
            fh.write(a.to_bytes(32, "little"))
            fh.write(struct.pack("<72I", *db_table(w)))
    return recs


def check(inp, outp):
    data = open(inp, "rb").read()
    res = open(outp, "rb").read()
    n = len(data) // 320
    bad = 0
    for k in range(n):
        rec = data[320 * k: 320 * (k + 1)]
        a = int.from_bytes(rec[:32], "little")
        tab = struct.unpack("<72I", rec[32:])
        w = sum(tab[j] << (29 * j) for j in range(9))  # W_0 = w
        r = int.from_bytes(res[32 * k: 32 * (k + 1)], "little")
        if r >= 2 * P or (r - a * w) % P:
            bad += 1
    print(f"{n} products, {bad} wrong")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "make":
        make(int(sys.argv[2]), sys.argv[3])
    else:
        sys.exit(1 if check(sys.argv[2], sys.argv[3]) else 0)
