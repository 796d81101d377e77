"""Inputs and the check for tools/microbench/mfma_mul.hip (the int8-MFMA constant product).

    python tools/mfma_mul_check.py make  N mfma_in.bin     # one random constant, N elements (+ edge cases)
    python tools/mfma_mul_check.py check mfma_in.bin mfma_out.bin

The check compares every output with a * w^k mod p (k = 1 and 64 chained products) for both forms
(MFMA column sums and the digit-basis VALU product) and checks the lazy range [0, 2p).
"""
import random
import struct
import sys
from fractions import Fraction

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from db_check import P, db_table  # noqa: E402

ITERS = 256


def balanced_digits(x):
    """32 signed bytes d_j in [-128, 127] with sum d_j 2^(8 j) = x (0 <= x < 2^254)."""
    out, c = [], 0
    for j in range(32):
        b = ((x >> (8 * j)) & 255) + c
        c = 1 if b >= 128 else 0
        out.append(b - 256 * c)
    assert c == 0 and sum(d << (8 * j) for j, d in enumerate(out)) == x
    return out


def constants(w):
    wi = [(w << (8 * i)) % P for i in range(32)]
    d = [balanced_digits(x) for x in wi]          # d[i][j]
    a = []                                        # lane l: row j = l & 31, i = 16 (l >> 5) + byte
    for lane in range(64):
        j, h = lane & 31, lane >> 5
        by = bytes((d[16 * h + t][j]) & 255 for t in range(16))
        a.append(struct.unpack("<4i", by))
    k = (128 * sum(wi)) % P + (1 << 12) * P
    assert k < 1 << 288
    kw = [(k >> (32 * g)) & 0xFFFFFFFF for g in range(9)]
    c224 = float(Fraction(1 << 224, P))
    blob = b"".join(struct.pack("<4i", *x) for x in a) + struct.pack("<9I", *kw) + b"\0" * 12
    blob += struct.pack("<dd", c224, 2.0 ** -20)
    return blob


def make(n, path):
    rng = random.Random(0x3FA5)
    w = rng.randrange(1, P)
    els = [0, 1, P - 1, 2 * P - 1, (1 << 256) - 1 if (1 << 256) - 1 < 2 * P else 2 * P - 2]
    els += [rng.randrange(0, 2 * P) for _ in range(n - len(els))]
    with open(path, "wb") as f:
        f.write(constants(w))
        f.write(struct.pack("<72I", *db_table(w)))
        f.write(struct.pack("<i", n))
        for x in els:
            f.write(x.to_bytes(32, "little"))
        f.write(w.to_bytes(32, "little"))   # (trailer: the constant, for the check)


def check(inp, outp):
    raw = open(inp, "rb").read()
    off = 64 * 16 + 36 + 12 + 16 + 72 * 4
    n = struct.unpack_from("<i", raw, off)[0]
    off += 4
    els = [int.from_bytes(raw[off + 32 * i: off + 32 * i + 32], "little") for i in range(n)]
    w = int.from_bytes(raw[off + 32 * n: off + 32 * n + 32], "little")
    out = open(outp, "rb").read()
    bad = 0
    for blk, (k, form) in enumerate(((1, "mfma"), (1, "digit basis"), (ITERS, "mfma"), (ITERS, "digit basis"))):
        wk = pow(w, k, P)
        base = blk * 32 * n
        for i in range(n):
            r = int.from_bytes(out[base + 32 * i: base + 32 * i + 32], "little")
            if r >= 2 * P or r % P != els[i] * wk % P:
                bad += 1
                if bad < 5:
                    print(f"{form} k={k} element {i}: got {r:#x}")
    print(f"{n} elements x 4 checks, {bad} wrong")
    return bad == 0


if __name__ == "__main__":
    if sys.argv[1] == "make":
        make(int(sys.argv[2]), sys.argv[3])
    else:
        sys.exit(0 if check(sys.argv[2], sys.argv[3]) else 1)
