"""CPU: the radix-2^29 arithmetic of the opt-in NTT pass kernel (stark-pure-rust_amd/csrc/fp29_dev.h,
ntt29.hip, STARK_NTT29=1) restated with exact integers.
  * the generated Shoup product (tools/gen_fe29_asm.py, csrc/fe29_asm.inc) emulated instruction by
    instruction for one lane: no 64-bit accumulator overflows and r = a*w mod p, r < 3p, normalised,
    for every input the kernel can feed it (limbs below 2^31.6, value below 2^261);
  * the borrowed images of 4p and 8p used by x - t + 4p / x - t + 8p: exact values, every limb at
    least as large as the subtracted operand's;
  * the butterfly schedule's limb growth (two levels of growth stay below the product's limit) and
    the table conversion wq = floor(w 2^261 / p) = 32 floor(w 2^256 / p) + floor(32 (w 2^256 mod p) / p);
  * the final canonical reduction's quotient estimate."""
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_fe29_asm as G  # noqa: E402

P = G.P
M29 = G.M29
K4 = [0x20000004, 0x3c3eb27d, 0x39709142, 0x3f4243cc, 0x36174a0b, 0x2b6d0301, 0x229b8503, 0x397098cf, 0x00c19138]
K8 = [0x20000008, 0x387d64fb, 0x32e12286, 0x3e84879a, 0x2c2e9418, 0x36da0604, 0x25370a07, 0x32e1319f, 0x01832272]
LIMIT = int(2 ** 31.6)   # product input limb bound (fp29_dev.h)


def limbs(x):
    return [(x >> (29 * i)) & M29 for i in range(9)]


def value(ls):
    return sum(v << (29 * i) for i, v in enumerate(ls))


def unnormalise(ls, rnd, top):
    """Same value, limbs pushed up towards `top` by borrowing from the next limb."""
    ls = list(ls)
    for i in range(8):
        room = (top - 1 - ls[i]) >> 29
        b = min(rnd.randrange(room + 1) if room > 0 else 0, ls[i + 1])
        ls[i + 1] -= b
        ls[i] += b << 29
    return ls


def test_generated_include_is_current():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_fe29_asm.py")], check=True,
                         capture_output=True, text=True).stdout
    with open(os.path.join(ROOT, "stark-pure-rust_amd", "csrc", "fe29_asm.inc")) as f:
        assert f.read() == out


def test_shoup29_stream_exact():
    rnd = random.Random(29)
    for t in range(1500):
        w = rnd.randrange(P) if t % 7 else rnd.choice([0, 1, P - 1])
        wq = (w << 261) // P
        kind = t % 3
        if kind == 0:
            a = rnd.randrange(P)
            al = limbs(a)
        elif kind == 1:                     # large values with limbs at the kernel's limit
            a = rnd.randrange(1 << 261)
            al = unnormalise(limbs(a), rnd, LIMIT)
        else:                               # lazy NTT values (< 64p), heavy limbs
            a = rnd.randrange(64 * P)
            al = unnormalise(limbs(a), rnd, LIMIT)
        assert value(al) == a and max(al) < LIMIT
        rl = G.emulate(al, limbs(w), limbs(wq))     # asserts no accumulator overflow
        r = value(rl)
        assert max(rl) <= M29
        assert r % P == a * w % P and r < 3 * P


def test_borrowed_multiples_of_p():
    for k, c in ((K4, 4), (K8, 8)):
        assert value(k) == c * P
        assert min(k[:8]) >= M29 and max(k) < 1 << 30
    # x - t + 4p never borrows a limb: t normalised with value < 3p (a product) or < 4p (an input)
    assert K4[8] >= ((4 * P - 1) >> 232) - 1 >= (3 * P) >> 232
    # x - t + 8p in the s = 0 step: t = x2 + x3 normalised, value < 8p when inputs are < 4p
    assert K8[8] >= ((8 * P - 1) >> 232) - 1


def test_butterfly_growth_stays_below_product_limit():
    # normalised limb < 2^29; each butterfly level adds < 2^30 per limb (t < 2^29 or K < 2^30);
    # a radix-4 step normalises x0 and x2, so a product input has at most two levels of growth
    assert M29 + 2 * ((1 << 30) - 1) < LIMIT
    # pass outputs (two levels) stored as u32 planes and read back as product inputs
    assert M29 + 2 * ((1 << 30) - 1) < 1 << 32


def test_butterfly_schedule_exact():
    """One radix-4 DIT step on random lazy inputs with the kernel's operations and normalisations."""
    rnd = random.Random(4)

    def mul(x, w):
        return G.emulate(x, limbs(w), limbs((w << 261) // P))

    def add(x, y):
        return [a + b for a, b in zip(x, y)]

    def subk(x, y, k=K4):
        out = [a + c - b for a, b, c in zip(x, y, k)]
        assert min(out) >= 0
        return out

    def norm(x):
        x = list(x)
        for i in range(8):
            x[i + 1] += x[i] >> 29
            x[i] &= M29
        return x

    for _ in range(200):
        # inputs as the previous step leaves them: two levels of growth, value < 40p
        xs = [unnormalise(limbs(rnd.randrange(40 * P)), rnd, M29 + 2 * (1 << 30)) for _ in range(4)]
        ws = [rnd.randrange(P) for _ in range(3)]
        x0, x1, x2, x3 = norm(xs[0]), xs[1], norm(xs[2]), xs[3]
        t1, t3 = mul(x1, ws[0]), mul(x3, ws[0])
        y0, y1 = add(x0, t1), subk(x0, t1)
        y2, y3 = add(x2, t3), subk(x2, t3)
        t2, t3b = mul(y2, ws[1]), mul(y3, ws[2])
        z0, z2 = add(y0, t2), subk(y0, t2)
        z1, z3 = add(y1, t3b), subk(y1, t3b)
        v = [value(x) for x in xs]
        e0 = (v[0] + v[1] * ws[0]) % P
        e1 = (v[0] - v[1] * ws[0]) % P
        e2 = (v[2] + v[3] * ws[0]) % P
        e3 = (v[2] - v[3] * ws[0]) % P
        assert value(z0) % P == (e0 + e2 * ws[1]) % P and value(z2) % P == (e0 - e2 * ws[1]) % P
        assert value(z1) % P == (e1 + e3 * ws[2]) % P and value(z3) % P == (e1 - e3 * ws[2]) % P
        for z in (z0, z1, z2, z3):
            assert max(z) < M29 + 2 * (1 << 30) and value(z) < 1 << 261


def test_table_conversion_formula():
    rnd = random.Random(5)
    for _ in range(500):
        w = rnd.randrange(P)
        m = (w << 256) % P
        q32 = (w << 256) // P
        assert q32 == (-m * pow(P, -1, 1 << 256)) % (1 << 256)
        assert (w << 261) // P == 32 * q32 + (32 * m) // P


def test_canonical_quotient_estimate():
    import numpy as np
    rnd = random.Random(6)
    assert P >> 232 == 3171406
    inv = np.float32(1.0 / 3171407.0 * (1.0 - 1.0 / (1 << 20)))
    for _ in range(2000):
        x = rnd.randrange(1 << 261)
        q = int(np.float32(np.float32(x >> 232) * inv))
        assert q <= x // P
        assert x - q * P < 3 * P
