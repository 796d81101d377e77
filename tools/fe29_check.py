"""Inputs for / check of tools/microbench/fe29_check.hip (fp29_dev.h building blocks on the GPU).
usage: fe29_check.py gen <in.bin> | fe29_check.py check <in.bin> <out.bin>"""
import random
import struct
import sys

P = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001
M29 = (1 << 29) - 1


def words(x, n=8):
    return [(x >> (32 * i)) & 0xffffffff for i in range(n)]


def val(ws, bits=32):
    return sum(w << (bits * i) for i, w in enumerate(ws))


def cases(n=4096):
    rnd = random.Random(7)
    out = []
    for t in range(n):
        a = rnd.randrange(P) if t % 4 else rnd.choice([0, 1, P - 1, (1 << 253)])
        b = rnd.randrange(P)
        w = rnd.randrange(P) if t % 5 else rnd.choice([0, 1, P - 1])
        out.append((a, b, w, (w << 256) % P))
    return out


def main():
    if sys.argv[1] == "gen":
        with open(sys.argv[2], "wb") as f:
            for a, b, w, m in cases():
                f.write(struct.pack("<32I", *(words(a) + words(b) + words(w) + words(m))))
        return
    cs = cases()
    raw = open(sys.argv[3], "rb").read()
    bad = {}
    for g, (a, b, w, m) in enumerate(cs):
        o = struct.unpack_from("<64I", raw, 256 * g)
        wq = (w << 261) // P
        checks = {
            "to32(from32)": val(o[0:8]) == a,
            "canonical": val(o[8:16]) == a,
            "mul(mont pair)": val(o[16:24]) == a * w % P,
            "mul_pair": val(o[24:32]) == a * w % P,
            "wq": val(o[32:41], 29) == wq,
            "subk": val(o[41:49]) == (a - b) % P,
            "add": val(o[49:57]) == (a + b) % P,
        }
        for k, ok in checks.items():
            if not ok:
                bad.setdefault(k, []).append(g)
    for k, v in bad.items():
        print(k, len(v), "bad, first", v[:5])
    print("ok" if not bad else "FAIL")


if __name__ == "__main__":
    main()
