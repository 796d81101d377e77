"""Digit-basis constant product (csrc/fe_db.h), checked on the CPU.

`tools/db_check.py:db_emulate` restates fe_mul_db step by step with exact integers and IEEE doubles;
here it is run on random and edge inputs in the NTT's lazy range [0, 4p + 2^224), on inputs whose quotient
estimate sits next to the margin, and the header's constants are checked against their definitions.
The GPU side is exercised bit-exactly by every NTT parity test (tests/test_gpu_ntt.py,
tests/test_gpu_large.py) and by tools/microbench/db_rate.hip (65,536 products vs Python).
"""
import os
import random
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import db_check as D  # noqa: E402

HDR = os.path.join(ROOT, "stark-pure-rust_amd", "csrc", "fe_db.h")


def _defines():
    out = {}
    for m in re.finditer(r"#define (STARK_DB_\w+) (\S+)", open(HDR).read()):
        out[m.group(1)] = m.group(2)
    return out


def test_header_constants():
    d = _defines()
    for j in range(9):
        assert int(d[f"STARK_DB_N{j}"].rstrip("u"), 16) == D.N_LIMBS[j]
    assert float(d["STARK_DB_C8"]) == D.C8
    assert float(d["STARK_DB_C7"]) == D.C7
    assert float(d["STARK_DB_MARGIN"]) == D.MARGIN
    assert int(d["STARK_DB_M29"].rstrip("u"), 16) == D.M29


def _check(a, w):
    r = D.db_emulate(a, D.db_table(w))
    assert 0 <= r < 2 * D.P and (r - a * w) % D.P == 0, (a, w, r)
    return r


def test_random_and_edges():
    rng = random.Random(11)
    edges_a = [0, 1, D.P - 1, D.P, 2 * D.P - 1, 2 * D.P, 3 * D.P, 4 * D.P - 1, 1 << 255, (1 << 224) * 0xC19139CB]
    edges_w = [0, 1, 2, D.P - 1, (D.P + 1) // 2, pow(7, (D.P - 1) // 4, D.P)]
    for a in edges_a:
        if a < 4 * D.P:
            for w in edges_w:
                _check(a, w)
    for _ in range(3000):
        _check(rng.randrange(4 * D.P), rng.randrange(D.P))
    # the radix-2^6 passes' lazy range reaches 4p + 2^224: the top word stays below 2^31.6 + 1
    top = 4 * D.P + (1 << 224) - 1
    for w in edges_w:
        _check(top, w)
    for _ in range(500):
        _check(rng.randrange(4 * D.P, top + 1), rng.randrange(D.P))


def test_quotient_next_to_margin():
    # a w = k p exactly (a = p, 2p, 3p) puts S / p on an integer: the estimate must stay below it
    # (q one short, r = p) and never above (r would be negative).
    rng = random.Random(12)
    short = 0
    for _ in range(300):
        w = rng.randrange(1, D.P)
        for m in (1, 2, 3):
            r = _check(m * D.P, w)
            short += r == D.P
    assert short > 0
    # and S / p just below an integer: a = k p - small
    for _ in range(300):
        w = rng.randrange(1, D.P)
        _check(rng.randrange(1, 4) * D.P - rng.randrange(1, 1 << 20), w)


def test_table_layout():
    w = 0x1234567890ABCDEF1234567890ABCDEF1234567890ABCDEF1234567890ABCDE % D.P
    t = D.db_table(w)
    assert len(t) == 72 and all(x < (1 << 29) for x in t)
    for i in range(8):
        assert sum(t[9 * i + j] << (29 * j) for j in range(9)) == (w << (32 * i)) % D.P
