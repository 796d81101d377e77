"""CPU: the generated modular products (tools/gen_fe_mul_asm.py, the inline asm in
stark-pure-rust_amd/csrc/fe_mul_asm.inc) emulated instruction by instruction with exact
integers for one lane: v_mad_u64_u32 / v_addc_co_u32 / v_sub(b)_co_u32 carry semantics, the
alternating accumulator pairs, the column shifts and the Shoup product's rare-correction branch.
  * Montgomery (single and the interleaved dual form): a*b*2^-256 mod p in [0, 2p) for a < 4p, b < p;
  * Shoup: a*w mod p in [0, 2p) for any a < 2^256, including inputs built to make the truncated
    quotient one short (the flagged correction path)."""
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_fe_mul_asm as G  # noqa: E402

P = 21888242871839275222246405745257275088548364400416034343698204186575808495617
M32 = (1 << 32) - 1
PINV = (-pow(P, -1, 1 << 32)) % (1 << 32)
R256 = 1 << 256


def _limbs(x):
    return [(x >> (32 * i)) & M32 for i in range(8)]


def _emulate(ops, regs: dict) -> dict:
    """Runs one lane of `ops` (exec = this lane) over `regs` (operand name -> u32)."""
    R = dict(regs)
    C = {"scc": 0}          # carry / mask SGPR pairs (one lane: 0 or 1)

    def val(x):
        if x == "0":
            return 0
        if x.startswith("0x"):
            return int(x, 16)
        if x.lstrip("-").isdigit():
            return int(x) & M32
        if x.startswith("v["):
            lo, hi = map(int, x[2:-1].split(":"))
            assert lo % 2 == 0 and hi == lo + 1, "64-bit operands are even-aligned pairs"
            return R[f"v{lo}"] | (R[f"v{hi}"] << 32)
        return R[x]

    def setv(x, v):
        if x.startswith("v["):
            lo, hi = map(int, x[2:-1].split(":"))
            R[f"v{lo}"], R[f"v{hi}"] = v & M32, (v >> 32) & M32
        else:
            R[x] = v & M32

    labels = {op[:-1]: i for i, op in enumerate(ops) if op.endswith(":")}
    pc = 0
    while pc < len(ops):
        op = ops[pc]
        pc += 1
        if op.endswith(":"):
            continue
        name, rest = op.split(" ", 1)
        args = [t.strip() for t in rest.split(",")]
        if name == "v_mad_u64_u32":
            d, c, x, y, s2 = args
            res = val(x) * val(y) + val(s2)
            C[c] = res >> 64
            setv(d, res)
        elif name in ("v_addc_co_u32", "v_addc_co_u32_e32"):
            d, c, x, y, ci = args
            s = val(x) + val(y) + C[ci]
            C[c] = s >> 32
            setv(d, s)
        elif name == "v_sub_co_u32":
            d, c, x, y = args
            s = val(x) - val(y)
            C[c] = 1 if s < 0 else 0
            setv(d, s)
        elif name == "v_subb_co_u32":
            d, c, x, y, ci = args
            s = val(x) - val(y) - C[ci]
            C[c] = 1 if s < 0 else 0
            setv(d, s)
        elif name == "v_cndmask_b32":
            d, x, y, m = args
            setv(d, val(y) if C[m] else val(x))
        elif name == "v_mul_lo_u32":
            d, x, y = args
            setv(d, val(x) * val(y))
        elif name == "v_mov_b32":
            d, x = args
            setv(d, val(x))
        elif name == "v_cmp_lt_u32":
            d, x, y = args
            C[d] = 1 if val(x) < val(y) else 0
        elif name == "s_and_b64":
            d, x, y = args
            C[d] = C[x] & (1 if y == "exec" else C[y])
        elif name == "s_cmp_eq_u64":
            x, y = args
            C["scc"] = 1 if C[x] == int(y) else 0
        elif name == "s_cbranch_scc1":
            if C["scc"]:
                pc = labels[args[0]]
        else:
            raise AssertionError(f"unexpected instruction {op}")
    return R


def _mont_regs(a, b, base_a, base_b, base_p=None, pinv=None):
    regs = {}
    for i, (x, y) in enumerate(zip(_limbs(a), _limbs(b))):
        regs[f"%{base_a + i}"] = x
        regs[f"%{base_b + i}"] = y
    if base_p is not None:
        for i, x in enumerate(_limbs(P)):
            regs[f"%{base_p + i}"] = x
        regs[pinv] = PINV
    return regs


def _out(R, base):
    return sum(R[f"%{base + i}"] << (32 * i) for i in range(8))


def _mont_cases():
    rnd = random.Random(7)
    # [0, 4p + 2^224): the lazy range of the radix-2^6 NTT passes, whose butterflies reduce by 2p only
    # when the top word exceeds 2p's (csrc/ntt.hip)
    top = 4 * P + (1 << 224) - 1
    cases = [(0, 0), (1, 1), (P - 1, P - 1), (4 * P - 1, P - 1), (4 * P - 1, 1), (2 ** 255, P - 1),
             (top, P - 1), (top, 1), (top, top % P)]
    return cases + [(rnd.randrange(4 * P), rnd.randrange(P)) for _ in range(1500)] + \
        [(rnd.randrange(4 * P, top + 1), rnd.randrange(P)) for _ in range(200)]


def test_generated_montgomery_product():
    assert PINV == 0xEFFFFFFF  # STARK_PINV32 in fp_dev.h
    r = [f"%{i}" for i in range(8)]
    ops = G.stream(r, [f"%{9 + i}" for i in range(8)], [f"%{17 + i}" for i in range(8)],
                   [f"%{25 + i}" for i in range(8)], "%33", "%8", [(0, 1), (2, 3)])
    rinv = pow(R256, -1, P)
    for a, b in _mont_cases():
        out = _out(_emulate(ops, _mont_regs(a, b, 9, 17, 25, "%33")), 0)
        assert out < 2 * P
        assert out % P == a * b * rinv % P


def test_generated_dual_product():
    """fe_mul_lazy2: two Montgomery products interleaved one for one (emit_dual's operand map)."""
    r, s = [f"%{i}" for i in range(8)], [f"%{8 + i}" for i in range(8)]
    p = [f"%{50 + i}" for i in range(8)]
    sa = G.stream(r, [f"%{18 + i}" for i in range(8)], [f"%{26 + i}" for i in range(8)], p, "%58", "%16",
                  [(0, 1), (2, 3)])
    sb = G.stream(s, [f"%{34 + i}" for i in range(8)], [f"%{42 + i}" for i in range(8)], p, "%58", "%17",
                  [(4, 5), (6, 7)])
    ops = [x for pr in zip(sa, sb) for x in pr]
    rinv = pow(R256, -1, P)
    cases = _mont_cases()
    for (a, b), (c, d) in zip(cases[:700], cases[700:1400]):
        regs = _mont_regs(a, b, 18, 26, 50, "%58")
        regs.update(_mont_regs(c, d, 34, 42))
        R = _emulate(ops, regs)
        x, y = _out(R, 0), _out(R, 8)
        assert x < 2 * P and y < 2 * P
        assert x % P == a * b * rinv % P and y % P == c * d * rinv % P


def _shoup_ops(qbase=None, rbase=None):
    """emit_shoup's operand map: r = %0..%7 (or pinned v[rbase + 2c]), q = %8.. unless in place,
    then cy, flag, a, w, wq, 2^256 - p."""
    r = [f"%{i}" for i in range(8)] if rbase is None else [f"v{rbase + 2 * i}" for i in range(8)]
    nq = 0 if qbase is not None else 8
    q = [f"%{8 + i}" for i in range(nq)]
    b = 8 + nq
    ops = G.shoup_stream(r, q, [f"%{b + 2 + i}" for i in range(8)], [f"%{b + 10 + i}" for i in range(8)],
                         [f"%{b + 18 + i}" for i in range(8)], [f"%{b + 26 + i}" for i in range(8)], f"%{b}",
                         [(0, 1), (2, 3)], f"%{b + 1}", qbase, rbase)
    tmp = q if qbase is None else [f"v{qbase + 2 * i}" for i in range(8)]
    return ops + G.csub2p_block(r, tmp, "a", f"%{b + 1}", G.P2), r, b


def _shoup(opsr, a, w):
    ops, r, b = opsr
    wq = w * R256 // P
    regs = {}
    for i in range(8):
        regs[f"%{b + 2 + i}"] = _limbs(a)[i]
        regs[f"%{b + 10 + i}"] = _limbs(w)[i]
        regs[f"%{b + 18 + i}"] = _limbs(wq)[i]
        regs[f"%{b + 26 + i}"] = G.NP[i]
    R = _emulate([o.replace("%=", "") for o in ops], regs)
    return sum(R[r[i]] << (32 * i) for i in range(8))


def _short_quotient(a, w):
    wq = w * R256 // P
    lo = sum(((a >> (32 * k)) & M32) * ((wq >> (32 * (c - k))) & M32) << (32 * c)
             for c in range(6) for k in range(c + 1))
    return (a * wq - lo) // R256 != a * wq // R256


@pytest.mark.parametrize("qbase,rbase", [(None, None), (4, None), (4, 20), (4, 36)])
def test_generated_shoup_product(qbase, rbase):
    assert sum(x << (32 * i) for i, x in enumerate(G.NP)) == R256 - P
    assert sum(x << (32 * i) for i, x in enumerate(G.P2)) == 2 * P
    ops = _shoup_ops(qbase, rbase)
    rnd = random.Random(11)
    cases = [(0, 0), (R256 - 1, P - 1), (4 * P - 1, P - 1), (1, 1), (R256 - 1, 1)]
    cases += [(rnd.randrange(4 * P), rnd.randrange(P)) for _ in range(800)]
    cases += [(rnd.randrange(R256), rnd.randrange(P)) for _ in range(400)]
    short = 0
    for _ in range(400):                      # a*wq = 2^100 mod 2^256: the dropped columns carry
        w = rnd.randrange(P)
        wq = w * R256 // P
        if wq % 2:
            a = (1 << 100) * pow(wq, -1, R256) % R256
            cases.append((a, w))
    for a, w in cases:
        r = _shoup(ops, a, w)
        short += _short_quotient(a, w)
        assert r < 2 * P, (a, w)
        assert r % P == a * w % P
    assert short > 50                         # the correction path was exercised


def test_committed_asm_is_generated():
    """fe_mul_asm.inc is exactly the generator's output."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_fe_mul_asm.py")], capture_output=True,
                         text=True, check=True).stdout
    inc = open(os.path.join(ROOT, "stark-pure-rust_amd", "csrc", "fe_mul_asm.inc")).read()
    assert out == inc
