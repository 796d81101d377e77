"""Shoup product by a constant in radix 2^29 (9 limbs), carry-free (the NTT pass kernel's product).

Element a = sum a_i 2^(29 i), limbs a_i < 2^31 (not necessarily normalised), value < 2^261.
Constant w < p canonical with w' = floor(w 2^261 / p), both normalised 9-limb images.
    q ~ floor(a w' / 2^261)   from columns 7..16 of a*w' (dropped columns 0..6 sum to < 2^-25 of 2^261)
    r = a w + q (2^261 - p) mod 2^261 = a w - q p     in [0, 3p), 9 normalised limbs
Every column is at most 18 products of < 2^60 plus a carry-in < 2^36, so a 64-bit accumulator never
overflows: no carry instructions at all.  Per column: v_mad_u64_u32 per product (the first one adds
the carry-in pair), then v_lshrrev_b64 for the next column's carry-in and v_and_b32 for the limb.
143 v_mad_u64_u32 + 18 v_lshrrev_b64 + 17 v_and_b32 (Shoup-32: 115 mads + 99 carry counts).

usage: python tools/gen_fe29_asm.py > stark-pure-rust_amd/csrc/fe29_asm.inc   (python ... test: emulation)"""

P = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001
M29 = (1 << 29) - 1
NP29 = [((1 << 261) - P) >> (29 * i) & M29 for i in range(9)]


def stream(r, q, a, w, wq, np, pairs):
    out = []
    st = {"k": 0, "fresh": True}

    def pair(k):
        return pairs[k & 1]

    def acc(k):
        lo, hi = pair(k)
        return f"v[{lo}:{hi}]"

    def mac(k, x, y, first, carry_in):
        src2 = "0" if (first and not carry_in) else acc(k)
        # the first product of column k adds the carry-in, which the shift left in the other pair
        out.append(f"v_mad_u64_u32 {acc(k)}, vcc, {x}, {y}, {src2}")

    def finish(k, limb_dst, carry_out):
        lo, hi = pair(k)
        if carry_out:
            out.append(f"v_lshrrev_b64 {acc(k + 1)}, 29, {acc(k)}")
        if limb_dst is not None:
            out.append(f"v_and_b32 {limb_dst}, {M29:#x}, v{lo}")

    # 1. q from columns 7..16 of a * w'
    for k in range(7, 17):
        terms = [(i, k - i) for i in range(max(0, k - 8), min(8, k) + 1)]
        for t, (i, j) in enumerate(terms):
            mac(k, a[i], wq[j], t == 0, k > 7)
        finish(k, q[k - 9] if k >= 9 else None, True)
    # q_8 = carry out of column 16 (its low word)
    out.append(f"v_mov_b32 {q[8]}, v{pair(17)[0]}")
    # 2. r = low 261 bits of a*w + q*np
    for k in range(9):
        terms = [(a[i], w[k - i]) for i in range(k + 1)] + [(q[i], np[k - i]) for i in range(k + 1)]
        for t, (x, y) in enumerate(terms):
            mac(k, x, y, t == 0, k > 0)
        finish(k, r[k], k < 8)
    return out


def emit(name: str) -> str:
    r = [f"%{i}" for i in range(9)]
    q = [f"%{9 + i}" for i in range(9)]
    a = [f"%{18 + i}" for i in range(9)]
    w = [f"%{27 + i}" for i in range(9)]
    wq = [f"%{36 + i}" for i in range(9)]
    np_ = [f"%{45 + i}" for i in range(9)]
    body = "\\n\\t".join(stream(r, q, a, w, wq, np_, [(0, 1), (2, 3)]))
    outs = ", ".join([f'"=&v"(r.l[{i}])' for i in range(9)] + [f'"=&v"(q{i})' for i in range(9)])
    ins = ", ".join([f'"v"(a.l[{i}])' for i in range(9)] + [f'"v"(w.l[{i}])' for i in range(9)] +
                    [f'"v"(wq.l[{i}])' for i in range(9)])
    ins_np = ", ".join(f'"s"(N{i})' for i in range(9))
    decl_n = ", ".join(f"N{i} = {NP29[i]:#010x}u" for i in range(9))
    return f'''// Shoup product by a constant in radix 2^29 (tools/gen_fe29_asm.py): r = a*w mod p in [0, 3p) with
// normalised limbs, for a < 2^261 with limbs < 2^31.6 and (w, wq) a normalised Shoup pair.
__device__ __forceinline__ fe29 {name}(const fe29& a, const fe29& w, const fe29& wq) {{
  fe29 r;
  uint32_t {", ".join(f"q{i}" for i in range(9))};
  const uint32_t {decl_n};
  asm("{body}"
      : {outs}
      : {ins},
        {ins_np}
      : "v0", "v1", "v2", "v3", "vcc");
  return r;
}}
'''


def emulate(a, w, wq):
    """Exact integer emulation of the stream (for the CPU test): returns the 9 output limbs."""
    accs = {}
    out = {}
    ops = stream([f"r{i}" for i in range(9)], [f"q{i}" for i in range(9)], [f"a{i}" for i in range(9)],
                 [f"w{i}" for i in range(9)], [f"wq{i}" for i in range(9)], [f"np{i}" for i in range(9)],
                 [(0, 1), (2, 3)])
    env = {}
    for i in range(9):
        env[f"a{i}"], env[f"w{i}"], env[f"wq{i}"], env[f"np{i}"] = a[i], w[i], wq[i], NP29[i]
    regs = {}

    def val(x):
        x = x.strip()
        if x.startswith("v["):
            lo, hi = x[2:-1].split(":")
            return regs.get(int(lo), 0) | (regs.get(int(hi), 0) << 32)
        if x.startswith("v"):
            return regs.get(int(x[1:]), 0)
        if x.startswith("0x"):
            return int(x, 16)
        if x.isdigit():
            return int(x)
        return env[x]

    def setv(x, v):
        x = x.strip()
        if x.startswith("v["):
            lo, hi = x[2:-1].split(":")
            regs[int(lo)] = v & 0xffffffff
            regs[int(hi)] = (v >> 32) & 0xffffffff
        elif x.startswith("v"):
            regs[int(x[1:])] = v & 0xffffffff
        else:
            env[x] = v & 0xffffffff

    for op in ops:
        mn, rest = op.split(" ", 1)
        args = [s.strip() for s in rest.split(",")]
        if mn == "v_mad_u64_u32":
            v = val(args[2]) * val(args[3]) + val(args[4])
            assert v < 1 << 64, "accumulator overflow"
            setv(args[0], v)
        elif mn == "v_lshrrev_b64":
            setv(args[0], val(args[2]) >> int(args[1]))
        elif mn == "v_and_b32":
            setv(args[0], val(args[1]) & val(args[2]))
        elif mn == "v_mov_b32":
            setv(args[0], val(args[1]))
        else:
            raise ValueError(mn)
    del accs, out
    return [env[f"r{i}"] for i in range(9)]


def selftest():
    import random
    rnd = random.Random(1)
    for t in range(2000):
        wv = rnd.randrange(P)
        wqv = (wv << 261) // P
        av = rnd.randrange(1 << 261) if t % 2 else rnd.randrange(8 * P)
        al = [(av >> (29 * i)) & M29 for i in range(9)]
        if t % 3 == 0:   # unnormalised limbs up to 2^31 with the same value
            for i in range(8):
                b = rnd.randrange(4)
                if al[i + 1] >= b:
                    al[i + 1] -= b
                    al[i] += b << 29
        assert sum(x << (29 * i) for i, x in enumerate(al)) == av and max(al) < 1 << 31
        rl = emulate(al, [(wv >> (29 * i)) & M29 for i in range(9)], [(wqv >> (29 * i)) & M29 for i in range(9)])
        rv = sum(x << (29 * i) for i, x in enumerate(rl))
        assert rv % P == av * wv % P and rv < 3 * P, (t, rv // P)
    return True


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "test":
        selftest()
        print("ok")
    else:
        print("// GENERATED by tools/gen_fe29_asm.py -- do not edit.  Included by fp29_dev.h.")
        print(emit("fe29_mul_shoup"))
