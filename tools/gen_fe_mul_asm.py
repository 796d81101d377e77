"""Generates stark-pure-rust_amd/csrc/fe_mul_asm.inc: the BN254 Montgomery
product as ONE inline-asm block (FIPS product scanning, 128 v_mad_u64_u32 into
a 96-bit column accumulator), and the DUAL form that interleaves two
independent products instruction by instruction.

Why one block: hipcc pads one wait state after every inline-asm block whose
outputs the next VALU touches, so the per-word-product asm of fp_dev.h costs a
`s_nop 0` per product.  Inside one block nothing is padded: VALU -> VALU
VGPR/SGPR dependencies interlock in hardware on CDNA (the only hazards in this
stream would be readlane/permlane/DPP/MFMA, none of which appear).

Why the dual form: a product is one serial dependency chain (every
v_mad_u64_u32 accumulates into the column the previous one wrote, every
v_addc_co_u32 counts the carry the previous mad wrote).  At the 4 waves per
SIMD the NTT pass kernel runs at, a lone chain leaves issue slots empty
(tools/microbench/mul_forms.hip: 121 G products/s at 4 waves/SIMD vs 142 at
8); two interleaved chains give each wave independent work for every slot.

Registers: the column accumulator (a 64-bit pair + a carry word) lives in the
fixed VGPRs v0-v3 (v4-v7 for the second product) declared as clobbers (inline
asm has no sub-register operand modifiers, and the column shift needs the
pairs' halves): two pairs alternate by column; m[j] lives in the output
register r[j] until r[j] is written; p's limbs and -p^-1 are SGPR operands
(one SGPR read per VOP3 is allowed).

Measured on gfx950 (tools/microbench/isa_rates.hip, mul_forms.hip): carry ops
are half rate in either encoding (VOP3 with an SGPR pair, or VOP2 with VCC:
4.1-4.2 cycles per wave64 instruction), so the VCC form buys nothing (+3 % at
4 waves/SIMD, -1 % at 8); the generator keeps it for the record.

usage: python tools/gen_fe_mul_asm.py > stark-pure-rust_amd/csrc/fe_mul_asm.inc
(included by fp_dev.h inside namespace stark)
"""


def stream(r, a, b, p, pinv, cy, pairs, carry="sgpr") -> list:
    """Instruction list of one Montgomery product r = a*b*2^-256 (lazy, [0, 2p))."""
    m = r          # m[j] lives in r[j]: last read in column j+7, r[j] first written at the end of column j+8
    out = []
    st = {"first": True, "col_first": True, "k": 0}

    def pair(k):
        return pairs[k & 1]

    def mac(x, y):
        lo, hi = pair(st["k"])
        c = pair(st["k"] + 1)[1]      # carry count: the other pair's high register
        acc = f"v[{lo}:{hi}]"
        src2 = "0" if st["first"] else acc
        out.append(f"v_mad_u64_u32 {acc}, {cy}, {x}, {y}, {src2}")
        if st["col_first"]:
            out.append(f"v_addc_co_u32 v{c}, {cy}, 0, 0, {cy}")
        elif carry == "vcc":
            out.append(f"v_addc_co_u32_e32 v{c}, vcc, 0, v{c}, vcc")
        else:
            out.append(f"v_addc_co_u32 v{c}, {cy}, v{c}, 0, {cy}")
        st["col_first"] = False
        st["first"] = False

    def shift():
        # P_{k+1} = (P_k.hi, carry count of column k)
        lo, hi = pair(st["k"])
        out.append(f"v_mov_b32 v{pair(st['k'] + 1)[0]}, v{hi}")
        st["k"] += 1

    for k in range(8):
        st["col_first"] = True
        for j in range(k):
            mac(a[j], b[k - j])
            mac(m[j], p[k - j])
        mac(a[k], b[0])
        out.append(f"v_mul_lo_u32 {m[k]}, v{pair(k)[0]}, {pinv}")
        mac(m[k], p[0])
        shift()
    for k in range(8, 15):
        st["col_first"] = True
        for j in range(k - 7, 8):
            mac(a[j], b[k - j])
            mac(m[j], p[k - j])
        out.append(f"v_mov_b32 {r[k - 8]}, v{pair(k)[0]}")
        if k < 14:
            shift()
    out.append(f"v_mov_b32 {r[7]}, v{pair(14)[1]}")   # column 15 = column 14's high word (< 2p: no carry)
    return out


def shoup_stream(r, q, a, w, wq, np, cy, pairs, flag, qbase=None, rbase=None) -> list:
    """Instruction list of one Shoup product r = a*w mod p, r in [0, 2p), for a < 2^256 and a
    constant w < p with wq = floor(w 2^256 / p):
      1. q ~ floor(a wq / 2^256) from columns 6..15 of a*wq (43 word products; the dropped
         columns 0..5 sum to < 7 * 2^224, so q is exact or one short);
      2. r = a w + q (2^256 - p) mod 2^256 = a w - q p (72 word products, column 7 without carries):
         exact q gives r in [0, 2p) (Shoup), a short one r in [p, 3p);
      3. q can only be short when the column-7 word of step 1 is >= 2^32 - 8 (probability 2^-29):
         `flag` (an SGPR pair) marks such lanes and the wave subtracts 2p where r >= 2p only then.
    115 v_mad_u64_u32 + 99 v_addc_co_u32 against the Montgomery product's 128 + 128 + 8 v_mul_lo.

    Column k accumulates in the 64-bit pair colpair(k) and counts its carry-outs in the high word of
    colpair(k + 1); the next column starts from (high word, carry count), one v_mov_b32 per column
    (64-bit operands are even-aligned, so a column's high word never starts the next aligned pair).
    qbase: q's columns 8..15 accumulate in their own pairs v[qbase + 2i : +1], so q_i is the low
    word where it was summed (no copy); otherwise two pairs alternate and q is copied out.
    rbase: likewise r_c is the low word of v[rbase + 2c : +1] (the caller pins r there)."""
    out = []
    st = {"first": True, "col_first": True, "k": 0, "count": True, "step": 1}

    def colpair(k):
        if st["step"] == 1 and qbase is not None and k >= 8:
            return (qbase + 2 * (k - 8), qbase + 2 * (k - 8) + 1)
        if st["step"] == 2 and rbase is not None:
            return (rbase + 2 * k, rbase + 2 * k + 1)
        return pairs[k & 1]

    def mac(x, y):
        lo, hi = colpair(st["k"])
        c = colpair(st["k"] + 1)[1]
        acc = f"v[{lo}:{hi}]"
        src2 = "0" if st["first"] else acc
        out.append(f"v_mad_u64_u32 {acc}, {cy}, {x}, {y}, {src2}")
        if st["count"]:
            if st["col_first"]:
                out.append(f"v_addc_co_u32 v{c}, {cy}, 0, 0, {cy}")
            else:
                out.append(f"v_addc_co_u32 v{c}, {cy}, v{c}, 0, {cy}")
        st["col_first"] = False
        st["first"] = False

    def shift():
        lo, hi = colpair(st["k"])
        out.append(f"v_mov_b32 v{colpair(st['k'] + 1)[0]}, v{hi}")
        st["k"] += 1

    if qbase is not None:
        q = [f"v{qbase + 2 * i}" for i in range(8)]
    # 1. q from columns 6..15 of a * wq
    st["k"] = 6
    for c in range(6, 15):
        st["col_first"] = True
        for i in range(max(0, c - 7), min(7, c) + 1):
            mac(a[i], wq[c - i])
        if c == 7:
            out.append(f"v_cmp_lt_u32 {flag}, -9, v{colpair(7)[0]}")    # column-7 word >= 2^32 - 8
        if c >= 8 and qbase is None:
            out.append(f"v_mov_b32 {q[c - 8]}, v{colpair(c)[0]}")
        if c < 14 or qbase is not None:
            shift()                     # with qbase, column 15's pair receives q_7 = column 14's high word
    if qbase is None:
        out.append(f"v_mov_b32 {q[7]}, v{colpair(14)[1]}")   # column 15: q < 2^256, no carry beyond
    # 2. r = low 256 bits of a*w + q*(2^256 - p)
    st["step"] = 2
    st["k"] = 0
    st["first"] = True
    for c in range(8):
        st["col_first"] = True
        st["count"] = c < 7            # column 7's carry-out leaves the 256 bits
        for i in range(c + 1):
            mac(a[i], w[c - i])
            mac(q[i], np[c - i])
        if rbase is None:
            out.append(f"v_mov_b32 {r[c]}, v{colpair(c)[0]}")
        if c < 7:
            shift()
    return out


def csub2p_block(r, tmp, label, flag, p2) -> list:
    """if (any lane flagged) r -= 2p where r >= 2p (r < 3p); flagged lanes only ever need it."""
    out = [f"s_and_b64 {flag}, {flag}, exec",
           f"s_cmp_eq_u64 {flag}, 0",
           f"s_cbranch_scc1 .Lshoup_ok%={label}"]
    # tmp = r - 2p (2p's limbs moved into tmp first: a borrow-in already uses the constant bus)
    for i in range(8):
        out.append(f"v_mov_b32 {tmp[i]}, {p2[i]:#010x}")
    out.append(f"v_sub_co_u32 {tmp[0]}, vcc, {r[0]}, {tmp[0]}")
    for i in range(1, 8):
        out.append(f"v_subb_co_u32 {tmp[i]}, vcc, {r[i]}, {tmp[i]}, vcc")
    for i in range(8):
        out.append(f"v_cndmask_b32 {r[i]}, {tmp[i]}, {r[i]}, vcc")
    out.append(f".Lshoup_ok%={label}:")
    return out


PROLOGUE = '''  const uint32_t P0 = STARK_P0, P1 = STARK_P1, P2 = STARK_P2, P3 = STARK_P3, P4 = STARK_P4, P5 = STARK_P5,
                 P6 = STARK_P6, P7 = STARK_P7, PINV = STARK_PINV32;'''


def ops(prefix, var, start):
    return [f"%{start + i}" for i in range(8)], ", ".join(f'"v"({var}.w[{i}])' for i in range(8))


def emit_single(name: str, carry: str = "sgpr") -> str:
    r = [f"%{i}" for i in range(8)]
    cy = "%8" if carry == "sgpr" else "vcc"
    a = [f"%{9 + i}" for i in range(8)]
    b = [f"%{17 + i}" for i in range(8)]
    p = [f"%{25 + i}" for i in range(8)]
    body = "\\n\\t".join(stream(r, a, b, p, "%33", cy, [(0, 1), (2, 3)], carry))
    clob = ", ".join(f'"v{x}"' for x in range(4)) + (', "vcc"' if carry == "vcc" else "")
    outs = ", ".join(f'"=&v"(r.w[{i}])' for i in range(8))
    ins_a = ", ".join(f'"v"(a.w[{i}])' for i in range(8))
    ins_b = ", ".join(f'"v"(b.w[{i}])' for i in range(8))
    ins_p = ", ".join(f'"s"(P{i})' for i in range(8))
    return f'''// Montgomery product a*b*2^-256 mod p, result in [0, 2p) (not reduced).
// Inputs < 2^256 with a*b < 2^256 * p (e.g. a < 4p, b < p).
__device__ __forceinline__ fe {name}(const fe& a, const fe& b) {{
  fe r;
  uint64_t cy;
{PROLOGUE}
  asm("{body}"
      : {outs}, "=&s"(cy)
      : {ins_a},
        {ins_b},
        {ins_p}, "s"(PINV)
      : {clob});
  (void)cy;
  return r;
}}
'''


def emit_dual(name: str) -> str:
    """r = a*b, s = c*d (two independent lazy Montgomery products), interleaved."""
    r = [f"%{i}" for i in range(8)]
    s = [f"%{8 + i}" for i in range(8)]
    cya, cyb = "%16", "%17"
    a = [f"%{18 + i}" for i in range(8)]
    b = [f"%{26 + i}" for i in range(8)]
    c = [f"%{34 + i}" for i in range(8)]
    d = [f"%{42 + i}" for i in range(8)]
    p = [f"%{50 + i}" for i in range(8)]
    pinv = "%58"
    sa = stream(r, a, b, p, pinv, cya, [(0, 1), (2, 3)])
    sb = stream(s, c, d, p, pinv, cyb, [(4, 5), (6, 7)])
    assert len(sa) == len(sb)
    body = "\\n\\t".join(x for pair in zip(sa, sb) for x in pair)
    clob = ", ".join(f'"v{x}"' for x in range(8))
    outs = ", ".join([f'"=&v"(r.w[{i}])' for i in range(8)] + [f'"=&v"(s.w[{i}])' for i in range(8)])
    ins = ", ".join([f'"v"(a.w[{i}])' for i in range(8)] + [f'"v"(b.w[{i}])' for i in range(8)] +
                    [f'"v"(c.w[{i}])' for i in range(8)] + [f'"v"(d.w[{i}])' for i in range(8)])
    ins_p = ", ".join(f'"s"(P{i})' for i in range(8))
    return f'''// Two independent Montgomery products r = a*b*2^-256, s = c*d*2^-256 (each in [0, 2p), same
// input bounds as fe_mul_lazy), their instruction streams interleaved one for one.
__device__ __forceinline__ void {name}(fe& r, fe& s, const fe& a, const fe& b, const fe& c, const fe& d) {{
  uint64_t cya, cyb;
{PROLOGUE}
  asm("{body}"
      : {outs}, "=&s"(cya), "=&s"(cyb)
      : {ins},
        {ins_p}, "s"(PINV)
      : {clob});
  (void)cya;
  (void)cyb;
}}
'''


NP = [0x0fffffff, 0xbc1e0a6c, 0x86468f6e, 0xd7cc17b7, 0x7e7ea7a2, 0x47afba49, 0x1ece5fd6, 0xcf9bb18d]  # 2^256 - p
P2 = [0xe0000002, 0x87c3eb27, 0xf372e122, 0x5067d090, 0x0302b0ba, 0x70a08b6d, 0xc2634053, 0x60c89ce5]  # 2p


def emit_shoup(name: str, qbase=None, rbase=None) -> str:
    """fe_mul_shoup (see shoup_stream).  qbase: q summed in place in clobbered pairs v[qbase..+15];
    rbase: r pinned to the even registers v[rbase + 2c] (the odd ones clobbered), so the result is
    read where it was summed -- two call sites whose results are live together use two rbases."""
    r = [f"%{i}" for i in range(8)] if rbase is None else [f"v{rbase + 2 * i}" for i in range(8)]
    nq = 0 if qbase is not None else 8
    q = [f"%{8 + i}" for i in range(nq)]
    base = 8 + nq                      # r's 8 outputs are operands %0..%7 pinned or not
    cy, flag = f"%{base}", f"%{base + 1}"
    a = [f"%{base + 2 + i}" for i in range(8)]
    w = [f"%{base + 10 + i}" for i in range(8)]
    wq = [f"%{base + 18 + i}" for i in range(8)]
    np_ = [f"%{base + 26 + i}" for i in range(8)]
    body_l = shoup_stream(r, q, a, w, wq, np_, cy, [(0, 1), (2, 3)], flag, qbase, rbase)
    tmp = q if qbase is None else [f"v{qbase + 2 * i}" for i in range(8)]
    body_l += csub2p_block(r, tmp, "a", flag, P2)    # q is dead by then: reuse it as the temporary
    body = "\\n\\t".join(body_l)
    outs = []
    if rbase is None:
        outs += [f'"=&v"(r.w[{i}])' for i in range(8)]
    else:
        outs += [f'"=&{{v{rbase + 2 * i}}}"(r.w[{i}])' for i in range(8)]
    outs += [f'"=&v"(q{i})' for i in range(nq)]
    clob = [f'"v{x}"' for x in range(4)]
    if qbase is not None:
        clob += [f'"v{x}"' for x in range(qbase, qbase + 16)]
    if rbase is not None:
        clob += [f'"v{rbase + 2 * i + 1}"' for i in range(8)]
    clob += ['"vcc"', '"scc"']
    ins = ", ".join([f'"v"(a.w[{i}])' for i in range(8)] + [f'"v"(w.w[{i}])' for i in range(8)] +
                    [f'"v"(wq.w[{i}])' for i in range(8)])
    ins_np = ", ".join(f'"s"(N{i})' for i in range(8))
    decl_n = ", ".join(f"N{i} = {NP[i]:#010x}u" for i in range(8))
    decl_q = f"  uint32_t {', '.join(f'q{i}' for i in range(nq))};\n" if nq else ""
    return f'''// Shoup product by a constant: r = a*w mod p in [0, 2p) for any a < 2^256, w < p canonical and
// wq = floor(w 2^256 / p) (tools/gen_fe_mul_asm.py shoup_stream: 115 v_mad_u64_u32).
__device__ __forceinline__ fe {name}(const fe& a, const fe& w, const fe& wq) {{
  fe r;
{decl_q}  uint64_t cy, flag;
  const uint32_t {decl_n};
  asm("{body}"
      : {", ".join(outs)}, "=&s"(cy), "=&s"(flag)
      : {ins},
        {ins_np}
      : {", ".join(clob)});
  (void)cy;
  (void)flag;
  return r;
}}
'''


if __name__ == "__main__":
    print("// GENERATED by tools/gen_fe_mul_asm.py -- do not edit.  Included by fp_dev.h.")
    print(emit_single("fe_mul_lazy"))
    print(emit_dual("fe_mul_lazy2"))
    print("// The VCC-carry (VOP2 addc) form of fe_mul_lazy: A/B reference only (tools/microbench/mul_forms.hip).")
    print(emit_single("fe_mul_lazy_vcc", "vcc"))
    # q summed in place (qbase=4) or r pinned (rbase) remove 8-16 v_mov_b32 per product but the
    # 20-36 clobbered VGPRs make the pass kernel spill: 1.878 / 1.903 ms vs 1.831 ms per 2^24
    # transform (r02 A/B), so the product keeps its copies.
    print(emit_shoup("fe_mul_shoup"))
