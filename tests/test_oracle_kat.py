"""CPU: pin the oracle (C restatement + pure-Python restatement) against the
reference's own known-answer vectors and the DFT definition."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden_vectors.json")))


def test_blake_kats(oracle):
    for v in KATS["blake"]["vectors"]:
        msg = bytes.fromhex(v["msg_hex"])
        assert oracle.blake2s(msg).hex() == v["digest_hex"]
        assert O.py_blake(msg).hex() == v["digest_hex"]


@pytest.mark.parametrize("length", [0, 1, 31, 32, 33, 63, 64, 65, 127, 128, 129, 256, 1000])
def test_blake_lengths(oracle, length):
    msg = bytes((7 * i + 3) & 0xFF for i in range(length))
    assert oracle.blake2s(msg) == hashlib.blake2s(msg).digest()


def test_pseudorandom_indices_kats(oracle):
    for v in KATS["pseudorandom_indices"]["vectors"]:
        seed = O.py_blake(v["seed_msg"].encode())
        assert oracle.get_pseudorandom_indices(seed, v["modulus"], v["count"], v["exclude"]) == v["out"]
        assert O.py_get_pseudorandom_indices(seed, v["modulus"], v["count"], v["exclude"]) == v["out"]


def test_pseudorandom_indices_exclude(oracle):
    seed = O.py_blake(b"exclude")
    for modulus, excl in ((128, 8), (1 << 20, 8), (1000, 3)):
        got = oracle.get_pseudorandom_indices(seed, modulus, 80, excl)
        assert got == O.py_get_pseudorandom_indices(seed, modulus, 80, excl)
        assert all(x % excl != 0 and x < modulus for x in got)


def test_merkle_16_kat(oracle):
    k = KATS["merkle_16"]
    leaves = [bytes.fromhex(h) for h in k["leaves_hex"]]
    for chunks in (1, 2, 4, 8, 16):
        root, paths = oracle.merkle(b"".join(leaves), 16, 4, [k["index"]], chunks=chunks)
        assert root.hex() == k["root_hex"]
        assert [d.hex() for d in paths[0]] == k["nodes_hex"]
    root, paths = O.py_merkle(leaves, [k["index"]])
    assert root.hex() == k["root_hex"] and [d.hex() for d in paths[0]] == k["nodes_hex"]


def test_merkle_4096_kat(oracle):
    k = KATS["merkle_4096"]
    leaf = bytes.fromhex(k["leaf_hex"])
    root, paths = oracle.merkle(leaf * k["n"], k["n"], 4, k["indices"], chunks=8)
    assert root.hex() == k["root_hex"]
    assert paths[0][0].hex() == k["proof0_node0_hex"]


def test_merkle_multi_core_vs_serial(oracle):
    """merkle_proof_in_place.rs:208-259: chunked (cpus=4) == serial, duplicates kept, caller order."""
    k = KATS["merkle_multi_core"]
    leaves = [i.to_bytes(4, "big") for i in range(16)]
    r1, p1 = oracle.merkle(b"".join(leaves), 16, 4, k["indices"], chunks=k["cpus"])
    r2, p2 = oracle.merkle(b"".join(leaves), 16, 4, k["indices"], chunks=1)
    r3, p3 = O.py_merkle(leaves, k["indices"])
    assert r1 == r2 == r3 and p1 == p2 == p3


def test_fp_codec_kat():
    k = KATS["fp_codec"]
    assert list(O.to_bytes_le(k["value"])) == k["bytes_le"]
    assert list(O.to_bytes_le(k["value"])[::-1]) == k["bytes_be"]
    assert O.from_bytes_le(bytes(k["bytes_le"])) == k["value"]


def test_from_bytes_le_reduces(oracle):
    # ff from_str reduces mod p (fp.rs:74-76): 2^256 - 1 -> (2^256 - 1) mod p
    b = b"\xff" * 32
    assert oracle.from_bytes_le(b) == (2 ** 256 - 1) % O.P == O.from_bytes_le(b)


def test_multi_inv_f7_kat():
    k = KATS["multi_inv_f7"]
    for v in k["vectors"]:
        assert O.py_multi_inv(v["in"], p=k["p"]) == v["out"]


def test_multi_inv_bn254(oracle):
    vals = O.from_limbs(O.random_elements(50, 9))
    vals[3] = 0
    vals[49] = 0
    got = O.from_limbs(oracle.multi_inv(O.to_limbs(vals)))
    assert got == O.py_multi_inv(vals)
    assert all((g * v) % O.P == (1 if v else 0) for g, v in zip(got, vals))


def test_expand_root_kats(oracle):
    k = KATS["expand_root_f7"]
    assert O.py_expand_root_of_unity(k["root"], p=k["p"]) == k["out"]
    assert len(oracle.expand_root_of_unity(O.root_of_unity(16))) == k["bn254_order_65536_len"]


def test_simple_ft_f7_kat():
    k = KATS["simple_ft_f7"]
    p, roots = k["p"], k["roots"]
    m = len(roots)
    for v in k["vectors"]:
        x = v["in"] + [0] * max(0, m - len(v["in"]))
        got = [sum(x[j] * roots[(i * j) % m] for j in range(m)) % p for i in range(m)]
        assert got == v["out"]


def test_serial_fft_f7_matches_dft():
    # serial_fft (fft.rs:150-193) over F17 (8 | 16): equals the DFT definition.
    p, n = 17, 8
    w = pow(3, (p - 1) // n, p)
    x = [5, 1, 0, 16, 7, 2, 3, 9]
    assert O.py_serial_fft(x, w, 3, p=p) == O.py_dft(x, w, n, p=p)


@pytest.mark.parametrize("log_n", [0, 1, 2, 5, 9])
@pytest.mark.parametrize("cpus", [1, 2, 8])
def test_oracle_fft_vs_dft(oracle, log_n, cpus):
    n = 1 << log_n
    c = O.random_elements(max(1, n - 3), 100 + log_n)
    w = O.root_of_unity(log_n)
    want = O.py_dft(O.from_limbs(c), w, n)
    assert O.from_limbs(oracle.best_fft(c, w, log_n, cpus=cpus)) == want
    back = O.from_limbs(oracle.inv_best_fft(O.to_limbs(want), w, log_n, cpus=cpus))
    assert back == O.from_limbs(c) + [0] * (n - len(c))


def test_golden_ntt_vectors(oracle):
    for v in GOLD["ntt"]:
        c = O.to_limbs([int(x) for x in v["coeffs"]])
        w = int(v["root"])
        assert O.from_limbs(oracle.best_fft(c, w, v["log_n"], cpus=4)) == [int(x) for x in v["forward"]]
        assert O.from_limbs(oracle.inv_best_fft(c, w, v["log_n"], cpus=2)) == [int(x) for x in v["inverse"]]


def test_golden_merkle_vectors(oracle):
    for v in GOLD["merkle"]:
        leaves = b"".join(O.to_bytes_le(x) for x in O.from_limbs(O.random_elements(v["n"], v["seed"])))
        root, paths = oracle.merkle(leaves, v["n"], 32, v["indices"], chunks=4)
        assert root.hex() == v["root"]
        assert [[d.hex() for d in p] for p in paths] == v["paths"]


def test_golden_fri_vectors(oracle):
    for v in GOLD["fri"]:
        n = 1 << v["log_n"]
        w = O.root_of_unity(v["log_n"])
        vals = oracle.best_fft(O.random_elements(n // 4, v["coeff_seed"]), w, v["log_n"], cpus=4)
        js = oracle.prove_low_degree_json(vals, w, n // 4, v["exclude"], chunks=4)
        assert hashlib.sha256(js.encode()).hexdigest() == v["json_sha256"]


def test_fri_c_vs_python(oracle):
    log_n = 8
    n = 1 << log_n
    w = O.root_of_unity(log_n)
    vals = oracle.best_fft(O.random_elements(n // 4, 77), w, log_n)
    a = oracle.prove_low_degree_json(vals, w, n // 4, 8, chunks=2)
    b = O.py_prove_low_degree_json(O.from_limbs(vals), w, n // 4, 8)
    assert a == b
    proof = json.loads(a)
    # maxdeg 64 > 16 -> one Middle layer, then maxdeg 16 <= 16 -> Last (fri.rs:88)
    assert [list(x)[0] for x in proof] == ["Middle", "Last"]
    assert len(proof[-1]["Last"]["last"]) == n // 4


def test_random_elements_canonical():
    a = O.from_limbs(O.random_elements(1000, 5))
    assert all(0 <= x < O.P for x in a)
    assert len(set(a)) == 1000


def test_multi_interp_4_and_eval_quartic(oracle):
    """The C multi_interp_4 (poly_utils.rs:449-511) against the Python lagrange_interp on 4 points
    (poly_utils.rs:409-439), and eval_quartic (:442-446) against direct evaluation: the interpolant
    passes through every point; a row with a repeated x has a zero denominator, which multi_inv maps
    to zero (its contributions vanish)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    from stark_verify import lagrange_interp
    rows = 40
    xs = O.from_limbs(O.random_elements(4 * rows, 71))
    ys = O.from_limbs(O.random_elements(4 * rows, 72))
    xs[4 * 7 + 2] = xs[4 * 7 + 1]  # row 7: duplicate x
    got = O.from_limbs(oracle.multi_interp_4(O.to_limbs(xs), O.to_limbs(ys)))
    for r in range(rows):
        c = got[4 * r:4 * r + 4]
        if r != 7:
            assert c == lagrange_interp(xs[4 * r:4 * r + 4], ys[4 * r:4 * r + 4])
            for k in range(4):
                x = xs[4 * r + k]
                assert (c[0] + c[1] * x + c[2] * x * x + c[3] * x ** 3) % O.P == ys[4 * r + k]
    px = O.from_limbs(O.random_elements(4 * rows, 73))
    at = O.from_limbs(O.random_elements(rows, 74))
    q = O.from_limbs(oracle.eval_quartic_multi(O.to_limbs(px), O.to_limbs(at)))
    for i in range(rows):
        p, x = px[4 * i:4 * i + 4], at[i]
        assert q[i] == (p[0] + p[1] * x + p[2] * x * x + p[3] * x ** 3) % O.P
