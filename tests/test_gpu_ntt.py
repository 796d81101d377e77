"""GPU parity: NTT / iNTT through the C ABI vs the oracle (bit-exact)."""
import json
import os

import numpy as np
import pytest

import oracle as O
import stark_amd as S

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden_vectors.json")))


def test_golden_ntt(ctx):
    for v in GOLD["ntt"]:
        c = O.to_limbs([int(x) for x in v["coeffs"]])
        w = int(v["root"])
        assert O.from_limbs(ctx.best_fft(c, w, v["log_n"])) == [int(x) for x in v["forward"]]
        assert O.from_limbs(ctx.inv_best_fft(c, w, v["log_n"])) == [int(x) for x in v["inverse"]]


@pytest.mark.parametrize("log_n", list(range(0, 19)))
def test_ntt_vs_oracle(ctx, oracle, log_n):
    n = 1 << log_n
    c = O.random_elements(n, 0x5EED0000 + log_n)
    w = O.root_of_unity(log_n)
    want = oracle.best_fft(c, w, log_n, cpus=8)
    got = ctx.best_fft(c, w, log_n)
    assert np.array_equal(got, want)
    want_i = oracle.inv_best_fft(c, w, log_n, cpus=8)
    got_i = ctx.inv_best_fft(c, w, log_n)
    assert np.array_equal(got_i, want_i)


@pytest.mark.parametrize("log_n,length", [(10, 1), (10, 77), (12, 1000), (16, 65535), (13, 0)])
def test_ntt_zero_padding(ctx, oracle, log_n, length):
    c = O.random_elements(max(length, 1), 11)[:length]
    w = O.root_of_unity(log_n)
    assert np.array_equal(ctx.best_fft(c, w, log_n), oracle.best_fft(c, w, log_n, cpus=8))


@pytest.mark.parametrize("log_n,zero_log", [(2, 1), (2, 2), (7, 3), (7, 7), (9, 1), (9, 4), (16, 2), (16, 3),
                                             (18, 3), (18, 6), (20, 3), (21, 7), (23, 3)])
def test_ntt_sparse_first_pass(ctx, oracle, log_n, zero_log):
    """Power-of-two inputs zero-padded by up to the first pass's radix take the sparse first pass
    (the padding is neither written nor read; the first copy stages are skipped): forward and inverse
    equal best_fft / inv_best_fft of the padded vector (fft.rs:327-379)."""
    length = 1 << (log_n - zero_log)
    c = O.random_elements(length, 900 + log_n * 10 + zero_log)
    w = O.root_of_unity(log_n)
    cpus = 16 if log_n >= 20 else 8
    assert np.array_equal(ctx.best_fft(c, w, log_n), oracle.best_fft(c, w, log_n, cpus=cpus))
    assert np.array_equal(ctx.inv_best_fft(c, w, log_n), oracle.inv_best_fft(c, w, log_n, cpus=cpus))


def test_ntt_extreme_values(ctx, oracle):
    # p-1 everywhere, zeros, ones: stresses the carry / reduction paths.
    log_n = 12
    n = 1 << log_n
    c = np.zeros((n, 4), dtype=np.uint64)
    c[: n // 3] = O.to_limbs([O.P - 1])[0]
    c[n // 3: n // 2] = O.to_limbs([1])[0]
    w = O.root_of_unity(log_n)
    assert np.array_equal(ctx.best_fft(c, w, log_n), oracle.best_fft(c, w, log_n, cpus=8))
    assert np.array_equal(ctx.inv_best_fft(c, w, log_n), oracle.inv_best_fft(c, w, log_n, cpus=8))


def test_ntt_other_root(ctx, oracle):
    # any primitive root of the right order, e.g. w^3 and w^-1
    log_n = 11
    w = pow(O.root_of_unity(log_n), 3, O.P)
    c = O.random_elements(1 << log_n, 99)
    assert np.array_equal(ctx.best_fft(c, w, log_n), oracle.best_fft(c, w, log_n, cpus=4))


def test_ntt_errors(ctx):
    w = O.root_of_unity(8)
    c = O.random_elements(300, 1)
    with pytest.raises(S.StarkError) as e:
        ctx.best_fft(c, w, 8)  # len > 2^log_n (fft.rs:162 assert)
    assert e.value.code == 1
    with pytest.raises(S.StarkError) as e:
        ctx.best_fft(c[:10], pow(w, 2, O.P), 8)  # root of order 128, not 256
    assert e.value.code == 2


@pytest.mark.parametrize("log_n", [20, 22, 24, 25, 26, 28])
def test_ntt_roundtrip_large(ctx, oracle, log_n):
    """fwd then inv == identity at full size (size-independent property); from 2^25 on two forward
    outputs are also checked against the oracle's Horner evaluation: 2^25 runs radix-512 passes
    (8, 8, 9), 2^26 the four-pass digit-basis plan (6, 6, 7, 7) whose third pass takes the two-level
    column twiddle with the digit-basis last step, and 2^28 (7, 7, 7, 7) the two-level column twiddle
    in its last two passes (no full last-pass table past 2^26).  (2^25..2^27 dense outputs are also
    pinned by digest in tests/test_gpu_large.py.)"""
    n = 1 << log_n
    if log_n < 27:
        c = O.random_elements(n, 0x5EED0000 + log_n)
    else:  # uniform below 2^252 < p, without the generator's 2^30-candidate temporaries
        c = np.random.default_rng(log_n).integers(0, 2**64, size=(n, 4), dtype=np.uint64)
        c[:, 3] >>= np.uint64(4)
    w = O.root_of_unity(log_n)
    d = ctx.alloc(n * 32)
    try:
        ctx.h2d(d, c)
        ctx.ntt_dev(d, log_n, 1, w, inverse=False)
        mid = np.empty_like(c)
        ctx.d2h(mid, d)
        assert not np.array_equal(mid, c)
        ctx.ntt_dev(d, log_n, 1, w, inverse=True)
        back = np.empty_like(c)
        ctx.d2h(back, d)
        assert np.array_equal(back, c)
        if log_n >= 25:
            rng = np.random.default_rng(log_n)
            idx = [int(i) for i in rng.integers(0, n, 2)]
            xs = O.to_limbs([pow(w, i, O.P) for i in idx])
            assert np.array_equal(oracle.eval_poly_multi(c, xs), mid[idx])
        if log_n > 20:
            return
        # spot-check 2 outputs of the forward transform against the DFT definition
        rng = np.random.default_rng(log_n)
        ci = O.from_limbs(c)
        for i in rng.integers(0, n, 2):
            wi = pow(w, int(i), O.P)
            acc, pw = 0, 1
            for x in ci:
                acc += x * pw
                pw = pw * wi % O.P
            assert O.from_limbs(mid[i])[0] == acc % O.P
    finally:
        ctx.free(d)


def test_ntt_dev_batch(ctx, oracle):
    log_n, batch = 10, 5
    n = 1 << log_n
    c = O.random_elements(n * batch, 3)
    w = O.root_of_unity(log_n)
    d = ctx.alloc(c.nbytes)
    try:
        ctx.h2d(d, c)
        ctx.ntt_dev(d, log_n, batch, w)
        got = np.empty_like(c)
        ctx.d2h(got, d)
    finally:
        ctx.free(d)
    for b in range(batch):
        assert np.array_equal(got[b * n:(b + 1) * n], oracle.best_fft(c[b * n:(b + 1) * n], w, log_n, cpus=4))


def test_expand_root_of_unity(ctx, oracle):
    w = O.root_of_unity(13)
    assert np.array_equal(ctx.expand_root_of_unity(w), oracle.expand_root_of_unity(w))
