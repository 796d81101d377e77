"""GPU parity at the sizes bench.py times.

* The dense 2^24 forward and inverse NTT through `stark_ntt_dev` -- the exact device-resident
  path the bench times (3 radix-256 Stockham passes, the last with the full twiddle table) --
  compared element for element with the oracle's best_fft / inv_best_fft (fft.rs:327-379) run
  live on the same input, and with the committed digests of tests/golden/large_digests.json.
* Config 2: the dense 2^20 forward and inverse, full vector, same two checks.
* prove_low_degree (fri.rs:46-224) at precision 2^23 on bench.py's FRI input, and mk_r1cs_proof
  (prove.rs:14-378) on the synthetic 2^20-step circuit: the JSON hashes to the digest of the
  oracle's JSON (tests/golden/make_large_golden.py generated both in the container).
* serial_fft / inv_serial_fft in place (`stark_fft_in_place`, fft.rs:150-193, 284-293).
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
BIG = json.load(open(os.path.join(HERE, "golden", "large_digests.json")))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
# Host threads for the live oracle: the GPU box's CPU share is 16 (power of two, as Worker::new
# splits parallel_fft, multicore.rs:43-45).
CPUS = 16


def _sha(a) -> str:
    if isinstance(a, str):
        a = a.encode()
    elif isinstance(a, np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.uint64).tobytes()
    return hashlib.sha256(a).hexdigest()


def _ntt_dev(ctx, c, log_n, w, inverse):
    d = ctx.alloc(c.nbytes)
    try:
        ctx.h2d(d, c)
        ctx.ntt_dev(d, log_n, 1, w, inverse=inverse)
        out = np.empty_like(c)
        ctx.d2h(out, d)
    finally:
        ctx.free(d)
    return out


@pytest.mark.parametrize("log_n", [20, 24])
def test_ntt_dense_full_vector_vs_oracle(ctx, oracle, log_n):
    rec = BIG[f"ntt_2^{log_n}"]
    c = O.random_elements(1 << log_n, 0x5EED0000 + log_n)
    assert _sha(c) == rec["input_sha256"]
    w = O.root_of_unity(log_n)
    fwd = _ntt_dev(ctx, c, log_n, w, inverse=False)
    assert _sha(fwd) == rec["forward_sha256"]
    assert np.array_equal(fwd, oracle.best_fft(c, w, log_n, cpus=CPUS))
    inv = _ntt_dev(ctx, c, log_n, w, inverse=True)
    assert _sha(inv) == rec["inverse_sha256"]
    assert np.array_equal(inv, oracle.inv_best_fft(c, w, log_n, cpus=CPUS))


@pytest.mark.parametrize("log_n", [25, 26, 27])
def test_ntt_dense_digest_beyond_bench(ctx, log_n):
    """Dense forward and inverse transforms past the bench size hash to the oracle's digests
    (tests/golden/make_large_golden.py --ntt 25,26,27): 2^25 = radices (8, 8, 9), 2^26 = the four
    digit-basis passes (6, 6, 7, 7) whose third pass takes the two-level column twiddle with the
    digit-basis last step, 2^27 = (9, 9, 9) past the full last-pass table (lo * hi column twiddle)."""
    rec = BIG.get(f"ntt_2^{log_n}")
    if rec is None:
        pytest.fail(f"large_digests.json has no ntt_2^{log_n} (run make_large_golden.py --ntt {log_n})")
    c = O.random_elements(1 << log_n, 0x5EED0000 + log_n)
    assert _sha(c) == rec["input_sha256"]
    w = O.root_of_unity(log_n)
    assert _sha(_ntt_dev(ctx, c, log_n, w, inverse=False)) == rec["forward_sha256"]
    assert _sha(_ntt_dev(ctx, c, log_n, w, inverse=True)) == rec["inverse_sha256"]


def test_ntt_2_24_host_entry_point(ctx):
    """best_fft on a host vector (H2D + the same passes + D2H) gives the same 2^24 output."""
    rec = BIG["ntt_2^24"]
    c = O.random_elements(1 << 24, 0x5EED0000 + 24)
    assert _sha(ctx.best_fft(c, O.root_of_unity(24), 24)) == rec["forward_sha256"]


def test_fri_2_23_vs_oracle_digest(ctx):
    rec = BIG["fri_2^23"]
    lf = 23
    nf = 1 << lf
    wf = O.root_of_unity(lf)
    coef = O.random_elements(nf // 4, 0x5EED0000 + lf)
    vals = ctx.best_fft(coef, wf, lf)
    assert _sha(vals) == rec["values_sha256"]
    js = ctx.prove_low_degree(vals, wf, nf // 4, 8).to_json()
    assert len(js) == rec["json_len"]
    assert _sha(js) == rec["json_sha256"]
    # the device-resident entry point bench.py times
    d = ctx.alloc(vals.nbytes)
    try:
        ctx.h2d(d, vals)
        js_dev = ctx.prove_low_degree_dev(d, nf, wf, nf // 4, 8).to_json()
    finally:
        ctx.free(d)
    assert _sha(js_dev) == rec["json_sha256"]


def test_synth_2_20_steps_proof_vs_oracle_digest(ctx):
    import synth_r1cs
    from stark_amd.r1cs import prove_with_witness
    rec = BIG["prove_synth_2^20_steps"]
    rs, ws = synth_r1cs.for_steps(20)
    assert _sha(rs) == rec["r1cs_sha256"] and _sha(ws) == rec["wtns_sha256"]
    js = prove_with_witness(ctx, rs, ws).to_json()
    assert len(js) == rec["json_len"]
    assert _sha(js) == rec["json_sha256"]


@pytest.mark.parametrize("log_n", [1, 2, 10, 18])
def test_fft_in_place_vs_oracle(ctx, oracle, log_n):
    n = 1 << log_n
    c = O.random_elements(n, 0x5EED0100 + log_n)
    w = O.root_of_unity(log_n)
    v = c.copy()
    ctx.serial_fft(v, w, log_n)
    assert np.array_equal(v, oracle.best_fft(c, w, log_n, cpus=8))
    ctx.inv_serial_fft(v, w, log_n)
    assert np.array_equal(v, c)
    u = c.copy()
    ctx.inv_serial_fft(u, w, log_n)
    assert np.array_equal(u, oracle.inv_best_fft(c, w, log_n, cpus=8))


def test_twiddle_cache_stays_under_cap(oracle):
    """The context's cached tables (the last pass's full twiddle table per size and direction, 2^log_n x
    32 B: 1 GiB at 2^25, 2 GiB at 2^26) stay under a 1 GiB cap while one context transforms 2^20 .. 2^27
    forward and inverse, and every transform still equals the oracle's digest (2^21 - 2^23: the round
    trip).  2^26's table does not fit the cap, so its last pass forms the twiddles from the two-level
    tables instead; 2^25's fits only after the others are evicted (least recently used first)."""
    import stark_amd as S
    cap = 1 << 30
    c = S.Context(0)
    try:
        c.set_cache_limit(cap)
        for log_n in range(20, 28):
            n = 1 << log_n
            x = O.random_elements(n, 0x5EED0000 + log_n)
            w = O.root_of_unity(log_n)
            fwd = _ntt_dev(c, x, log_n, w, inverse=False)
            m = c.memory()
            assert m["cache_limit"] == cap and m["cached"] <= cap, (log_n, m)
            rec = BIG.get(f"ntt_2^{log_n}")
            if rec:
                assert _sha(x) == rec["input_sha256"]
                assert _sha(fwd) == rec["forward_sha256"], log_n
                assert _sha(_ntt_dev(c, x, log_n, w, inverse=True)) == rec["inverse_sha256"], log_n
            else:
                assert np.array_equal(_ntt_dev(c, fwd, log_n, w, inverse=True), x), log_n
            assert c.memory()["cached"] <= cap, log_n
            del x, fwd
        assert c.memory()["resident"] >= c.memory()["cached"]
        c.set_cache_limit(0)  # frees every cached table at once
        assert c.memory()["cached"] == 0
        x = O.random_elements(1 << 24, 0x5EED0000 + 24)
        assert _sha(_ntt_dev(c, x, 24, O.root_of_unity(24), inverse=False)) == BIG["ntt_2^24"]["forward_sha256"]
        assert c.memory()["cached"] == 0
    finally:
        c.close()
