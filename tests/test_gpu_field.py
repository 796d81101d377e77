"""Field-vector entry points on the GPU against the oracle: multi_interp_4 and eval_quartic
(poly_utils.rs:442-511), the field linear combination (the L combination's shape, prove.rs:287-322)
and the LDE (prove.rs:100-101: inv_best_fft then best_fft of the zero-padded coefficients)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows", [1, 40, 1000, 70000])
def test_multi_interp_4(ctx, oracle, rows):
    xs = O.random_elements(4 * rows, 81 + rows)
    ys = O.random_elements(4 * rows, 82 + rows)
    if rows > 1:
        xs[4 * (rows // 2) + 3] = xs[4 * (rows // 2)]  # a repeated x: zero denominators map to zero
    assert np.array_equal(ctx.multi_interp_4(xs, ys), oracle.multi_interp_4(xs, ys))


def test_multi_interp_4_fri_rows(ctx, oracle):
    """The FRI shape: row i's points are x0 * zeta^j (fri.rs:135-150)."""
    log_n = 12
    n = 1 << log_n
    w = O.root_of_unity(log_n)
    q = n // 4
    xs = [pow(w, i + j * q, O.P) for i in range(q) for j in range(4)]
    ys = O.random_elements(n, 90)
    X = O.to_limbs(xs)
    assert np.array_equal(ctx.multi_interp_4(X, ys), oracle.multi_interp_4(X, ys))


@pytest.mark.parametrize("n", [1, 333, 50000])
def test_eval_quartic_multi(ctx, oracle, n):
    p = O.random_elements(4 * n, 91 + n)
    x = O.random_elements(n, 92 + n)
    assert np.array_equal(ctx.eval_quartic_multi(p, x), oracle.eval_quartic_multi(p, x))


@pytest.mark.parametrize("n_cols,n", [(1, 10), (9, 4096), (17, 1000)])
def test_lincomb(ctx, n_cols, n):
    cols = O.random_elements(n_cols * n, 93 + n_cols)
    k = O.random_elements(n_cols, 94 + n)
    c = O.from_limbs(cols)
    kv = O.from_limbs(k)
    want = [sum(kv[j] * c[j * n + i] for j in range(n_cols)) % O.P for i in range(n)]
    assert O.from_limbs(ctx.lincomb(cols, k)) == want


# (13, 3), (12, 4), (10, 6), (8, 8): a radix-2^8 first pass (the 16 x 16 split) skipping 2, 4, 6 and all 8
# copy stages of the zero-padded input
# (17, 3): the 2^20 plan (8, 4, 8); (12, 2), (9, 5), (19, 2): radix-2^7 sparse first passes (plans (7, 7) and (7, 7, 7), the 8 x 16
# kColSparse instance) that skip 1 and 5 copy stages
@pytest.mark.parametrize("log_steps,log_blowup", [(4, 3), (7, 3), (13, 3), (15, 3), (10, 1), (4, 8), (12, 6),
                                                  (12, 4), (10, 6), (8, 8), (12, 2), (9, 5), (19, 2), (17, 3)])
def test_lde(ctx, oracle, log_steps, log_blowup):
    log_prec = log_steps + log_blowup
    g2 = O.root_of_unity(log_prec)
    g1 = pow(g2, 1 << log_blowup, O.P)
    v = O.random_elements(1 << log_steps, 95 + log_prec)
    coeffs = oracle.inv_best_fft(v, g1, log_steps, cpus=8)
    want = oracle.best_fft(coeffs, g2, log_prec, cpus=8)
    assert np.array_equal(ctx.lde(v, g1, log_blowup, g2), want)


def test_lde_dev_batch(ctx, oracle):
    log_steps, log_blowup, batch = 11, 3, 3
    log_prec = log_steps + log_blowup
    g2 = O.root_of_unity(log_prec)
    g1 = pow(g2, 8, O.P)
    v = O.random_elements(batch << log_steps, 96)
    d_in = torch.from_numpy(v.view(np.int64).copy()).cuda()
    d_out = torch.empty((batch << log_prec, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.lde_dev(d_in.data_ptr(), d_out.data_ptr(), log_steps, log_blowup, batch, g1, g2)
    ctx.synchronize()
    got = d_out.cpu().numpy().view(np.uint64).reshape(-1, 4)
    n, m = 1 << log_steps, 1 << log_prec
    for b in range(batch):
        coeffs = oracle.inv_best_fft(v[b * n:(b + 1) * n], g1, log_steps, cpus=8)
        assert np.array_equal(got[b * m:(b + 1) * m], oracle.best_fft(coeffs, g2, log_prec, cpus=8))


def test_lde_rejects_mismatched_roots(ctx):
    from stark_amd import StarkError
    g2 = O.root_of_unity(10)
    with pytest.raises(StarkError):
        ctx.lde(O.random_elements(128, 97), pow(g2, 4, O.P), 3, g2)  # g1 must be g2^8
