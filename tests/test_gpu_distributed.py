"""GPU: the four-step multi-GPU NTT with libstark_hip local steps.  On the
one-GPU test box both ranks share GPU 0 and exchange through gloo; the 8-GPU
bench uses the same code with RCCL ("nccl")."""
import datetime
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

import oracle as O
from ranks import run_ranks  # noqa: E402

pytestmark = pytest.mark.gpu


def _worker_cyclic(rank, world, port, log_n, inverse, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import faulthandler
    faulthandler.dump_traceback_later(90, exit=True)   # a stuck rank prints its stack and exits
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=80))
    import stark_amd as S
    from stark_amd.distributed import GpuOps, cyclic_ntt
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(0)
    n = 1 << log_n
    full = O.random_elements(n, 0x5EED0000 + log_n)
    x = torch.from_numpy(full[rank::world].copy().view(np.int64)).cuda()
    y = cyclic_ntt(x, log_n, O.root_of_unity(log_n), GpuOps(ctx), inverse=inverse)
    torch.cuda.synchronize()
    out_q.put((rank, y.cpu().numpy().view(np.uint64).copy()))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,log_n,inverse", [(2, 12, False), (2, 17, True), (4, 16, False), (8, 15, True)])
def test_cyclic_ntt_gpu(world, log_n, inverse):
    parts = dict(run_ranks(_worker_cyclic, world, (log_n, inverse), timeout=110))
    n = 1 << log_n
    M, c = n // world, n // world // world
    got = np.zeros((n, 4), dtype=np.uint64)
    for r in range(world):
        out = parts[r].reshape(world, c, 4)
        for k1 in range(world):
            got[r * c + k1 * M: r * c + k1 * M + c] = out[k1]
    o = O.Oracle()
    full = O.random_elements(n, 0x5EED0000 + log_n)
    w = O.root_of_unity(log_n)
    want = o.inv_best_fft(full, w, log_n, cpus=8) if inverse else o.best_fft(full, w, log_n, cpus=8)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("log_g,inverse", [(1, False), (2, True), (3, False), (3, True), (4, False)])
def test_ntt_strided(ctx, oracle, log_g, inverse):
    G, stride = 1 << log_g, 1000
    a = O.random_elements(G * stride, 17 + log_g)
    d = ctx.alloc(a.nbytes)
    try:
        ctx.h2d(d, a)
        w = O.root_of_unity(log_g)
        ctx.ntt_strided_dev(d, log_g, stride, w, inverse=inverse)
        got = np.empty_like(a)
        ctx.d2h(got, d)
    finally:
        ctx.free(d)
    want = a.reshape(G, stride, 4).copy()
    f = oracle.inv_best_fft if inverse else oracle.best_fft
    for i in range(0, stride, 97):
        want[:, i] = f(want[:, i].copy(), w, log_g, cpus=1)
        assert np.array_equal(got.reshape(G, stride, 4)[:, i], want[:, i])


@pytest.mark.parametrize("log_g,inverse", [(1, False), (3, False), (3, True), (4, True)])
def test_ntt_strided_tw(ctx, oracle, log_g, inverse):
    """The receiver-side twiddle fused into the strided DFT: d[i + stride j] *= t^(j (base + i)) first."""
    G, stride, log_order, base = 1 << log_g, 1000, 20, 123456
    a = O.random_elements(G * stride, 31 + log_g)
    t = O.root_of_unity(log_order)
    d = ctx.alloc(a.nbytes)
    try:
        ctx.h2d(d, a)
        w = O.root_of_unity(log_g)
        ctx.ntt_strided_tw_dev(d, log_g, stride, w, t, log_order, base, inverse=inverse)
        got = np.empty_like(a)
        ctx.d2h(got, d)
    finally:
        ctx.free(d)
    want = a.reshape(G, stride, 4).copy()
    f = oracle.inv_best_fft if inverse else oracle.best_fft
    mask = (1 << log_order) - 1
    for i in range(0, stride, 97):
        col = [v * pow(t, (j * (base + i)) & mask, O.P) % O.P for j, v in enumerate(O.from_limbs(want[:, i]))]
        want[:, i] = f(O.to_limbs(col), w, log_g, cpus=1)
        assert np.array_equal(got.reshape(G, stride, 4)[:, i], want[:, i])


def _worker_merkle(rank, world, port, log_m, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import faulthandler
    faulthandler.dump_traceback_later(90, exit=True)   # a stuck rank prints its stack and exits
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=80))
    import stark_amd as S
    from stark_amd.distributed import DistributedMerkle, GpuOps
    torch.cuda.set_device(0)
    ctx = S.Context(0)
    m = 1 << log_m
    full = O.random_elements(world * m, 99)
    shard = torch.from_numpy(full[rank * m:(rank + 1) * m].copy().view(np.int64)).cuda()
    dm = DistributedMerkle(GpuOps(ctx))
    root = dm.commit(shard, m, 32)
    n = world * m
    idx = [0, n - 1, 3, n // 2 + 7, 3]
    proofs = dm.gen_proofs(idx)
    out_q.put((rank, root, [(p.leaf, p.nodes) for p in proofs]))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,log_m", [(2, 12), (4, 10)])
def test_distributed_merkle_gpu(world, log_m):
    res = run_ranks(_worker_merkle, world, (log_m,), timeout=110)
    n = world << log_m
    blob = O.random_elements(n, 99).tobytes()
    idx = [0, n - 1, 3, n // 2 + 7, 3]
    want_root, want_paths = O.Oracle().merkle(blob, n, 32, idx)
    for _, root, proofs in res:
        assert root == want_root
        for k, (leaf, nodes) in enumerate(proofs):
            assert leaf == blob[idx[k] * 32:(idx[k] + 1) * 32]
            assert list(nodes) == want_paths[k]


def _worker(rank, world, port, log_n, inverse, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import faulthandler
    faulthandler.dump_traceback_later(90, exit=True)   # a stuck rank prints its stack and exits
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=80))
    import stark_amd as S
    from stark_amd.distributed import GpuOps, four_step_ntt
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(0)
    n = 1 << log_n
    M = n // world
    full = O.random_elements(n, 0x5EED0000 + log_n)
    x = torch.from_numpy(full[rank * M:(rank + 1) * M].copy().view(np.int64)).cuda()
    y = four_step_ntt(x, log_n, O.root_of_unity(log_n), GpuOps(ctx), inverse=inverse)
    torch.cuda.synchronize()
    out_q.put((rank, y.cpu().numpy().view(np.uint64).copy()))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,log_n,inverse", [(2, 12, False), (2, 17, True), (4, 16, False)])
def test_four_step_ntt_gpu(world, log_n, inverse):
    parts = dict(run_ranks(_worker, world, (log_n, inverse), timeout=110))
    got = np.concatenate([parts[r] for r in range(world)])
    o = O.Oracle()
    n = 1 << log_n
    full = O.random_elements(n, 0x5EED0000 + log_n)
    w = O.root_of_unity(log_n)
    want = o.inv_best_fft(full, w, log_n, cpus=8) if inverse else o.best_fft(full, w, log_n, cpus=8)
    assert np.array_equal(got, want)


def test_transpose_and_twiddle(ctx):
    rows, cols = 37, 70
    a = O.random_elements(rows * cols, 3)
    d = ctx.alloc(a.nbytes)
    e = ctx.alloc(a.nbytes)
    try:
        ctx.h2d(d, a)
        ctx.transpose_dev(d, e, rows, cols)
        t = np.empty_like(a)
        ctx.d2h(t, e)
        assert np.array_equal(t.reshape(cols, rows, 4), a.reshape(rows, cols, 4).transpose(1, 0, 2))
        w = O.root_of_unity(12)
        ctx.twiddle2d_dev(d, rows, cols, 5, 9, w, 12)
        g = np.empty_like(a)
        ctx.d2h(g, d)
        vals = O.from_limbs(a)
        want = [v * pow(w, ((5 + i // cols) * (9 + i % cols)) % 4096, O.P) % O.P for i, v in enumerate(vals)]
        assert O.from_limbs(g) == want
    finally:
        ctx.free(d)
        ctx.free(e)


def _worker_rccl_world1(rank, world, port, out_q):
    """Backend "nccl" (RCCL) at world 1 on the box's one GPU: the code the 8-GPU bench runs --
    cyclic_ntt_pipelined's async all_to_all_single on RCCL's stream, the plain cyclic_ntt exchange
    and DistributedMerkle's all_gather_object -- with trivial exchanges."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import faulthandler
    faulthandler.dump_traceback_later(100, exit=True)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"),
                            timeout=datetime.timedelta(seconds=90))
    import stark_amd as S
    from stark_amd.distributed import DistributedMerkle, GpuOps, cyclic_ntt, cyclic_ntt_pipelined
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(0)
    ops = GpuOps(ctx)
    log_n = 14
    n = 1 << log_n
    w = O.root_of_unity(log_n)
    ins = [O.random_elements(n, 0x5EED0400 + i) for i in range(2)]
    pairs = [(torch.from_numpy(h.view(np.int64).copy()).cuda(), torch.empty((n, 4), dtype=torch.int64).cuda())
             for h in ins]
    cyclic_ntt_pipelined(pairs, 2, log_n, w, ops)
    torch.cuda.synchronize()
    res = {"pipelined": [b.cpu().numpy().view(np.uint64).copy() for _, b in pairs]}
    x = torch.from_numpy(ins[0].view(np.int64).copy()).cuda()
    res["cyclic"] = cyclic_ntt(x, log_n, w, ops).cpu().numpy().view(np.uint64).copy()
    leaves = torch.from_numpy(ins[1].view(np.int64).copy()).cuda()
    res["merkle_root"] = DistributedMerkle(ops).commit(leaves, n, 32)
    torch.cuda.synchronize()
    # prove_distributed over RCCL: the status all-reduce, the device-tensor all-gathers of the tree
    # digests and of the openings, the device roots (k, special_x) -- at world 1
    import hashlib
    from stark_amd.dprove import GpuProverOps, prove_distributed
    fix = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "r1cs")
    r1 = open(os.path.join(fix, "pedersen_test.r1cs"), "rb").read()
    wt = open(os.path.join(fix, "pedersen_test.wtns"), "rb").read()
    st = {}
    js = prove_distributed(GpuProverOps(ctx), r1, wt, stats=st)
    res["pedersen_sha"] = hashlib.sha256(js.encode()).hexdigest()
    res["host_syncs"] = st["host_syncs"]
    out_q.put(res)
    ctx.close()
    dist.destroy_process_group()


def test_rccl_world1_pipelined_and_merkle():
    res = run_ranks(_worker_rccl_world1, 1, timeout=110)[0]
    o = O.Oracle()
    log_n = 14
    w = O.root_of_unity(log_n)
    ins = [O.random_elements(1 << log_n, 0x5EED0400 + i) for i in range(2)]
    for h, got in zip(ins, res["pipelined"]):
        assert np.array_equal(got, o.best_fft(h, w, log_n, cpus=8))
    assert np.array_equal(res["cyclic"], o.best_fft(ins[0], w, log_n, cpus=8))
    root, _ = o.merkle(ins[1].tobytes(), 1 << log_n, 32)
    assert res["merkle_root"] == root
    import json
    golden = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "r1cs_proofs.json")))
    assert res["pedersen_sha"] == golden["pedersen_test"]["json_sha256"]
    assert res["host_syncs"] <= 7


@pytest.mark.parametrize("g", [1, 2, 8, 64])
def test_merkle_top_and_root_dev(ctx, oracle, g):
    """stark_merkle_root_dev + stark_merkle_top_dev (the distributed commit's device-side top tree,
    merkle_proof_in_place.rs:176-180) against the single tree's root and the host Blake2s."""
    import stark_amd as S
    m = 16
    leaves = O.random_elements(g * m, 0x5EED0500 + g).tobytes()
    want_root, _ = oracle.merkle(leaves, g * m, 32)
    roots = torch.empty(g * 32, dtype=torch.uint8, device="cuda")
    trees = []
    for c in range(g):
        t = S.MerkleProofInPlace(ctx)
        blob = torch.from_numpy(np.frombuffer(leaves[c * m * 32:(c + 1) * m * 32], dtype=np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        t.update_dev(blob.data_ptr(), m, 32, stream=ctx.stream)
        ctx.check(ctx.lib.stark_merkle_root_dev(t.h, roots[32 * c:].data_ptr(), ctx.stream), "root_dev")
        trees.append((t, blob))
    levels = torch.zeros(max(g - 1, 1) * 32, dtype=torch.uint8, device="cuda")
    ctx.check(ctx.lib.stark_merkle_top_dev(ctx.h, roots.data_ptr(), g, levels.data_ptr(), ctx.stream), "top_dev")
    ctx.synchronize()
    got = (levels if g > 1 else roots).cpu().numpy().tobytes()[-32:]
    assert got == want_root
    # every level equals pairwise host hashing of the level below
    lv = [roots.cpu().numpy().tobytes()[32 * i:32 * (i + 1)] for i in range(g)]
    flat, at = levels.cpu().numpy().tobytes(), 0
    while len(lv) > 1:
        lv = [O.py_blake(lv[2 * i] + lv[2 * i + 1]) for i in range(len(lv) // 2)]
        assert flat[at:at + 32 * len(lv)] == b"".join(lv)
        at += 32 * len(lv)


@pytest.mark.parametrize("world,rank", [(1, 0), (4, 3)])
def test_fri_fold_dev_root_equals_host_root(ctx, world, rank):
    """stark_fri_fold_dev_root (special_x from a device-resident root, fri.rs:135) = stark_fri_fold_dev
    (the same root from the host), including a root >= p (reduced mod p)."""
    from stark_amd import _limbs, _p64
    log_n = 12
    n = 1 << log_n
    w = O.root_of_unity(log_n)
    vals = torch.from_numpy(O.random_elements(n // world, 0x5EED0600 + world).view(np.int64).copy()).cuda()
    for root in (bytes(range(32)), b"\xff" * 32):
        d_root = torch.from_numpy(np.frombuffer(root, dtype=np.uint8).copy()).cuda()
        a = torch.empty(n // 4 // world * 32, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        torch.cuda.synchronize()
        rl = _limbs(w)
        ctx.check(ctx.lib.stark_fri_fold_dev(ctx.h, vals.data_ptr(), a.data_ptr(), n, _p64(rl), root, world, rank,
                                             ctx.stream), "fold")
        ctx.check(ctx.lib.stark_fri_fold_dev_root(ctx.h, vals.data_ptr(), b.data_ptr(), n, _p64(rl), d_root.data_ptr(),
                                                  world, rank, ctx.stream), "fold_root")
        ctx.synchronize()
        assert torch.equal(a, b)


@pytest.mark.parametrize("log_n,log_g,rank,inverse", [(15, 3, 5, False), (15, 3, 7, True), (12, 1, 1, False),
                                                     (20, 2, 2, True), (8, 4, 9, False)])
def test_cyclic_ntt_local_fused_twiddle(ctx, oracle, log_n, log_g, rank, inverse):
    """stark_cyclic_ntt_local_dev = the rank's M-point best_fft (root w^G) followed by the twiddle
    w^(rank k) (w^-1 and inv_best_fft for the inverse): the one-exchange distributed NTT's first step
    with the twiddle in the last pass's store."""
    G = 1 << log_g
    M = 1 << (log_n - log_g)
    w = O.root_of_unity(log_n)
    x = O.random_elements(M, 0x5EED0700 + log_n + rank)
    d = torch.from_numpy(x.view(np.int64).copy()).cuda()
    torch.cuda.synchronize()
    ctx.cyclic_ntt_local_dev(d.data_ptr(), log_n, log_g, rank, w, inverse=inverse, stream=ctx.stream)
    ctx.synchronize()
    got = O.from_limbs(d.cpu().numpy().view(np.uint64).reshape(-1, 4))
    wl = pow(w, G, O.P)
    base = oracle.inv_best_fft(x, wl, log_n - log_g, cpus=8) if inverse else oracle.best_fft(x, wl, log_n - log_g, cpus=8)
    wt = pow(w, O.P - 2, O.P) if inverse else w
    step = pow(wt, rank, O.P)
    want, t = [], 1
    for v in O.from_limbs(base):
        want.append(v * t % O.P)
        t = t * step % O.P
    assert got == want


def _local_step_want(oracle, x, log_n, log_g, rank):
    w = O.root_of_unity(log_n)
    base = oracle.best_fft(x, pow(w, 1 << log_g, O.P), log_n - log_g, cpus=8)
    step, want, t = pow(w, rank, O.P), [], 1
    for v in O.from_limbs(base):
        want.append(v * t % O.P)
        t = t * step % O.P
    return want


@pytest.mark.parametrize("cap_units", [0, 1, 3])
def test_cyclic_ntt_local_post_table_under_cache_cap(oracle, cap_units):
    """the sender-side post table of G = 8 under a cache cap that cannot hold it
    (0: built for the call and freed), or holds it or the last pass's full table but not both (1.5 and
    3.5 x M x 32 B with other tables competing).  The table a transform is using is never evicted by
    the full table that transform's last pass reserves; every result equals the oracle's."""
    import stark_amd as S
    log_n, log_g = 18, 3
    M = 1 << (log_n - log_g)
    c = S.Context(0)
    try:
        c.set_cache_limit(M * 32 * cap_units + M * 16)
        for rank in (1, 6, 1):  # a second rank's table evicts (or replaces) the first's
            x = O.random_elements(M, 0x5EED0900 + rank)
            d = torch.from_numpy(x.view(np.int64).copy()).cuda()
            torch.cuda.synchronize()
            c.cyclic_ntt_local_dev(d.data_ptr(), log_n, log_g, rank, O.root_of_unity(log_n), stream=c.stream)
            c.synchronize()
            got = O.from_limbs(d.cpu().numpy().view(np.uint64).reshape(-1, 4))
            assert got == _local_step_want(oracle, x, log_n, log_g, rank), (cap_units, rank)
            m = c.memory()
            assert m["cached"] <= m["cache_limit"], m
    finally:
        c.close()
