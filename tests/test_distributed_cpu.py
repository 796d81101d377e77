"""CPU (gloo): the multi-GPU four-step NTT orchestration
(stark_amd/distributed.py) at world sizes 2 and 4, with the local steps done
by the oracle, checked bit-exactly against the oracle's single-process NTT."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

import oracle as O
from ranks import run_ranks  # noqa: E402


class OracleOps:
    """Local steps on the host with the oracle (test infrastructure)."""

    def __init__(self):
        self.o = O.Oracle()

    @staticmethod
    def _u64(t):
        return t.numpy().view(np.uint64).reshape(-1, 4)

    def ntt(self, t, log_len, batch, root, inverse):
        a = self._u64(t)
        n = 1 << log_len
        for b in range(batch):
            seg = a[b * n:(b + 1) * n]
            f = self.o.inv_best_fft if inverse else self.o.best_fft
            seg[:] = f(seg.copy(), root, log_len, cpus=1)

    def ntt_strided(self, t, log_g, stride, root, inverse):
        a = self._u64(t).reshape(1 << log_g, stride, 4)
        f = self.o.inv_best_fft if inverse else self.o.best_fft
        for i in range(stride):
            a[:, i] = f(a[:, i].copy(), root, log_g, cpus=1)

    def ntt_strided_tw(self, t, log_g, stride, root, inverse, tw_root, log_order, tw_base):
        a = self._u64(t).reshape(1 << log_g, stride, 4)
        mask = (1 << log_order) - 1
        for j in range(1, 1 << log_g):
            vals = O.from_limbs(a[j])
            a[j] = O.to_limbs([v * pow(tw_root, (j * (tw_base + i)) & mask, O.P) % O.P for i, v in enumerate(vals)])
        self.ntt_strided(t, log_g, stride, root, inverse)

    def merkle_commit(self, shard, m, leaf_len):
        self._leaves = bytes(shard.numpy().view(np.uint8)) if hasattr(shard, "numpy") else bytes(shard)
        self._m, self._ll = m, leaf_len
        root, _ = self.o.merkle(self._leaves, m, leaf_len)
        return root

    def merkle_open(self, local_indices):
        """(leaves k x leaf_len, nodes k x depth x 32) of the local subtree."""
        _, paths = self.o.merkle(self._leaves, self._m, self._ll, list(local_indices))
        leaves = b"".join(self._leaves[i * self._ll:(i + 1) * self._ll] for i in local_indices)
        nodes = b"".join(b"".join(p) for p in paths)
        return np.frombuffer(leaves, dtype=np.uint8), np.frombuffer(nodes, dtype=np.uint8)

    def transpose(self, src, dst, rows, cols):
        s = self._u64(src).reshape(rows, cols, 4)
        self._u64(dst)[:] = s.transpose(1, 0, 2).reshape(-1, 4)

    def twiddle2d(self, t, rows, cols, row_base, col_base, root, log_order):
        a = self._u64(t)
        vals = O.from_limbs(a)
        mask = (1 << log_order) - 1
        for i in range(rows):
            for j in range(cols):
                e = ((row_base + i) * (col_base + j)) & mask
                vals[i * cols + j] = vals[i * cols + j] * pow(root, e, O.P) % O.P
        a[:] = O.to_limbs(vals)


def _worker(rank, world, port, log_n, inverse, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stark_amd.distributed import four_step_ntt
    n = 1 << log_n
    M = n // world
    full = O.random_elements(n, 0x5EED0000 + log_n)
    x = torch.from_numpy(full[rank * M:(rank + 1) * M].copy().view(np.int64))
    w = O.root_of_unity(log_n)
    y = four_step_ntt(x, log_n, w, OracleOps(), inverse=inverse)
    out_q.put((rank, y.numpy().view(np.uint64).copy()))
    dist.barrier()
    dist.destroy_process_group()


def _worker_pipelined(rank, world, port, log_n, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stark_amd.distributed import cyclic_ntt, cyclic_ntt_pipelined
    n = 1 << log_n
    w = O.root_of_unity(log_n)
    ops = OracleOps()
    # Three transforms on two buffer pairs: transform 2 reuses pair 0 after transform 0's exchange.
    shards = [torch.from_numpy(O.random_elements(n, 500 + 10 * s)[rank::world].copy().view(np.int64))
              for s in range(2)]
    want0 = cyclic_ntt(shards[0], log_n, w, ops)
    want1 = cyclic_ntt(shards[1], log_n, w, ops)
    want2 = cyclic_ntt(_local_after(shards[0], log_n, w, ops), log_n, w, ops)
    pairs = [(shards[0].clone(), torch.empty_like(shards[0])), (shards[1].clone(), torch.empty_like(shards[1]))]
    cyclic_ntt_pipelined(pairs, 2, log_n, w, ops)
    ok = torch.equal(pairs[0][1], want0) and torch.equal(pairs[1][1], want1)
    cyclic_ntt_pipelined(pairs, 3, log_n, w, ops)   # 3rd transform: pair 0 again, its shard already local-transformed twice
    ok = ok and torch.equal(pairs[0][1], want2)
    out_q.put((rank, ok))
    dist.destroy_process_group()


def _local_after(shard, log_n, w, ops):
    """The shard a third transform on pair 0 sees: cyclic_ntt_local applied twice in place."""
    from stark_amd.distributed import cyclic_ntt_local
    y = shard.clone()
    cyclic_ntt_local(y, log_n, w, ops, in_place=True)
    cyclic_ntt_local(y, log_n, w, ops, in_place=True)
    return y


@pytest.mark.parametrize("world,log_n", [(2, 8), (4, 10)])
def test_cyclic_ntt_pipelined_gloo(world, log_n):
    """bench.py's N > 1 schedule (exchange i overlapping local NTT i+1, two buffer pairs) produces
    exactly cyclic_ntt's result for every transform."""
    res = dict(run_ranks(_worker_pipelined, world, (log_n,), timeout=300))
    assert all(res.values())


def _worker_cyclic(rank, world, port, log_n, inverse, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stark_amd.distributed import cyclic_ntt
    n = 1 << log_n
    full = O.random_elements(n, 0x5EED0000 + log_n)
    x = torch.from_numpy(full[rank::world].copy().view(np.int64))   # cyclic: x[rank + G j]
    y = cyclic_ntt(x, log_n, O.root_of_unity(log_n), OracleOps(), inverse=inverse)
    out_q.put((rank, y.numpy().view(np.uint64).copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,log_n,inverse", [(2, 6, False), (2, 9, True), (4, 8, False), (4, 10, True),
                                                 (8, 12, False), (8, 9, True)])
def test_cyclic_ntt_gloo(world, log_n, inverse):
    """One-exchange layout: rank r gets X[r c + i + M k1] at out[k1 c + i]."""
    parts = dict(run_ranks(_worker_cyclic, world, (log_n, inverse), timeout=300))
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
    want = o.inv_best_fft(full, w, log_n, cpus=4) if inverse else o.best_fft(full, w, log_n, cpus=4)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("world,log_n,inverse", [(2, 6, False), (2, 9, True), (4, 8, False), (4, 10, True),
                                                 (8, 12, False)])
def test_four_step_ntt_gloo(world, log_n, inverse):
    parts = dict(run_ranks(_worker, world, (log_n, inverse), timeout=300))
    got = np.concatenate([parts[r] for r in range(world)])
    o = O.Oracle()
    n = 1 << log_n
    full = O.random_elements(n, 0x5EED0000 + log_n)
    w = O.root_of_unity(log_n)
    want = o.inv_best_fft(full, w, log_n, cpus=4) if inverse else o.best_fft(full, w, log_n, cpus=4)
    assert np.array_equal(got, want)


def _worker_merkle(rank, world, port, log_m, leaf_len, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stark_amd.distributed import DistributedMerkle
    m = 1 << log_m
    rng = np.random.default_rng(7)
    blob = rng.integers(0, 256, size=world * m * leaf_len, dtype=np.uint8)
    shard = torch.from_numpy(blob[rank * m * leaf_len:(rank + 1) * m * leaf_len].copy())
    dm = DistributedMerkle(OracleOps())
    root = dm.commit(shard, m, leaf_len)
    n = world * m
    idx = [0, n - 1, 5 % n, n // 2, 5 % n, (n * 3) // 4 + 1]
    proofs = dm.gen_proofs(idx)
    out_q.put((rank, root, [(p.leaf, p.nodes) for p in proofs]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,log_m,leaf_len", [(2, 5, 32), (4, 6, 40), (8, 3, 256)])
def test_distributed_merkle_gloo(world, log_m, leaf_len):
    """Per-rank subtrees + all-gathered roots = the single tree (root and paths)."""
    res = run_ranks(_worker_merkle, world, (log_m, leaf_len), timeout=300)
    m = 1 << log_m
    n = world * m
    rng = np.random.default_rng(7)
    blob = bytes(rng.integers(0, 256, size=n * leaf_len, dtype=np.uint8))
    idx = [0, n - 1, 5 % n, n // 2, 5 % n, (n * 3) // 4 + 1]
    want_root, want_paths = O.Oracle().merkle(blob, n, leaf_len, idx)
    for _, root, proofs in res:
        assert root == want_root
        for k, (leaf, nodes) in enumerate(proofs):
            assert leaf == blob[idx[k] * leaf_len:(idx[k] + 1) * leaf_len]
            assert list(nodes) == want_paths[k]
