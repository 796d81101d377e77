"""Multi-GPU four-step NTT: one transform of n = G * M elements sharded over
G ranks (one process per GPU), block distribution in and out:

    rank r holds x[r M : (r+1) M]  ->  rank r holds X[r M : (r+1) M]

with X[k] = sum_j x[j] w^(j k) exactly as best_fft (packages/fri/src/fft.rs:327-357).
The reference is single-process; this module is the
MI355X-native way to scale the hot path across the xGMI-connected GPUs of one
node.  Derivation (j = g M + m, k = h M + q1 + G q2, t = q2 + (M/G) h):

    S[m][q1] = sum_g x[g M + m] wG^(g q1)                (G-point DFTs, wG = w^M)
    T[q1][m] = S[m][q1] w^(m q1)                          (four-step twiddle)
    X[h M + q1 + G q2] = sum_m T[q1][m] wM^(m t)          (M-point DFTs, wM = w^G)

Three all-to-alls (RCCL over xGMI with backend "nccl"; each moves (G-1)/G of
the shard, 1/G of it per peer link) and three local transposes; all local
arithmetic runs in libstark_hip.  `ops` abstracts the local steps so the same
orchestration is tested on CPU with gloo (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import P


def _exchange(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """all_to_all_single of equal chunks; gloo needs host tensors."""
    if dist.get_backend(group) == "gloo" and inp.is_cuda:
        o = torch.empty_like(out, device="cpu")
        dist.all_to_all_single(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, group=group)


def four_step_ntt(x: torch.Tensor, log_n: int, root: int, ops, inverse: bool = False, group=None) -> torch.Tensor:
    """Distributed forward (or inverse, inv_best_fft semantics) NTT.

    x: this rank's block, shape (M, 4) int64 (canonical u64 limbs), M = n / G.
    Returns a new (M, 4) tensor with this rank's block of the result.
    """
    G = dist.get_world_size(group)
    r = dist.get_rank(group)
    n = 1 << log_n
    M = n // G
    if M * G != n or M % G != 0 or x.shape[0] != M:
        raise ValueError(f"four_step_ntt: need M = n/G divisible by G (n=2^{log_n}, G={G}, block={x.shape[0]})")
    log_m = M.bit_length() - 1
    log_g = G.bit_length() - 1
    w = root % P
    if G == 1:
        y = x.clone()
        ops.ntt(y, log_n, 1, w, inverse)
        return y
    w_tw = pow(w, P - 2, P) if inverse else w   # the twiddle uses w^-1 for the inverse
    c = M // G
    # 1) all-to-all: chunk q of every block goes to rank q -> R1[g][ml] = x_g[r c + ml]
    r1 = torch.empty_like(x)
    _exchange(r1, x, group)
    # 2) G-point DFTs over g for each ml
    t1 = torch.empty_like(x)
    ops.transpose(r1, t1, G, c)                      # (G, c) -> (c, G)
    ops.ntt(t1, log_g, c, pow(w, M, P), inverse)     # batch c of G-point transforms, root w^M
    # 3) twiddle w^(m q1), m = r c + ml
    ops.twiddle2d(t1, c, G, r * c, 0, w_tw, log_n)
    # 4) all-to-all: row q1 to rank q1 -> R2 = T[r][m], m in [0, M) in order
    u = torch.empty_like(x)
    ops.transpose(t1, u, c, G)                       # (c, G) -> (G, c)
    r2 = torch.empty_like(x)
    _exchange(r2, u, group)
    # 5) M-point DFT over m, root w^G
    ops.ntt(r2, log_m, 1, pow(w, G, P), inverse)
    # 6) all-to-all: t-chunk h to rank h -> R3[q1][q2] = X[r M + q1 + G q2]
    r3 = torch.empty_like(x)
    _exchange(r3, r2, group)
    # 7) natural order: out[q2 G + q1] = R3[q1][q2]
    out = torch.empty_like(x)
    ops.transpose(r3, out, G, c)
    return out


def cyclic_ntt(x: torch.Tensor, log_n: int, root: int, ops, inverse: bool = False, group=None,
               out: torch.Tensor = None, in_place: bool = False) -> torch.Tensor:
    """Distributed NTT with ONE all-to-all: cyclic distribution in, chunked out.

    Input: rank r holds u_r[j2] = x[r + G j2], j2 < M (shape (M, 4), M = n / G).
    Output: rank r holds out[k1][i] = X[r c + i + M k1], k1 < G, i < c = M / G
    (G runs of c consecutive outputs, M apart).  With j = j1 + G j2 and
    k = k2 + M k1:

        X[k2 + M k1] = sum_j1 wG^(j1 k1) * w^(j1 k2) * DFT_M(u_j1)[k2]

    so each rank runs its M-point NTT (root w^G) and the twiddle w^(r k2)
    locally, one all_to_all_single sends chunk k2 in [s c, (s+1) c) to rank s,
    and the G-point DFTs over j1 (root w^M) run locally across the received
    chunks (stark_ntt_strided_dev: no transposes).  The inverse uses the same
    steps with inverse transforms and w^-1 in the twiddle (n^-1 = M^-1 G^-1).
    The block-in/block-out `four_step_ntt` needs three exchanges for the same
    transform; this layout is the one-exchange form.  in_place=True lets the
    local transform overwrite x (no copy); `out` receives the result if given.
    """
    G = dist.get_world_size(group)
    y = cyclic_ntt_local(x, log_n, root, ops, inverse, group, in_place)
    if G == 1:
        return y
    z = torch.empty_like(y) if out is None else out
    _exchange(z, y, group)                                          # z[j1][i] = Y_j1[r c + i]
    cyclic_ntt_finish(z, log_n, root, ops, inverse, group)
    return z


def _fused_twiddle(ops, G: int) -> bool:
    """Where the twiddle w^(r k2) goes: into the sender's last local pass (one product per element,
    stark_cyclic_ntt_local_dev) from G = 8 on; below that the receiver's strided DFT applies it as a
    chain of (G-1)/G products per element more cheaply.  One GPU, 2^24 per rank
    (profiles/r04_distributed_local_step.txt): G = 2 1.685 vs 1.764 ms, G = 4 1.753 vs 1.779, G = 8
    1.816 vs 1.792 (receiver vs sender)."""
    return hasattr(ops, "cyclic_local") and G >= 8


def cyclic_ntt_local(x: torch.Tensor, log_n: int, root: int, ops, inverse: bool = False, group=None,
                     in_place: bool = False) -> torch.Tensor:
    """cyclic_ntt's first step: this rank's M-point NTT (root w^G), plus the twiddle w^(+-r k2) when
    the ops cannot fuse it into the last step.  With G == 1 it is the whole transform.  The result is
    what the exchange sends."""
    G = dist.get_world_size(group)
    n = 1 << log_n
    M = n // G
    if M * G != n or M % G != 0 or x.shape[0] != M:
        raise ValueError(f"cyclic_ntt: need M = n/G divisible by G (n=2^{log_n}, G={G}, shard={x.shape[0]})")
    w = root % P
    y = x if in_place else x.clone()
    if G == 1:
        ops.ntt(y, log_n, 1, w, inverse)
        return y
    log_m = M.bit_length() - 1
    if _fused_twiddle(ops, G):
        # M-point NTT (root w^G) with the twiddle w^(+-r k2) in its last pass's store
        ops.cyclic_local(y, log_n, G.bit_length() - 1, dist.get_rank(group), w, inverse)
        return y
    ops.ntt(y, log_m, 1, pow(w, G, P), inverse)                     # M-point, root w^G
    if not hasattr(ops, "ntt_strided_tw"):
        ops.twiddle2d(y, 1, M, dist.get_rank(group), 0, pow(w, P - 2, P) if inverse else w, log_n)
    return y


def cyclic_ntt_finish(z: torch.Tensor, log_n: int, root: int, ops, inverse: bool = False, group=None) -> None:
    """cyclic_ntt's last step on the received chunks z[j1][i] = Y_j1[r c + i]: the twiddle
    w^(+-j1 (r c + i)) (applied here, fused into the strided kernel, when the ops have
    ntt_strided_tw) and the G-point DFTs over j1 (root w^M), in place."""
    G = dist.get_world_size(group)
    r = dist.get_rank(group)
    n = 1 << log_n
    M = n // G
    c = M // G
    w = root % P
    log_g = G.bit_length() - 1
    if hasattr(ops, "ntt_strided_tw") and not _fused_twiddle(ops, G):
        ops.ntt_strided_tw(z, log_g, c, pow(w, M, P), inverse, pow(w, P - 2, P) if inverse else w, log_n, r * c)
    else:  # the twiddle was applied before the exchange (cyclic_ntt_local)
        ops.ntt_strided(z, log_g, c, pow(w, M, P), inverse)


def cyclic_ntt_pipelined(pairs, k: int, log_n: int, root: int, ops, inverse: bool = False, group=None) -> None:
    """k independent cyclic_ntt transforms with the exchange of transform i overlapping the local NTT
    of transform i+1: transform i runs on pairs[i % len(pairs)] = (shard, out), the shard transformed
    in place and the result left in out.  With backend "nccl" the all-to-all runs on RCCL's stream
    while this stream computes; every transform is complete when the call returns (on the stream)."""
    pending = None
    for i in range(k):
        a, b = pairs[i % len(pairs)]
        cyclic_ntt_local(a, log_n, root, ops, inverse, group, in_place=True)
        work = dist.all_to_all_single(b, a, group=group, async_op=True)
        if pending is not None:
            pending[0].wait()
            cyclic_ntt_finish(pending[1], log_n, root, ops, inverse, group)
        pending = (work, b)
    if pending is not None:
        pending[0].wait()
        cyclic_ntt_finish(pending[1], log_n, root, ops, inverse, group)


class GpuOps:
    """Local steps on this rank's GPU through libstark_hip (kernels on the
    torch current stream, so they order with the RCCL collectives)."""

    def __init__(self, ctx):
        self.ctx = ctx

    @staticmethod
    def _stream() -> int:
        from . import torch_stream
        return torch_stream()

    def ntt(self, t: torch.Tensor, log_len: int, batch: int, root: int, inverse: bool) -> None:
        self.ctx.ntt_dev(t.data_ptr(), log_len, batch, root, inverse=inverse, stream=self._stream())

    def ntt_strided(self, t: torch.Tensor, log_g: int, stride: int, root: int, inverse: bool) -> None:
        self.ctx.ntt_strided_dev(t.data_ptr(), log_g, stride, root, inverse=inverse, stream=self._stream())

    def cyclic_local(self, t: torch.Tensor, log_n: int, log_g: int, rank: int, root: int, inverse: bool) -> None:
        """The local M-point NTT with its twiddle fused into the last pass (stark_cyclic_ntt_local_dev)."""
        self.ctx.cyclic_ntt_local_dev(t.data_ptr(), log_n, log_g, rank, root, inverse=inverse, stream=self._stream())

    def ntt_strided_tw(self, t: torch.Tensor, log_g: int, stride: int, root: int, inverse: bool, tw_root: int,
                       log_order: int, tw_base: int) -> None:
        self.ctx.ntt_strided_tw_dev(t.data_ptr(), log_g, stride, root, tw_root, log_order, tw_base,
                                    inverse=inverse, stream=self._stream())

    def transpose(self, src: torch.Tensor, dst: torch.Tensor, rows: int, cols: int) -> None:
        self.ctx.transpose_dev(src.data_ptr(), dst.data_ptr(), rows, cols, 1, stream=self._stream())

    def merkle_commit(self, shard: torch.Tensor, m: int, leaf_len: int) -> torch.Tensor:
        """Subtree over this rank's m leaves (device tensor of m * leaf_len bytes); its root as a (32,)
        device tensor, copied on the stream (no host round trip)."""
        from . import MerkleProofInPlace
        self._tree = MerkleProofInPlace(self.ctx)
        self._tree.update_dev(shard.data_ptr(), m, leaf_len, stream=self._stream())
        out = torch.empty(32, dtype=torch.uint8, device=shard.device)
        self.ctx.check(self.ctx.lib.stark_merkle_root_dev(self._tree.h, out.data_ptr(), self._stream()),
                       "merkle_root_dev")
        return out

    def merkle_top(self, roots: torch.Tensor, G: int) -> torch.Tensor:
        """The G - 1 digests above G subtree roots (device), the root last (stark_merkle_top_dev)."""
        out = torch.empty(max(G - 1, 1) * 32, dtype=torch.uint8, device=roots.device)
        if G > 1:
            self.ctx.check(self.ctx.lib.stark_merkle_top_dev(self.ctx.h, roots.data_ptr(), G, out.data_ptr(),
                                                             self._stream()), "merkle_top")
        return out[:(G - 1) * 32]

    def merkle_open(self, local_indices) -> tuple:
        """(leaves k x leaf_len, nodes k x depth x 32) byte arrays of the local subtree."""
        ps = self._tree.gen_proofs(local_indices)
        depth = max(self._tree.width().bit_length() - 1, 0)
        leaves = np.frombuffer(b"".join(p.leaf for p in ps), dtype=np.uint8).reshape(len(ps), -1)
        nodes = np.frombuffer(b"".join(b"".join(p.nodes) for p in ps), dtype=np.uint8).reshape(len(ps), depth, 32)
        return leaves, nodes

    def twiddle2d(self, t: torch.Tensor, rows: int, cols: int, row_base: int, col_base: int, root: int,
                  log_order: int) -> None:
        self.ctx.twiddle2d_dev(t.data_ptr(), rows, cols, row_base, col_base, root, log_order,
                               stream=self._stream())


class DistributedMerkle:
    """Blake2s Merkle commitment of n = G * m leaves sharded in rank order
    (rank r holds leaves [r m, (r+1) m)), one GPU per rank.

    commit(): every rank builds its subtree on its GPU (`ops.merkle_commit`, root left in HBM); the G
    subtree roots are all-gathered as one (G, 32) tensor (RCCL with backend "nccl", device memory) and
    the top log2(G) levels are hashed on the device (`ops.merkle_top`); one download brings the levels
    to the host.  The root is the single-tree root: the reference itself builds 2^k subtrees and a top
    tree over their roots (gen_multi_proofs_multi_core, merkle_proof_in_place.rs:106-206).

    gen_proofs(indices): each rank opens the indices inside its shard (leaf + subtree siblings); one
    padded tensor all-gather brings every rank's openings to every rank (the byte count of each rank's
    part follows from the indices, known everywhere), which appends the top-tree siblings and returns
    them in the caller's order, duplicates kept (merkle_proof_in_place.rs:191-205).
    """

    def __init__(self, ops, group=None):
        self.ops = ops
        self.group = group
        self.G = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        self.levels = []      # top tree: levels[0] = subtree roots, ..., levels[-1] = [root]
        self.m = 0
        self.leaf_len = 0

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """(G, *t.shape) concatenation of every rank's t (host tensors under gloo)."""
        host = dist.get_backend(self.group) == "gloo" and t.is_cuda
        src = t.cpu() if host else t
        parts = [torch.empty_like(src) for _ in range(self.G)]
        dist.all_gather(parts, src, group=self.group)
        return torch.stack(parts).to(t.device)

    def commit(self, shard, m: int, leaf_len: int) -> bytes:
        if m == 0 or m & (m - 1) or self.G & (self.G - 1):
            raise ValueError("DistributedMerkle: power-of-two shard size and world size required")
        self.m, self.leaf_len = m, leaf_len
        local = self.ops.merkle_commit(shard, m, leaf_len)
        if isinstance(local, (bytes, bytearray)):        # host-side ops (the CPU tests' oracle ops)
            local = torch.frombuffer(bytearray(local), dtype=torch.uint8)
        roots = self._all_gather(local).reshape(-1)     # (G * 32,)
        if hasattr(self.ops, "merkle_top"):
            levels = torch.cat([roots, self.ops.merkle_top(roots, self.G)]).cpu().numpy().tobytes()
        else:
            from . import blake
            lv = [roots.cpu().numpy().tobytes()[32 * i:32 * (i + 1)] for i in range(self.G)]
            levels = b"".join(lv)
            while len(lv) > 1:
                lv = [blake(lv[2 * i] + lv[2 * i + 1]) for i in range(len(lv) // 2)]
                levels += b"".join(lv)
        self.levels, at, w = [], 0, self.G
        while w >= 1:
            self.levels.append([levels[at + 32 * i:at + 32 * (i + 1)] for i in range(w)])
            at += 32 * w
            w //= 2
        return self.levels[-1][0]

    def root(self) -> bytes:
        return self.levels[-1][0]

    def gen_proofs(self, indices) -> list:
        from . import Proof
        idx = np.asarray(list(indices), dtype=np.int64)
        m, G, ll = self.m, self.G, self.leaf_len
        depth = m.bit_length() - 1
        owner = idx // m
        mine = np.nonzero(owner == self.r)[0]
        per = ll + depth * 32
        counts = [int(np.count_nonzero(owner == p)) for p in range(G)]
        width = max(max(counts), 1) * per
        blob = np.zeros(width, dtype=np.uint8)
        if len(mine):
            leaves, nodes = self.ops.merkle_open([int(i) - self.r * m for i in idx[mine]])
            part = np.concatenate([np.asarray(leaves, dtype=np.uint8).reshape(len(mine), ll),
                                   np.asarray(nodes, dtype=np.uint8).reshape(len(mine), depth * 32)], axis=1)
            blob[:part.size] = part.reshape(-1)
        t = torch.from_numpy(blob)
        if dist.get_backend(self.group) == "nccl":
            t = t.to(torch.device("cuda", torch.cuda.current_device()))
        allb = self._all_gather(t).cpu().numpy()      # (G, width)
        out = [None] * len(idx)
        at = [0] * G
        for k, i in enumerate(idx):
            p = int(owner[k])
            row = allb[p, at[p] * per:(at[p] + 1) * per].tobytes()
            at[p] += 1
            pos = p
            top = []
            for lv in self.levels[:-1]:   # siblings of the subtree root up to the top
                top.append(lv[pos ^ 1])
                pos >>= 1
            out[k] = Proof(row[:ll], [row[ll + 32 * d:ll + 32 * (d + 1)] for d in range(depth)] + top)
        return out
