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

    def merkle_commit(self, shard: torch.Tensor, m: int, leaf_len: int) -> bytes:
        """Subtree over this rank's m leaves (device tensor of m * leaf_len bytes)."""
        from . import MerkleProofInPlace
        self._tree = MerkleProofInPlace(self.ctx)
        self._tree.update_dev(shard.data_ptr(), m, leaf_len, stream=self._stream())
        torch.cuda.current_stream().synchronize()
        self._tree.gen_proofs([])  # sets the root (MerkleProofInPlace::get_root semantics)
        return self._tree.get_root()

    def merkle_open(self, local_indices) -> list:
        return [(p.leaf, p.nodes) for p in self._tree.gen_proofs(local_indices)]

    def twiddle2d(self, t: torch.Tensor, rows: int, cols: int, row_base: int, col_base: int, root: int,
                  log_order: int) -> None:
        self.ctx.twiddle2d_dev(t.data_ptr(), rows, cols, row_base, col_base, root, log_order,
                               stream=self._stream())


class DistributedMerkle:
    """Blake2s Merkle commitment of n = G * m leaves sharded in rank order
    (rank r holds leaves [r m, (r+1) m)), one GPU per rank.

    commit(): every rank builds its subtree on its GPU (`ops.merkle_commit`);
    the G subtree roots are all-gathered (RCCL with backend "nccl") and the
    top log2(G) levels are hashed on the host.  The root is the single-tree
    root: the reference itself builds 2^k subtrees and a top tree over their
    roots (gen_multi_proofs_multi_core, merkle_proof_in_place.rs:106-206).

    gen_proofs(indices): each rank opens the indices inside its shard (leaf +
    subtree siblings) and appends the top-tree siblings; the proofs are
    all-gathered so every rank returns them in the caller's order, duplicates
    kept (merkle_proof_in_place.rs:191-205).
    """

    def __init__(self, ops, group=None):
        self.ops = ops
        self.group = group
        self.G = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        self.levels = []      # top tree: levels[0] = subtree roots, ..., levels[-1] = [root]
        self.m = 0

    def _all_gather_bytes(self, b: bytes) -> list:
        out = [None] * self.G
        dist.all_gather_object(out, b, group=self.group)
        return out

    def commit(self, shard, m: int, leaf_len: int) -> bytes:
        if m == 0 or m & (m - 1) or self.G & (self.G - 1):
            raise ValueError("DistributedMerkle: power-of-two shard size and world size required")
        self.m = m
        local = self.ops.merkle_commit(shard, m, leaf_len)
        from . import blake
        roots = self._all_gather_bytes(local)
        self.levels = [roots]
        while len(self.levels[-1]) > 1:
            lv = self.levels[-1]
            self.levels.append([blake(lv[2 * i] + lv[2 * i + 1]) for i in range(len(lv) // 2)])
        return self.levels[-1][0]

    def root(self) -> bytes:
        return self.levels[-1][0]

    def gen_proofs(self, indices) -> list:
        from . import Proof
        idx = list(indices)
        mine = [(k, i - self.r * self.m) for k, i in enumerate(idx) if i // self.m == self.r]
        local = self.ops.merkle_open([li for _, li in mine]) if mine else []
        part = [(k, leaf, nodes) for (k, _), (leaf, nodes) in zip(mine, local)]
        parts = [None] * self.G
        dist.all_gather_object(parts, part, group=self.group)
        out = [None] * len(idx)
        for p in parts:
            for k, leaf, nodes in p:
                pos = idx[k] // self.m
                top = []
                for lv in self.levels[:-1]:   # siblings of the subtree root up to the top
                    top.append(lv[pos ^ 1])
                    pos >>= 1
                out[k] = Proof(leaf, list(nodes) + top)
        return out
