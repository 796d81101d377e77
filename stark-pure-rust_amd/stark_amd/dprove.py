"""One R1CS STARK proof (mk_r1cs_proof, packages/r1cs-stark/src/prove.rs:14-378)
shared by G = world_size GPUs of one node, one process per GPU.

The proof is byte-identical to the single-GPU prover's (and the reference's).
Layout: the precision domain is split by residue class; rank r owns the
evaluation points i = r + G*j.  With G | 8 (the extension factor) this makes
almost the whole proof local (csrc/r1cs.hip `dprove_begin`):

  * LDE: each column's polynomial has degree < steps <= precision/G, so its
    values at r + G*j are one precision/G-point coset NTT: no exchange at all;
  * constraints: every shifted read (-8, +k*8, +2k*8) is a multiple of G;
  * FRI: the fold of row i reads i + t*n/4, all in i's class while G | n/4,
    so each layer's column is residue-class distributed again.

Only the Merkle commitments mix classes.  DistTree hashes the local leaves,
exchanges the 32-B leaf digests with one all-to-all (RCCL over xGMI with
backend "nccl"), builds the rank's contiguous subtree, all-gathers the G
subtree roots and hashes the top log2(G) levels: the reference's own
subtree + top-tree split (merkle_proof_in_place.rs:106-206), so the root is
the single tree's.  Small trees (fewer than G leaves per rank) are all-gathered
and built whole on every rank.  Openings: a leaf comes from its class owner,
the lower path from the subtree owner, the top path from the roots; one
all_gather_object collects every opening of the proof, rank 0 renders the
StarkProof JSON (utils.rs:122-130).

The transcript (m_root -> k, l_root -> positions, FRI roots -> special_x, ys)
is recomputed identically on every rank from the all-gathered roots.

`ops` abstracts the per-rank device work: GpuProverOps runs it in
libstark_hip on this rank's GPU; tests/test_dprove_cpu.py runs the same
orchestration with an oracle-backed ops under gloo.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import P, blake, get_pseudorandom_indices

EXTENSION_FACTOR = 8        # r1cs-stark/src/utils.rs:135
SPOT_CHECK_SECURITY_FACTOR = 80  # utils.rs:136


def _exchange(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """all_to_all_single of equal chunks (gloo needs host tensors)."""
    if dist.get_backend(group) == "gloo" and inp.is_cuda:
        o = torch.empty_like(out, device="cpu")
        dist.all_to_all_single(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, group=group)


def _all_gather_tensor(t: torch.Tensor, G: int, group=None) -> torch.Tensor:
    """(G, *t.shape) concatenation of every rank's t."""
    host = dist.get_backend(group) == "gloo" and t.is_cuda
    src = t.cpu() if host else t
    parts = [torch.empty_like(src) for _ in range(G)]
    dist.all_gather(parts, src, group=group)
    return torch.stack(parts).to(t.device)


def _all_gather_object(obj, G: int, group=None) -> list:
    out = [None] * G
    dist.all_gather_object(out, obj, group=group)
    return out


class DistTree:
    """Blake2s Merkle tree over n leaves held by residue class (rank r holds
    leaves r, r + G, ...; n_local = n / G of them, leaf_len bytes each)."""

    def __init__(self, ops, group=None):
        self.ops = ops
        self.group = group
        self.G = dist.get_world_size(group)
        self.r = dist.get_rank(group)

    def commit(self, leaves, n_local: int, leaf_len: int) -> bytes:
        G = self.G
        self.leaves, self.n_local, self.leaf_len = leaves, n_local, leaf_len
        self.n = n_local * G
        dig = self.ops.leaf_digests(leaves, n_local, leaf_len)      # (n_local * 32,) uint8
        self.tree = self.ops.new_tree()
        if n_local % G or G == 1:
            # Few leaves: every rank builds the whole tree from all the digests.
            self.blocked = False
            alld = _all_gather_tensor(dig, G, self.group).reshape(-1)
            self.root = self.tree.build(alld, self.n, G)
            self.top = []
            return self.root
        self.blocked = True
        recv = torch.empty_like(dig)
        _exchange(recv, dig, self.group)          # chunk s of class r -> rank s; rank s gets G chunks
        sub = self.tree.build(recv, n_local, G)   # leaves [r n_local, (r+1) n_local)
        roots = _all_gather_object(sub, G, self.group)
        self.top = [roots]
        while len(self.top[-1]) > 1:
            lv = self.top[-1]
            self.top.append([blake(lv[2 * i] + lv[2 * i + 1]) for i in range(len(lv) // 2)])
        self.root = self.top[-1][0]
        return self.root

    def contributions(self, indices) -> tuple:
        """This rank's parts of the openings: {k: leaf bytes}, {k: lower path}."""
        G, r, m = self.G, self.r, self.n_local
        mine_leaf = [(k, i) for k, i in enumerate(indices) if i % G == r]
        leaves = {}
        if mine_leaf:
            got = self.ops.gather(self.leaves, self.leaf_len, [i // G for _, i in mine_leaf])
            leaves = {k: b for (k, _), b in zip(mine_leaf, got)}
        if self.blocked:
            mine_path = [(k, i - r * m) for k, i in enumerate(indices) if i // m == r]
        else:
            mine_path = [(k, i) for k, i in enumerate(indices)] if r == 0 else []
        paths = {}
        if mine_path:
            got = self.tree.open([li for _, li in mine_path])
            paths = {k: nodes for (k, _), nodes in zip(mine_path, got)}
        return leaves, paths

    def top_path(self, index: int) -> list:
        if not self.blocked:
            return []
        pos = index // self.n_local
        out = []
        for lv in self.top[:-1]:
            out.append(lv[pos ^ 1])
            pos >>= 1
        return out


def _from_bytes_le(b: bytes) -> int:
    return int.from_bytes(b, "little") % P


def _k_values(m_root: bytes) -> list:
    """prove.rs:274-283 (mk_seed + from_str of the BE digest)."""
    return [1] + [int.from_bytes(blake(m_root + bytes([i])), "big") % P for i in range(1, 11)]


class _Branches(ctypes.Structure):
    _fields_ = [("leaves", ctypes.c_char_p), ("nodes", ctypes.c_char_p), ("k", ctypes.c_size_t),
                ("leaf_len", ctypes.c_size_t), ("depth", ctypes.c_size_t)]


class _FriLayer(ctypes.Structure):
    _fields_ = [("root2", ctypes.c_char_p), ("column", _Branches), ("poly", _Branches)]


def _branches(proofs, leaf_len: int, depth: int, keep: list) -> _Branches:
    lv = b"".join(p[0] for p in proofs)
    nd = b"".join(b"".join(p[1]) for p in proofs)
    keep += [lv, nd]
    return _Branches(lv, nd, len(proofs), leaf_len, depth)


def render_json(lib, m_root, l_root, a_root, main, main_depth, lcomb, l_depth, layers, last_values) -> str:
    """stark_r1cs_proof_json_from_parts: serde_json of StarkProof (utils.rs:122-130)."""
    keep = []
    mb = _branches(main, 256, main_depth, keep)
    lb = _branches(lcomb, 32, l_depth, keep)
    arr = (_FriLayer * max(len(layers), 1))()
    for i, (root2, col, cdepth, poly, pdepth) in enumerate(layers):
        keep.append(root2)
        arr[i] = _FriLayer(root2, _branches(col, 32, cdepth, keep), _branches(poly, 32, pdepth, keep))
    last = b"".join(last_values)
    cap = 64 + 4 * (len(b"".join(keep)) + len(last) + 96) + 64 * (len(main) + len(lcomb) + 200 * (len(layers) + 1))
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    rc = lib.stark_r1cs_proof_json_from_parts(m_root, l_root, a_root, ctypes.byref(mb), ctypes.byref(lb),
                                              ctypes.cast(arr, ctypes.c_void_p), len(layers), last,
                                              len(last_values), buf, cap, ctypes.byref(n))
    if rc != 0 or n.value >= cap:
        raise RuntimeError(f"stark_r1cs_proof_json_from_parts failed ({rc}, {n.value} >= {cap})")
    return buf.raw[:n.value].decode()


def prove_distributed(ops, r1cs: bytes, wtns: bytes, group=None):
    """prove_with_witness (run.rs:310-452) over the G ranks of `group`.
    Every rank calls it; rank 0 returns the StarkProof JSON, the others None."""
    G = dist.get_world_size(group)
    r = dist.get_rank(group)
    if G & (G - 1) or G > EXTENSION_FACTOR:
        raise ValueError(f"prove_distributed: world size must be a power of two <= 8 (got {G})")
    h = ops.begin(r1cs, wtns, G, r)
    try:
        status, info = ops.info(h)
        codes = _all_gather_object(status, G, group)
        if any(codes):
            ops.raise_status(next(c for c in codes if c), "prove_distributed")
        prec, n_local, os_, g2, a_root = info
        skips = EXTENSION_FACTOR
        log_prec = prec.bit_length() - 1
        # Main tree over the 256-B rows (prove.rs:235-264) -> k -> L (prove.rs:274-322) -> L tree.
        main = DistTree(ops, group)
        m_root = main.commit(ops.rows(h), n_local, 256)
        lvals = ops.lincomb(h, m_root, _k_values(m_root))
        ltree = DistTree(ops, group)
        l_root = ltree.commit(lvals, n_local, 32)
        # prove_low_degree(L, g2, precision/4, skips) (prove.rs:367, fri.rs:46-224), layer by layer.
        layers = []
        vals, n, w, deg, mtree, mroot = lvals, prec, g2, prec // 4, ltree, l_root
        while deg > 16:
            q = n // 4
            col = ops.fold(vals, n, w, mroot, G, r)
            t2 = DistTree(ops, group)
            root2 = t2.commit(col, q // G, 32)
            ys = get_pseudorandom_indices(root2, q, 40, skips)              # fri.rs:181-189
            poly_idx = [y + q * j for y in ys for j in range(4)]           # fri.rs:193-204
            layers.append((root2, t2, ys, mtree, poly_idx, (q.bit_length() - 1)))
            vals, n, w, deg, mtree, mroot = col, q, pow(w, 4, P), deg // 4, t2, root2
        last_local = ops.to_host(vals, n // G)
        # Spot checks (prove.rs:337-362).
        positions = get_pseudorandom_indices(l_root, prec, SPOT_CHECK_SECURITY_FACTOR, skips)
        aug = []
        for j in positions:
            aug += [j, (j + prec - skips) % prec, (j + os_ // 3 * skips) % prec, (j + os_ // 3 * 2 * skips) % prec]
        reqs = [(main, aug), (ltree, positions)]
        for (_, t2, ys, mt, poly_idx, _) in layers:
            reqs += [(t2, ys), (mt, poly_idx)]
        parts = [t.contributions(idx) for t, idx in reqs]
        allparts = _all_gather_object((parts, last_local), G, group)
        if r != 0:
            return None
        proofs = []
        for q_i, (t, idx) in enumerate(reqs):
            out = []
            for k, i in enumerate(idx):
                leaf = next(p[0][q_i][0][k] for p in allparts if k in p[0][q_i][0])
                lower = next(p[0][q_i][1][k] for p in allparts if k in p[0][q_i][1])
                out.append((leaf, list(lower) + t.top_path(i)))
            proofs.append(out)
        last_values = []
        chunks = [p[1] for p in allparts]
        for j in range(n // G):
            for rr in range(G):
                last_values.append(chunks[rr][32 * j:32 * (j + 1)])
        fri_parts = []
        for li, (root2, t2, ys, mt, poly_idx, log_q) in enumerate(layers):
            fri_parts.append((root2, proofs[2 + 2 * li], log_q, proofs[3 + 2 * li], log_q + 2))
        return render_json(ops.lib, m_root, l_root, a_root, proofs[0], log_prec, proofs[1], log_prec, fri_parts,
                           last_values)
    finally:
        ops.end(h)


class GpuProverOps:
    """The per-rank steps on this rank's GPU through libstark_hip; kernels go to
    torch's current stream so they order with the RCCL collectives."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.lib = ctx.lib
        self.dev = torch.device("cuda", torch.cuda.current_device())

    @staticmethod
    def _stream():
        return torch.cuda.current_stream().cuda_stream

    @staticmethod
    def _ptr(buf) -> int:
        return buf.data_ptr() if isinstance(buf, torch.Tensor) else int(buf)

    def raise_status(self, code, where):
        from . import StarkError
        raise StarkError(code, where)

    def begin(self, r1cs: bytes, wtns: bytes, G: int, r: int):
        from . import _vp
        h = _vp()
        self.ctx.check(self.lib.stark_dprove_begin_bytes(self.ctx.h, G, r, r1cs, len(r1cs), wtns, len(wtns),
                                                         self._stream(), ctypes.byref(h)), "dprove_begin")
        return h

    def info(self, h):
        from . import _u64p
        v = [ctypes.c_size_t(0) for _ in range(3)]
        g2 = np.zeros(4, dtype=np.uint64)
        a_root = ctypes.create_string_buffer(32)
        rc = self.lib.stark_dprove_info(h, *[ctypes.byref(x) for x in v], g2.ctypes.data_as(_u64p), a_root)
        g2i = sum(int(g2[k]) << (64 * k) for k in range(4))
        return rc, (v[0].value, v[1].value, v[2].value, g2i, a_root.raw)

    def end(self, h):
        self.lib.stark_dprove_free(h)

    def rows(self, h) -> int:
        from . import _vp
        p = _vp()
        self.ctx.check(self.lib.stark_dprove_rows(h, ctypes.byref(p)), "dprove_rows")
        return p.value

    def lincomb(self, h, m_root: bytes, k: list) -> int:
        from . import _vp
        p = _vp()
        self.ctx.check(self.lib.stark_dprove_lincomb(h, m_root, ctypes.byref(p)), "dprove_lincomb")
        return p.value

    def leaf_digests(self, leaves, n: int, leaf_len: int) -> torch.Tensor:
        out = torch.empty(n * 32, dtype=torch.uint8, device=self.dev)
        self.ctx.check(self.lib.stark_merkle_leaf_digests_dev(self.ctx.h, self._ptr(leaves), n, leaf_len,
                                                              out.data_ptr(), self._stream()), "leaf_digests")
        return out

    def new_tree(self):
        return _GpuTree(self)

    def gather(self, buf, row_bytes: int, local_indices) -> list:
        from . import _szp
        idx = np.ascontiguousarray(np.asarray(local_indices, dtype=np.uint64))
        out = ctypes.create_string_buffer(len(idx) * row_bytes)
        self.ctx.check(self.lib.stark_gather_rows_dev(self.ctx.h, self._ptr(buf), row_bytes, idx.ctypes.data_as(_szp),
                                                      len(idx), out, self._stream()), "gather_rows")
        raw = out.raw
        return [raw[i * row_bytes:(i + 1) * row_bytes] for i in range(len(idx))]

    def fold(self, vals, n: int, root: int, m_root: bytes, G: int, r: int) -> torch.Tensor:
        from . import _limbs, _p64
        col = torch.empty(n // 4 // G * 32, dtype=torch.uint8, device=self.dev)
        rl = _limbs(root)
        self.ctx.check(self.lib.stark_fri_fold_dev(self.ctx.h, self._ptr(vals), col.data_ptr(), n, _p64(rl), m_root,
                                                   G, r, self._stream()), "fri_fold")
        return col

    def to_host(self, buf, count: int) -> bytes:
        out = ctypes.create_string_buffer(max(count * 32, 1))
        torch.cuda.current_stream().synchronize()
        self.ctx.check(self.lib.stark_memcpy_d2h(self.ctx.h, out, self._ptr(buf), count * 32), "d2h")
        return out.raw[:count * 32]


class _GpuTree:
    def __init__(self, ops: GpuProverOps):
        from . import MerkleProofInPlace
        self.ops = ops
        self.t = MerkleProofInPlace(ops.ctx)

    def build(self, digests: torch.Tensor, n: int, interleave: int) -> bytes:
        self.t.update_digests_dev(digests.data_ptr(), n, interleave, stream=self.ops._stream())
        torch.cuda.current_stream().synchronize()
        self.t.gen_proofs([])      # sets the root (MerkleProofInPlace::get_root semantics)
        return self.t.get_root()

    def open(self, local_indices) -> list:
        return [p.nodes for p in self.t.gen_proofs(local_indices)]
