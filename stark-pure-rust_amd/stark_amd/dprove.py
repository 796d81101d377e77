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
from .verify import _Branches, _FriLayer

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

    def open_plan(self, idx: np.ndarray) -> list:
        """This rank's gathers for opening leaves idx: (rows request, path request).
        A leaf comes from its class owner, the lower path from the subtree owner
        (or rank 0 when the tree is whole on every rank)."""
        G, r, m = self.G, self.r, self.n_local
        leaf_local = idx[idx % G == r] // G
        if self.blocked:
            path_local = idx[idx // m == r] - r * m
        else:
            path_local = idx if r == 0 else idx[:0]
        return [("rows", self.leaves, self.leaf_len, m, leaf_local), ("tree", self.tree, path_local)]

    def assemble(self, idx: np.ndarray, parts: list) -> tuple:
        """(k x leaf_len leaves, k x depth x 32 nodes) from every rank's (leaf blob, node blob)."""
        G, m, k = self.G, self.n_local, len(idx)
        depth = self.n.bit_length() - 1
        leaves = np.empty((k, self.leaf_len), dtype=np.uint8)
        nodes = np.empty((k, depth, 32), dtype=np.uint8)
        low = (m.bit_length() - 1) if self.blocked else depth
        for p, (lb, nb) in enumerate(parts):
            sel = idx % G == p
            leaves[sel] = np.frombuffer(lb, dtype=np.uint8).reshape(-1, self.leaf_len)
            psel = (idx // m == p) if self.blocked else np.full(k, p == 0)
            if psel.any():
                nodes[psel, :low] = np.frombuffer(nb, dtype=np.uint8).reshape(-1, low, 32)
        if self.blocked:
            pos = idx // m
            for lvl, lv in enumerate(self.top[:-1]):
                arr = np.frombuffer(b"".join(lv), dtype=np.uint8).reshape(-1, 32)
                nodes[:, low + lvl] = arr[pos ^ 1]
                pos = pos >> 1
        return leaves, nodes


def _k_values(m_root: bytes) -> list:
    """prove.rs:274-283 (mk_seed + from_str of the BE digest)."""
    return [1] + [int.from_bytes(blake(m_root + bytes([i])), "big") % P for i in range(1, 11)]


def _branches(opened, keep: list) -> _Branches:
    leaves, nodes = opened
    lv, nd = leaves.tobytes(), nodes.tobytes()
    keep += [lv, nd]
    return _Branches(lv, nd, leaves.shape[0], leaves.shape[1], nodes.shape[1])


def render_json(lib, m_root, l_root, a_root, main, lcomb, layers, last: bytes) -> str:
    """stark_r1cs_proof_json_from_parts: serde_json of StarkProof (utils.rs:122-130).
    main / lcomb / each layer's column and poly: (leaves k x leaf_len, nodes k x depth x 32) arrays."""
    keep = []
    mb = _branches(main, keep)
    lb = _branches(lcomb, keep)
    arr = (_FriLayer * max(len(layers), 1))()
    for i, (root2, col, poly) in enumerate(layers):
        keep.append(root2)
        arr[i] = _FriLayer(root2, _branches(col, keep), _branches(poly, keep))
    total = sum(len(x) for x in keep) + len(last) + 96
    nproofs = main[0].shape[0] + lcomb[0].shape[0] + sum(c[0].shape[0] + q[0].shape[0] for _, c, q in layers)
    cap = 256 + 4 * total + 32 * nproofs + 64 * len(layers)
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    rc = lib.stark_r1cs_proof_json_from_parts(m_root, l_root, a_root, ctypes.byref(mb), ctypes.byref(lb),
                                              ctypes.cast(arr, ctypes.c_void_p), len(layers), last,
                                              len(last) // 32, buf, cap, ctypes.byref(n))
    if rc != 0 or n.value >= cap:
        raise RuntimeError(f"stark_r1cs_proof_json_from_parts failed ({rc}, {n.value} >= {cap})")
    return buf.raw[:n.value].decode()


class _Phases:
    """STARK_PROFILE=1: wall-clock of each phase on this rank (stderr)."""

    def __init__(self, rank: int):
        import os
        import time
        self.on = os.environ.get("STARK_PROFILE", "0") not in ("", "0")
        self.rank, self.time = rank, time.perf_counter
        self.t0 = self.last = self.time()

    def mark(self, what: str):
        if self.on:
            import sys
            now = self.time()
            print(f"[dprove r{self.rank}] {what}: {1e3 * (now - self.last):.3f} ms (total {1e3 * (now - self.t0):.3f})",
                  file=sys.stderr)
            self.last = now


# FRI layers of at most 2^FRI_TAIL_LOG values are not worth a collective each: their
# values go to rank 0, which proves the rest of the FRI recursion alone (one device-resident
# prove_low_degree, no per-layer host round trip).  The proof is the same.
FRI_TAIL_LOG = 16
_EMPTY_LAST = '{"Last":{"last":[]}}]}'


def prove_distributed(ops, r1cs: bytes, wtns: bytes, group=None, fri_tail_log: int = FRI_TAIL_LOG, circuit=None):
    """prove_with_witness (run.rs:310-452) over the G ranks of `group`.
    Every rank calls it; rank 0 returns the StarkProof JSON, the others None.
    circuit: this rank's DistCircuit (the .r1cs-only work done once; r1cs is then unused)."""
    G = dist.get_world_size(group)
    r = dist.get_rank(group)
    ph = _Phases(r)
    if G & (G - 1) or G > EXTENSION_FACTOR:
        raise ValueError(f"prove_distributed: world size must be a power of two <= 8 (got {G})")
    # A rank that fails must not leave the others blocked in a collective: every rank
    # reports its status first and all of them raise together.
    h, status, info = None, 0, None
    try:
        h = ops.begin(r1cs, wtns, G, r, circuit)
        status, info = ops.info(h)
    except Exception as e:  # noqa: BLE001 - re-raised below on every rank
        status = getattr(e, "code", -1) or -1
    try:
        codes = _all_gather_object(status, G, group)
        if any(codes):
            ops.raise_status(next(c for c in codes if c), "prove_distributed")
        prec, n_local, os_, g2, a_root = info
        ph.mark("trace + LDE + constraints (begin)")
        skips = EXTENSION_FACTOR
        log_prec = prec.bit_length() - 1
        # Main tree over the 256-B rows (prove.rs:235-264) -> k -> L (prove.rs:274-322) -> L tree.
        main = DistTree(ops, group)
        m_root = main.commit(ops.rows(h), n_local, 256)
        ph.mark("main tree")
        lvals = ops.lincomb(h, m_root, _k_values(m_root))
        ltree = DistTree(ops, group)
        l_root = ltree.commit(lvals, n_local, 32)
        ph.mark("L + L tree")
        # prove_low_degree(L, g2, precision/4, skips) (prove.rs:367, fri.rs:46-224), layer by layer.
        layers = []
        vals, n, w, deg, mtree, mroot = lvals, prec, g2, prec // 4, ltree, l_root
        while deg > 16 and n > (1 << fri_tail_log):
            q = n // 4
            col = ops.fold(vals, n, w, mroot, G, r)
            t2 = DistTree(ops, group)
            root2 = t2.commit(col, q // G, 32)
            ys = get_pseudorandom_indices(root2, q, 40, skips)              # fri.rs:181-189
            poly_idx = [y + q * j for y in ys for j in range(4)]           # fri.rs:193-204
            layers.append((root2, t2, ys, mtree, poly_idx, (q.bit_length() - 1)))
            vals, n, w, deg, mtree, mroot = col, q, pow(w, 4, P), deg // 4, t2, root2
        last_local = ops.to_host(vals, n // G)
        ph.mark(f"FRI ({len(layers)} layers)")
        # Spot checks (prove.rs:337-362).
        positions = get_pseudorandom_indices(l_root, prec, SPOT_CHECK_SECURITY_FACTOR, skips)
        aug = []
        for j in positions:
            aug += [j, (j + prec - skips) % prec, (j + os_ // 3 * skips) % prec, (j + os_ // 3 * 2 * skips) % prec]
        reqs = [(main, aug), (ltree, positions)]
        for (_, t2, ys, mt, poly_idx, _) in layers:
            reqs += [(t2, ys), (mt, poly_idx)]
        reqs = [(t, np.asarray(idx, dtype=np.uint64)) for t, idx in reqs]
        plan = [g for t, idx in reqs for g in t.open_plan(idx)]
        got = ops.open_batch(plan)        # one gather launch for every opening held here
        mine = [(got[2 * i][0], got[2 * i + 1][1]) for i in range(len(reqs))]
        allparts = _all_gather_object((mine, last_local), G, group)
        ph.mark("openings")
        if r != 0:
            return None
        opened = [t.assemble(idx, [p[0][i] for p in allparts]) for i, (t, idx) in enumerate(reqs)]
        chunks = np.stack([np.frombuffer(p[1], dtype=np.uint8).reshape(-1, 32) for p in allparts], axis=1)
        values = chunks.reshape(-1, 32).tobytes()   # value r + G j is rank r's j-th
        fri_parts = [(root2, opened[2 + 2 * li], opened[3 + 2 * li]) for li, (root2, *_rest) in enumerate(layers)]
        if deg <= 16:
            js = render_json(ops.lib, m_root, l_root, a_root, opened[0], opened[1], fri_parts, values)
        else:
            # The remaining layers [Middle.., Last] of prove_low_degree_rec on this layer's values,
            # spliced in place of an empty Last.
            tail = ops.fri_tail(values, n, w, deg, skips)
            js = render_json(ops.lib, m_root, l_root, a_root, opened[0], opened[1], fri_parts, b"")
            assert js.endswith(_EMPTY_LAST) and tail.startswith("[") and tail.endswith("]")
            js = js[:-len(_EMPTY_LAST)] + tail[1:] + "}"
        ph.mark("assembly + JSON")
        return js
    finally:
        if h is not None:
            ops.end(h)


class DistCircuit:
    """A circuit prepared on this rank for prove_distributed (stark_dprove_circuit_new): the
    slot tables and this rank's coset LDEs of K, F0-F2, IDX, PIDX and Zb inverses stay in HBM,
    so each proof extends only S, P and A (cf. stark_amd.r1cs.R1csCircuit on one GPU)."""

    def __init__(self, ctx, r1cs: bytes, group=None):
        from . import _vp
        self.ctx = ctx
        self.G = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        self.h = _vp()
        ctx.check(ctx.lib.stark_dprove_circuit_new(ctx.h, self.G, self.r, r1cs, len(r1cs), ctypes.byref(self.h)),
                  "dprove_circuit_new")

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.stark_r1cs_circuit_free(self.h)
        except Exception:
            pass


class _OpenReq(ctypes.Structure):
    _fields_ = [("tree", ctypes.c_void_p), ("d_rows", ctypes.c_void_p), ("row_bytes", ctypes.c_size_t),
                ("n_rows", ctypes.c_size_t), ("idx", ctypes.POINTER(ctypes.c_size_t)), ("k", ctypes.c_size_t),
                ("leaves_out", ctypes.c_void_p), ("nodes_out", ctypes.c_void_p)]


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

    def begin(self, r1cs: bytes, wtns: bytes, G: int, r: int, circuit=None):
        from . import _vp
        h = _vp()
        if circuit is not None:
            if (circuit.G, circuit.r) != (G, r):
                raise ValueError("DistCircuit prepared for another rank / world size")
            self.ctx.check(self.lib.stark_dprove_begin_circuit(self.ctx.h, circuit.h, wtns, len(wtns), self._stream(),
                                                               ctypes.byref(h)), "dprove_begin")
        else:
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

    def open_batch(self, plan) -> list:
        """stark_open_batch over ("rows", buf, row_bytes, n_rows, idx) / ("tree", tree, idx)
        requests: a list of (leaf blob, node blob) per request."""
        from . import _szp
        reqs = (_OpenReq * max(len(plan), 1))()
        keep, outs = [], []
        for i, g in enumerate(plan):
            if g[0] == "rows":
                _, buf, row_bytes, n_rows, idx = g
                tree, rows, leaf_len, depth = None, self._ptr(buf), row_bytes, 0
            else:
                _, tr, idx = g
                tree, rows, n_rows, row_bytes = tr.t.h, None, 0, 0
                leaf_len, depth = 32, max(tr.t.width().bit_length() - 1, 0)
            idx = np.ascontiguousarray(idx, dtype=np.uint64)
            lo = ctypes.create_string_buffer(max(len(idx) * leaf_len, 1))
            no = ctypes.create_string_buffer(max(len(idx) * depth * 32, 1))
            keep += [idx, lo, no]
            outs.append((lo, len(idx) * leaf_len, no, len(idx) * depth * 32))
            reqs[i] = _OpenReq(tree, rows, row_bytes, n_rows, idx.ctypes.data_as(_szp), len(idx),
                               ctypes.cast(lo, ctypes.c_void_p), ctypes.cast(no, ctypes.c_void_p))
        torch.cuda.current_stream().synchronize()   # trees were built on this stream
        self.ctx.check(self.lib.stark_open_batch(self.ctx.h, ctypes.cast(reqs, ctypes.c_void_p), len(plan),
                                                 self._stream()), "open_batch")
        return [(lo.raw[:nl], no.raw[:nn]) for lo, nl, no, nn in outs]

    def fri_tail(self, values: bytes, n: int, root: int, max_deg_plus_1: int, excl: int) -> str:
        """prove_low_degree on the full layer (rank 0): its serde JSON."""
        v = np.frombuffer(values, dtype=np.uint64).reshape(-1, 4)
        return self.ctx.prove_low_degree(v, root, max_deg_plus_1, excl).to_json()

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
