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
subtree roots as one (G, 32) device tensor and hashes the top log2(G) levels on
the device: the reference's own subtree + top-tree split
(merkle_proof_in_place.rs:106-206), so the root is the single tree's.  Small
trees (fewer than G leaves per rank) are all-gathered and built whole on every
rank.

Nothing in the commit phase waits for the host: each root stays in HBM and
feeds the next step on the stream (k and L from the main root, special_x and
the fold from each FRI layer's root), and every collective is stream-ordered
under RCCL.  The roots come down in ONE batched copy after the last FRI layer;
the host then derives the transcript's indices (l_root -> positions, each
root2 -> ys; the same transcript on every rank), every rank gathers the
openings it holds in one zero-copy launch, and one tensor all-gather (sizes
known on every rank from the layout) brings them to rank 0, which renders the
StarkProof JSON (utils.rs:122-130).  Host-synchronising steps per proof: the
begin call, the status reduction, the roots download, the opening gather and
its collective (`stats["host_syncs"]`).

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

    def commit(self, leaves, n_local: int, leaf_len: int) -> None:
        """Enqueues the commitment; the root is `d_root()` (device) until `set_host` brings the levels."""
        G = self.G
        self.leaves, self.n_local, self.leaf_len = leaves, n_local, leaf_len
        self.n = n_local * G
        dig = self.ops.leaf_digests(leaves, n_local, leaf_len)      # (n_local * 32,) uint8
        self.tree = self.ops.new_tree()
        if n_local % G or G == 1:
            # Few leaves: every rank builds the whole tree from all the digests.
            self.blocked = False
            alld = _all_gather_tensor(dig, G, self.group).reshape(-1)
            self.tree.build(alld, self.n, G)
            self.d_levels = self.tree.root_tensor()
            return
        self.blocked = True
        recv = torch.empty_like(dig)
        _exchange(recv, dig, self.group)          # chunk s of class r -> rank s; rank s gets G chunks
        self.tree.build(recv, n_local, G)         # leaves [r n_local, (r+1) n_local)
        roots = _all_gather_tensor(self.tree.root_tensor(), G, self.group).reshape(-1)   # (G * 32,)
        # subtree roots, then the G - 1 digests above them (the root last), all on the device
        self.d_levels = torch.cat([roots, self.ops.merkle_top(roots, G)])

    def d_root(self) -> torch.Tensor:
        return self.d_levels[-32:]

    def set_host(self, levels: bytes) -> None:
        """The downloaded levels: self.root and (blocked) self.top, the subtree roots and the levels above."""
        self.root = levels[-32:]
        self.top = []
        if self.blocked:
            at, w = 0, self.G
            while w >= 1:
                self.top.append([levels[at + 32 * i:at + 32 * (i + 1)] for i in range(w)])
                at += 32 * w
                w //= 2

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

    def _low(self) -> int:
        depth = self.n.bit_length() - 1
        return (self.n_local.bit_length() - 1) if self.blocked else depth

    def blob_sizes(self, idx: np.ndarray, p: int) -> tuple:
        """Bytes of rank p's (leaf blob, node blob) for opening idx (what its open_plan gathers)."""
        G, m = self.G, self.n_local
        leaves = int(np.count_nonzero(idx % G == p)) * self.leaf_len
        paths = int(np.count_nonzero(idx // m == p)) if self.blocked else (len(idx) if p == 0 else 0)
        return leaves, paths * self._low() * 32

    def assemble(self, idx: np.ndarray, parts: list) -> tuple:
        """(k x leaf_len leaves, k x depth x 32 nodes) from every rank's (leaf blob, node blob)."""
        G, m, k = self.G, self.n_local, len(idx)
        depth = self.n.bit_length() - 1
        leaves = np.empty((k, self.leaf_len), dtype=np.uint8)
        nodes = np.empty((k, depth, 32), dtype=np.uint8)
        low = self._low()
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
    """Per-phase time of one proof on this rank: host wall-clock at each mark and, on a GPU, a HIP event
    on the proof's stream (the device time line, read after the proof's last synchronisation).
    STARK_PROFILE=1 also prints the host marks (stderr).  host_syncs counts the steps that wait for
    the device or for another rank."""

    def __init__(self, rank: int, device: bool):
        import os
        import time
        self.on = os.environ.get("STARK_PROFILE", "0") not in ("", "0")
        self.rank, self.time, self.device = rank, time.perf_counter, device
        self.t0 = self.last = self.time()
        self.marks = []   # (name, host seconds since the previous mark, device event or None)
        self.ev0 = self._event()
        self.host_syncs = 0

    def _event(self):
        if not self.device:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def mark(self, what: str):
        now = self.time()
        self.marks.append((what, now - self.last, self._event()))
        if self.on:
            import sys
            print(f"[dprove r{self.rank}] {what}: {1e3 * (now - self.last):.3f} ms (total {1e3 * (now - self.t0):.3f})",
                  file=sys.stderr)
        self.last = now

    def sync(self, n: int = 1):
        self.host_syncs += n

    def report(self) -> dict:
        """{phase: {"host_ms", "device_ms"}} (device_ms from the events, after everything completed)."""
        out, prev = {}, self.ev0
        for what, dt, ev in self.marks:
            rec = {"host_ms": round(1e3 * dt, 3)}
            if ev is not None and prev is not None:
                ev.synchronize()
                rec["device_ms"] = round(prev.elapsed_time(ev), 3)
            out[what] = rec
            prev = ev
        return {"phases": out, "host_syncs": self.host_syncs, "total_ms": round(1e3 * (self.last - self.t0), 3)}


# FRI layers of at most 2^FRI_TAIL_LOG values are not worth a collective each: their
# values go to rank 0, which proves the rest of the FRI recursion alone (one device-resident
# prove_low_degree, no per-layer host round trip).  The proof is the same.
FRI_TAIL_LOG = 16
_EMPTY_LAST = '{"Last":{"last":[]}}]}'


def _status_max(code: int, group=None, dev=None) -> int:
    """The largest status code over the ranks (0 = every rank ok): one small all-reduce."""
    t = torch.tensor([int(code)], dtype=torch.int64,
                     device=dev if dev is not None and dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.cpu()[0])


def _gather_to_rank0(blobs: list, sizes: list, G: int, r: int, group=None, dev=None):
    """Rank 0 gets every rank's blobs (blobs[i] bytes, rank p's sizes in sizes[p][i], known on every
    rank): one padded tensor all-gather (device memory under RCCL).  Returns [per rank [bytes...]] on
    rank 0, None elsewhere."""
    totals = [sum(sz) for sz in sizes]
    width = max(max(totals), 1)
    mine = np.zeros(width, dtype=np.uint8)
    flat = b"".join(blobs)
    assert len(flat) == totals[r], (len(flat), totals[r])
    mine[:len(flat)] = np.frombuffer(flat, dtype=np.uint8)
    t = torch.from_numpy(mine)
    if dev is not None and dist.get_backend(group) == "nccl":
        t = t.to(dev)
    allt = _all_gather_tensor(t, G, group).cpu().numpy()   # (G, width)
    if r != 0:
        return None
    out = []
    for p in range(G):
        row, at, parts = allt[p].tobytes(), 0, []
        for n in sizes[p]:
            parts.append(row[at:at + n])
            at += n
        out.append(parts)
    return out


def prove_distributed(ops, r1cs: bytes, wtns: bytes, group=None, fri_tail_log: int = FRI_TAIL_LOG, circuit=None,
                      stats: dict | None = None):
    """prove_with_witness (run.rs:310-452) over the G ranks of `group`.
    Every rank calls it; rank 0 returns the StarkProof JSON, the others None.
    circuit: this rank's DistCircuit (the .r1cs-only work done once; r1cs is then unused).
    stats: filled (when given) with this rank's per-phase times and host-synchronising step count.
    On a GPU every step runs on torch's current stream (GpuProverOps): the library's kernels,
    torch's copies and the collectives share one stream order."""
    G = dist.get_world_size(group)
    r = dist.get_rank(group)
    dev = getattr(ops, "dev", None)
    ph = _Phases(r, dev is not None and dev.type == "cuda")
    if G & (G - 1) or G > EXTENSION_FACTOR:
        raise ValueError(f"prove_distributed: world size must be a power of two <= 8 (got {G})")
    # A rank that fails must not leave the others blocked in a collective: every rank
    # reports its status first and all of them raise together.
    h, status, info = None, 0, None
    try:
        h = ops.begin(r1cs, wtns, G, r, circuit)   # trace, LDE, constraints (ends with a stream sync)
        status, info = ops.info(h)
    except Exception as e:  # noqa: BLE001 - re-raised below on every rank
        status = getattr(e, "code", -1) or -1
        if status < 0:
            status = 1 << 20
    ph.sync(2)   # begin ends with a stream synchronisation; info reads the transcript back
    try:
        worst = _status_max(status, group, dev)
        ph.sync()
        if worst:
            ops.raise_status(worst, "prove_distributed")
        prec, n_local, os_, g2, a_root = info
        ph.mark("begin: trace + LDE + constraints")
        skips = EXTENSION_FACTOR
        # Main tree over the 256-B rows (prove.rs:235-264) -> k -> L (prove.rs:274-322) -> L tree, each
        # root consumed on the device.
        main = DistTree(ops, group)
        main.commit(ops.rows(h), n_local, 256)
        ph.mark("main tree")
        lvals = ops.lincomb(h, main.d_root())
        ltree = DistTree(ops, group)
        ltree.commit(lvals, n_local, 32)
        ph.mark("L + L tree")
        # prove_low_degree(L, g2, precision/4, skips) (prove.rs:367, fri.rs:46-224), layer by layer; the
        # fold's special_x comes from the previous tree's root on the device.
        layers = []
        vals, n, w, deg, mtree = lvals, prec, g2, prec // 4, ltree
        while deg > 16 and n > (1 << fri_tail_log):
            q = n // 4
            col = ops.fold(vals, n, w, mtree.d_root(), G, r)
            t2 = DistTree(ops, group)
            t2.commit(col, q // G, 32)
            layers.append((t2, mtree, q))
            vals, n, w, deg, mtree = col, q, pow(w, 4, P), deg // 4, t2
        ph.mark(f"FRI folds + trees ({len(layers)} layers)")
        # Every root and top level, and this rank's share of the last layer, in one download.
        trees = [main, ltree] + [t2 for t2, _, _ in layers]
        host = ops.to_host_many([t.d_levels for t in trees] + [(vals, n // G * 32)])
        ph.sync()
        for t, b in zip(trees, host):
            t.set_host(b)
        last_local = host[-1]
        m_root, l_root = main.root, ltree.root
        # Spot checks (prove.rs:337-362) and the FRI openings (fri.rs:181-205), from the roots.
        positions = get_pseudorandom_indices(l_root, prec, SPOT_CHECK_SECURITY_FACTOR, skips)
        aug = []
        for j in positions:
            aug += [j, (j + prec - skips) % prec, (j + os_ // 3 * skips) % prec, (j + os_ // 3 * 2 * skips) % prec]
        reqs = [(main, aug), (ltree, positions)]
        for (t2, mt, q) in layers:
            ys = get_pseudorandom_indices(t2.root, q, 40, skips)             # fri.rs:181-189
            reqs += [(t2, ys), (mt, [y + q * j for y in ys for j in range(4)])]   # fri.rs:193-204
        reqs = [(t, np.asarray(idx, dtype=np.uint64)) for t, idx in reqs]
        ph.mark("roots download + transcript")
        plan = [g for t, idx in reqs for g in t.open_plan(idx)]
        got = ops.open_batch(plan)        # one gather launch for every opening held here
        ph.sync(2)   # the stream (trees built) and the gather's own completion
        blobs = []
        for i in range(len(reqs)):
            blobs += [got[2 * i][0], got[2 * i + 1][1]]
        blobs.append(last_local)
        sizes = [[x for t, idx in reqs for x in t.blob_sizes(idx, p)] + [len(last_local)] for p in range(G)]
        allparts = _gather_to_rank0(blobs, sizes, G, r, group, dev)
        ph.sync()
        ph.mark("openings gathered")
        if r != 0:
            return None
        opened = [t.assemble(idx, [(allparts[p][2 * i], allparts[p][2 * i + 1]) for p in range(G)])
                  for i, (t, idx) in enumerate(reqs)]
        chunks = np.stack([np.frombuffer(allparts[p][-1], dtype=np.uint8).reshape(-1, 32) for p in range(G)], axis=1)
        values = chunks.reshape(-1, 32).tobytes()   # value r + G j is rank r's j-th
        fri_parts = [(t2.root, opened[2 + 2 * li], opened[3 + 2 * li]) for li, (t2, _, _) in enumerate(layers)]
        if deg <= 16:
            js = render_json(ops.lib, m_root, l_root, a_root, opened[0], opened[1], fri_parts, values)
        else:
            # The remaining layers [Middle.., Last] of prove_low_degree_rec on this layer's values,
            # spliced in place of an empty Last.
            tail = ops.fri_tail(values, n, w, deg, skips)
            js = render_json(ops.lib, m_root, l_root, a_root, opened[0], opened[1], fri_parts, b"")
            assert js.endswith(_EMPTY_LAST) and tail.startswith("[") and tail.endswith("]")
            js = js[:-len(_EMPTY_LAST)] + tail[1:] + "}"
        ph.mark("assembly + JSON (rank 0)")
        return js
    finally:
        if stats is not None:
            stats.update(ph.report())
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
        from . import torch_stream
        return torch_stream()

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

    def lincomb(self, h, d_m_root: torch.Tensor) -> int:
        """k from the main tree's root (in HBM) and L at this rank's points, asynchronously."""
        from . import _vp
        p = _vp()
        self.ctx.check(self.lib.stark_dprove_lincomb_dev(h, d_m_root.data_ptr(), ctypes.byref(p)), "dprove_lincomb")
        return p.value

    def merkle_top(self, roots: torch.Tensor, G: int) -> torch.Tensor:
        """The G - 1 digests above G subtree roots (device), level by level, the root last."""
        out = torch.empty((G - 1) * 32, dtype=torch.uint8, device=self.dev)
        self.ctx.check(self.lib.stark_merkle_top_dev(self.ctx.h, roots.data_ptr(), G, out.data_ptr(), self._stream()),
                       "merkle_top")
        return out

    def to_host_many(self, items: list) -> list:
        """Bytes of each item (a uint8 tensor, or (buffer, nbytes)) in one device-to-host copy."""
        parts = []
        for it in items:
            if isinstance(it, tuple):
                buf, nb = it
                if not isinstance(buf, torch.Tensor):   # a raw device pointer (no FRI layer ran)
                    parts.append(self.to_host(buf, nb // 32))
                    continue
                it = buf.reshape(-1)[:nb]
            parts.append(it.reshape(-1))
        dev = [x for x in parts if isinstance(x, torch.Tensor)]
        flat = torch.cat(dev).cpu().numpy().tobytes() if dev else b""
        out, at = [], 0
        for x in parts:
            if isinstance(x, torch.Tensor):
                out.append(flat[at:at + x.numel()])
                at += x.numel()
            else:
                out.append(x)
        return out

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

    def fold(self, vals, n: int, root: int, d_m_root: torch.Tensor, G: int, r: int) -> torch.Tensor:
        """The layer's fold with special_x from its Merkle root in HBM (no host round trip)."""
        from . import _limbs, _p64
        col = torch.empty(n // 4 // G * 32, dtype=torch.uint8, device=self.dev)
        rl = _limbs(root)
        self.ctx.check(self.lib.stark_fri_fold_dev_root(self.ctx.h, self._ptr(vals), col.data_ptr(), n, _p64(rl),
                                                        d_m_root.data_ptr(), G, r, self._stream()), "fri_fold")
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

    def build(self, digests: torch.Tensor, n: int, interleave: int) -> None:
        self.keep = digests       # read by the build's kernels on the stream
        self.t.update_digests_dev(digests.data_ptr(), n, interleave, stream=self.ops._stream())

    def root_tensor(self) -> torch.Tensor:
        """The root digest copied into a (32,) device tensor on the stream."""
        out = torch.empty(32, dtype=torch.uint8, device=self.ops.dev)
        self.ops.ctx.check(self.ops.lib.stark_merkle_root_dev(self.t.h, out.data_ptr(), self.ops._stream()),
                           "merkle_root_dev")
        return out
