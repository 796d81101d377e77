"""CPU (gloo): the distributed prover's orchestration (stark_amd/dprove.py) at
world sizes 1-8 with every per-rank step done on the host by the oracle (test
infrastructure), checked against the golden StarkProof digest of the
single-process prover.  Covers the residue-class layout, the digest
all-to-all + subtree + top-tree commitments (blocked and all-gathered), the
transcript, the per-class FRI folds and the opening assembly."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

import oracle as O
from ranks import run_ranks  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "r1cs")
P = O.P


def _u8(b: bytes) -> torch.Tensor:
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy())


def _levels(lv: list) -> list:
    out = [lv]
    while len(lv) > 1:
        lv = [O.py_blake(lv[2 * i] + lv[2 * i + 1]) for i in range(len(lv) // 2)]
        out.append(lv)
    return out


class _PyTree:
    """Blake2s tree over given leaf digests (interleaved residue-class chunks)."""

    def build(self, digests: torch.Tensor, n: int, interleave: int) -> None:
        raw = bytes(digests.numpy())
        chunk = n // interleave
        self.levels = _levels([raw[32 * (r * chunk + m):32 * (r * chunk + m + 1)]
                               for m in range(chunk) for r in range(interleave)])

    def root_tensor(self) -> torch.Tensor:
        return _u8(self.levels[-1][0])

    def open(self, idx) -> list:
        out = []
        for i in idx:
            nodes, pos = [], i
            for lv in self.levels[:-1]:
                nodes.append(lv[pos ^ 1])
                pos >>= 1
            out.append(nodes)
        return out


class OracleProverOps:
    """dprove.py's per-rank steps on the host (oracle rows sliced to the rank's
    residue class; L, the FRI fold and the hashing restated in Python)."""

    def __init__(self):
        import stark_amd
        import r1cs as R
        self.R = R
        self.o = O.Oracle()
        self.lib = stark_amd.load_library()   # host-only JSON renderer

    def raise_status(self, code, where):
        raise RuntimeError(f"{where}: {code}")

    def begin(self, r1cs, wtns, G, r, circuit=None):
        tr = self.R.build_trace(self.R.read_r1cs(r1cs), self.R.read_witness(wtns))
        rows, a_root = self.R.r1cs_rows(self.o, tr, cpus=2)
        prec = len(rows) // 256
        local = b"".join(rows[256 * i:256 * (i + 1)] for i in range(r, prec, G))
        return {"G": G, "r": r, "prec": prec, "os": len(tr.coefficients), "rows": local, "a_root": a_root,
                "g2": O.root_of_unity(prec.bit_length() - 1)}

    def info(self, h):
        return 0, (h["prec"], h["prec"] // h["G"], h["os"], h["g2"], h["a_root"])

    def end(self, h):
        pass

    def rows(self, h):
        return h["rows"]

    def lincomb(self, h, m_root_t):
        """L = k0 D1 + ... + k10 S at this rank's points (prove.rs:287-322), k from m_root (prove.rs:274-283)."""
        from stark_amd.dprove import _k_values
        k = _k_values(bytes(m_root_t.numpy()))
        G, r, prec, rows = h["G"], h["r"], h["prec"], h["rows"]
        steps = prec // 8
        g2s = pow(h["g2"], steps, P)
        out = []
        for j in range(prec // G):
            f = [int.from_bytes(rows[256 * j + 32 * c:256 * j + 32 * (c + 1)], "little") for c in range(8)]
            p, a, s, d1, d2, d3, b2, b3 = f
            xs = pow(g2s, r + G * j, P)
            acc = (k[0] * d1 + k[1] * d2 + k[2] * d3 + k[3] * p + k[4] * p * xs + k[5] * b2 + k[6] * b2 * xs
                   + k[7] * b3 + k[8] * b3 * xs + k[9] * a + k[10] * s) % P
            out.append(acc.to_bytes(32, "little"))
        return b"".join(out)

    def leaf_digests(self, leaves, n, leaf_len):
        return _u8(b"".join(O.py_blake(leaves[leaf_len * i:leaf_len * (i + 1)]) for i in range(n)))

    def new_tree(self):
        return _PyTree()

    def merkle_top(self, roots_t, G):
        raw = bytes(roots_t.numpy())
        lv = _levels([raw[32 * i:32 * (i + 1)] for i in range(G)])
        return _u8(b"".join(b"".join(x) for x in lv[1:]))

    def to_host_many(self, items):
        out = []
        for it in items:
            if isinstance(it, tuple):
                buf, nb = it
                out.append(bytes(buf.numpy()[:nb]) if isinstance(buf, torch.Tensor) else bytes(buf[:nb]))
            else:
                out.append(bytes(it.numpy()))
        return out

    def open_batch(self, plan):
        out = []
        for g in plan:
            if g[0] == "rows":
                _, buf, row_bytes, _, idx = g
                out.append((b"".join(bytes(buf[row_bytes * int(i):row_bytes * (int(i) + 1)]) for i in idx), b""))
            else:
                _, tree, idx = g
                out.append((b"", b"".join(b"".join(nodes) for nodes in tree.open([int(i) for i in idx]))))
        return out

    def fold(self, vals, n, root, m_root_t, G, r):
        """Column rows r + G j: the cubic through (w^(i + t n/4), v[i + t n/4]) at special_x (fri.rs:135-164)."""
        sx = int.from_bytes(bytes(m_root_t.numpy()), "little") % P
        q = n // 4
        ql = q // G
        v = [int.from_bytes(vals[32 * i:32 * (i + 1)], "little") for i in range(n // G)]
        out = []
        for j in range(ql):
            i = r + G * j
            xs = [pow(root, i + t * q, P) for t in range(4)]
            ys = [v[j + t * ql] for t in range(4)]
            acc = 0
            for a in range(4):
                num, den = 1, 1
                for b in range(4):
                    if a != b:
                        num = num * (sx - xs[b]) % P
                        den = den * (xs[a] - xs[b]) % P
                acc = (acc + ys[a] * num * pow(den, P - 2, P)) % P
            out.append(acc.to_bytes(32, "little"))
        return b"".join(out)

    def fri_tail(self, values, n, root, max_deg_plus_1, excl):
        v = np.frombuffer(values, dtype=np.uint64).reshape(-1, 4)
        return self.o.prove_low_degree_json(v, root, max_deg_plus_1, excl)

    def to_host(self, buf, count):
        return bytes(buf[:32 * count])


def _worker(rank, world, port, name, tail_log, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stark_amd.dprove import prove_distributed
    r1 = open(os.path.join(FIX, f"{name}.r1cs"), "rb").read()
    wt = open(os.path.join(FIX, f"{name}.wtns"), "rb").read()
    js = prove_distributed(OracleProverOps(), r1, wt, fri_tail_log=tail_log)
    out_q.put((rank, hashlib.sha256(js.encode()).hexdigest() if js is not None else None))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world,tail_log", [("compute", 1, 0), ("compute", 2, 0), ("compute", 4, 16),
                                                 ("compute", 8, 0), ("poseidon3_test", 4, 12)])
def test_prove_distributed_gloo(name, world, tail_log):
    """tail_log 0: every FRI layer distributed; else layers of <= 2^tail_log values on rank 0."""
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))
    res = dict(run_ranks(_worker, world, (name, tail_log), timeout=600))
    assert res[0] == golden[name]["json_sha256"]
    assert all(res[r] is None for r in range(1, world))


def _worker_bad(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from stark_amd.dprove import prove_distributed
    r1 = open(os.path.join(FIX, "compute.r1cs"), "rb").read()
    wt = open(os.path.join(FIX, "compute.wtns"), "rb").read()
    if rank == 1:
        wt = wt[:len(wt) // 2]          # one rank gets a truncated witness
    try:
        prove_distributed(OracleProverOps(), r1, wt)
        out_q.put((rank, "no error"))
    except Exception as e:  # noqa: BLE001
        out_q.put((rank, type(e).__name__))
    dist.barrier()
    dist.destroy_process_group()


def test_prove_distributed_failure_raises_on_every_rank():
    """A rank whose set-up fails must not leave the others blocked in a collective."""
    world = 2
    res = dict(run_ranks(_worker_bad, world, (), timeout=300))
    assert all(v != "no error" for v in res.values()), res
