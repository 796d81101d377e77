"""Device groups (include/stark_hip.h `stark_group_*`): one call over G GPUs from one process.

The reference parallelises each call over the thread pool the call builds for itself
(`Worker::new` inside best_fft, packages/fri/src/fft.rs:332; commitment/src/multicore.rs:43-45).
A Group is that pool with GPUs as its workers, created once.  Its methods keep the reference's
names and return what the single-context calls return, bit for bit:

    Group.best_fft / inv_best_fft          fft.rs:327-379 (one-exchange cyclic NTT across members)
    Group.merkle() -> GroupMerkleTree      MerkleTree trait, merkle_tree.rs:60-73 (subtree + top tree)
    Group.prove_with_witness               run.rs:310-452 (one proof shared by the members)
    Group.circuit(r1cs).prove(wtns)        the same with the .r1cs-only work prepared once

The members exchange data by peer copies pulled on their own streams (xGMI between devices, a
device-to-device copy when members share a GPU), all inside libstark_hip: no torch.distributed,
no collective library, no process per GPU.  A device list may repeat a device (G contexts on one
GPU run the same code), which is how the one-GPU test box covers G = 2, 4, 8.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import Proof, StarkError, _elems, _limbs, _out_array, _p64, _vp, load_library


def _lib():
    return load_library()


class Group:
    """G = len(devices) members (1, 2, 4 or 8); a device may repeat."""

    def __init__(self, devices):
        self.lib = _lib()
        devs = list(devices)
        arr = (ctypes.c_int * len(devs))(*devs)
        h = _vp()
        rc = self.lib.stark_group_create(arr, len(devs), ctypes.byref(h))
        if rc != 0:
            raise StarkError(rc, "stark_group_create")
        self.h = h
        self.devices = devs
        self.G = len(devs)

    def close(self):
        if self.h:
            self.lib.stark_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, where: str):
        if rc != 0:
            raise StarkError(rc, where, self.lib.stark_group_last_error(self.h).decode())

    def ctx_handle(self, i: int) -> int:
        return self.lib.stark_group_ctx(self.h, i)

    def synchronize(self):
        self.check(self.lib.stark_group_synchronize(self.h), "group_synchronize")

    # ---- fri::fft -------------------------------------------------------------------------------
    def best_fft(self, coefficients, root_of_unity, log_order_of_root: int, out=None) -> np.ndarray:
        """fft.rs:327-357 over the group (`out`: a caller buffer, as Context.best_fft)."""
        c = _elems(coefficients)
        out = _out_array(out, log_order_of_root)
        self.check(self.lib.stark_group_best_fft(self.h, _p64(c), len(c), _p64(_limbs(root_of_unity)),
                                                 log_order_of_root, _p64(out)), "group_best_fft")
        return out

    def inv_best_fft(self, evaluations, root_of_unity, log_order_of_root: int, out=None) -> np.ndarray:
        """fft.rs:359-379 over the group (`out` as in best_fft)."""
        c = _elems(evaluations)
        out = _out_array(out, log_order_of_root)
        self.check(self.lib.stark_group_inv_best_fft(self.h, _p64(c), len(c), _p64(_limbs(root_of_unity)),
                                                     log_order_of_root, _p64(out)), "group_inv_best_fft")
        return out

    def ntt_dev(self, shards, outs, log_n: int, root, inverse: bool = False) -> None:
        """stark_group_ntt_dev: member r's device shard x[r + G j] -> outs[r] (asynchronous)."""
        a = (_vp * self.G)(*[int(p) for p in shards])
        b = (_vp * self.G)(*[int(p) for p in outs])
        self.check(self.lib.stark_group_ntt_dev(self.h, a, b, log_n, _p64(_limbs(root)), 1 if inverse else 0),
                   "group_ntt_dev")

    # ---- commitment ---------------------------------------------------------------------------
    def merkle(self) -> "GroupMerkleTree":
        return GroupMerkleTree(self)

    # ---- r1cs-stark ---------------------------------------------------------------------------
    def prove_with_witness(self, r1cs: bytes, wtns: bytes):
        """run.rs:310-452: one StarkProof computed by the members together."""
        from .r1cs import StarkProof
        h = _vp()
        self.check(self.lib.stark_group_prove_r1cs_bytes(self.h, r1cs, len(r1cs), wtns, len(wtns), ctypes.byref(h)),
                   "group_prove_r1cs_bytes")
        return StarkProof(self.lib, h)

    def circuit(self, r1cs: bytes) -> "GroupCircuit":
        return GroupCircuit(self, r1cs)


class GroupMerkleTree:
    """MerkleTree<Vec<u8>, BlakeDigest> (merkle_tree.rs:60-73) over the group's members."""

    def __init__(self, group: Group):
        self.g = group
        h = _vp()
        group.check(group.lib.stark_group_merkle_new(group.h, ctypes.byref(h)), "group_merkle_new")
        self.h = h
        self.leaf_len = 0

    def __del__(self):
        try:
            if self.h and self.g.h:   # (a tree outliving its closed group is left to the process)
                self.g.lib.stark_group_merkle_free(self.h)
        except Exception:
            pass

    def width(self) -> int:
        return self.g.lib.stark_group_merkle_width(self.h)

    def update_bytes(self, blob: bytes, n: int, leaf_len: int) -> None:
        self.leaf_len = leaf_len
        self.g.check(self.g.lib.stark_group_merkle_update(self.h, blob, n, leaf_len), "group_merkle_update")

    def update_dev(self, blocks, n: int, leaf_len: int) -> None:
        self.leaf_len = leaf_len
        arr = (_vp * self.g.G)(*[int(p) for p in blocks] + [0] * (self.g.G - len(blocks)))
        self.g.check(self.g.lib.stark_group_merkle_update_dev(self.h, arr, n, leaf_len), "group_merkle_update_dev")

    def get_root(self) -> bytes:
        out = ctypes.create_string_buffer(32)
        n = ctypes.c_size_t(0)
        self.g.check(self.g.lib.stark_group_merkle_get_root(self.h, out, ctypes.byref(n)), "group_get_root")
        return out.raw[:n.value]

    def gen_proofs(self, indices) -> list:
        idx = list(indices)
        k = len(idx)
        depth = max(self.width().bit_length() - 1, 0)
        arr = (ctypes.c_size_t * max(k, 1))(*idx)
        leaves = ctypes.create_string_buffer(max(k * self.leaf_len, 1))
        nodes = ctypes.create_string_buffer(max(k * depth * 32, 1))
        self.g.check(self.g.lib.stark_group_merkle_gen_proofs(self.h, arr, k, leaves, nodes), "group_gen_proofs")
        lr, nr = leaves.raw, nodes.raw
        return [Proof(lr[i * self.leaf_len:(i + 1) * self.leaf_len],
                      [nr[(i * depth + d) * 32:(i * depth + d + 1) * 32] for d in range(depth)]) for i in range(k)]


class GroupCircuit:
    """A circuit prepared on every member (stark_group_circuit_new): each proof extends only S, P, A."""

    def __init__(self, group: Group, r1cs: bytes):
        self.g = group
        self.hs = (_vp * group.G)()
        group.check(group.lib.stark_group_circuit_new(group.h, r1cs, len(r1cs), self.hs), "group_circuit_new")

    def prove(self, wtns: bytes):
        from .r1cs import StarkProof
        h = _vp()
        self.g.check(self.g.lib.stark_group_prove_r1cs_circuit(self.g.h, self.hs, wtns, len(wtns), ctypes.byref(h)),
                     "group_prove_r1cs_circuit")
        return StarkProof(self.g.lib, h)

    def __del__(self):
        try:
            for p in self.hs:
                if p and self.g.h:
                    self.g.lib.stark_r1cs_circuit_free(p)
        except Exception:
            pass
