"""GPU: device groups (include/stark_hip.h stark_group_*, csrc/group.hip) -- one call over G members in
one process, the multi-GPU path of the C ABI.  On the one-GPU test box the G members are G contexts on
device 0; the peer-copy transport and every other line of the code are the ones an 8-GPU group runs.

Parity, per the reference items the group entry points keep:
  * best_fft / inv_best_fft (fft.rs:327-379): equal to the oracle's restatement at 2^20 (and small sizes),
    and to the committed digests of the bench's 2^24 input;
  * MerkleTree (merkle_tree.rs:60-73, merkle_proof_in_place.rs:106-206): root and paths equal the oracle's
    single tree;
  * prove_with_witness (run.rs:310-452): the StarkProof JSON equals the golden digests (poseidon3 =
    BASELINE config 4, pedersen = config 3) and, at G = 8, the oracle's digest of the 2^20-step synthetic
    proof (config 5's stand-in), cold and with a prepared circuit."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "r1cs")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))
BIG = json.load(open(os.path.join(ROOT, "tests", "golden", "large_digests.json")))


def _group(G):
    from stark_amd.group import Group
    return Group([0] * G)


def _sha(a) -> str:
    return hashlib.sha256(a.tobytes() if hasattr(a, "tobytes") else a).hexdigest()


def _fixture(name):
    return (open(os.path.join(FIX, f"{name}.r1cs"), "rb").read(), open(os.path.join(FIX, f"{name}.wtns"), "rb").read())


@pytest.mark.parametrize("G", [1, 2, 4, 8])
@pytest.mark.parametrize("log_n,length", [(3, 5), (6, 64), (10, 700), (10, 0), (16, 1 << 14)])
def test_group_best_fft_small_vs_oracle(oracle, G, log_n, length):
    """Zero padding (len < 2^log_n, down to an empty input), both directions, from sizes the group does not
    split (n < G^2: member 0 alone, and a one-member group) to sizes it does."""
    g = _group(G)
    try:
        c = O.random_elements(max(length, 1), 0x5EED0600 + log_n)[:length]
        w = O.root_of_unity(log_n)
        assert np.array_equal(g.best_fft(c, w, log_n), oracle.best_fft(c, w, log_n, cpus=8))
        assert np.array_equal(g.inv_best_fft(c, w, log_n), oracle.inv_best_fft(c, w, log_n, cpus=8))
    finally:
        g.close()


@pytest.mark.parametrize("G", [2, 4, 8])
def test_group_best_fft_2_20_vs_oracle(oracle, G):
    """Config 2's size: forward and inverse equal the oracle (and the committed digests)."""
    rec = BIG["ntt_2^20"]
    c = O.random_elements(1 << 20, 0x5EED0000 + 20)
    assert _sha(c) == rec["input_sha256"]
    w = O.root_of_unity(20)
    g = _group(G)
    try:
        fwd = g.best_fft(c, w, 20)
        assert _sha(fwd) == rec["forward_sha256"]
        inv = g.inv_best_fft(c, w, 20)
        assert _sha(inv) == rec["inverse_sha256"]
        if G == 8:
            assert np.array_equal(fwd, oracle.best_fft(c, w, 20, cpus=16))
    finally:
        g.close()


@pytest.mark.parametrize("G", [4, 8])
def test_group_best_fft_2_24_digest(G):
    """The bench's 2^24 input through the group equals the oracle's digests (forward and inverse)."""
    rec = BIG["ntt_2^24"]
    c = O.random_elements(1 << 24, 0x5EED0000 + 24)
    w = O.root_of_unity(24)
    g = _group(G)
    try:
        assert _sha(g.best_fft(c, w, 24)) == rec["forward_sha256"]
        assert _sha(g.inv_best_fft(c, w, 24)) == rec["inverse_sha256"]
    finally:
        g.close()


@pytest.mark.parametrize("G", [2, 8])
def test_group_ntt_dev_layout(oracle, G):
    """stark_group_ntt_dev's documented layout: cyclic shards in, member r holds X[r c + i + M k1] at
    k1 c + i; a second call on the same buffers (reused allocations) gives the same.  Device memory
    comes from the member contexts (stark_group_ctx + stark_dev_alloc)."""
    import ctypes
    log_n = 14
    n = 1 << log_n
    M, c = n // G, n // G // G
    x = O.random_elements(n, 0x5EED0700)
    w = O.root_of_unity(log_n)
    want = oracle.best_fft(x, w, log_n, cpus=8)
    g = _group(G)
    lib = g.lib
    bufs = []
    try:
        for r in range(G):
            for _ in range(2):
                p = ctypes.c_void_p()
                assert lib.stark_dev_alloc(g.ctx_handle(r), M * 32, ctypes.byref(p)) == 0
                bufs.append((r, p.value))
        shards = [bufs[2 * r][1] for r in range(G)]
        outs = [bufs[2 * r + 1][1] for r in range(G)]
        for _ in range(2):
            for r in range(G):
                src = np.ascontiguousarray(x[r::G])
                assert lib.stark_memcpy_h2d(g.ctx_handle(r), shards[r], src.ctypes.data, src.nbytes) == 0
            g.ntt_dev(shards, outs, log_n, w)
            g.synchronize()
            for r in range(G):
                got = np.empty((M, 4), dtype=np.uint64)
                assert lib.stark_memcpy_d2h(g.ctx_handle(r), got.ctypes.data, outs[r], got.nbytes) == 0
                got = got.reshape(G, c, 4)
                for k1 in range(G):
                    assert np.array_equal(got[k1], want[r * c + M * k1: r * c + M * k1 + c])
    finally:
        for r, p in bufs:
            lib.stark_dev_free(g.ctx_handle(r), p)
        g.close()


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("log_n,leaf_len", [(2, 32), (12, 32), (16, 256), (10, 40)])
def test_group_merkle_vs_oracle(oracle, G, log_n, leaf_len):
    """Root and paths equal the oracle's single tree (gen_multi_proofs_multi_core,
    merkle_proof_in_place.rs:106-206); n < G puts the tree on member 0; duplicates and caller order
    kept; get_root is empty before gen_proofs (merkle_tree.rs:66, H::default())."""
    n = 1 << log_n
    rng = np.random.default_rng(log_n * 131 + leaf_len + G)
    blob = rng.integers(0, 256, n * leaf_len, dtype=np.uint8).tobytes()
    idx = [0, n - 1, n // 2, 1 % n, n // 3, 0]
    root, paths = oracle.merkle(blob, n, leaf_len, idx, chunks=4)
    g = _group(G)
    try:
        t = g.merkle()
        t.update_bytes(blob, n, leaf_len)
        assert t.get_root() == b""
        proofs = t.gen_proofs(idx)
        assert t.get_root() == root
        assert [p.nodes for p in proofs] == paths
        assert [p.leaf for p in proofs] == [blob[i * leaf_len:(i + 1) * leaf_len] for i in idx]
        from stark_amd import verify_multi_branch
        verify_multi_branch(root, idx, proofs)
    finally:
        del t
        g.close()


@pytest.mark.parametrize("name,G", [("compute", 1), ("compute", 2), ("compute", 8), ("poseidon3_test", 4),
                                    ("pedersen_test", 2), ("pedersen_test", 8), ("bits", 4)])
def test_group_prove_vs_golden(name, G):
    """One proof over G members equals the golden StarkProof digest (BASELINE config 4: poseidon3 on 4)."""
    r1, wt = _fixture(name)
    g = _group(G)
    try:
        js = g.prove_with_witness(r1, wt).to_json()
        assert hashlib.sha256(js.encode()).hexdigest() == GOLD[name]["json_sha256"]
        js2 = g.prove_with_witness(r1, wt).to_json()   # the group's reused buffers and trees
        assert js2 == js
    finally:
        g.close()


@pytest.mark.parametrize("G", [2, 8])
def test_group_prepared_circuit(G):
    """A circuit prepared on every member; pedersen and a synthetic circuit with two witnesses."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth_r1cs
    from stark_amd import Context
    from stark_amd.r1cs import prove_with_witness
    g = _group(G)
    try:
        r1, wt = _fixture("pedersen_test")
        circ = g.circuit(r1)
        assert hashlib.sha256(circ.prove(wt).to_json().encode()).hexdigest() == GOLD["pedersen_test"]["json_sha256"]
        del circ
        r1, _ = synth_r1cs.for_steps(13)
        circ = g.circuit(r1)
        ctx = Context(0)
        try:
            for inputs in [(5, 6), (7, 8)]:
                _, wt = synth_r1cs.for_steps(13, inputs=inputs)
                assert circ.prove(wt).to_json() == prove_with_witness(ctx, r1, wt).to_json()
        finally:
            ctx.close()
        del circ
    finally:
        g.close()


@pytest.mark.parametrize("prepared", [False, True])
def test_group_prove_synth_2_20_vs_oracle_digest(prepared):
    """BASELINE config 5's stand-in at its size (2^20 steps, precision 2^23) over 8 members equals the
    oracle's StarkProof digest (tests/golden/large_digests.json)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth_r1cs
    want = BIG["prove_synth_2^20_steps"]["json_sha256"]
    r1, wt = synth_r1cs.for_steps(20)
    g = _group(8)
    try:
        if prepared:
            circ = g.circuit(r1)
            js = circ.prove(wt).to_json()
            del circ
        else:
            js = g.prove_with_witness(r1, wt).to_json()
        assert hashlib.sha256(js.encode()).hexdigest() == want
    finally:
        g.close()


def test_group_errors():
    """Reference panics become status codes: a bad member count, a non-power-of-two length, a bad root,
    proofs before update."""
    from stark_amd import StarkError
    from stark_amd.group import Group
    with pytest.raises(StarkError):
        Group([0, 0, 0])
    g = _group(2)
    try:
        c = O.random_elements(8, 1)
        with pytest.raises(StarkError) as e:
            g.best_fft(c, O.root_of_unity(3), 2)       # len > 2^log_n (fft.rs:162)
        assert e.value.code == 1
        with pytest.raises(StarkError) as e:
            g.best_fft(c, 5, 10)                        # not a primitive 2^10-th root
        assert e.value.code == 2
        t = g.merkle()
        with pytest.raises(StarkError) as e:
            t.gen_proofs([0])
        assert e.value.code == 7
        with pytest.raises(StarkError) as e:
            t.update_bytes(b"\0" * 96, 3, 32)           # merkle_proof_in_place.rs:113
        assert e.value.code == 1
        del t
    finally:
        g.close()
