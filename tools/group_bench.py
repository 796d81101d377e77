"""Device-group timings (include/stark_hip.h stark_group_*): one process drives G GPUs through the C ABI.

    python tools/group_bench.py --devices 0,1,2,3,4,5,6,7 [--log-shard 24] [--reps 5]

Prints one JSON object:
  * group_ntt_2^k: one 2^(log_shard + log2 G)-point transform per call (2^log_shard points per member,
    cyclic shards in HBM, stark_group_ntt_dev + stark_group_synchronize), host wall-clock per call
    (median), elements/s over the whole transform; its output checked against the plain one-GPU
    stark_ntt_dev of the same vector when that fits one member (log_shard + log2 G <= 26), member 0;
  * group_best_fft_2^20 / _2^24 digests vs tests/golden/large_digests.json (the host entry point);
  * group_merkle: 2^log_shard 32-B leaves per member (device blocks), root equal to member 0's single tree
    of the same leaves when they fit;
  * group_prove_*: pedersen_test (config 3) and poseidon3_test (config 4) and the synthetic 2^20-step
    circuit (config 5's stand-in), cold prove_with_witness over the group, digests vs the goldens.
No torch: the library's own device memory (stark_dev_alloc on the member contexts).  bench.py --gpus N
runs this on rank 0 over devices 0..N-1 (the other ranks wait on a CPU barrier); on the one-GPU test box
it runs with a repeated device (--devices 0,0,0,0), which times the code path, not a scaling figure.
"""
import argparse
import ctypes
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-pure-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def sha(b) -> str:
    return hashlib.sha256(b.tobytes() if hasattr(b, "tobytes") else b).hexdigest()


def med_wall(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0")
    ap.add_argument("--log-shard", type=int, default=24)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-prove", action="store_true")
    args = ap.parse_args()
    import oracle as O
    import stark_amd as S
    from stark_amd.group import Group
    devices = [int(x) for x in args.devices.split(",")]
    G = len(devices)
    log_g = G.bit_length() - 1
    out = {"group_devices": devices, "group_members": G,
           "group_transport": "peer copies pulled on member streams (hipMemcpyPeerAsync across devices, "
                              "device-to-device within one)"}
    big = json.load(open(os.path.join(ROOT, "tests", "golden", "large_digests.json")))
    g = Group(devices)
    lib = g.lib

    def alloc(r, nbytes):
        p = ctypes.c_void_p()
        g.check(lib.stark_dev_alloc(g.ctx_handle(r), nbytes, ctypes.byref(p)), "dev_alloc")
        return p.value

    def h2d(r, ptr, a):
        a = np.ascontiguousarray(a)
        g.check(lib.stark_memcpy_h2d(g.ctx_handle(r), ptr, a.ctypes.data, a.nbytes), "h2d")

    def d2h(r, a, ptr):
        g.check(lib.stark_memcpy_d2h(g.ctx_handle(r), a.ctypes.data, ptr, a.nbytes), "d2h")

    # ---- NTT: one 2^(log_shard + log G) transform, 2^log_shard points per member (weak scaling) ----
    ls = args.log_shard
    log_n = ls + log_g
    M = 1 << ls
    w = O.root_of_unity(log_n)
    rng = np.random.default_rng(log_n)
    shards, outs, hosts = [], [], []
    for r in range(G):
        x = rng.integers(0, 2**63, (M, 4), dtype=np.uint64)
        x[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
        hosts.append(x)
        shards.append(alloc(r, M * 32))
        outs.append(alloc(r, M * 32))
        h2d(r, shards[r], x)
    g.ntt_dev(shards, outs, log_n, w)     # warm: twiddle tables
    g.synchronize()
    for r in range(G):
        h2d(r, shards[r], hosts[r])
    g.ntt_dev(shards, outs, log_n, w)
    g.synchronize()
    if G > 1 and log_n <= 26:
        # the same vector (x[r + G j] = member r's j-th) transformed by member 0 alone
        full = np.empty((1 << log_n, 4), dtype=np.uint64)
        for r in range(G):
            full[r::G] = hosts[r]
        ref = np.empty_like(full)
        d = alloc(0, full.nbytes)
        try:
            h2d(0, d, full)
            c0 = g.ctx_handle(0)
            rl = S._limbs(w)
            g.check(lib.stark_ntt_dev(c0, d, log_n, 1, S._p64(rl), 0, None), "ntt_dev")
            g.check(lib.stark_ctx_synchronize(c0), "sync")
            d2h(0, ref, d)
        finally:
            lib.stark_dev_free(g.ctx_handle(0), d)
        c = M // G
        ok = True
        for r in range(G):
            got = np.empty((M, 4), dtype=np.uint64)
            d2h(r, got, outs[r])
            got = got.reshape(G, c, 4)
            for k1 in range(G):
                ok &= bool(np.array_equal(got[k1], ref[r * c + M * k1: r * c + M * k1 + c]))
        out[f"group_ntt_2^{log_n}_bitexact_vs_one_gpu"] = ok
        del full, ref

    def step():
        g.ntt_dev(shards, outs, log_n, w)
        g.synchronize()
    step()
    ms = med_wall(step, max(args.reps, 5))
    out[f"group_ntt_2^{log_n}_ms"] = round(ms, 4)
    out[f"group_ntt_2^{log_n}_elems_per_s"] = (1 << log_n) / (ms / 1000.0)
    out["group_ntt_timing"] = (f"host wall-clock median per call (stark_group_ntt_dev + stark_group_synchronize), "
                               f"2^{ls} points per member, input destroyed in place (timing only)")
    # ---- Merkle: 2^log_shard 32-B leaves per member ----
    t = g.merkle()
    n_leaves = M * G
    t.update_dev(outs, n_leaves, 32)
    t.gen_proofs([])
    root = t.get_root()
    ms = med_wall(lambda: t.update_dev(outs, n_leaves, 32), max(args.reps, 5))
    out[f"group_merkle_2^{log_n}x32B_ms"] = round(ms, 4)
    out[f"group_merkle_2^{log_n}x32B_leaves_per_s"] = n_leaves / (ms / 1000.0)
    if G > 1 and log_n <= 26:
        blob = np.empty((n_leaves, 4), dtype=np.uint64)
        for r in range(G):
            d2h(r, blob[r * M:(r + 1) * M], outs[r])
        # member 0's context as a plain single tree over all the leaves
        h = ctypes.c_void_p()
        g.check(lib.stark_merkle_new(g.ctx_handle(0), ctypes.byref(h)), "merkle_new")
        try:
            g.check(lib.stark_merkle_update(h, blob.tobytes(), n_leaves, 32), "merkle_update")
            g.check(lib.stark_merkle_gen_proofs(h, None, 0, None, None), "gen_proofs")
            r0 = ctypes.create_string_buffer(32)
            k = ctypes.c_size_t(0)
            lib.stark_merkle_get_root(h, r0, ctypes.byref(k))
            out[f"group_merkle_2^{log_n}_root_equals_single_tree"] = r0.raw == root
        finally:
            lib.stark_merkle_free(h)
        del blob
    del t
    for r in range(G):
        lib.stark_dev_free(g.ctx_handle(r), shards[r])
        lib.stark_dev_free(g.ctx_handle(r), outs[r])
    # ---- host entry points vs the oracle digests ----
    for k in (20, 24):
        rec = big[f"ntt_2^{k}"]
        x = O.random_elements(1 << k, 0x5EED0000 + k)
        wk = O.root_of_unity(k)
        out[f"group_best_fft_2^{k}_bitexact_vs_oracle_digest"] = sha(g.best_fft(x, wk, k)) == rec["forward_sha256"]
        out[f"group_inv_best_fft_2^{k}_bitexact_vs_oracle_digest"] = \
            sha(g.inv_best_fft(x, wk, k)) == rec["inverse_sha256"]
        if k == 24:
            hout = np.empty((1 << k, 4), dtype=np.uint64)  # a caller buffer, touched by the first call
            out["group_best_fft_host_2^24_ms_pcie_inclusive"] = round(
                med_wall(lambda: g.best_fft(x, wk, k, out=hout), 3), 2)
    # ---- proofs ----
    if not args.no_prove:
        fix = os.path.join(ROOT, "tests", "golden", "r1cs")
        golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))
        import synth_r1cs
        cases = [("pedersen", *(open(os.path.join(fix, f"pedersen_test.{e}"), "rb").read() for e in ("r1cs", "wtns")),
                  golden["pedersen_test"]["json_sha256"]),
                 ("poseidon3", *(open(os.path.join(fix, f"poseidon3_test.{e}"), "rb").read() for e in ("r1cs", "wtns")),
                  golden["poseidon3_test"]["json_sha256"])]
        rs, ws = synth_r1cs.for_steps(20)
        cases.append(("synth_2^20_steps", rs, ws, big["prove_synth_2^20_steps"]["json_sha256"]))
        for key, r1, wt, want in cases:
            js = g.prove_with_witness(r1, wt).to_json()
            out[f"group_prove_{key}_bitexact"] = sha(js.encode()) == want
            out[f"group_prove_{key}_ms"] = round(min(
                med_wall(lambda: g.prove_with_witness(r1, wt).to_json(), 1) for _ in range(3)), 3)
        c = g.circuit(rs)
        out["group_prove_synth_2^20_steps_prepared_bitexact"] = \
            sha(c.prove(ws).to_json().encode()) == big["prove_synth_2^20_steps"]["json_sha256"]
        out["group_prove_synth_2^20_steps_prepared_ms"] = round(min(
            med_wall(lambda: c.prove(ws).to_json(), 1) for _ in range(3)), 3)
        del c
        out["group_prove_timing"] = "host wall-clock, best of 3 (cold prove_with_witness / prepared circuit)"
    g.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
