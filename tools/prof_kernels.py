"""Workload for rocprofv3 counter passes (tools/pmc_round.sh): the bench's dominant kernels on
device-resident synthetic data, a few dispatches each, nothing else.
    WHAT=ntt|merkle|merkle32 (2^24 x 32-B trees alone)|all (default all) | prover (the synthetic 2^20-step proof, the sha256_2_test stand-in:
    REPS cold prove_with_witness calls, then REPS from a prepared circuit); REPS=5;
    STARK_LIB=<path> times another build of the library
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "stark-pure-rust_amd"))
import oracle as O  # noqa: E402  (synthetic input generator only)
import stark_amd as S  # noqa: E402


def main():
    what = os.environ.get("WHAT", "all")
    reps = int(os.environ.get("REPS", "5"))
    log_n = 24
    n = 1 << log_n
    if os.environ.get("STARK_LIB"):
        S.load_library(os.path.abspath(os.environ["STARK_LIB"]))
    ctx = S.Context(0)
    if what == "prover":
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import synth_r1cs
        from stark_amd.r1cs import R1csCircuit, prove_with_witness
        rs, ws = synth_r1cs.for_steps(int(os.environ.get("LOG_STEPS", "20")))
        for _ in range(reps):
            prove_with_witness(ctx, rs, ws).to_json()
        c = R1csCircuit(ctx, rs)
        for _ in range(reps):
            c.prove(ws).to_json()
        del c
        ctx.close()
        print("prof_kernels done", what, reps)
        return
    host = O.random_elements(n, 0x5EED0000 + log_n)
    d = ctx.alloc(n * 32)
    ctx.h2d(d, host)
    w = O.root_of_unity(log_n)
    if what in ("ntt", "all"):
        ctx.ntt_dev(d, log_n, 1, w)          # twiddle tables outside the counted steady state
        for _ in range(reps):
            ctx.ntt_dev(d, log_n, 1, w)
        ctx.synchronize()
    if what in ("merkle", "merkle32", "all"):
        t = S.MerkleProofInPlace(ctx)
        for _ in range(reps):
            t.update_dev(d, n, 32)
        for _ in range(reps if what != "merkle32" else 0):
            t.update_dev(d, n // 8, 256)
        ctx.synchronize()
        del t
    ctx.free(d)
    ctx.close()
    print("prof_kernels done", what, reps)


if __name__ == "__main__":
    main()
