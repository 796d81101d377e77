"""Same-process A/B of libstark_hip builds (the one parameterised A/B driver; variants are built by
tools/build_variant.sh into variants/, which is git-ignored).

Each build is loaded with its own ctypes handle and context; the timed loops alternate between the
builds in rounds so that clock and thermal drift hit every build alike.  For each build and case it
prints the median ms per call and a digest of the output, which must agree across builds.

usage: python tools/ab_libs.py [--cases ntt20,ntt24,ntt26,intt24,lde20] [--reps 30] [--rounds 5] lib.so ...
"""
import argparse
import ctypes
import hashlib
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

vp = ctypes.c_void_p
u64p = ctypes.POINTER(ctypes.c_uint64)


def bind(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.stark_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.stark_ntt_dev.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, u64p, ctypes.c_int, vp]
    lib.stark_ctx_destroy.argtypes = [vp]
    h = vp()
    assert lib.stark_ctx_create(0, ctypes.byref(h)) == 0
    return lib, h


def limbs(x):
    return (ctypes.c_uint64 * 4)(*[(x >> (64 * k)) & (2**64 - 1) for k in range(4)])


def make_case(name):
    """(log_n, batch, inverse) of a case name: ntt20 = forward 2^20, intt24 = inverse 2^24, ntt20x8 ..."""
    inv = name.startswith("i")
    body = name[4:] if inv else name[3:]
    log_n, _, batch = body.partition("x")
    return int(log_n), int(batch or 1), inv


def main():
    import oracle as O
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="ntt20,ntt24")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    builds = [bind(p) for p in a.libs]
    out = {"libs": [os.path.basename(p) for p in a.libs], "cases": {}}
    for case in a.cases.split(","):
        log_n, batch, inv = make_case(case)
        n = batch << log_n
        rng = np.random.default_rng(log_n)
        x = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
        x[:, 3] >>= np.uint64(4)
        src = torch.from_numpy(x.view(np.uint8).reshape(-1).copy()).cuda()
        bufs = [torch.empty_like(src) for _ in builds]
        root = limbs(O.root_of_unity(log_n))
        digests = []
        for (lib, h), b in zip(builds, bufs):  # warm-up and output digest
            b.copy_(src)
            assert lib.stark_ntt_dev(h, b.data_ptr(), log_n, batch, root, int(inv), stream.cuda_stream) == 0
            torch.cuda.synchronize()
            digests.append(hashlib.sha256(b.cpu().numpy().tobytes()).hexdigest()[:16])
        times = [[] for _ in builds]
        for _ in range(a.rounds):
            for i, ((lib, h), b) in enumerate(zip(builds, bufs)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.reps):
                    lib.stark_ntt_dev(h, b.data_ptr(), log_n, batch, root, int(inv), stream.cuda_stream)
                e1.record()
                e1.synchronize()
                times[i].append(e0.elapsed_time(e1) / a.reps)
        out["cases"][case] = {"ms_median": [round(statistics.median(t), 4) for t in times],
                              "ms_min": [round(min(t), 4) for t in times], "digest": digests,
                              "digests_equal": len(set(digests)) == 1}
        print(json.dumps({case: out["cases"][case]}), flush=True)
    for lib, h in builds:
        lib.stark_ctx_destroy(h)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
