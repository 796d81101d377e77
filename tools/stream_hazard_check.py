"""Cross-stream hazard check of a libstark_hip build: multi-pass NTTs on two
streams of ONE context, enqueued with no host synchronisation, against the same transforms run one at a
time.  Binds only stark_ctx_create / stark_ntt_dev / stark_ctx_destroy, so any build of the library
(e.g. the round-4 one, before its context buffers were ordered across streams) can be checked.

usage: python tools/stream_hazard_check.py <libstark_hip.so> [rounds]
Prints one JSON line: the mismatching transforms per round (fresh context: first use of each size on
both streams at once; warm: tables built beforehand)."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import oracle as O
    lib = ctypes.CDLL(sys.argv[1])
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    vp = ctypes.c_void_p
    lib.stark_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.stark_ntt_dev.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                  ctypes.c_int, vp]
    lib.stark_ctx_destroy.argtypes = [vp]
    torch.cuda.set_device(0)

    def ctx_new():
        h = vp()
        assert lib.stark_ctx_create(0, ctypes.byref(h)) == 0
        return h

    def root(l):
        w = O.root_of_unity(l)
        return (ctypes.c_uint64 * 4)(*[(w >> (64 * k)) & (2**64 - 1) for k in range(4)])

    def ntt(h, t, l, b, stream):
        assert lib.stark_ntt_dev(h, t.data_ptr(), l, b, root(l), 0, stream) == 0

    jobs = [(22, 2), (24, 1), (22, 2), (24, 1)]
    rng = np.random.default_rng(7)
    inputs = []
    for l, b in jobs:
        c = rng.integers(0, 2**64, size=(b << l, 4), dtype=np.uint64)
        c[:, 3] >>= np.uint64(4)
        inputs.append(torch.from_numpy(c.view(np.uint8).reshape(-1).copy()))
    dig = lambda t: hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()
    h = ctx_new()
    want = []
    for (l, b), x in zip(jobs, inputs):
        t = x.cuda()
        torch.cuda.synchronize()
        ntt(h, t, l, b, None)
        torch.cuda.synchronize()
        want.append(dig(t))
    lib.stark_ctx_destroy(h)
    out = {"lib": os.path.basename(sys.argv[1]), "rounds": rounds}
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for mode in ("fresh", "warm"):
        h = ctx_new()
        if mode == "warm":
            for l, b in jobs[:2]:
                ntt(h, torch.zeros((b << l) * 32, dtype=torch.uint8, device="cuda"), l, b, None)
            torch.cuda.synchronize()
        bad = []
        for rnd in range(rounds):
            ts = [x.cuda() for x in inputs]
            torch.cuda.synchronize()
            for i, ((l, b), t) in enumerate(zip(jobs, ts)):
                ntt(h, t, l, b, streams[(i + rnd) % 2].cuda_stream)
            torch.cuda.synchronize()
            bad.append([i for i, t in enumerate(ts) if dig(t) != want[i]])
        lib.stark_ctx_destroy(h)
        out[mode + "_mismatches_per_round"] = bad
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
