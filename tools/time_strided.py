"""Times the one-exchange distributed NTT's local compute on one GPU (stark_amd/distributed.py
cyclic_ntt, no exchange): the rank's 2^24-point NTT (root w^G) alone, and followed by the cross-rank
G-point DFT with its fused twiddle (stark_ntt_strided_tw_dev) for G = 2, 4, 8 -- what one rank of
bench.py --gpus G computes per step besides the all-to-all.  Env: REPS (50)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-pure-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402  (input and roots only)
import stark_amd as S  # noqa: E402


def main():
    reps = int(os.environ.get("REPS", "50"))
    ctx = S.Context(0)
    log_m = 24
    M = 1 << log_m
    x = torch.from_numpy(O.random_elements(M, 0x5EED0000 + 27).view(np.int64).copy()).cuda()
    torch.cuda.synchronize()
    s = ctx.stream

    def timeit(fn):
        for _ in range(5):
            fn()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        ctx.synchronize()
        return (time.perf_counter() - t0) * 1000 / reps

    for G in (1, 2, 4, 8):
        log_g = G.bit_length() - 1
        log_n = log_m + log_g
        w = O.root_of_unity(log_n)
        wl = pow(w, G, O.P)
        c = M // G

        def step():  # receiver-side twiddle, fused into the strided DFT
            ctx.ntt_dev(x.data_ptr(), log_m, 1, wl, inverse=False, stream=s)
            if G > 1:
                ctx.ntt_strided_tw_dev(x.data_ptr(), log_g, c, pow(w, M, O.P), w, log_n, 0, inverse=False, stream=s)
        ms = timeit(step)
        print(f"G={G}: local 2^24 NTT{' + strided DFT with the twiddle' if G > 1 else ''}: {ms:.3f} ms", flush=True)
        if G > 1:
            ms2 = timeit(lambda: ctx.ntt_strided_tw_dev(x.data_ptr(), log_g, c, pow(w, M, O.P), w, log_n, 0,
                                                        inverse=False, stream=s))
            print(f"G={G}:   strided DFT with the twiddle alone: {ms2:.3f} ms", flush=True)

            def fused():  # the twiddle in the local NTT's last store (stark_cyclic_ntt_local_dev)
                ctx.cyclic_ntt_local_dev(x.data_ptr(), log_n, log_g, 3 % G, w, inverse=False, stream=s)
                ctx.ntt_strided_dev(x.data_ptr(), log_g, c, pow(w, M, O.P), inverse=False, stream=s)
            print(f"G={G}: fused local NTT + strided DFT: {timeit(fused):.3f} ms", flush=True)
            ms3 = timeit(lambda: ctx.cyclic_ntt_local_dev(x.data_ptr(), log_n, log_g, 3 % G, w, inverse=False,
                                                          stream=s))
            print(f"G={G}:   fused local NTT alone: {ms3:.3f} ms", flush=True)
            ms4 = timeit(lambda: ctx.ntt_strided_dev(x.data_ptr(), log_g, c, pow(w, M, O.P), inverse=False, stream=s))
            print(f"G={G}:   strided DFT alone: {ms4:.3f} ms", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
