"""GPU parity of the opt-in radix-2^29 NTT kernels (run with STARK_NTT29=1; tests/test_gpu_ntt29.py):
forward / inverse best_fft against the oracle at every pass plan from 2^2 to 2^20 (one to three
passes, odd and even radices), batched device transforms, and the LDE's sparse first pass
(inv_best_fft + zero padding + best_fft, prove.rs:100-101).  Exit status 0 when all agree."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402  (the checker)
import stark_amd as S  # noqa: E402


def main():
    assert os.environ.get("STARK_NTT29") == "1"
    ctx = S.Context(0)
    o = O.Oracle()
    bad = []
    for log_n in list(range(2, 19)) + [20]:
        w = O.root_of_unity(log_n)
        c = O.random_elements(1 << log_n, 0x2900 + log_n)
        want = o.best_fft(c, w, log_n, cpus=8)
        if not np.array_equal(ctx.best_fft(c, w, log_n), want):
            bad.append(f"fwd 2^{log_n}")
        if not np.array_equal(ctx.inv_best_fft(want, w, log_n), c):
            bad.append(f"inv 2^{log_n}")
    for log_steps, log_blowup in ((6, 3), (10, 3), (13, 3), (16, 3)):
        log_prec = log_steps + log_blowup
        g2 = O.root_of_unity(log_prec)
        g1 = pow(g2, 1 << log_blowup, O.P)
        v = O.random_elements(1 << log_steps, 0x2a00 + log_prec)
        want = o.best_fft(o.inv_best_fft(v, g1, log_steps, cpus=8), g2, log_prec, cpus=8)
        if not np.array_equal(ctx.lde(v, g1, log_blowup, g2), want):
            bad.append(f"lde 2^{log_steps}x{1 << log_blowup}")
    ctx.close()
    print("ntt29 parity:", "ok" if not bad else "MISMATCH " + ", ".join(bad), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
