"""Times the batched LDE (stark_lde_dev: iNTT over steps then the sparse NTT over
steps * 2^blowup) in isolation, per batch, for comparison with the prover's own
LDE launches (tools/time_r1cs.py under rocprofv3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import oracle as O  # noqa: E402  (roots only)
import stark_amd as S  # noqa: E402


def main():
    log_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    pad_gb = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0   # extra resident allocation (footprint test)
    ctx = S.Context(0)
    pad = torch.empty(int(pad_gb * (1 << 30)), dtype=torch.uint8, device="cuda") if pad_gb else None  # noqa: F841
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    g2 = O.root_of_unity(log_steps + 3)
    g1 = pow(g2, 8, O.P)
    for batch in (1, 2, 8):
        n = 1 << log_steps
        src = torch.randint(-2**63, 2**63 - 1, (batch * n, 4), dtype=torch.int64, device="cuda")
        src[:, 3] &= 0x0FFFFFFFFFFFFFFF
        work = src.clone()
        out = torch.empty((batch * n * 8, 4), dtype=torch.int64, device="cuda")
        f = lambda: (work.copy_(src), ctx.lde_dev(work.data_ptr(), out.data_ptr(), log_steps, 3, batch, g1, g2,  # noqa
                                                  stream=s.cuda_stream))
        for _ in range(3):
            f()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(10):
            f()
        b.record(s)
        b.synchronize()
        print(f"LDE 2^{log_steps} -> 2^{log_steps + 3} x {batch}: {a.elapsed_time(b) / 10:.3f} ms", flush=True)
        # The same after the GPU idled (host work between proofs): clock ramp-up effects.
        import time
        for idle in (0.0002, 0.001, 0.002, 0.005, 0.02):
            ts = []
            for _ in range(5):
                s.synchronize()
                time.sleep(idle)
                a.record(s)
                f()
                b.record(s)
                b.synchronize()
                ts.append(a.elapsed_time(b))
            print(f"   after {idle * 1e3:.1f} ms idle: {min(ts):.3f} .. {max(ts):.3f} ms", flush=True)
        del src, work, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
