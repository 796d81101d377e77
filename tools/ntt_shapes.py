"""Per-element cost of batched NTT shapes (stark_ntt_dev, forward, HBM-resident):
ps per element per radix-2 stage for batch x 2^log_n, to compare the LDE's
batched 2^23 transforms with the 2^24 headline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import oracle as O  # noqa: E402  (roots only)
import stark_amd as S  # noqa: E402


def main():
    ctx = S.Context(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    shapes = [(24, 1), (23, 2), (23, 8), (22, 16), (20, 64), (26, 1), (24, 4)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]]
    for log_n, batch in shapes:
        n = 1 << log_n
        t = torch.randint(-2**63, 2**63 - 1, (batch * n, 4), dtype=torch.int64, device="cuda")
        t[:, 3] &= 0x0FFFFFFFFFFFFFFF
        w = O.root_of_unity(log_n)
        f = lambda: ctx.ntt_dev(t.data_ptr(), log_n, batch, w, inverse=False, stream=s.cuda_stream)  # noqa: E731
        f()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(5):
            f()
        b.record(s)
        b.synchronize()
        ms = a.elapsed_time(b) / 5
        print(f"2^{log_n} x {batch}: {ms:.3f} ms, {ms * 1e9 / (batch * n * log_n):.2f} ps/elem/stage", flush=True)
        del t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
