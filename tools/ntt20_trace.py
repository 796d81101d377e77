"""2^20 forward NTTs back to back on one stream, for a kernel trace (rocprofv3 --kernel-trace): the three
passes' durations against the gaps between them.   python tools/ntt20_trace.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]
import stark_amd as S  # noqa: E402
import oracle as O  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    ctx = S.Context(0)
    g = torch.Generator(device="cuda:0").manual_seed(20)
    t = torch.randint(-2**63, 2**63 - 1, (1 << 20, 4), dtype=torch.int64, device="cuda:0", generator=g)
    t[:, 3] &= 0x0FFFFFFFFFFFFFFF
    w = O.root_of_unity(20)
    s = torch.cuda.Stream()
    for _ in range(reps):
        ctx.ntt_dev(t.data_ptr(), 20, 1, w, inverse=False, stream=s.cuda_stream)
    s.synchronize()
    ctx.close()
    print("done", reps)


if __name__ == "__main__":
    main()
