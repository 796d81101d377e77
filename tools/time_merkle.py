"""Merkle build timings (MerkleProofInPlace::update on device leaves) for the bench's
leaf shapes: 2^24 x 32 B, 2^21 x 256 B, 2^20 x 40 B.  Prints one JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-pure-rust_amd"))
import stark_amd as S  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(0)
    n = 1 << 24
    buf = torch.randint(0, 2**62, (n, 4), dtype=torch.int64, device="cuda:0")
    tree = S.MerkleProofInPlace(ctx)
    out = {}
    for cnt, ll in ((n, 32), (n // 8, 256), (1 << 20, 40)):
        for _ in range(3):
            tree.update_dev(buf.data_ptr(), cnt, ll, stream=stream.cuda_stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            tree.update_dev(buf.data_ptr(), cnt, ll, stream=stream.cuda_stream)
        b.record(stream)
        b.synchronize()
        ms = a.elapsed_time(b) / reps
        out[f"2^{cnt.bit_length() - 1}x{ll}B"] = {"ms": round(ms, 4), "leaves_per_s": cnt / (ms / 1e3)}
    print(json.dumps(out))
    del tree
    ctx.close()


if __name__ == "__main__":
    main()
