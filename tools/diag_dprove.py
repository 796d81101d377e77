"""Diagnostic: repeat the world-G prepared (DistCircuit) proof of the synthetic 2^20-step circuit with every
rank on the one GPU (gloo), and on a mismatch against the single-GPU proof report which part of the
StarkProof differs (the JSON's top-level fields, and the first differing byte).

    python tools/diag_dprove.py [world 8] [runs 4] [prepared 1]
"""
import datetime
import hashlib
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]

from ranks import run_ranks  # noqa: E402


def _worker(rank, world, port, prepared, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=180))
    import stark_amd as S
    from stark_amd.dprove import DistCircuit, GpuProverOps, prove_distributed
    import synth_r1cs
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(0)
    r1, wt = synth_r1cs.for_steps(20)
    if prepared:
        circ = DistCircuit(ctx, r1)
        js = prove_distributed(GpuProverOps(ctx), None, wt, circuit=circ)
    else:
        circ = None
        js = prove_distributed(GpuProverOps(ctx), r1, wt)
    out_q.put((rank, js if rank == 0 else None))
    dist.barrier()
    del circ
    ctx.close()
    dist.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    prepared = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
    import stark_amd as S
    from stark_amd.r1cs import prove_with_witness
    import synth_r1cs
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "large_digests.json")))["prove_synth_2^20_steps"]
    ref = None
    for k in range(runs):
        res = dict(run_ranks(_worker, world, (prepared,), timeout=230))
        js = res[0]
        ok = hashlib.sha256(js.encode()).hexdigest() == want["json_sha256"]
        print(f"run {k}: world {world} prepared {prepared}: {'ok' if ok else 'MISMATCH'}", flush=True)
        if ok:
            continue
        if ref is None:
            ctx = S.Context(0)
            r1, wt = synth_r1cs.for_steps(20)
            ref = prove_with_witness(ctx, r1, wt).to_json()
            ctx.close()
        a, b = json.loads(js), json.loads(ref)
        for key in b:
            if a.get(key) != b[key]:
                va, vb = a.get(key), b[key]
                detail = ""
                if isinstance(vb, list) and isinstance(va, list):
                    idx = [i for i in range(min(len(va), len(vb))) if va[i] != vb[i]]
                    detail = f" (len {len(va)} vs {len(vb)}; {len(idx)} differing entries, first {idx[:5]})"
                print(f"  field {key!r} differs{detail}", flush=True)
        i = next((i for i in range(min(len(js), len(ref))) if js[i] != ref[i]), None)
        print(f"  first differing byte {i} of {len(ref)}: got {js[max(0, i - 40):i + 40]!r}", flush=True)


if __name__ == "__main__":
    main()
