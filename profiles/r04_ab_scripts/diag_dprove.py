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
    if os.environ.get("DIAG_POISON_TORCH"):  # every torch.empty / empty_like filled with 0xA5 bytes
        _empty, _empty_like = torch.empty, torch.empty_like

        def _poison(t):
            if t.numel() and t.is_contiguous():
                t.view(torch.uint8).fill_(0xA5)
            return t
        torch.empty = lambda *a, **k: _poison(_empty(*a, **k))
        torch.empty_like = lambda *a, **k: _poison(_empty_like(*a, **k))
    import stark_amd as S
    if os.environ.get("STARK_LIB"):
        S.load_library(os.environ["STARK_LIB"])
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
    hold = None
    if os.environ.get("DIAG_PARENT_GPU"):  # like pytest's session context: the parent holds a GPU context
        if os.environ.get("STARK_LIB"):
            S.load_library(os.environ["STARK_LIB"])
        hold = S.Context(0)
        r1h, wth = synth_r1cs.for_steps(14)
        prove_with_witness(hold, r1h, wth).to_json()
    for k in range(runs):
        alt = os.environ.get("DIAG_ALTERNATE")  # a cold proof before each prepared one, as the test file runs them
        if alt:
            res0 = dict(run_ranks(_worker, world, (False,), timeout=230))
            ok0 = hashlib.sha256(res0[0].encode()).hexdigest() == want["json_sha256"]
            print(f"run {k}: world {world} cold: {'ok' if ok0 else 'MISMATCH'}", flush=True)
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
