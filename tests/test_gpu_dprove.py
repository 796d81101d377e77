"""GPU: one StarkProof shared by `world` ranks (stark_amd/dprove.py with
libstark_hip's per-rank steps).  On the one-GPU test box the ranks share GPU 0
and exchange through gloo; the 8-GPU bench runs the same code over RCCL.
The proof must equal the single-GPU / oracle proof byte for byte."""
import datetime
import hashlib
import json
import os
import sys

import pytest
import torch
import torch.distributed as dist
from ranks import run_ranks

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "r1cs")


def _worker(rank, world, port, name, log_synth, tail_log, out_q):
    import faulthandler
    faulthandler.dump_traceback_later(90, exit=True)   # a stuck rank prints its stack and exits
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=80))
    import stark_amd as S
    from stark_amd.dprove import GpuProverOps, prove_distributed
    from stark_amd.r1cs import prove_with_witness
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(0)
    if name:
        r1 = open(os.path.join(FIX, f"{name}.r1cs"), "rb").read()
        wt = open(os.path.join(FIX, f"{name}.wtns"), "rb").read()
    else:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import synth_r1cs
        r1, wt = synth_r1cs.for_steps(log_synth)
    js = prove_distributed(GpuProverOps(ctx), r1, wt, fri_tail_log=tail_log)
    single = prove_with_witness(ctx, r1, wt).to_json() if rank == 0 and not name else None
    digest = lambda s: hashlib.sha256(s.encode()).hexdigest() if s is not None else None
    out_q.put((rank, digest(js), digest(single)))
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


def _run(world, name, log_synth=0, tail_log=16):
    res = {r: (a, b) for r, a, b in run_ranks(_worker, world, (name, log_synth, tail_log), timeout=110)}
    assert all(res[r][0] is None for r in range(1, world))
    return res[0]


@pytest.mark.parametrize("name,world,tail_log", [("compute", 2, 0), ("compute", 8, 16), ("poseidon3_test", 4, 0),
                                                 ("pedersen_test", 2, 16), ("pedersen_test", 8, 12), ("bits", 4, 0)])
def test_prove_distributed_gpu(name, world, tail_log):
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))
    got, _ = _run(world, name, tail_log=tail_log)
    assert got == golden[name]["json_sha256"]


@pytest.mark.parametrize("world", [1, 4])
def test_prove_distributed_gpu_synthetic(world):
    """A 2^14-step synthetic circuit: the distributed proof equals the single-GPU proof."""
    got, single = _run(world, None, 14)
    assert got == single


def _worker_circuit(rank, world, port, out_q):
    import faulthandler
    faulthandler.dump_traceback_later(90, exit=True)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=80))
    import stark_amd as S
    from stark_amd.dprove import DistCircuit, GpuProverOps, prove_distributed
    from stark_amd.r1cs import prove_with_witness
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth_r1cs
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(0)
    r1, _ = synth_r1cs.for_steps(13)
    circ = DistCircuit(ctx, r1)
    got = []
    for inputs in [(5, 6), (7, 8)]:
        _, wt = synth_r1cs.for_steps(13, inputs=inputs)
        js = prove_distributed(GpuProverOps(ctx), None, wt, circuit=circ)
        if rank == 0:
            got.append(hashlib.sha256(js.encode()).hexdigest() ==
                       hashlib.sha256(prove_with_witness(ctx, r1, wt).to_json().encode()).hexdigest())
    r1p, wtp = open(os.path.join(FIX, "pedersen_test.r1cs"), "rb").read(), open(os.path.join(FIX, "pedersen_test.wtns"), "rb").read()
    js = prove_distributed(GpuProverOps(ctx), None, wtp, circuit=DistCircuit(ctx, r1p))
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))
    if rank == 0:
        got.append(hashlib.sha256(js.encode()).hexdigest() == golden["pedersen_test"]["json_sha256"])
    out_q.put((rank, got))
    dist.barrier()
    del circ
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 4])
def test_prove_distributed_prepared_circuit(world):
    """DistCircuit: two witnesses of one synthetic circuit equal the single-GPU proofs; pedersen_test
    equals the golden digest."""
    res = dict(run_ranks(_worker_circuit, world, (), timeout=110))
    assert res[0] == [True, True, True]


def _worker_synth20(rank, world, port, prepared, out_q):
    """The sha256_2_test stand-in (synthetic 2^20-step circuit, precision 2^23) through the multi-rank
    prover: rank 0's StarkProof JSON digest, to be compared with the oracle's
    (tests/golden/large_digests.json, mk_r1cs_proof restated in oracle/r1cs.c, prove.rs:14-378)."""
    import faulthandler
    faulthandler.dump_traceback_later(200, exit=True)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=180))
    import stark_amd as S
    from stark_amd.dprove import DistCircuit, GpuProverOps, prove_distributed
    sys.path.insert(0, os.path.join(ROOT, "tools"))
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


def _differing_fields(js, ctx):
    """On a wrong digest: which StarkProof fields differ from the single-GPU proof, and where."""
    from stark_amd.r1cs import prove_with_witness
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth_r1cs
    r1, wt = synth_r1cs.for_steps(20)
    a, b = json.loads(js), json.loads(prove_with_witness(ctx, r1, wt).to_json())
    out = []
    for key in b:
        if a.get(key) != b[key]:
            va, vb = a.get(key), b[key]
            if isinstance(va, list) and isinstance(vb, list):
                idx = [i for i in range(min(len(va), len(vb))) if va[i] != vb[i]]
                out.append(f"{key}: {len(idx)} of {len(vb)} entries differ, first {idx[:6]}")
            else:
                out.append(f"{key}: differs")
    return "; ".join(out)


@pytest.mark.parametrize("world,prepared", [(4, False), (8, False), (8, True)])
def test_prove_distributed_synth_2_20_vs_oracle_digest(world, prepared):
    """BASELINE config 5's stand-in at its size: one proof of the synthetic 2^20-step circuit over
    `world` ranks (cold, and from a DistCircuit) equals the oracle's StarkProof byte for byte
    (the digest tests/test_gpu_large.py pins the single-GPU prover to)."""
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "large_digests.json")))["prove_synth_2^20_steps"]
    res = dict(run_ranks(_worker_synth20, world, (prepared,), timeout=230))
    got = hashlib.sha256(res[0].encode()).hexdigest()
    if got != want["json_sha256"]:
        import stark_amd as S
        c = S.Context(0)
        try:
            detail = _differing_fields(res[0], c)
        finally:
            c.close()
        pytest.fail(f"digest {got} != {want['json_sha256']}: {detail}")
