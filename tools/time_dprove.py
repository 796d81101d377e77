"""Times stark_amd.dprove.prove_distributed (one proof over all ranks) against the
single-GPU prover.  Run one rank per GPU:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/time_dprove.py [log_steps]
STARK_BENCH_BACKEND=gloo rehearses several ranks on one GPU; STARK_PROFILE=1 prints phases."""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import stark_amd as S  # noqa: E402
import synth_r1cs  # noqa: E402
from stark_amd.dprove import GpuProverOps, prove_distributed  # noqa: E402
from stark_amd.r1cs import prove_with_witness  # noqa: E402


def main():
    log_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    backend = os.environ.get("STARK_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = S.Context(local)
    ops = GpuProverOps(ctx)
    rs, ws = synth_r1cs.for_steps(log_steps)
    js = prove_distributed(ops, rs, ws)
    ts = []
    for _ in range(reps):
        dist.barrier()
        t0 = time.perf_counter()
        prove_distributed(ops, rs, ws)
        dist.barrier()
        ts.append(time.perf_counter() - t0)
    if rank == 0:
        single = prove_with_witness(ctx, rs, ws).to_json()
        t1 = time.perf_counter()
        prove_with_witness(ctx, rs, ws).to_json()
        t_single = time.perf_counter() - t1
        print(f"2^{log_steps} steps, {world} ranks ({backend}): distributed {1e3 * min(ts):.2f} ms, "
              f"single GPU {1e3 * t_single:.2f} ms, identical={hashlib.sha256(js.encode()).digest() == hashlib.sha256(single.encode()).digest()}")
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
