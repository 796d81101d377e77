"""GPU: one context driven from two streams with no host synchronisation between the calls, the way
the distributed prover drives it (its circuit on the context stream, its proof steps on the caller's
torch stream, the FRI tail back on the context stream).  Every result must equal the one the same
call gives alone: the context's shared buffers (the NTT ping-pong, the batch inverse's scratch, the
fold's special_x slot) and its lazily filled tables (the last pass's full twiddle table) are ordered
across streams by the library (csrc/api.hip buf_acquire / fill_wait).

Reference: fft.rs:150-251 (the transform), fri.rs:135-164 (the fold), prove.rs:14-378 (the proof)."""
import datetime
import hashlib
import json
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
from ranks import run_ranks

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "r1cs")


def _rand(n, seed):
    """n uniform elements below 2^252 < p as a (n, 4) uint64 array."""
    c = np.random.default_rng(seed).integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    c[:, 3] >>= np.uint64(4)
    return c


def _dev(a: np.ndarray) -> torch.Tensor:
    """The elements as a device byte tensor (32 B each)."""
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()


def _host(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64).reshape(-1, 4)


def test_ntt_two_streams_oracle_small(ctx, oracle):
    """2^12 forward on stream A and 2^13 inverse on stream B, enqueued back to back: both equal the
    oracle (fft.rs:150-251)."""
    import oracle as O
    a, b = _rand(1 << 12, 1), _rand(1 << 13, 2)
    wa, wb = O.root_of_unity(12), O.root_of_unity(13)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ta, tb = _dev(a), _dev(b)
    torch.cuda.synchronize()
    ctx.ntt_dev(ta.data_ptr(), 12, 1, wa, inverse=False, stream=sa.cuda_stream)
    ctx.ntt_dev(tb.data_ptr(), 13, 1, wb, inverse=True, stream=sb.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(_host(ta), oracle.best_fft(a, wa, 12, cpus=4))
    assert np.array_equal(_host(tb), oracle.inv_best_fft(b, wb, 13, cpus=4))


@pytest.mark.parametrize("fresh", [True, False])
def test_ntt_two_streams_shared_scratch_and_full_table(fresh):
    """Multi-pass transforms (2^22 x 2 and 2^24, each with a last-pass full table) on two streams
    of one context, several rounds with no host synchronisation: equal to the same transforms run
    alone.  fresh: the first use of each size happens on the two streams at once (stream A's call
    publishes the full table while its fill is still queued; stream B's call must wait for it)."""
    import oracle as O
    import stark_amd as S
    jobs = [(22, 2, 11), (24, 1, 12), (22, 2, 13), (24, 1, 14)]
    inputs = [_rand(b << l, seed) for l, b, seed in jobs]
    roots = {l: O.root_of_unity(l) for l, _, _ in jobs}
    # The reference results: each transform alone on the context stream of its own context.
    ref_ctx = S.Context(0)
    want = []
    try:
        for (l, b, _), x in zip(jobs, inputs):
            t = _dev(x)
            torch.cuda.synchronize()
            ref_ctx.ntt_dev(t.data_ptr(), l, b, roots[l])
            ref_ctx.synchronize()
            want.append(hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest())
    finally:
        ref_ctx.close()
    c = S.Context(0)
    try:
        if not fresh:  # tables built and complete before the concurrent rounds
            for l, b, _ in jobs[:2]:
                t = torch.zeros((b << l) * 32, dtype=torch.uint8, device="cuda")
                c.ntt_dev(t.data_ptr(), l, b, roots[l])
            c.synchronize()
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for rnd in range(3):
            ts = [_dev(x) for x in inputs]
            torch.cuda.synchronize()
            for i, ((l, b, _), t) in enumerate(zip(jobs, ts)):
                s = streams[(i + rnd) % 2]
                c.ntt_dev(t.data_ptr(), l, b, roots[l], stream=s.cuda_stream)
            torch.cuda.synchronize()
            got = [hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest() for t in ts]
            assert got == want, f"round {rnd}: transforms differ from their single-stream results"
    finally:
        c.close()


def test_fold_then_context_stream_fri(ctx):
    """The distributed fold on a torch stream (special_x in the context's slot 15) followed at once by
    prove_low_degree on the context stream (slots 0-14) and another fold: every output equals the
    same call run alone (fri.rs:135-164, 46-224)."""
    import oracle as O
    log_n = 14
    n = 1 << log_n
    w = O.root_of_unity(log_n)
    vals = _rand(n, 21)
    root_a, root_b = bytes(range(32)), bytes(range(100, 132))
    s = torch.cuda.Stream()

    def fold(root_bytes, stream):
        v = _dev(vals)
        col = torch.empty(n // 4 * 32, dtype=torch.uint8, device="cuda")
        r = torch.tensor(list(root_bytes), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        from stark_amd import _limbs, _p64
        rl = _limbs(w)
        ctx.check(ctx.lib.stark_fri_fold_dev_root(ctx.h, v.data_ptr(), col.data_ptr(), n, _p64(rl), r.data_ptr(),
                                                  1, 0, stream), "fri_fold")
        return v, col, r

    # alone
    _, c1, _ = fold(root_a, s.cuda_stream)
    torch.cuda.synchronize()
    want_fold = _host(c1).copy()
    want_fri = ctx.prove_low_degree(vals, w, n // 4, 8).to_json()
    # back to back across the two streams
    keep = fold(root_a, s.cuda_stream)
    got_fri = ctx.prove_low_degree(vals, w, n // 4, 8).to_json()
    keep2 = fold(root_a, s.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(_host(keep[1]), want_fold)
    assert np.array_equal(_host(keep2[1]), want_fold)
    assert got_fri == want_fri
    _, c3, _ = fold(root_b, s.cuda_stream)
    torch.cuda.synchronize()
    assert not np.array_equal(_host(c3), want_fold)  # special_x really comes from the root


def _worker_streams(rank, world, port, out_q):
    """One rank: a DistCircuit built on the context stream, then proofs begun on two different torch
    streams and on the context stream, back to back (prepared and cold), each compared with the
    golden digest / the single-GPU proof."""
    import faulthandler
    faulthandler.dump_traceback_later(100, exit=True)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    import stark_amd as S
    from stark_amd.dprove import DistCircuit, GpuProverOps, prove_distributed
    torch.cuda.set_device(0)
    ctx = S.Context(0)
    r1 = open(os.path.join(FIX, "pedersen_test.r1cs"), "rb").read()
    wt = open(os.path.join(FIX, "pedersen_test.wtns"), "rb").read()
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))["pedersen_test"]["json_sha256"]
    circ = DistCircuit(ctx, r1)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    got = []
    for stream, prepared in [(sa, True), (sb, True), (sa, False), (None, True), (sb, False)]:
        with torch.cuda.stream(stream if stream is not None else torch.cuda.default_stream()):
            js = prove_distributed(GpuProverOps(ctx), None if prepared else r1, wt, fri_tail_log=12,
                                   circuit=circ if prepared else None)
        if rank == 0:
            got.append(hashlib.sha256(js.encode()).hexdigest() == golden)
    out_q.put((rank, got))
    dist.barrier()
    del circ
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_prove_distributed_across_streams(world):
    """pedersen_test through prove_distributed five times from one context, alternating the stream the
    proof's steps run on (two torch streams and the default one) and the prepared / cold path: every
    proof equals the golden StarkProof digest (prove.rs:14-378, run.rs:310-452)."""
    res = dict(run_ranks(_worker_streams, world, (), timeout=110))
    assert res[0] == [True] * 5
