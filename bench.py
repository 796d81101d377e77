"""Benchmark of the FRI-prover hot path on MI355X (BASELINE.json metric:
"2^24-pt NTT field-elems/sec + Merkle leaves/sec; end-to-end proof wall-clock").

A step is one forward NTT over BN254 Fr on HBM-resident synthetic data
(BASELINE.md generator) with 2^24 points per GPU.  `value` = field elements of
the transform per second.  The N=1 line also carries the Merkle leaves/s (2^24
32-B leaves), the 2^20 forward+inverse pair (config 2) and an FRI prove
wall-clock.

N > 1 GPUs: one process per GPU (torch.distributed.run, backend "nccl" = RCCL);
the GPUs jointly transform ONE 2^(24+log2 N)-point vector with the one-exchange
distributed NTT (stark_amd/distributed.py `cyclic_ntt`: cyclic distribution in,
chunked out; local 2^24-point NTT + twiddle, one RCCL all-to-all over xGMI,
local N-point DFTs).  Per-GPU work is fixed, so scaling is weak; timing is
barrier-bracketed and the max over ranks is used.
"""
import argparse
import datetime
import hashlib
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "stark-pure-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

S = None  # stark_amd, imported in main() once this process is known to be a rank

HBM_PEAK_GBS = 8000.0          # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
# Issue cost of a wave64 VALU instruction on a 16-lane SIMD: one quad-cycle.  The hardware's own count
# of VALU quad-cycles (SQ_ACTIVE_INST_VALU) equals SQ_INSTS_VALU on these kernels, and the measured
# mixed streams (64-bit mads, carry chains, alignbit/xor) issue at 4.0 cycles per instruction
# (tools/microbench/mix_rates.hip, profiles/r02_mix_rates.txt).
ISSUE_CYCLES = 4.0
SIMDS = 1024
# The constant products alone with their constants in LDS, 4 waves/SIMD, same run
# (tools/microbench/db_rate.hip, profiles/r02_db_product.txt): Shoup 138.7 G/s, digit basis 200.0 G/s.
SHOUP_PRODUCT_PEAK = 138.71e9
DB_PRODUCT_PEAK = 199.98e9
LOG_N = 24
PROFILE = os.path.join(ROOT, "profiles", "r06_summary.json")
PMC = os.path.join(ROOT, "profiles", "r06_pmc_ntt.json")
LARGE = os.path.join(ROOT, "tests", "golden", "large_digests.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--log-n", type=int, default=LOG_N)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks and rendezvous only (CPU test of the --gpus N launcher)")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args) -> int | None:
    """`bench.py --gpus N` with N > 1 and no launcher around it: start torch.distributed.run as a
    CHILD process (one rank per GPU, rendezvous on 127.0.0.1) before anything touches the GPU, wait,
    and hand back its exit code (its stdout, the rank-0 JSON line, is inherited).  Under a launcher
    the requested N must be the world it started.  Returns None when this process is a rank."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus <= 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.run(cmd).returncode
    if int(world) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    return None


def sha256(a) -> str:
    if isinstance(a, str):
        a = a.encode()
    elif isinstance(a, np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.uint64).tobytes()
    return hashlib.sha256(a).hexdigest()


def large_digests() -> dict:
    try:
        return json.load(open(LARGE))
    except (OSError, ValueError):
        return {}


def host_cpus():
    """(physical cores of the host, CPUs this process may use).  The reference's Worker::new takes
    num_cpus::get_physical() threads and parallel_fft splits into 2^floor(log2) of them
    (multicore.rs:43-45, fft.rs:332-351); the GPU box grants one job a share of the host (its
    OMP_NUM_THREADS), so the baseline uses the smaller of the two."""
    phys = set()
    cur = {}
    try:
        for line in open("/proc/cpuinfo"):
            if ":" in line:
                k, v = (x.strip() for x in line.split(":", 1))
                cur[k] = v
            elif cur:
                phys.add((cur.get("physical id", "0"), cur.get("core id", cur.get("processor"))))
                cur = {}
        if cur:
            phys.add((cur.get("physical id", "0"), cur.get("core id", cur.get("processor"))))
    except OSError:
        pass
    physical = len(phys) or (os.cpu_count() or 1)
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or allowed
    return physical, min(allowed, share)


def synthetic(n, seed):
    import oracle as O  # the synthetic generator only; not the checker here
    return O.random_elements(n, seed)


def timed_events(fn, stream, reps):
    """Average ms per call of fn() on `stream`, HIP events around the region."""
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record(stream)
    for _ in range(reps):
        fn()
    end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / reps


def steady_ms(fn, stream, target_ms=60.0):
    """Average ms per call of fn() at a steady clock: the card ramps its clock up from idle over
    several ms (profiles/r03_clock_ramp_probe.txt: a 2^24 NTT reads 2.0 ms over 5 calls after idle,
    1.63 ms over 50), so ~30 ms of untimed calls first, then timed_events over >= target_ms."""
    fn()
    one = max(timed_events(fn, stream, 1), 1e-3)
    for _ in range(max(2, int(30.0 / one))):
        fn()
    return timed_events(fn, stream, max(5, int(target_ms / one)))


def median_ms(fn, stream, reps=25, warm=3):
    """BASELINE.md's timing: the median of `reps` (>= 20) timed calls after `warm` untimed ones, each
    call bracketed by its own HIP event pair on `stream` (the launch stream), after ~30 ms of untimed
    calls so the clock has ramped (steady_ms).  Returns (median ms, [every call's ms])."""
    fn()
    one = max(timed_events(fn, stream, 1), 1e-3)
    for _ in range(max(warm, int(30.0 / one))):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    ev[-1][1].synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2] if len(ts) % 2 else 0.5 * (ts[len(ts) // 2 - 1] + ts[len(ts) // 2]), ts


def median_host_ms(fn, reps=21, warm=3):
    """Host-to-host median of `reps` calls of a synchronous fn (host buffers in and out)."""
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1000.0)
    ts.sort()
    return ts[len(ts) // 2]


def _smi_power():
    """(socket power W, power cap W, sclk MHz) from rocm-smi, or None (a child process, never exec)."""
    import re
    try:
        out = subprocess.run(["rocm-smi", "--showpower", "--showmaxpower", "--showclocks", "--json"],
                             capture_output=True, text=True, timeout=15).stdout
        card = next(iter(json.loads(out).values()))
        pw = float(next(v for k, v in card.items() if "Package Power" in k and "Max" not in k))
        cap = next((float(v) for k, v in card.items() if "Max" in k and "Power" in k), None)
        sclk = int(re.search(r"\((\d+)Mhz", card["sclk clock speed:"]).group(1))
        return pw, cap, sclk
    except Exception:  # noqa: BLE001  (no rocm-smi or an unexpected format: no power figure)
        return None


def power_under_load(step, sync, secs=2.5):
    """Board power and shader clock while `step` runs back to back (tools/power_probe.py): the NTT
    pass kernels run at the package power limit, which is what sets their clock."""
    import statistics
    import threading
    samples, stop = [], threading.Event()

    def sampler():
        time.sleep(0.8)
        while not stop.is_set():
            r = _smi_power()
            if r:
                samples.append(r)
            time.sleep(0.3)

    th = threading.Thread(target=sampler)
    th.start()
    t0 = time.time()
    while time.time() - t0 < secs:
        for _ in range(20):
            step()
        sync()
    stop.set()
    th.join()
    if not samples:
        return None
    pw = statistics.median(x[0] for x in samples)
    cap = samples[0][1]
    out = {"board_power_w": pw, "power_cap_w": cap, "sclk_mhz": statistics.median(x[2] for x in samples),
           "samples": len(samples), "source": "rocm-smi --showpower --showmaxpower --showclocks"}
    if cap:
        out["power_frac"] = round(pw / cap, 3)
    return out


def end_to_end(ctx):
    """prove_with_witness wall-clock on the reference's pedersen_test fixture and on a
    synthetic 2^20-step circuit (stand-in for sha256_2_test, whose .r1cs is not shipped)."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth_r1cs
    from stark_amd.r1cs import prove_with_witness
    fix = os.path.join(ROOT, "tests", "golden", "r1cs")
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))
    out = {}
    big = large_digests().get("prove_synth_2^20_steps", {})

    def synth_ms(reps):
        rs, ws = synth_r1cs.for_steps(20)
        js20 = prove_with_witness(ctx, rs, ws).to_json()
        if big:
            out["prove_synth_2^20_steps_bitexact_vs_oracle_digest"] = sha256(js20) == big.get("json_sha256")
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            prove_with_witness(ctx, rs, ws).to_json()
            ts.append(time.perf_counter() - t0)
        return min(ts) if ts else None

    # One untimed pass first: the multi-MB host buffers of the trace and the JSON only stop
    # page-faulting once glibc's dynamic mmap threshold has grown past them (it grows when such
    # a chunk is freed), as in any long-running prover process.
    synth_ms(0)
    r1 = open(os.path.join(fix, "pedersen_test.r1cs"), "rb").read()
    wt = open(os.path.join(fix, "pedersen_test.wtns"), "rb").read()
    js = prove_with_witness(ctx, r1, wt).to_json()
    out["prove_pedersen_bitexact_vs_golden"] = \
        hashlib.sha256(js.encode()).hexdigest() == golden["pedersen_test"]["json_sha256"]
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        prove_with_witness(ctx, r1, wt).to_json()
        ts.append(time.perf_counter() - t0)
    out["prove_pedersen_ms"] = round(min(ts) * 1000.0, 3)
    for name in ("compute", "poseidon3_test"):          # configs 1 and 4 (single GPU), bit-exact
        r1n = open(os.path.join(fix, f"{name}.r1cs"), "rb").read()
        wtn = open(os.path.join(fix, f"{name}.wtns"), "rb").read()
        jsn = prove_with_witness(ctx, r1n, wtn).to_json()
        tn = []
        for _ in range(5):
            t0 = time.perf_counter()
            prove_with_witness(ctx, r1n, wtn).to_json()
            tn.append(time.perf_counter() - t0)
        short = name.split("_")[0]
        out[f"prove_{short}_ms"] = round(min(tn) * 1000.0, 3)
        out[f"prove_{short}_bitexact_vs_golden"] = \
            hashlib.sha256(jsn.encode()).hexdigest() == golden[name]["json_sha256"]
    out["prove_synth_2^20_steps_ms"] = round(synth_ms(3) * 1000.0, 3)
    # The same proofs from a prepared circuit (R1csCircuit: the .r1cs-only work, including the LDEs of
    # K, F0-F2, IDX, PIDX, done once outside the timed region): a prover serving many witnesses of
    # one circuit.  Labelled separately; the lines above are the cold prove_with_witness.
    from stark_amd.r1cs import R1csCircuit

    def prepared_ms(r1b, wtb, reps):
        c = R1csCircuit(ctx, r1b)
        c.prove(wtb).to_json()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            c.prove(wtb).to_json()
            ts.append(time.perf_counter() - t0)
        return round(min(ts) * 1000.0, 3), c
    out["prove_pedersen_prepared_circuit_ms"], c = prepared_ms(r1, wt, 5)
    out["prove_pedersen_prepared_circuit_bitexact"] = \
        hashlib.sha256(c.prove(wt).to_json().encode()).hexdigest() == golden["pedersen_test"]["json_sha256"]
    del c
    rs, ws = synth_r1cs.for_steps(20)
    out["prove_synth_2^20_steps_prepared_circuit_ms"], c = prepared_ms(rs, ws, 3)
    # The verifier (verify_with_file_path on bytes, run.rs:556-592): cold (circuit extensions built per
    # call) on pedersen_test and on the synthetic 2^20-step proof; both must accept.
    from stark_amd.verify import verify_with_wtns
    js_s = c.prove(ws).to_json()
    del c
    for key, (rb, wb, jb) in (("pedersen", (r1, wt, js)), ("synth_2^20_steps", (rs, ws, js_s))):
        # The proof as the file's bytes (run.rs:556-592 reads the JSON file): a 3 MB str would be
        # re-encoded by the Python wrapper in every timed call (0.1-0.2 ms of the host's memcpy and page faults).
        jb = jb.encode()
        ok = verify_with_wtns(ctx, rb, wb, jb)
        tv = []
        for _ in range(10):
            t0 = time.perf_counter()
            verify_with_wtns(ctx, rb, wb, jb)
            tv.append(time.perf_counter() - t0)
        out[f"verify_{key}_ms"] = round(min(tv) * 1000.0, 3)
        out[f"verify_{key}_accepts"] = bool(ok)
    return out


def distributed_prove(ctx, world, rank, on_gloo, local):
    """One StarkProof shared by all ranks (stark_amd/dprove.py: residue-class layout, digest all-to-alls
    over RCCL): pedersen_test checked bit-exact against the golden digest, and the synthetic 2^20-step
    circuit (sha256_2_test stand-in) timed, max over ranks."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth_r1cs
    from stark_amd.dprove import GpuProverOps, prove_distributed
    ops = GpuProverOps(ctx)
    fix = os.path.join(ROOT, "tests", "golden", "r1cs")
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))
    out = {}
    r1 = open(os.path.join(fix, "pedersen_test.r1cs"), "rb").read()
    wt = open(os.path.join(fix, "pedersen_test.wtns"), "rb").read()
    js = prove_distributed(ops, r1, wt)
    if rank == 0:
        out["prove_pedersen_distributed_bitexact_vs_golden"] = \
            hashlib.sha256(js.encode()).hexdigest() == golden["pedersen_test"]["json_sha256"]

    def timed(rs, ws, reps, circuit=None):
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            prove_distributed(ops, rs, ws, circuit=circuit)
        dist.barrier()
        t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64,
                         device="cpu" if on_gloo else f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return round(float(t.cpu()[0]) * 1000.0, 3)

    out["prove_pedersen_distributed_ms"] = timed(r1, wt, 3)
    # config 4: poseidon3_test over the N GPUs, bit-exact against the golden digest
    r1p = open(os.path.join(fix, "poseidon3_test.r1cs"), "rb").read()
    wtp = open(os.path.join(fix, "poseidon3_test.wtns"), "rb").read()
    jsp = prove_distributed(ops, r1p, wtp)
    if rank == 0:
        out["prove_poseidon3_distributed_bitexact_vs_golden"] = \
            hashlib.sha256(jsp.encode()).hexdigest() == golden["poseidon3_test"]["json_sha256"]
    out["prove_poseidon3_distributed_ms"] = timed(r1p, wtp, 3)
    # The sha256_2_test stand-in (synthetic 2^20 steps, precision 2^23): the untimed first proof (it
    # also warms the twiddles and arenas) is checked against the oracle's StarkProof digest
    # (tests/golden/large_digests.json), so the timing below never stands without its parity flag.
    want = large_digests().get("prove_synth_2^20_steps", {}).get("json_sha256")
    rs, ws = synth_r1cs.for_steps(20)
    js20 = prove_distributed(ops, rs, ws)
    if rank == 0:
        out["prove_synth_2^20_steps_distributed_bitexact_vs_oracle_digest"] = sha256(js20) == want
    out["prove_synth_2^20_steps_distributed_ms"] = timed(rs, ws, 3)
    # One more proof with this rank's per-phase times (host wall-clock and the device time line from
    # HIP events on the proof's stream) and its count of host-synchronising steps (stark_amd/dprove.py).
    st = {}
    dist.barrier()
    prove_distributed(ops, rs, ws, stats=st)
    if rank == 0:
        out["prove_synth_2^20_steps_distributed_phases_rank0"] = st
    # Prepared circuit per rank (DistCircuit: the .r1cs-only work outside the timed region), labelled.
    from stark_amd.dprove import DistCircuit
    circ = DistCircuit(ctx, rs)
    js20 = prove_distributed(ops, None, ws, circuit=circ)
    if rank == 0:
        out["prove_synth_2^20_steps_distributed_prepared_circuit_bitexact_vs_oracle_digest"] = sha256(js20) == want
    del js20
    out["prove_synth_2^20_steps_distributed_prepared_circuit_ms"] = timed(None, ws, 3, circ)
    del circ
    return out


MERKLE_SQ = os.path.join(ROOT, "profiles", "r04_pmc_merkle32.json")
CPU_PROVE_2_20 = os.path.join(ROOT, "profiles", "r04_cpu_prove_synth_2_20.json")


XGMI_LINK_GBS = 153.0  # one xGMI link, one direction (MI355X: 7 links per GPU, task brief)


def group_extras(world: int, rank: int, on_gloo: bool) -> dict:
    """The C ABI's multi-GPU path (stark_group_*: one process drives the N GPUs through peer copies,
    include/stark_hip.h) timed on the same node: rank 0 runs tools/group_bench.py over devices 0..N-1 as a
    child process while the other ranks wait on a CPU (gloo) barrier with their GPUs idle.  A failure or a
    time-out is reported in the line; the headline is unaffected."""
    cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=400))
    out = {}
    if rank == 0:
        # (the one-GPU gloo rehearsal runs the same code with its N members on device 0: labelled as such)
        devs = ",".join("0" if on_gloo else str(i) for i in range(world))
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "group_bench.py"), "--devices", devs],
                               capture_output=True, text=True, timeout=240)
            if r.returncode == 0 and r.stdout.strip():
                out = {"group": json.loads(r.stdout.strip().splitlines()[-1])}
                if on_gloo:
                    out["group"]["note"] = "rehearsal: every member on device 0 (code path, not a scaling figure)"
            else:
                out = {"group_error": f"rc {r.returncode}: {r.stderr[-300:]}"}
        except Exception as e:  # noqa: BLE001 - reported in the line
            out = {"group_error": repr(e)[:300]}
    dist.barrier(group=cpu_group)
    return out


def distributed_phases(buf, log_total, w_total, ops, stream, on_gloo, local, reps=5) -> dict:
    """Median device time of each phase of one distributed step (the timed loop's transform, run
    unpipelined with HIP events on the step's stream between the phases), max over ranks: the local
    M-point NTT (stark_amd/distributed.py cyclic_ntt_local), the all-to-all, the cross-rank G-point
    DFT (cyclic_ntt_finish)."""
    from stark_amd.distributed import _exchange, cyclic_ntt_finish, cyclic_ntt_local
    a = buf.clone()
    z = torch.empty_like(a)
    names = ("local_ms", "exchange_ms", "finish_ms")
    got = {k: [] for k in names}
    for _ in range(reps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        dist.barrier()
        torch.cuda.synchronize()
        ev[0].record()
        y = cyclic_ntt_local(a, log_total, w_total, ops, in_place=True)
        ev[1].record()
        _exchange(z, y)
        ev[2].record()
        cyclic_ntt_finish(z, log_total, w_total, ops)
        ev[3].record()
        ev[3].synchronize()
        for i, k in enumerate(names):
            got[k].append(ev[i].elapsed_time(ev[i + 1]))
    med = torch.tensor([statistics.median(got[k][1:]) for k in names], dtype=torch.float64,
                       device="cpu" if on_gloo else f"cuda:{local}")
    dist.all_reduce(med, op=dist.ReduceOp.MAX)
    return dict(zip(names, (round(float(x), 4) for x in med.cpu())))


def distributed_roofline(ph: dict, n: int, world: int, log_n: int, plan: list, on_gloo: bool) -> dict:
    """The distributed step's rooflines, kept apart: its HBM-bound local kernels (the M-point NTT's pass
    launches and the strided G-point DFT, each 64 B per element read + written) at this
    rank's shard, and the all-to-all's bytes ((G-1)/G of the 32-B shard leave each rank, one G-th to
    each peer) against the direct xGMI links (G-1 of them at XGMI_LINK_GBS per rank)."""
    local_bytes = 64.0 * n * 2
    local_ms = ph["local_ms"] + ph["finish_ms"]
    achieved = local_bytes / (local_ms / 1000.0) / 1e9
    x_bytes = (world - 1) / world * n * 32.0
    x_peak = (world - 1) * XGMI_LINK_GBS
    x_ach = x_bytes / (ph["exchange_ms"] / 1000.0) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
            "traffic_note": "no counter pass of the distributed step (the committed PMC profiles are the "
                            "1-GPU transform's)",
            "kernel": f"local: {len(plan)} NTT pass launches (radices 2^{plan}) of this rank's 2^{log_n}-point "
                      "transform + the strided G-point DFT across the received chunks",
            "algorithmic_bytes_per_rank": local_bytes, "phases_ms": ph,
            "step_ms_unpipelined": round(sum(ph.values()), 4),
            "exchange": {"bound": "host-staged gloo (rehearsal: not an xGMI figure)" if on_gloo
                         else f"xGMI: {world - 1} direct links per rank", "bytes_per_rank": x_bytes,
                         "ms": ph["exchange_ms"], "achieved": round(x_ach, 2), "peak": x_peak, "unit": "GB/s",
                         "frac": round(x_ach / x_peak, 4)}}


def merkle_valu_roofline(n: int, ms: float) -> dict:
    """Blake2s issue roofline of a 2^log n x 32-B tree build: n leaf compressions (one 32-B block
    each) + n - 1 node compressions (64-B blocks) = 2n - 1.  From the committed counter passes over
    2^24 x 32-B tree builds alone (tools/pmc_round.sh ... merkle32): per build, the VALU instructions
    of every launch (SQ_INSTS_VALU, weighted by launches per build) x 4 cycles / 1024 SIMDs over the
    launches' elapsed cycles (GRBM_GUI_ACTIVE / 8) -- each dispatch at its own clock, so clock-free;
    and the instructions per compression."""
    comp = 2 * n - 1
    out = {"compressions": comp, "achieved_compressions_per_s": comp / (ms / 1000.0)}
    try:
        prof = json.load(open(MERKLE_SQ))["kernels"]
        builds = min(v["dispatches_per_pass"] for k, v in prof.items() if "merkle_build_kernel<true>" in k)
        need = took = insts = 0.0
        for k, v in prof.items():
            if "merkle" not in k or "GRBM_GUI_ACTIVE" not in v or "SQ_INSTS_VALU" not in v:
                continue
            w = v["dispatches_per_pass"] / builds
            insts += w * v["SQ_INSTS_VALU"]
            need += w * (v["SQ_INSTS_VALU"] - v.get("SQ_ACTIVE_INST_VALU2", 0.0)) * ISSUE_CYCLES / SIMDS
            took += w * v["GRBM_GUI_ACTIVE"] / 8
        leaf = next(v for k, v in prof.items() if "merkle_build_kernel<true>" in k)
        out.update({"valu_insts_per_compression": round(insts * 64 / comp, 1),
                    "issue_cycles_per_wave64_instruction": ISSUE_CYCLES,
                    "issue_cycles_per_build": round(need), "elapsed_cycles_per_build": round(took),
                    "frac": round(need / took, 4),
                    "leaf_kernel_issue_frac": round(leaf["valu_issue_frac"], 4),
                    "leaf_kernel_clock_ghz": round(leaf.get("effective_clock_ghz", 0), 3),
                    "sq_profile": os.path.relpath(MERKLE_SQ, ROOT)})
    except (OSError, KeyError, ValueError, StopIteration):
        pass
    return out


def ntt_products(log_n: int, plan: list) -> tuple:
    """Modular products of one forward 2^log_n transform, counted from csrc/ntt.hip's pass kernel:
    each radix-4 step multiplies 4 of every 4 elements (w_{2m}^jj twice, w_{4m}^jj, w_{4m}^(jj+m)),
    the s = 0 step of an even radix only by w_{4m}^(jj+m) (n/4), an odd radix runs a product-free
    radix-2 stage 0 first; every pass after the first multiplies each element by its column twiddle,
    one product from a table (t16 when Ns R <= 2^l16, or the last pass's full table for 2^17..2^26)
    or two in the lo * hi form.  Returns (all products, digit-basis products): the radix-4 steps
    before the last one of every pass use the digit-basis product (ntt.hip DbPlan,
    radices 2^4..2^8).  Radices >= 2^5 run their first step with twiddles (s = 2 even, s = 1 odd)
    jj-major, and its jj = 0 butterflies (n/16 even, n/8 odd) skip the products by w^0 = 1 (three of
    their four).  Radix 2^8 runs 16 x 16 (ntt.hip DbPlan::four): w_4 (n/4), the jj-major step (13n/16),
    one Shoup twiddle per element (n), w_4 (n/4), the last step (13n/16: its a = 0 waves multiply by w_4
    only); every product but the twiddles by the digit basis."""
    n = 1 << log_n
    l16 = 18 if log_n >= 25 else min(log_n, 16)
    total, db, ns = 0, 0, 0
    for i, r in enumerate(plan):
        if r == 8:
            total += 50 * n // 16
            db += 34 * n // 16
        elif r % 2:
            steps = n * ((r - 1) // 2)
        else:
            steps = n * (r // 2 - 1) + n // 4
        if r != 8:
            skip = 0 if r < 5 else 3 * n // 8 if r % 2 else 3 * n // 16
            total += steps - skip
            if 4 <= r <= 7:
                db += steps - skip  # every radix-4 step, the last from the table staged per tile
        if ns:
            last = i == len(plan) - 1
            table = ns + r <= l16 or (last and log_n > l16 and 17 <= log_n <= 26)
            total += n * (1 if table else 2)
        ns += r
    return total, db


def main():
    global S
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    backend = os.environ.get("STARK_BENCH_BACKEND", "nccl")
    if args.launch_check:
        # The launcher's CPU rehearsal: rendezvous, one collective, report the world that ran.
        if world > 1:
            dist.init_process_group("gloo", init_method="env://", timeout=datetime.timedelta(seconds=120))
            t = torch.tensor([1.0])
            dist.all_reduce(t)
            world_seen = int(t.item())
            dist.destroy_process_group()
        else:
            world_seen = 1
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_in_all_reduce": world_seen}))
        return
    import stark_amd
    S = stark_amd
    # One rank per GPU.  (local % device_count and STARK_BENCH_BACKEND=gloo exist only to rehearse
    # the N > 1 path with several ranks on a one-GPU box; the driver's runs use RCCL, one GPU per rank.)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", init_method="env://", device_id=torch.device(f"cuda:{local}"),
                                    timeout=datetime.timedelta(seconds=300))
        else:
            dist.init_process_group(backend, init_method="env://", timeout=datetime.timedelta(seconds=300))
    ctx = S.Context(local)
    # Every library launch and every RCCL collective goes to this stream, so
    # the HIP events below bracket exactly the timed work.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    log_n = args.log_n                      # per-GPU shard: 2^log_n elements
    n = 1 << log_n
    log_total = log_n + (world.bit_length() - 1)
    import oracle as O
    w_total = O.root_of_unity(log_total)
    w = O.root_of_unity(log_n)
    host = synthetic(n, 0x5EED0000 + log_total + 7919 * rank)
    buf = torch.from_numpy(host.view(np.int64)).to(f"cuda:{local}")
    torch.cuda.synchronize()
    dptr = buf.data_ptr()
    big = large_digests()
    parity = {}
    gpu_fwd = None
    if world == 1:
        # Parity of the exact timed path (stark_ntt_dev, device-resident) on the step's input:
        # forward and inverse against the oracle's digests (tests/golden/large_digests.json);
        # the CPU baseline below re-checks the forward output element for element.
        chk = buf.clone()
        ctx.ntt_dev(chk.data_ptr(), log_n, 1, w, inverse=False, stream=sptr)
        stream.synchronize()
        gpu_fwd = chk.cpu().numpy().view(np.uint64).reshape(-1, 4).copy()
        chk.copy_(buf)
        ctx.ntt_dev(chk.data_ptr(), log_n, 1, w, inverse=True, stream=sptr)
        stream.synchronize()
        gpu_inv = chk.cpu().numpy().view(np.uint64).reshape(-1, 4)
        rec = big.get(f"ntt_2^{log_n}")
        if rec and sha256(host) == rec["input_sha256"]:
            parity[f"ntt_2^{log_n}_fwd_bitexact_vs_oracle_digest"] = sha256(gpu_fwd) == rec["forward_sha256"]
            parity[f"ntt_2^{log_n}_inv_bitexact_vs_oracle_digest"] = sha256(gpu_inv) == rec["inverse_sha256"]
        del chk, gpu_inv
        torch.cuda.empty_cache()
    pipelined = world > 1 and dist.get_backend() == "nccl"
    if world > 1:
        from stark_amd.distributed import GpuOps, cyclic_ntt, cyclic_ntt_pipelined
        ops = GpuOps(ctx)
        bufs = [buf, torch.empty_like(buf)]
        state = {"i": 0}

        def step():
            # in place on this rank's shard, result into the other buffer (ping-pong)
            a, b = bufs[state["i"]], bufs[1 - state["i"]]
            cyclic_ntt(a, log_total, w_total, ops, out=b, in_place=True)
            state["i"] ^= 1

        if pipelined:
            # Steps are independent transforms (two shards in flight): the all-to-all of step i
            # (RCCL stream) overlaps the local NTT of step i+1 (this stream); step i's cross-rank
            # DFT runs once its exchange is done.  Every step is still a complete transform.
            pairs = [(buf, torch.empty_like(buf)),
                     (torch.from_numpy(synthetic(n, 0x5EED1000 + 7919 * rank).view(np.int64)).to(f"cuda:{local}"),
                      torch.empty_like(buf))]

            def run_steps(k):
                cyclic_ntt_pipelined(pairs, k, log_total, w_total, ops)
    else:
        def step():
            ctx.ntt_dev(dptr, log_n, 1, w, inverse=False, stream=sptr)

    if not pipelined:
        def run_steps(k):
            for _ in range(k):
                step()

    run_steps(args.warmup)
    # Clock settle: the card ramps its clock up over the first ~10-20 ms of load after the host-side
    # parity checks left it idle (profiles/r03_clock_ramp_probe.txt), so ~30 ms of untimed steps follow
    # the W warmup steps (the same count on every rank: the steps hold collectives; in the JSON line).
    torch.cuda.synchronize()
    ts = time.perf_counter()
    run_steps(1)
    torch.cuda.synchronize()
    settle = torch.tensor([min(1000, int(0.03 / max(time.perf_counter() - ts, 1e-5)) + 1)], dtype=torch.int64,
                          device="cpu" if world > 1 and dist.get_backend() == "gloo" else f"cuda:{local}")
    if world > 1:
        dist.all_reduce(settle, op=dist.ReduceOp.MAX)
    settle = int(settle.cpu()[0])
    run_steps(settle - 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_ms = timed_events(lambda: run_steps(args.steps), stream, 1) / args.steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    on_gloo = world > 1 and dist.get_backend() == "gloo"
    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if on_gloo else f"cuda:{local}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.cpu()[0])
    ms_per_step = elapsed * 1000.0 / args.steps
    value = world * n * args.steps / elapsed

    extras = dict(parity)
    if not args.no_extras and world == 1:
        # config 2: 2^20 forward + inverse pair; each direction checked against the oracle's digest
        n20 = 1 << 20
        w20 = O.root_of_unity(20)
        h20 = synthetic(n20, 0x5EED0000 + 20)
        b20 = torch.from_numpy(h20.view(np.int64)).to(f"cuda:{local}")
        rec20 = big.get("ntt_2^20", {})
        ctx.ntt_dev(b20.data_ptr(), 20, 1, w20, inverse=False, stream=sptr)
        stream.synchronize()
        f20 = sha256(b20.cpu().numpy().view(np.uint64))
        b20.copy_(torch.from_numpy(h20.view(np.int64)))
        ctx.ntt_dev(b20.data_ptr(), 20, 1, w20, inverse=True, stream=sptr)
        stream.synchronize()
        i20 = sha256(b20.cpu().numpy().view(np.uint64))
        b20.copy_(torch.from_numpy(h20.view(np.int64)))
        torch.cuda.synchronize()
        if rec20:
            extras["ntt_2^20_fwd_bitexact_vs_oracle_digest"] = f20 == rec20["forward_sha256"]
            extras["ntt_2^20_inv_bitexact_vs_oracle_digest"] = i20 == rec20["inverse_sha256"]

        def pair():
            ctx.ntt_dev(b20.data_ptr(), 20, 1, w20, inverse=False, stream=sptr)
            ctx.ntt_dev(b20.data_ptr(), 20, 1, w20, inverse=True, stream=sptr)
        pair()
        pair_ms, _ = median_ms(pair, stream, reps=25)
        stream.synchronize()
        ok = bool(np.array_equal(b20.cpu().numpy().view(np.uint64).reshape(-1, 4), h20))
        extras["ntt_2^20_fwd_inv_ms"] = round(pair_ms, 4)
        extras["ntt_2^20_fwd_inv_timing"] = "median of 25 event-timed pairs after warm-up"
        extras["ntt_2^20_fwd_inv_roundtrip_exact"] = ok
        # The host-buffer entry point (best_fft on a host Vec: H2D + NTT + D2H), PCIe-inclusive;
        # reported beside `value`, never as it.
        hc = host.copy()
        hout = np.empty_like(hc)
        extras["best_fft_host_2^24_ms_pcie_inclusive"] = round(
            median_host_ms(lambda: ctx.best_fft(hc, w, log_n, out=hout), reps=21, warm=2), 2)
        extras["best_fft_host_2^24_timing"] = ("host-to-host median of 21 calls (H2D + NTT + D2H) into a caller "
                                               "buffer already touched, as the reference's in-place best_fft "
                                               "writes the caller's Vec (a fresh buffer per call adds its page "
                                               "faults: about 70 ms for 512 MB)")
        del hc
        # BASELINE.md's timing of the headline transform: the median of 25 event-timed calls after
        # warm-up (`value` above is the contract's mean over the K barrier-bracketed steps).
        med, ts = median_ms(lambda: ctx.ntt_dev(dptr, log_n, 1, w, inverse=False, stream=sptr), stream, reps=25)
        extras[f"ntt_2^{log_n}_median_ms"] = round(med, 4)
        extras[f"ntt_2^{log_n}_median_elems_per_s"] = n / (med / 1000.0)
        extras[f"ntt_2^{log_n}_min_max_ms"] = [round(ts[0], 4), round(ts[-1], 4)]
        # Size sweep 2^20..2^26 (north star: synthetic traces of 2^20-2^26 field elements), forward NTT,
        # HBM-resident; elements uniform below 2^252 (< p), generated on the device.
        sweep = {}
        for ls in (20, 22, 24, 26):
            g = torch.Generator(device=f"cuda:{local}").manual_seed(ls)
            t = torch.randint(-2**63, 2**63 - 1, ((1 << ls), 4), dtype=torch.int64, device=f"cuda:{local}",
                              generator=g)
            t[:, 3] &= 0x0FFFFFFFFFFFFFFF
            ws = O.root_of_unity(ls)
            ctx.ntt_dev(t.data_ptr(), ls, 1, ws, inverse=False, stream=sptr)
            ms, _ = median_ms(lambda: ctx.ntt_dev(t.data_ptr(), ls, 1, ws, inverse=False, stream=sptr), stream,
                              reps=25)
            sweep[f"2^{ls}"] = {"ms": round(ms, 4), "elems_per_s": (1 << ls) / (ms / 1000.0),
                                "hbm_frac": round(64.0 * (1 << ls) / (ms / 1000.0) / 1e9 / HBM_PEAK_GBS, 5)}
            del t
        torch.cuda.empty_cache()
        extras["ntt_sweep"] = sweep
        extras["ntt_sweep_timing"] = "median of 25 event-timed transforms per size after warm-up"
        # inverse 2^24 throughput
        ctx.ntt_dev(dptr, log_n, 1, w, inverse=True, stream=sptr)   # warm: builds the w^-1 tables
        inv_ms, _ = median_ms(lambda: ctx.ntt_dev(dptr, log_n, 1, w, inverse=True, stream=sptr), stream, reps=25)
        extras["intt_2^24_elems_per_s"] = n / (inv_ms / 1000.0)
        # Merkle: 2^24 leaves of 32 B (canonical Fp, the FRI / L-tree leaves)
        tree = S.MerkleProofInPlace(ctx)
        tree.update_dev(dptr, n, 32, stream=sptr)
        stream.synchronize()
        tree.gen_proofs([])
        # The CPU baseline below rebuilds this tree from the same leaves (the buffer's current contents:
        # the timed loop transformed it in place) and compares roots.
        merkle_root = tree.get_root()
        merkle_leaves = buf.cpu().numpy().tobytes() if rank == 0 and not args.no_cpu_baseline else None
        mk_ms, _ = median_ms(lambda: tree.update_dev(dptr, n, 32, stream=sptr), stream, reps=25)
        extras["merkle_2^24x32B_leaves_per_s"] = n / (mk_ms / 1000.0)
        extras["merkle_2^24x32B_ms"] = round(mk_ms, 4)
        extras["merkle_timing"] = "median of 25 event-timed builds after warm-up"
        extras["merkle_roofline_frac"] = round(96.0 * n / (mk_ms / 1000.0) / 1e9 / HBM_PEAK_GBS, 5)
        extras["merkle_valu_roofline"] = merkle_valu_roofline(n, mk_ms)
        # Secondary leaf shapes: 256-B leaves (the main tree's P|A|S|D1..B3 rows; the same
        # 512 MiB buffer read as 2^21 rows) and 2^20 x 40-B accumulator leaves.
        for cnt, ll, key in ((n // 8, 256, "merkle_2^21x256B"), (1 << 20, 40, "merkle_2^20x40B")):
            tree.update_dev(dptr, cnt, ll, stream=sptr)
            t_ms, _ = median_ms(lambda: tree.update_dev(dptr, cnt, ll, stream=sptr), stream, reps=25)
            extras[f"{key}_leaves_per_s"] = cnt / (t_ms / 1000.0)
            extras[f"{key}_ms"] = round(t_ms, 4)
        del tree
        # FRI prove wall clock at precision 2^23 (largest a reference proof can use, fri/src/utils.rs:88),
        # the proof checked against the oracle's digest (same input as make_large_golden.py).
        lf = 23
        nf = 1 << lf
        wf = O.root_of_unity(lf)
        coef = synthetic(nf // 4, 0x5EED0000 + lf)
        hf = np.zeros((nf, 4), dtype=np.uint64)
        hf[: nf // 4] = coef
        bf = torch.from_numpy(hf.view(np.int64)).to(f"cuda:{local}")
        torch.cuda.synchronize()
        ctx.ntt_dev(bf.data_ptr(), lf, 1, wf, stream=sptr)
        stream.synchronize()
        proof = ctx.prove_low_degree_dev(bf.data_ptr(), nf, wf, nf // 4, 8)
        fri_json_sha = sha256(proof.to_json())
        if big.get("fri_2^23"):
            extras["fri_2^23_bitexact_vs_oracle_digest"] = fri_json_sha == big["fri_2^23"]["json_sha256"]
        extras["fri_prove_2^23_ms"] = round(median_host_ms(
            lambda: ctx.prove_low_degree_dev(bf.data_ptr(), nf, wf, nf // 4, 8), reps=21, warm=2), 3)
        extras["fri_prove_timing"] = "host-to-host median of 21 proofs (device-resident input, proof on the host)"
        extras["fri_layers"] = len(proof)
        fri_vals = bf.cpu().numpy().view(np.uint64).reshape(-1, 4).copy()  # the CPU baseline's input
        del bf, proof
        # End-to-end proof wall-clock (config 3: pedersen_test full prove on 1 GPU):
        # prove_with_witness = .r1cs/.wtns bytes -> trace -> mk_r1cs_proof -> StarkProof JSON.
        try:
            extras.update(end_to_end(ctx))
        except Exception as e:  # the headline line is still printed; the failure is reported in it
            extras["end_to_end_error"] = repr(e)[:300]
        # Board power while the NTT and the Merkle build run back to back (after every timing above, so
        # the heat does not skew them): the NTT sits at the package power limit, which sets its clock.
        pwr = power_under_load(lambda: ctx.ntt_dev(dptr, log_n, 1, w, inverse=False, stream=sptr), stream.synchronize)
        if pwr:
            extras["power_during_ntt"] = pwr
        ptree = S.MerkleProofInPlace(ctx)
        pwr = power_under_load(lambda: ptree.update_dev(dptr, n, 32, stream=sptr), stream.synchronize)
        if pwr:
            extras["power_during_merkle"] = pwr
        del ptree

    if not args.no_extras and world > 1:
        # Distributed Merkle commitment (north star: per-GPU subtrees combined across ranks):
        # 2^log_n 32-B leaves per GPU, subtree roots all-gathered, top levels on the host.
        from stark_amd.distributed import DistributedMerkle
        dm = DistributedMerkle(ops)
        dm.commit(bufs[0], n, 32)
        dist.barrier()
        t_m = time.perf_counter()
        reps = 3
        for _ in range(reps):
            dm.commit(bufs[0], n, 32)
        dist.barrier()
        tm = torch.tensor([time.perf_counter() - t_m], dtype=torch.float64,
                          device="cpu" if on_gloo else f"cuda:{local}")
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        extras["merkle_distributed_leaves_per_s"] = world * n * reps / float(tm.cpu()[0])
        extras["merkle_distributed_ms"] = round(float(tm.cpu()[0]) * 1000.0 / reps, 3)
        # The timed loop's schedule gives the same transform as the plain cyclic_ntt: one fresh
        # shard through both, compared bit for bit on every rank.
        fresh = torch.from_numpy(synthetic(n, 0x5EED2000 + 7919 * rank).view(np.int64)).to(f"cuda:{local}")
        ref = cyclic_ntt(fresh, log_total, w_total, ops)
        if pipelined:
            pairs[0][0].copy_(fresh)
            run_steps(1)
            got = pairs[0][1]
        else:
            got = cyclic_ntt(fresh, log_total, w_total, ops)
        same = torch.tensor([1.0 if torch.equal(got, ref) else 0.0], dtype=torch.float64,
                            device="cpu" if on_gloo else f"cuda:{local}")
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        extras["distributed_schedule_matches_cyclic_ntt"] = bool(float(same.cpu()[0]) == 1.0)
        try:
            extras.update(distributed_prove(ctx, world, rank, on_gloo, local))
        except Exception as e:  # symmetric failures still print the headline line
            extras["distributed_prove_error"] = repr(e)[:300]
        extras.update(group_extras(world, rank, on_gloo))

    # Roofline of the dominant kernel, ntt_pass_kernel: one 2^log_n transform is len(plan)
    # launches; achieved = SURVEY 8(d)'s algorithmic 64 B per element per transform (read 32 +
    # write 32) x n / transform time (HIP events on the launch stream).
    ntt_bytes = 64.0 * n
    if world > 1:
        # The distributed step, phase by phase (its own roofline below, nothing from a 1-GPU profile):
        # this rank's local M-point transform, the all-to-all, the cross-rank G-point DFT.
        dphase = distributed_phases(buf, log_total, w_total, ops, stream, on_gloo, local)
        ev_ms = dphase["local_ms"]
    achieved = ntt_bytes / (ev_ms / 1000.0) / 1e9
    plan = S.ntt_plan(log_n)
    passes = len(plan)
    # The pass kernels of this transform (csrc/ntt.hip ntt_pass_kernel<LOG_R, COL>: COL = 0 first pass,
    # 2 Shoup t16 column twiddles, 1 the last pass's full table): per-launch HBM bytes and rocprof times
    # from the committed profile of this exact command line (tools/profile_round.sh), VALU issue from the
    # committed counter passes over 2^24 transforms alone (tools/pmc_round.sh ... ntt).
    traffic = prof_avg = prof_med = None
    knames, sq, timed = [], {}, None
    try:
        if world > 1:
            raise OSError("the committed profiles are of the 1-GPU transform")
        prof = json.load(open(PROFILE))
        knames = sorted(k for k in prof["kernels"] if "ntt_pass_kernel" in k)
        if log_n == 24 and knames and all(k in prof["pmc_bytes_per_launch"] for k in knames):
            # HBM bytes of one transform: per-launch FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md)
            # summed over the transform's launches.
            traffic = sum(prof["pmc_bytes_per_launch"][k]["hbm_bytes"] for k in knames)
            prof_avg = sum(prof["kernels"][k]["avg_ns"] for k in knames) / 1e6
            prof_med = sum(prof["kernels"][k]["steady_median_ns"] for k in knames) / 1e6
            timed = prof.get("timed_region")
    except (OSError, KeyError, ValueError):
        pass
    try:
        if log_n == 24 and world == 1:
            pmc = json.load(open(PMC))["kernels"]
            sq = {k: v for k, v in pmc.items() if "ntt_pass_kernel" in k and "valu_issue_frac" in v}
    except (OSError, KeyError, ValueError):
        pass
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_over_algorithmic": round(traffic / ntt_bytes, 3) if traffic else None,
                "kernel": f"{passes} NTT pass launches (radices 2^{plan}) per 2^{log_n} transform",
                "ms_per_transform": round(ev_ms, 4), "avg_launch_ms": round(ev_ms / passes, 4),
                "rocprof_ms_per_transform_avg": round(prof_avg, 4) if prof_avg else None,
                "rocprof_ms_per_transform_steady_median": round(prof_med, 4) if prof_med else None,
                "rocprof_kernels": knames, "rocprof_summary": os.path.relpath(PROFILE, ROOT)}
    if world > 1:
        roofline = distributed_roofline(dphase, n, world, log_n, plan, on_gloo)
    if timed:  # the profiled run's kernels over its own timed steps vs that run's ms_per_step
        roofline["rocprof_timed_region_ms_per_transform"] = round(timed["kernel_ms_per_transform"], 4)
        roofline["rocprof_run_ms_per_step"] = round(timed["bench_ms_per_step_same_run"], 4)
    modmuls, db_muls = ntt_products(log_n, plan)
    # The transform's products at the standalone rates of their two forms (the rest of the pass, the
    # butterflies, LDS traffic and the Montgomery full-table column twiddle, priced at nothing).
    peak = modmuls / (db_muls / DB_PRODUCT_PEAK + (modmuls - db_muls) / SHOUP_PRODUCT_PEAK)
    valu = {"bound": "VALU issue: one quad-cycle (4 cycles) per wave64 VALU instruction on a 16-lane SIMD",
            "modmuls_per_transform": modmuls, "digit_basis_modmuls_per_transform": db_muls,
            "achieved_modmul_per_s": modmuls / (ev_ms / 1000.0),
            "product_peak_per_s": round(peak), "shoup_product_peak_per_s": SHOUP_PRODUCT_PEAK,
            "digit_basis_product_peak_per_s": DB_PRODUCT_PEAK}
    valu["product_frac"] = round(valu["achieved_modmul_per_s"] / peak, 4)
    if sq:
        # Issue fraction of the transform, each dispatch priced at ITS OWN clock: per pass,
        # (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) x 4 / 1024 SIMDs = the SIMD cycles its VALU
        # instructions occupy (one quad-cycle each, less the quad-cycles that issued two), over
        # GRBM_GUI_ACTIVE / 8 XCDs = the cycles it took, both from the same dispatch
        # (tools/pmc_summary.py); summed over the transform's passes.  Clock-free and <= 1.
        need = sum((v["SQ_INSTS_VALU"] - v.get("SQ_ACTIVE_INST_VALU2", 0.0)) * ISSUE_CYCLES / SIMDS
                   for v in sq.values())
        took = sum(v["GRBM_GUI_ACTIVE"] / 8 for v in sq.values())
        insts = sum(v["SQ_INSTS_VALU"] for v in sq.values())
        valu.update({"sq_insts_valu_per_transform": insts,
                     "valu_lane_insts_per_element": round(insts * 64 / n, 1),
                     "issue_cycles_per_transform": round(need), "elapsed_cycles_per_transform": round(took),
                     "frac": round(need / took, 4),
                     "per_pass": {k: {"frac": round(v["valu_issue_frac"], 4),
                                      "frac_4cyc": round(v.get("valu_issue_frac_4cyc", 0), 4),
                                      "clock_ghz": round(v.get("effective_clock_ghz", 0), 3),
                                      "dual_issue_share": round(v.get("valu_dual_issue_share", 0), 4),
                                      "class_share": {c: round(x, 3) for c, x in v.get("valu_class_share", {}).items()}}
                                  for k, v in sq.items()},
                     "sq_profile": os.path.relpath(PMC, ROOT)})
        # The same instruction count priced at the clock rocm-smi sampled under this bench's NTT loop
        # (reads up to ~10 % above the in-kernel clock, so this figure is a lower estimate).
        sclk = extras.get("power_during_ntt", {}).get("sclk_mhz")
        if sclk:
            valu["frac_at_sampled_sclk"] = round(need / (sclk * 1e6) * 1e3 / ev_ms, 4)
        roofline["valu_issue_frac"] = valu["frac"]
    if "power_during_ntt" in extras:
        roofline["power_during_ntt"] = extras["power_during_ntt"]

    cpu = None
    if rank == 0 and world > 1 and not args.no_cpu_baseline:
        # One rank's share on the host: best_fft (fft.rs:327-357, the oracle's C restatement with the
        # Worker split's 2^floor(log2 cores) threads) of this rank's 2^log_n shard.  The reference has no
        # multi-node form; the whole job's CPU time is world times this.
        o = O.Oracle()
        physical, usable = host_cpus()
        threads = 1 << (min(physical, usable).bit_length() - 1)
        t2 = time.perf_counter()
        o.best_fft(host, w, log_n, cpus=threads)
        tc = time.perf_counter() - t2
        cpu = {"value": n / tc, "unit": "field-elems/s", "cores": threads, "threads": threads,
               "host_physical_cores": physical, "cpus_granted": usable, "kind": "port",
               "sample": f"rank 0's 2^{log_n}-element shard as one 2^{log_n}-point best_fft (oracle C restatement "
                         f"of fft.rs parallel_fft, {threads} threads), {tc:.2f} s; the whole 2^{log_total} job on "
                         f"this host would be {world} such shards or more",
               "scope": "one rank's shard (per-GPU work of the weak-scaling step)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # The reference algorithm on the host: the oracle's C restatement of best_fft / parallel_fft
        # (fft.rs:195-251, 327-357) with T = 2^floor(log2(cores)) threads as Worker::new splits it,
        # on the SAME input as the GPU step; its output is compared with the GPU's element for element.
        o = O.Oracle()
        physical, usable = host_cpus()
        cores = min(physical, usable)
        threads = 1 << (cores.bit_length() - 1)
        t2 = time.perf_counter()
        cpu_out = o.best_fft(host, w, log_n, cpus=threads)
        tc = time.perf_counter() - t2
        cpu = {"value": n / tc, "unit": "field-elems/s", "cores": threads, "threads": threads,
               "host_physical_cores": physical, "cpus_granted": usable, "kind": "port",
               "sample": f"one 2^{log_n}-point best_fft on the bench step's input (oracle C restatement of "
                         f"fft.rs parallel_fft, {threads} threads = 2^floor(log2 min(physical cores {physical}, "
                         f"CPUs granted {usable}))), {tc:.2f} s",
               "gpu_output_bitexact": bool(gpu_fwd is not None and np.array_equal(cpu_out, gpu_fwd))}
        extras[f"ntt_2^{log_n}_bitexact_vs_cpu_baseline"] = cpu["gpu_output_bitexact"]
        del cpu_out
        if not args.no_extras:
            # The metric's other legs beside their GPU numbers, same inputs, each CPU output compared with
            # the GPU's (one timed run each: ~10-40 s of CPU work).
            legs = {}
            # Merkle: gen_multi_proofs_multi_core (merkle_proof_in_place.rs:106-206) over the same 2^24
            # x 32-B leaves.  The reference hashes every leaf and layer on one thread (it never calls
            # worker.scope); its 2^floor(log2 cpus) subtrees run one after another.
            t3 = time.perf_counter()
            cpu_root, _ = o.merkle(merkle_leaves, n, 32, chunks=threads)
            tm = time.perf_counter() - t3
            del merkle_leaves
            legs["merkle_2^24x32B"] = {
                "value": n / tm, "unit": "leaves/s", "ms": round(tm * 1000.0, 1), "cores": 1, "threads": 1,
                "kind": "port", "sample": f"one build of the bench's 2^24 x 32-B tree, {threads} subtrees hashed "
                                          "in sequence on one thread (oracle C restatement)",
                "gpu_root_bitexact": bool(cpu_root == merkle_root)}
            # FRI: prove_low_degree (fri.rs:46-224) on the bench's precision-2^23 input, single-threaded
            # like the reference (its Merkle builds are sequential and its fold is a serial loop).
            t3 = time.perf_counter()
            cpu_fri = o.prove_low_degree_json(fri_vals, wf, nf // 4, 8, chunks=threads)
            tf = time.perf_counter() - t3
            legs["fri_prove_2^23"] = {
                "value": round(tf * 1000.0, 1), "unit": "ms", "cores": 1, "threads": 1, "kind": "port",
                "sample": "one prove_low_degree at precision 2^23 (maxdeg 2^21, exclude 8) on the bench's input "
                          "(oracle C restatement)",
                "gpu_json_bitexact": bool(sha256(cpu_fri) == fri_json_sha)}
            del cpu_fri
            # Config 2's pair on the CPU: best_fft then inv_best_fft of the 2^20 input (fft.rs:327-379).
            t3 = time.perf_counter()
            f20c = o.best_fft(h20, w20, 20, cpus=threads)
            b20c = o.inv_best_fft(f20c, w20, 20, cpus=threads)
            t20 = time.perf_counter() - t3
            legs["ntt_2^20_fwd_inv"] = {
                "value": round(t20 * 1000.0, 1), "unit": "ms", "cores": threads, "threads": threads, "kind": "port",
                "sample": "best_fft + inv_best_fft of the bench's 2^20 input (oracle C restatement of parallel_fft)",
                "roundtrip_exact": bool(np.array_equal(b20c, h20))}
            del f20c, b20c
            # End-to-end: the oracle's restatement of mk_r1cs_proof on compute (config 1) and pedersen_test.
            import r1cs as R
            trc = R.build_trace(*R.load_fixture(os.path.join(ROOT, "tests", "golden", "r1cs"), "compute"))
            t3 = time.perf_counter()
            R.mk_r1cs_proof_json(o, trc, cpus=threads)
            legs["prove_compute"] = {"value": round((time.perf_counter() - t3) * 1000.0, 2), "unit": "ms",
                                     "cores": threads, "threads": threads, "kind": "port",
                                     "sample": "one mk_r1cs_proof of compute (oracle C restatement)"}
            tr = R.build_trace(*R.load_fixture(os.path.join(ROOT, "tests", "golden", "r1cs"), "pedersen_test"))
            t3 = time.perf_counter()
            R.mk_r1cs_proof_json(o, tr, cpus=threads)
            extras["prove_pedersen_cpu_port_ms"] = round((time.perf_counter() - t3) * 1000.0, 1)
            extras["prove_pedersen_cpu_port_threads"] = threads
            legs["prove_pedersen"] = {"value": extras["prove_pedersen_cpu_port_ms"], "unit": "ms", "cores": threads,
                                      "threads": threads, "kind": "port",
                                      "sample": "one mk_r1cs_proof of pedersen_test (oracle C restatement)"}
            # The 2^20-step proof on the CPU port takes minutes, so it is timed once by
            # tools/cpu_prove_baseline.py on the GPU box and committed; reported here with its source.
            try:
                rec = json.load(open(CPU_PROVE_2_20))
                rec["timed_in_this_run"] = False
                rec["provenance"] = (f"committed round-4 record ({os.path.relpath(CPU_PROVE_2_20, ROOT)}), "
                                     "not timed in this run")
                legs["prove_synth_2^20_steps"] = rec
            except (OSError, ValueError):
                pass
            extras["cpu_baselines"] = legs

    if rank == 0:
        # N > 1: the metric names the workload the GPUs share (one 2^(24 + log2 N)-point transform)
        metric = "2^24-pt NTT field-elems/sec" if world == 1 else \
            f"2^{log_total}-pt distributed NTT field-elems/sec (2^{log_n} per GPU)"
        line = {"metric": metric, "value": value, "unit": "field-elems/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "clock_settle_steps": settle, "ms_per_step": ms_per_step,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32x8 (BN254 Fr)",
                "data": "synthetic (splitmix64 uniform in [0,p), BASELINE.md)",
                "config": {"workload": f"forward NTT 2^{log_total} BN254 Fr, natural order, HBM-resident"
                                       + (f", distributed over {world} GPUs (cyclic in / chunked out, one RCCL "
                                          "all-to-all)" if world > 1 else ""),
                           "global_batch": 1, "seq_len": n * world, "shard_per_gpu": n,
                           "parallelism": f"distributed NTT x{world} (one all-to-all)" if world > 1 else "single GPU"},
                "roofline": roofline, "valu_roofline": valu, "cpu_baseline": cpu}
        line.update(extras)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
