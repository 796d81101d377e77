"""Wall-clock of the GPU-resident mk_r1cs_proof on the reference fixtures and
on synthetic circuits (tools/synth_r1cs.py).  Usage:
    python tools/time_r1cs.py [--reps 3] [--synth 16,18,20] [--fixtures pedersen_test]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "tools")]

import stark_amd as S  # noqa: E402
from stark_amd.r1cs import R1csCircuit, R1csTrace, prove_with_witness  # noqa: E402
import synth_r1cs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--synth", default="16,18,20")
    ap.add_argument("--fixtures", default="poseidon3_test,pedersen_test")
    ap.add_argument("--prepared", action="store_true", help="prove through R1csCircuit (prepared once)")
    a = ap.parse_args()
    ctx = S.Context(0)
    cases = []
    for name in [x for x in a.fixtures.split(",") if x]:
        d = os.path.join(ROOT, "tests", "golden", "r1cs")
        cases.append((name, open(f"{d}/{name}.r1cs", "rb").read(), open(f"{d}/{name}.wtns", "rb").read()))
    for k in [int(x) for x in a.synth.split(",") if x]:
        r, w = synth_r1cs.for_steps(k)
        cases.append((f"synth_2^{k}", r, w))
    for name, r, w in cases:
        t0 = time.perf_counter()
        tr = R1csTrace(r, w)
        t_trace = time.perf_counter() - t0
        dims = tr.dims()
        times = []
        circ = R1csCircuit(ctx, r) if a.prepared else None
        for i in range(a.reps + 1):
            t1 = time.perf_counter()
            p = circ.prove(w) if circ else prove_with_witness(ctx, r, w)
            js = p.to_json()
            times.append(time.perf_counter() - t1)
        print(f"{name}: original_steps={dims['original_steps']} host_trace_build={t_trace * 1e3:.1f} ms "
              f"prove first={times[0] * 1e3:.1f} ms best={min(times[1:]) * 1e3:.1f} ms json={len(js)} B",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
