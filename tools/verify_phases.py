"""Host phase times of the cold verifier (STARK_PROFILE=1 prints the library's phase clock on stderr):
prove a fixture (or `synthK`, the synthetic 2^K-step circuit) once, then verify_with_wtns N times, printing
each call's wall-clock.   python tools/verify_phases.py [pedersen_test | synth20] [N]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]
import stark_amd as S  # noqa: E402
from stark_amd.r1cs import prove_with_witness  # noqa: E402
from stark_amd.verify import verify_with_wtns  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "pedersen_test"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    ctx = S.Context(0)
    if name.startswith("synth"):  # synthK: the synthetic 2^K-step circuit (tools/synth_r1cs.py)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import synth_r1cs
        r1, wt = synth_r1cs.for_steps(int(name[5:]))
    else:
        fix = os.path.join(ROOT, "tests", "golden", "r1cs")
        r1 = open(os.path.join(fix, f"{name}.r1cs"), "rb").read()
        wt = open(os.path.join(fix, f"{name}.wtns"), "rb").read()
    js = prove_with_witness(ctx, r1, wt).to_json().encode()
    for i in range(reps):
        t = time.perf_counter()
        verify_with_wtns(ctx, r1, wt, js)
        print(f"verify {i}: {(time.perf_counter() - t) * 1e3:.3f} ms", file=sys.stderr, flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
