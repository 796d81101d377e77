"""A/B of the verifier (cold verify_with_wtns and prepared verify_circuit on pedersen_test) across library
builds, one process per build:  python tools/time_verify_libs.py a.so b.so ... [--reps 30] [--synth]"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]
import stark_amd as S
S.load_library(LIB)
from stark_amd.r1cs import R1csCircuit, prove_with_witness
from stark_amd.verify import verify_circuit, verify_with_wtns
import r1cs as R
d = os.path.join(ROOT, "tests", "golden", "r1cs")
r1 = open(f"{d}/pedersen_test.r1cs", "rb").read()
wt = open(f"{d}/pedersen_test.wtns", "rb").read()
ctx = S.Context(0)
jb = prove_with_witness(ctx, r1, wt).to_json().encode()
h = R.read_r1cs(r1).header
pub = R.read_witness(wt)[:1 + h.n_public_inputs + h.n_public_outputs]
c = R1csCircuit(ctx, r1)
def best(fn):
    ts = []
    for _ in range(REPS + 1):
        t = time.perf_counter(); fn(); ts.append(time.perf_counter() - t)
    ts = sorted(ts[1:])
    return ts[0] * 1e3, ts[len(ts) // 2] * 1e3
cb, cm = best(lambda: verify_with_wtns(ctx, r1, wt, jb))
pb, pm = best(lambda: verify_circuit(ctx, c, pub, jb))
print(f"{os.path.basename(LIB)}: cold best {cb:.3f} median {cm:.3f} ms  prepared best {pb:.3f} median {pm:.3f} ms", flush=True)
if SYNTH:
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth_r1cs
    rs, ws = synth_r1cs.for_steps(20)
    js = R1csCircuit(ctx, rs).prove(ws).to_json().encode()
    assert verify_with_wtns(ctx, rs, ws, js)
    REPS = 5
    sb, sm = best(lambda: verify_with_wtns(ctx, rs, ws, js))
    print(f"{os.path.basename(LIB)}: 2^20-step cold best {sb:.3f} median {sm:.3f} ms", flush=True)
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--synth", action="store_true", help="also the cold verify of a synthetic 2^20-step proof")
    a = ap.parse_args()
    for lib in a.libs:
        code = f"ROOT = {ROOT!r}\nLIB = {os.path.abspath(lib)!r}\nREPS = {a.reps}\nSYNTH = {a.synth}\n" + CHILD
        subprocess.run([sys.executable, "-c", code], check=True)


if __name__ == "__main__":
    main()
