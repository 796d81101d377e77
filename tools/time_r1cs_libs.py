"""A/B of the 2^k-step synthetic proof (cold) across library builds, one process per build:
    python tools/time_r1cs_libs.py a.so b.so ... [--steps 20] [--reps 4] [--fixture pedersen_test]
(--fixture: a reference fixture from tests/golden/r1cs instead of the synthetic circuit)"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "tools")]
import stark_amd as S
S.load_library(LIB)
from stark_amd.r1cs import prove_with_witness
import synth_r1cs
if FIXTURE:
    d = os.path.join(ROOT, "tests", "golden", "r1cs")
    r, w = open(f"{d}/{FIXTURE}.r1cs", "rb").read(), open(f"{d}/{FIXTURE}.wtns", "rb").read()
else:
    r, w = synth_r1cs.for_steps(STEPS)
ctx = S.Context(0)
ts = []
for i in range(REPS + 1):
    t = time.perf_counter(); p = prove_with_witness(ctx, r, w); js = p.to_json(); ts.append(time.perf_counter() - t)
print(f"{os.path.basename(LIB)}: best {min(ts[1:]) * 1e3:.2f} ms  median {sorted(ts[1:])[len(ts[1:]) // 2] * 1e3:.2f} ms", flush=True)
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--fixture", default="")
    a = ap.parse_args()
    for lib in a.libs:
        code = (f"ROOT = {ROOT!r}\nLIB = {os.path.abspath(lib)!r}\nSTEPS = {a.steps}\nREPS = {a.reps}\nFIXTURE = {a.fixture!r}\n" + CHILD)
        subprocess.run([sys.executable, "-c", code], check=True)


if __name__ == "__main__":
    main()
