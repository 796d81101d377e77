"""A/B of the 2^k-step synthetic proof (cold) across library builds, one process per build:
    python tools/time_r1cs_libs.py a.so b.so ... [--steps 20] [--reps 4]"""
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
    a = ap.parse_args()
    for lib in a.libs:
        code = (f"ROOT = {ROOT!r}\nLIB = {os.path.abspath(lib)!r}\nSTEPS = {a.steps}\nREPS = {a.reps}\n" + CHILD)
        subprocess.run([sys.executable, "-c", code], check=True)


if __name__ == "__main__":
    main()
