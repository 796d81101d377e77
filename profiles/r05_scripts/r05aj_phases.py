# host phases of repeated cold 2^20-step proofs: the library's STARK_PROFILE phase clock (stderr) plus the
# Python side (the call, to_json, the previous proof's release)
import os, sys, time
R = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
sys.path[:0] = [os.path.join(R, "stark-pure-rust_amd"), os.path.join(R, "tools")]
import stark_amd as S
from stark_amd.r1cs import prove_with_witness
import synth_r1cs
FX = os.environ.get("FIXTURE", "")
if FX:
    d = os.path.join(R, "tests", "golden", "r1cs")
    r, w = open(f"{d}/{FX}.r1cs", "rb").read(), open(f"{d}/{FX}.wtns", "rb").read()
else:
    r, w = synth_r1cs.for_steps(20)
ctx = S.Context(0)
p = None
for i in range(int(os.environ.get("REPS", "5"))):
    t0 = time.perf_counter()
    p = None
    t1 = time.perf_counter()
    q = prove_with_witness(ctx, r, w)
    t2 = time.perf_counter()
    js = q.to_json()
    t3 = time.perf_counter()
    p = q
    print(f"[py] release {1e6 * (t1 - t0):.0f} us  call {1e6 * (t2 - t1):.0f} us  to_json {1e6 * (t3 - t2):.0f} us  "
          f"total {1e6 * (t3 - t0):.0f} us", file=sys.stderr, flush=True)
