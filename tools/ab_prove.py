"""Same-box A/B of whole proofs across library builds (any ABI revision: raw ctypes, no header check), one
child process per build per round, rounds alternating so that clock and thermal drift hit every build alike:
    python tools/ab_prove.py [--fixtures compute,pedersen_test] [--reps 20] [--rounds 3] a.so b.so ...
Fixtures are names under tests/golden/r1cs or synthK (the synthetic 2^K-step circuit).
Prints per build and fixture the best and median host wall-clock of prove_with_witness on raw bytes
(stark_prove_r1cs_bytes + reading the JSON) and the JSON's digest (must agree across builds)."""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import ctypes, hashlib, json, os, sys, time
lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
vp = ctypes.c_void_p
lib.stark_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
lib.stark_prove_r1cs_bytes.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]
lib.stark_r1cs_proof_json_view.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]
lib.stark_r1cs_proof_free.argtypes = [vp]
ctx = vp()
assert lib.stark_ctx_create(0, ctypes.byref(ctx)) == 0
out = {}
d = os.path.join(sys.argv[2], "tests", "golden", "r1cs")
for name in sys.argv[3].split(","):
    if name.startswith("synth"):  # synthK: the synthetic 2^K-step circuit (tools/synth_r1cs.py)
        sys.path.insert(0, os.path.join(sys.argv[2], "tools"))
        import synth_r1cs
        r, w = synth_r1cs.for_steps(int(name[5:]))
    else:
        r, w = open(f"{d}/{name}.r1cs", "rb").read(), open(f"{d}/{name}.wtns", "rb").read()
    ts, dig = [], None
    for i in range(int(sys.argv[4]) + 2):
        t = time.perf_counter()
        p = vp()
        assert lib.stark_prove_r1cs_bytes(ctx, r, len(r), w, len(w), ctypes.byref(p)) == 0
        q, n = vp(), ctypes.c_size_t()
        lib.stark_r1cs_proof_json_view(p, ctypes.byref(q), ctypes.byref(n))
        js = ctypes.string_at(q.value, n.value)
        lib.stark_r1cs_proof_free(p)
        ts.append(time.perf_counter() - t)
        dig = hashlib.sha256(js).hexdigest()[:16]
    out[name] = {"ms": [round(x * 1e3, 4) for x in ts[2:]], "digest": dig}
print(json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixtures", default="compute,pedersen_test")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    res = {lib: {} for lib in a.libs}
    for _ in range(a.rounds):
        for lib in a.libs:
            r = subprocess.run([sys.executable, "-c", CHILD, lib, ROOT, a.fixtures, str(a.reps)], capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                print(f"{lib}: rc {r.returncode} {r.stderr[-500:]}", flush=True)
                continue
            for name, v in json.loads(r.stdout.strip().splitlines()[-1]).items():
                e = res[lib].setdefault(name, {"ms": [], "digest": v["digest"]})
                e["ms"] += v["ms"]
                e["digest_stable"] = e.get("digest_stable", True) and e["digest"] == v["digest"]
    for lib, per in res.items():
        for name, e in per.items():
            print(f"{os.path.basename(lib):12s} {name:16s} best {min(e['ms']):8.3f} ms  median "
                  f"{statistics.median(e['ms']):8.3f} ms  n={len(e['ms'])}  digest {e['digest']}", flush=True)


if __name__ == "__main__":
    main()
