"""Same-box A/B of the host-buffer best_fft (stark_best_fft / stark_inv_best_fft: pageable host vectors in and
out, PCIe inclusive) across library builds, one child process per build per round.
    python tools/ab_host_fft.py [--log-n 24] [--reps 5] [--rounds 3] a.so b.so ...
Prints per build the median ms of best_fft and of inv_best_fft and the output digest (must agree)."""
import argparse
import json
import os
import statistics
import subprocess
import sys

CHILD = r'''
import ctypes, hashlib, json, sys, time
import numpy as np
lib = ctypes.CDLL(sys.argv[1])
vp = ctypes.c_void_p
u64p = ctypes.POINTER(ctypes.c_uint64)
lib.stark_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
lib.stark_best_fft.argtypes = [vp, u64p, ctypes.c_size_t, u64p, ctypes.c_uint32, u64p]
lib.stark_inv_best_fft.argtypes = [vp, u64p, ctypes.c_size_t, u64p, ctypes.c_uint32, u64p]
lib.stark_expand_root_of_unity = None
log_n, reps = int(sys.argv[2]), int(sys.argv[3])
n = 1 << log_n
p = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001
w = pow(7, (p - 1) >> log_n, p)
root = (ctypes.c_uint64 * 4)(*[(w >> (64 * k)) & (2**64 - 1) for k in range(4)])
rng = np.random.default_rng(5)
x = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
x[:, 3] &= np.uint64((1 << 60) - 1)
out = np.empty_like(x)
back = np.empty_like(x)
ctx = vp()
assert lib.stark_ctx_create(0, ctypes.byref(ctx)) == 0
P = lambda a: a.ctypes.data_as(u64p)
fw, iv = [], []
for i in range(reps + 1):
    t = time.perf_counter(); assert lib.stark_best_fft(ctx, P(x), n, root, log_n, P(out)) == 0; fw.append(time.perf_counter() - t)
    t = time.perf_counter(); assert lib.stark_inv_best_fft(ctx, P(out), n, root, log_n, P(back)) == 0; iv.append(time.perf_counter() - t)
print(json.dumps({"fwd": [1e3 * v for v in fw[1:]], "inv": [1e3 * v for v in iv[1:]],
                  "digest": hashlib.sha256(out.tobytes()).hexdigest()[:16], "roundtrip": bool((back == x).all())}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    res = {lib: {"fwd": [], "inv": []} for lib in a.libs}
    for _ in range(a.rounds):
        for lib in a.libs:
            r = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(lib), str(a.log_n), str(a.reps)],
                               capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                print(f"{lib}: rc {r.returncode} {r.stderr[-400:]}", flush=True)
                continue
            v = json.loads(r.stdout.strip().splitlines()[-1])
            res[lib]["fwd"] += v["fwd"]
            res[lib]["inv"] += v["inv"]
            res[lib]["digest"] = v["digest"]
            res[lib]["roundtrip"] = v["roundtrip"]
    for lib, v in res.items():
        print(f"{os.path.basename(lib):12s} 2^{a.log_n} best_fft median {statistics.median(v['fwd']):8.2f} ms  "
              f"inv_best_fft median {statistics.median(v['inv']):8.2f} ms  digest {v.get('digest')}  "
              f"roundtrip {v.get('roundtrip')}", flush=True)


if __name__ == "__main__":
    main()
