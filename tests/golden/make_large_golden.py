"""Generates tests/golden/large_digests.json: SHA-256 digests of the ORACLE's outputs at the
sizes bench.py times, so a GPU run can be checked at full size without the oracle's minutes of
CPU work.  Everything here is computed by the C restatement (oracle/oracle.c,
oracle/r1cs.c), which tests/test_oracle_kat.py pins to the reference's known-answer vectors and
to the DFT definition:

* ntt 2^24 forward and inverse (fft.rs:327-379 best_fft / inv_best_fft) on bench.py's rank-0
  input: random_elements(2^24, 0x5EED0000 + 24), w = 7^((p-1)/2^24);
* ntt 2^20 forward and inverse (config 2) on random_elements(2^20, 0x5EED0000 + 20);
* ntt 2^25, 2^26 and 2^27 forward and inverse on random_elements(2^k, 0x5EED0000 + k): the plans
  (8, 8, 9), (6, 6, 7, 7) and (9, 9, 9) -- the radix-2^9 passes, the four-pass digit-basis plan with
  its two-level-table column twiddles, and (2^27, past the full last-pass table) the lo * hi column
  twiddle of the last pass;
* prove_low_degree (fri.rs:46-224) at precision 2^23 on bench.py's FRI input: the evaluations of
  random_elements(2^21, 0x5EED0000 + 23) zero-padded to 2^23, maxdeg 2^21, exclude 8;
* mk_r1cs_proof (prove.rs:14-378) on the synthetic 2^20-step circuit tools/synth_r1cs.for_steps(20)
  (the stand-in for sha256_2_test, whose .r1cs the reference does not ship).

Digests are over the raw little-endian limb bytes (vectors) or the StarkProof/FriProof JSON.

    python tests/golden/make_large_golden.py [--threads T] [--ntt 20,24,25,26,27] [--ntt-only]
    (~3-5 min on 8 cores for the default sizes and the proofs; 2^25..2^27 add ~10 min)
"""
import argparse
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402

OUT = os.path.join(HERE, "large_digests.json")


def sha(a) -> str:
    if isinstance(a, str):
        a = a.encode()
    elif isinstance(a, np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.uint64).tobytes()
    return hashlib.sha256(a).hexdigest()


def random_coeffs(log_n: int) -> np.ndarray:
    return O.random_elements(1 << (log_n - 2), 0x5EED0000 + log_n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--skip-proof", action="store_true")
    ap.add_argument("--ntt", default="20,24", help="NTT sizes (log2) to digest")
    ap.add_argument("--ntt-only", action="store_true", help="only the NTT digests")
    args = ap.parse_args()
    T = 1 << (args.threads.bit_length() - 1)
    o = O.Oracle()
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    out["generator"] = "tests/golden/make_large_golden.py (oracle C restatement)"
    for log_n in [int(x) for x in args.ntt.split(",") if x]:
        t0 = time.time()
        c = O.random_elements(1 << log_n, 0x5EED0000 + log_n)
        w = O.root_of_unity(log_n)
        fwd = o.best_fft(c, w, log_n, cpus=T)
        inv = o.inv_best_fft(c, w, log_n, cpus=T)
        out[f"ntt_2^{log_n}"] = {"input": f"random_elements(2^{log_n}, 0x5EED0000 + {log_n})",
                                 "root": f"root_of_unity({log_n})",
                                 "input_sha256": sha(c), "forward_sha256": sha(fwd), "inverse_sha256": sha(inv),
                                 "forward_head": [str(x) for x in O.from_limbs(fwd[:2])]}
        print(f"ntt 2^{log_n}: {time.time() - t0:.1f} s", flush=True)
        del c, fwd, inv
        json.dump(out, open(OUT, "w"), indent=1)
    if args.ntt_only:
        return
    lf = 23
    t0 = time.time()
    nf = 1 << lf
    wf = O.root_of_unity(lf)
    coef = random_coeffs(lf)
    vals = o.best_fft(coef, wf, lf, cpus=T)
    js = o.prove_low_degree_json(vals, wf, nf // 4, 8, chunks=T)
    out["fri_2^23"] = {"input": "best_fft(random_elements(2^21, 0x5EED0000 + 23) zero-padded, root_of_unity(23))",
                       "max_deg_plus_1": nf // 4, "exclude": 8, "values_sha256": sha(vals),
                       "json_sha256": sha(js), "json_len": len(js)}
    print(f"fri 2^23: {time.time() - t0:.1f} s", flush=True)
    if not args.skip_proof:
        import r1cs as R
        import synth_r1cs
        t0 = time.time()
        rs, ws = synth_r1cs.for_steps(20)
        tr = R.build_trace(R.read_r1cs(rs), R.read_witness(ws))
        print(f"synth 2^20 trace: {time.time() - t0:.1f} s", flush=True)
        js = R.mk_r1cs_proof_json(o, tr, cpus=T)
        out["prove_synth_2^20_steps"] = {"input": "tools/synth_r1cs.for_steps(20)",
                                         "r1cs_sha256": sha(rs), "wtns_sha256": sha(ws),
                                         "json_sha256": sha(js), "json_len": len(js)}
        print(f"proof 2^20 steps: {time.time() - t0:.1f} s", flush=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
