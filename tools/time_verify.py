"""Verifier wall-clock split: cold (stark_verify_with_witness: circuit built per call) versus a
prepared circuit (stark_verify_r1cs_circuit), and the FRI host verifier alone."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]
import stark_amd as S  # noqa: E402
from stark_amd.r1cs import R1csCircuit, prove_with_witness  # noqa: E402
from stark_amd.verify import verify_circuit, verify_low_degree_proof, verify_with_wtns  # noqa: E402
import r1cs as R  # noqa: E402
import oracle as O  # noqa: E402


def best(fn, reps=5):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 3)


def main():
    ctx = S.Context(0)
    fix = os.path.join(ROOT, "tests", "golden", "r1cs")
    r1 = open(os.path.join(fix, "pedersen_test.r1cs"), "rb").read()
    wt = open(os.path.join(fix, "pedersen_test.wtns"), "rb").read()
    js = prove_with_witness(ctx, r1, wt).to_json()
    jb = js.encode()
    h = R.read_r1cs(r1).header
    pub = R.read_witness(wt)[:1 + h.n_public_inputs + h.n_public_outputs]
    c = R1csCircuit(ctx, r1)
    out = {"json_bytes": len(jb)}
    out["cold_ms"] = best(lambda: verify_with_wtns(ctx, r1, wt, jb))
    out["prepared_ms"] = best(lambda: verify_circuit(ctx, c, pub, jb))
    out["circuit_build_ms"] = best(lambda: R1csCircuit(ctx, r1))
    p = json.loads(js)
    log_p = 18
    out["fri_host_ms"] = best(lambda: verify_low_degree_proof(bytes(p["l_root"]), O.root_of_unity(log_p),
                                                              p["fri_proof"], (1 << log_p) // 4, 8))
    print(json.dumps(out))
    del c
    ctx.close()


if __name__ == "__main__":
    main()
