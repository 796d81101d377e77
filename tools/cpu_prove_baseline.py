"""CPU baseline of the end-to-end leg: the oracle's C restatement of mk_r1cs_proof (prove.rs:14-378,
oracle/r1cs.c) on the synthetic 2^20-step circuit (tools/synth_r1cs.py, the sha256_2_test stand-in),
with T = 2^floor(log2 min(physical cores, CPUs granted)) threads as bench.py's cpu_baseline.  Its JSON
is checked against the oracle digest in tests/golden/large_digests.json.  Too slow for every bench
run, so it runs once per round on the GPU box and bench.py reports the committed record:

    python tools/cpu_prove_baseline.py gpurun_out/cpu_prove_synth_2_20.json
    (then copy to profiles/r0N_cpu_prove_synth_2_20.json)
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402
import r1cs as R  # noqa: E402
import synth_r1cs  # noqa: E402
from bench import host_cpus  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "cpu_prove_synth_2_20.json")
    physical, usable = host_cpus()
    threads = 1 << (min(physical, usable).bit_length() - 1)
    o = O.Oracle()
    rs, ws = synth_r1cs.for_steps(20)
    t0 = time.perf_counter()
    tr = R.build_trace(R.read_r1cs(rs), R.read_witness(ws))
    t1 = time.perf_counter()
    js = R.mk_r1cs_proof_json(o, tr, cpus=threads)
    t2 = time.perf_counter()
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "large_digests.json")))["prove_synth_2^20_steps"]
    rec = {"value": round((t2 - t1) * 1000.0, 1), "unit": "ms", "cores": threads, "threads": threads,
           "host_physical_cores": physical, "cpus_granted": usable, "kind": "port",
           "sample": "one mk_r1cs_proof of the synthetic 2^20-step circuit (precision 2^23), oracle C "
                     "restatement; the trace build (Python restatement of run.rs) not included",
           "trace_build_python_ms": round((t1 - t0) * 1000.0, 1),
           "json_bitexact_vs_oracle_digest": hashlib.sha256(js.encode()).hexdigest() == want["json_sha256"],
           "source": "tools/cpu_prove_baseline.py on the GPU box"}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
