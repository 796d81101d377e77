"""Generates the committed golden vectors under tests/golden/ with the
pure-Python restatement in oracle/oracle.py (exact integers; NTTs by the DFT
definition).  The reference itself (Rust) cannot be built or run in this
environment, so these vectors are pinned to the reference through the
restatement, which tests/test_oracle_kat.py checks against every known-answer
vector the reference's tests hold (reference_kats.json).

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import oracle as O  # noqa: E402


def main():
    out = {"ntt": [], "merkle": [], "fri": []}
    # NTT: out[i] = sum_j c_j w^(ij), w = 7^((p-1)/n); short inputs are zero padded (best_fft).
    for log_n, length, seed in ((0, 1, 1), (1, 2, 2), (3, 5, 3), (4, 16, 4), (6, 40, 5), (8, 256, 6)):
        n = 1 << log_n
        c = O.from_limbs(O.random_elements(length, 0x5EED0000 + seed))
        w = O.root_of_unity(log_n)
        y = O.py_dft(c, w, n)
        winv = pow(w, O.P - 2, O.P)
        inv = [v * pow(n, O.P - 2, O.P) % O.P for v in O.py_dft(c + [0] * (n - length), winv, n)]
        out["ntt"].append({"log_n": log_n, "root": str(w), "coeffs": [str(v) for v in c],
                           "forward": [str(v) for v in y], "inverse": [str(v) for v in inv]})
    # Merkle over 32-B canonical field elements (the FRI / L-tree leaves).
    for log_n, idx in ((0, [0]), (3, [5, 0, 5]), (10, [1, 1023, 512, 7])):
        n = 1 << log_n
        leaves = [O.to_bytes_le(v) for v in O.from_limbs(O.random_elements(n, 0xABC + log_n))]
        root, paths = O.py_merkle(leaves, idx)
        out["merkle"].append({"n": n, "leaf_len": 32, "seed": 0xABC + log_n, "indices": idx, "root": root.hex(),
                              "paths": [[d.hex() for d in p] for p in paths]})
    # FRI over the evaluations of a random polynomial of degree < n/4 (BASELINE.md synthetic input).
    for log_n, excl in ((7, 8), (9, 8), (10, 0)):
        n = 1 << log_n
        w = O.root_of_unity(log_n)
        coeffs = O.from_limbs(O.random_elements(n // 4, 0x5EED0000 + log_n))
        vals = O.py_dft(coeffs, w, n)
        js = O.py_prove_low_degree_json(vals, w, n // 4, excl)
        rec = {"log_n": log_n, "exclude": excl, "coeff_seed": 0x5EED0000 + log_n,
               "json_sha256": hashlib.sha256(js.encode()).hexdigest(), "json_len": len(js)}
        out["fri"].append(rec)
    with open(os.path.join(HERE, "golden_vectors.json"), "w") as f:
        json.dump(out, f)
    print("wrote golden_vectors.json")


if __name__ == "__main__":
    main()
