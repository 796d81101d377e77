"""Copies the reference's own R1CS/witness test fixtures (data files under
packages/r1cs-stark/tests/) into this directory, so the GPU box -- where
/root/reference does not exist -- can run the end-to-end prover tests.

These are inputs (circom binary R1CS + witness files), not source.  Run from
the repo root:  python tests/golden/r1cs/copy_fixtures.py
"""
import os
import shutil

SRC = "/root/reference/packages/r1cs-stark/tests"
DST = os.path.dirname(os.path.abspath(__file__))
FILES = [
    "compute.r1cs", "compute.wtns", "compute.r1cs.json",
    "poseidon3_test.r1cs", "poseidon3_test.wtns",
    "pedersen_test.r1cs", "pedersen_test.wtns",
    "bits.r1cs", "bits.wtns",
]

if __name__ == "__main__":
    for f in FILES:
        shutil.copyfile(os.path.join(SRC, f), os.path.join(DST, f))
        print("copied", f, os.path.getsize(os.path.join(DST, f)))
