"""The C ABI from non-Python callers making exactly the calls of the Rust shim in INTEGRATION.md:
* tests/abi_client/shim_flow.cpp: best_fft -> MerkleProofInPlace new/update/gen_proofs/get_root ->
  prove_low_degree -> serde JSON; its outputs equal the oracle's best_fft (fft.rs:327-357), Merkle root
  and paths (merkle_proof_in_place.rs:106-206) and FRI proof JSON (fri.rs:46-224);
* tests/abi_client/prover_flow.cpp: the whole-prover routes (prove_with_witness on raw bytes, run.rs:
  310-452; mk_r1cs_proof on the exported trace vectors, prove.rs:14) and a StarkProof rebuilt from the
  structured parts (roots, branches, FRI layers) as the shim builds StarkProof<H> without serde; all
  four texts equal the golden StarkProof digests;
* tests/abi_client/group_flow.cpp: the device-group entry points (stark_group_*)
  at G = 2, 4, 8 members on one GPU: best_fft / inv_best_fft equal the oracle, the group Merkle root and
  paths equal the oracle's single tree, and the group's proofs (cold and prepared) equal the golden digests.
CPU: the programs build and link against libstark_hip.so."""
import os
import struct
import subprocess

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
CLIENT = os.path.join(HERE, "abi_client")
BIN = os.path.join(CLIENT, "shim_flow")
PROVER = os.path.join(CLIENT, "prover_flow")
GROUP = os.path.join(CLIENT, "group_flow")
FIX = os.path.join(HERE, "golden", "r1cs")


@pytest.mark.parametrize("prog", [BIN, PROVER, GROUP])
def test_client_builds_and_links(prog):
    subprocess.run(["make", "-s", "-C", CLIENT], check=True)
    out = subprocess.run(["ldd", prog], capture_output=True, text=True, check=True).stdout
    assert "libstark_hip.so" in out and "not found" not in out.split("libstark_hip.so")[1].splitlines()[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["compute", "pedersen_test"])
def test_prover_client_matches_golden(tmp_path, name):
    """Both whole-prover routes, as the library serialises them and as rebuilt from the parts, equal
    the golden StarkProof (tests/golden/r1cs_proofs.json, oracle/r1cs.c restating prove.rs:14-378)."""
    import hashlib
    import json
    assert os.path.exists(PROVER), "build() compiles tests/abi_client/prover_flow"
    want = json.load(open(os.path.join(HERE, "golden", "r1cs_proofs.json")))[name]["json_sha256"]
    r = subprocess.run([PROVER, os.path.join(FIX, f"{name}.r1cs"), os.path.join(FIX, f"{name}.wtns"), str(tmp_path)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    for f in ("bytes.json", "bytes_parts.json", "mk.json", "mk_parts.json"):
        assert hashlib.sha256((tmp_path / f).read_bytes()).hexdigest() == want, f


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,exclude", [(12, 8), (16, 8), (10, 0)])
def test_client_matches_oracle(oracle, tmp_path, log_n, exclude):
    assert os.path.exists(BIN), "build() compiles tests/abi_client/shim_flow"
    n = 1 << log_n
    coeffs = O.random_elements(n // 4, 0x5EED0300 + log_n)
    w = O.root_of_unity(log_n)
    idx = [0, 1, n - 1, 5, 5, n // 2 + 3]
    blob = struct.pack("<4I", log_n, len(coeffs), len(idx), exclude) + O.to_limbs([w]).tobytes() + \
        coeffs.tobytes() + np.array(idx, dtype=np.uint64).tobytes()
    (tmp_path / "in.bin").write_bytes(blob)
    r = subprocess.run([BIN, str(tmp_path / "in.bin"), str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    evals = np.frombuffer((tmp_path / "evals.bin").read_bytes(), dtype=np.uint64).reshape(-1, 4)
    assert np.array_equal(evals, oracle.best_fft(coeffs, w, log_n, cpus=8))
    root, paths = oracle.merkle(evals.tobytes(), n, 32, idx, chunks=4)
    assert (tmp_path / "merkle_root.bin").read_bytes() == root
    nodes = (tmp_path / "merkle_nodes.bin").read_bytes()
    assert [[nodes[(i * log_n + d) * 32:(i * log_n + d + 1) * 32] for d in range(log_n)]
            for i in range(len(idx))] == paths
    leaves = (tmp_path / "merkle_leaves.bin").read_bytes()
    assert leaves == b"".join(evals[i].tobytes() for i in idx)
    want = oracle.prove_low_degree_json(evals, w, n // 4, exclude, chunks=4)
    assert (tmp_path / "fri.json").read_text() == want


@pytest.mark.gpu
@pytest.mark.parametrize("G,name", [(2, "compute"), (4, "poseidon3_test"), (8, "pedersen_test")])
def test_group_client_matches_oracle(oracle, tmp_path, G, name):
    """The group entry points from C++ (G members on device 0): NTT and inverse vs the oracle, the Merkle
    root and paths vs the oracle's single tree, and both proofs vs the golden digest."""
    import hashlib
    import json
    assert os.path.exists(GROUP), "build() compiles tests/abi_client/group_flow"
    log_n = 16
    n = 1 << log_n
    coeffs = O.random_elements(n // 4 + 5, 0x5EED0800 + G)
    w = O.root_of_unity(log_n)
    idx = [0, 1, n - 1, 7, 7, n // 2 + 3, n // G]
    blob = struct.pack("<4I", log_n, len(coeffs), len(idx), 0) + O.to_limbs([w]).tobytes() + \
        coeffs.tobytes() + np.array(idx, dtype=np.uint64).tobytes()
    (tmp_path / "in.bin").write_bytes(blob)
    r = subprocess.run([GROUP, str(G), str(tmp_path / "in.bin"), os.path.join(FIX, f"{name}.r1cs"),
                        os.path.join(FIX, f"{name}.wtns"), str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    evals = np.frombuffer((tmp_path / "evals.bin").read_bytes(), dtype=np.uint64).reshape(-1, 4)
    assert np.array_equal(evals, oracle.best_fft(coeffs, w, log_n, cpus=8))
    back = np.frombuffer((tmp_path / "inv.bin").read_bytes(), dtype=np.uint64).reshape(-1, 4)
    assert np.array_equal(back[:len(coeffs)], coeffs) and not back[len(coeffs):].any()
    root, paths = oracle.merkle(evals.tobytes(), n, 32, idx, chunks=4)
    assert (tmp_path / "merkle_root.bin").read_bytes() == root
    nodes = (tmp_path / "merkle_nodes.bin").read_bytes()
    assert [[nodes[(i * log_n + d) * 32:(i * log_n + d + 1) * 32] for d in range(log_n)]
            for i in range(len(idx))] == paths
    assert (tmp_path / "merkle_leaves.bin").read_bytes() == b"".join(evals[i].tobytes() for i in idx)
    want = json.load(open(os.path.join(HERE, "golden", "r1cs_proofs.json")))[name]["json_sha256"]
    for f in ("proof.json", "proof_circuit.json"):
        assert hashlib.sha256((tmp_path / f).read_bytes()).hexdigest() == want, f
