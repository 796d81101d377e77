"""The proof JSON writer's byte arrays (fri.hip json_bytes_at; serde_json of Vec<u8> / [u8; 32], as
StarkProof is written by run.rs:549 and FriProof by fri.rs:16-26): the AVX-512 digits
(host_json_v512.cpp) and the scalar table path must both give exactly json.dumps' compact text.
stark_r1cs_proof_json_from_parts renders a whole StarkProof on the host (no GPU), once per path in
its own process (the path is chosen once per process; STARK_JSON_SIMD=0 forces the scalar one)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytest.importorskip("stark_amd")

HERE = os.path.dirname(os.path.abspath(__file__))

# leaf lengths around the 16-byte groups (the SIMD path covers whole groups, the rest is scalar) and
# the proof's own 32 / 256; byte values include every digit-count boundary
LEAF_LENS = [1, 2, 15, 16, 17, 31, 32, 33, 48, 63, 64, 65, 100, 256]


def _parts(seed, main_leaf, lcomb_leaf):
    rng = np.random.default_rng(seed)

    def arr(*shape):
        a = rng.integers(0, 256, size=shape, dtype=np.uint8)
        flat = a.reshape(-1)
        edge = np.array([0, 9, 10, 99, 100, 199, 200, 255], dtype=np.uint8)
        flat[: min(len(flat), len(edge))] = edge[: len(flat)]
        return a

    def branches(k, leaf_len, depth):
        return arr(k, leaf_len), arr(k, depth, 32)

    roots = [bytes(arr(32)) for _ in range(3)]
    main = branches(12, main_leaf, 5)
    lcomb = branches(7, lcomb_leaf, 3)
    # FRI leaves are 32-B field elements (the writer refuses other lengths)
    layers = [(bytes(arr(32)), branches(3 + i, 32, 1 + i), branches(2 + i, 32, 2 + i)) for i in range(4)]
    last = bytes(arr(9 * 32))
    return roots, main, lcomb, layers, last


def _cases():
    return [(11 + i, ll, LEAF_LENS[-1 - i]) for i, ll in enumerate(LEAF_LENS)]


def _expected(roots, main, lcomb, layers, last):
    def br(b):
        leaves, nodes = b
        return [{"leaf": leaves[i].tolist(), "nodes": nodes[i].tolist()} for i in range(leaves.shape[0])]

    fri = [{"Middle": {"root2": list(r2), "column_branches": br(c), "poly_branches": br(p)}} for r2, c, p in layers]
    fri.append({"Last": {"last": [list(last[i:i + 32]) for i in range(0, len(last), 32)]}})
    doc = {"m_root": list(roots[0]), "l_root": list(roots[1]), "a_root": list(roots[2]),
           "main_branches": br(main), "linear_comb_branches": br(lcomb), "fri_proof": fri}
    return json.dumps(doc, separators=(",", ":"))


@pytest.mark.parametrize("simd", ["1", "0"])
def test_proof_json_from_parts_equals_serde_text(tmp_path, simd):
    child = (
        "import json, sys\n"
        f"sys.path.insert(0, {HERE!r})\n"
        "import stark_amd as S\n"
        "from stark_amd.dprove import render_json\n"
        "from test_json_writer import _parts, _cases\n"
        "lib = S.load_library()\n"
        "out = []\n"
        "for seed, ml, ll in _cases():\n"
        "    roots, main, lcomb, layers, last = _parts(seed, ml, ll)\n"
        "    out.append(render_json(lib, *roots, main, lcomb, layers, last))\n"
        f"open({str(tmp_path / 'out.json')!r}, 'w').write(json.dumps(out))\n"
        "print(lib.stark_json_simd_width())\n")
    env = dict(os.environ, STARK_JSON_SIMD=simd)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(os.path.dirname(HERE), "stark-pure-rust_amd"),
                                         env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    width = int(r.stdout.strip().splitlines()[-1])
    assert width in (1, 64)
    if simd == "0":
        assert width == 1
    got = json.loads((tmp_path / "out.json").read_text())
    assert len(got) == len(_cases())
    for text, (seed, ml, ll) in zip(got, _cases()):
        assert text == _expected(*_parts(seed, ml, ll)), (seed, ml, ll)


def test_fri_leaves_must_be_32_bytes():
    import stark_amd as S
    from stark_amd.dprove import render_json
    roots, main, lcomb, layers, last = _parts(3, 32, 32)
    bad = [(layers[0][0], (layers[0][1][0][:, :16], layers[0][1][1]), layers[0][2])]
    with pytest.raises(RuntimeError):  # the library's STARK_ERR_BAD_ARG
        render_json(S.load_library(), *roots, main, lcomb, bad, last)
