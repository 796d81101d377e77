"""The proof reader's AVX-512 path for u8 arrays (host_json_v512.cpp json_u8s_v512, used by the verifier's
serde_json reader, verify.hip Json::bytes_to): on compact text "d,d,...,d]" it must give exactly the
numbers serde_json reads, and on anything else -- leading zeros, values above 255, four digits,
whitespace, empty slots, a missing ']', too many numbers -- it must decline (nullptr), so that the
scalar reader (covered by tests/test_gpu_verify.py) decides.  A C++ client calls it on this host."""
import os
import random
import subprocess

import pytest

S = pytest.importorskip("stark_amd")

HERE = os.path.dirname(os.path.abspath(__file__))
CLIENT = os.path.join(HERE, "abi_client")


def _model(text, mx):
    vals, i = [], 0
    while True:
        j = i
        while j < len(text) and text[j].isdigit():
            j += 1
        d = text[i:j]
        if not 1 <= len(d) <= 3 or (len(d) > 1 and d[0] == "0") or int(d) > 255:
            return None
        vals.append(int(d))
        if len(vals) > mx or j >= len(text):
            return None
        if text[j] == "]":
            return vals, j + 1
        if text[j] != ",":
            return None
        i = j + 1


def _cases():
    rng = random.Random(5)
    edge = [0, 1, 9, 10, 99, 100, 199, 200, 254, 255]
    out = []
    for n in list(range(1, 70)) + [100, 255, 1000]:
        vals = [rng.choice(edge) if rng.random() < 0.3 else rng.randrange(256) for _ in range(n)]
        body = ",".join(map(str, vals)) + "]"
        tail = rng.choice(["", ",\"nodes\":[[1,2]]}", "]}", ",[3]"])
        out.append((n, body + tail))
        out.append((n - 1, body + tail))  # one number too many
        # single mutations: each must be declined unless the model still accepts
        for bad in ["05", "256", "1000", " 1", "1 ", "", "a", "-1", "00", "300"]:
            k = rng.randrange(n)
            m = list(map(str, vals))
            m[k] = bad
            out.append((n, ",".join(m) + "]" + tail))
        out.append((n, body[:-1]))                  # no ']'
        out.append((n, body[:-1] + ",]"))           # trailing comma
        out.append((n, body.replace(",", ",,", 1)))  # an empty slot
    out.append((4, "]"))
    return out


def test_simd_u8_arrays_match_serde(tmp_path):
    lib = S.load_library()
    if lib.stark_json_simd_width() != 64:
        pytest.skip("this CPU has no AVX-512 VBMI2: the reader uses its scalar loop only")
    subprocess.run(["make", "-s", "-C", CLIENT, "json_u8s"], check=True)
    cases = _cases()
    inp = "".join(f"{mx}\t{t}\n" for mx, t in cases)
    r = subprocess.run([os.path.join(CLIENT, "json_u8s")], input=inp, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = r.stdout.splitlines()
    assert len(got) == len(cases)
    accepted = 0
    for (mx, text), g in zip(cases, got):
        want = _model(text, mx)
        if want is None:
            assert g == "null", (mx, text[:80], g)
        else:
            vals, end = want
            accepted += 1
            assert g == f"ok {len(vals)} {end} {bytes(vals).hex()}", (mx, text[:80], g)
    assert accepted >= 70  # (every well-formed case with room for its numbers)
