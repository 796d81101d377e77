"""Board power and clocks while one kernel stream runs back to back (is the pass kernel power-bound?).
Runs stark_ntt_dev 2^24 (WHAT=ntt) or the Merkle build (WHAT=merkle) for ~SECS
seconds and samples `rocm-smi --showpower --showclocks` from a side thread; prints one JSON line."""
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "stark-pure-rust_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402  (input generator)
import stark_amd as S  # noqa: E402


def smi():
    try:
        return subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--json"], capture_output=True,
                              text=True, timeout=20).stdout
    except Exception as e:  # noqa: BLE001
        return repr(e)


def main():
    what = os.environ.get("WHAT", "ntt")
    secs = float(os.environ.get("SECS", "6"))
    ctx = S.Context(0)
    n = 1 << 24
    d = ctx.alloc(n * 32)
    ctx.h2d(d, O.random_elements(n, 0x5EED0018))
    w = O.root_of_unity(24)
    tree = S.MerkleProofInPlace(ctx) if what == "merkle" else None
    step = (lambda: tree.update_dev(d, n, 32)) if tree else (lambda: ctx.ntt_dev(d, 24, 1, w))
    samples = []
    stop = threading.Event()

    def sampler():
        time.sleep(1.5)
        while not stop.is_set():
            samples.append(smi())
            time.sleep(0.5)

    th = threading.Thread(target=sampler)
    idle = smi()
    th.start()
    t0 = time.time()
    k = 0
    while time.time() - t0 < secs:
        for _ in range(50):
            step()
        ctx.synchronize()
        k += 50
    stop.set()
    th.join()
    print(json.dumps({"what": what, "steps": k,
                      "ms_per_step": (time.time() - t0) * 1e3 / k, "idle": idle, "busy": samples[:6]}))


if __name__ == "__main__":
    main()
