"""Times stark_ntt_dev (2^log_n forward, HBM-resident) for one or more builds
of libstark_hip.so given on the command line (A/B in one process)."""
import ctypes
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (synthetic input generator only)


def main():
    log_n = int(os.environ.get("LOG_N", "24"))
    libs = sys.argv[1:]
    n = 1 << log_n
    host = O.random_elements(n, 0x5EED0000 + log_n)
    w = O.to_limbs([O.root_of_unity(log_n)])[0]
    u64p = ctypes.POINTER(ctypes.c_uint64)
    results = {}
    for path in libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        lib.stark_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        lib.stark_ntt_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, u64p,
                                      ctypes.c_int, ctypes.c_void_p]
        lib.stark_dev_alloc.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
        lib.stark_memcpy_h2d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.stark_ctx_synchronize.argtypes = [ctypes.c_void_p]
        ctx = ctypes.c_void_p()
        assert lib.stark_ctx_create(0, ctypes.byref(ctx)) == 0
        d = ctypes.c_void_p()
        assert lib.stark_dev_alloc(ctx, n * 32, ctypes.byref(d)) == 0
        lib.stark_memcpy_h2d(ctx, d, host.ctypes.data, n * 32)
        wp = w.ctypes.data_as(u64p)
        if os.environ.get("WHAT") == "merkle":   # Merkle commit of n 32-B leaves instead
            lib.stark_merkle_new.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
            lib.stark_merkle_update_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                    ctypes.c_size_t, ctypes.c_void_p]
            tree = ctypes.c_void_p()
            assert lib.stark_merkle_new(ctx, ctypes.byref(tree)) == 0
            step = lambda: lib.stark_merkle_update_dev(tree, d, n, 32, None)  # noqa: E731
        else:
            step = lambda: lib.stark_ntt_dev(ctx, d, log_n, 1, wp, 0, None)  # noqa: E731
        for _ in range(int(os.environ.get("WARM", "3"))):
            step()
        lib.stark_ctx_synchronize(ctx)
        reps = int(os.environ.get("REPS", "20"))
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        lib.stark_ctx_synchronize(ctx)
        ms = (time.perf_counter() - t0) * 1000 / reps
        results[path] = ms
        # Every build ran the same WARM + REPS in-place transforms of the same input: equal digests = equal outputs.
        lib.stark_memcpy_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        back = np.empty_like(host)
        lib.stark_memcpy_d2h(ctx, back.ctypes.data, d, n * 32)
        lib.stark_ctx_synchronize(ctx)
        dig = hashlib.sha256(back.tobytes()).hexdigest()[:16]
        print(f"{path}: {ms:.3f} ms  ({n / ms / 1e6:.3f} G elems/s)  out {dig}", flush=True)


if __name__ == "__main__":
    main()
