"""Times stark_lde_dev (the prover's LDE: iNTT over 2^log_steps then the sparse NTT over 8x the points,
prove.rs:100-124) for one or more builds of libstark_hip.so given on the command line (A/B in one
process), batch 8 columns as the cold 2^20-step proof runs it.  Env: LOG_STEPS (20), BATCH (8), REPS (20).
Prints ms per LDE and a digest of the extended columns (equal digests = equal outputs)."""
import ctypes
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (inputs and roots only)


def main():
    log_steps = int(os.environ.get("LOG_STEPS", "20"))
    batch = int(os.environ.get("BATCH", "8"))
    reps = int(os.environ.get("REPS", "20"))
    n = 1 << log_steps
    host = O.random_elements(n * batch, 0x5EED7000 + log_steps)
    g2 = O.to_limbs([O.root_of_unity(log_steps + 3)])[0]
    g1 = O.to_limbs([pow(O.root_of_unity(log_steps + 3), 8, O.P)])[0]
    u64p = ctypes.POINTER(ctypes.c_uint64)
    for path in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.abspath(path))
        lib.stark_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        lib.stark_dev_alloc.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
        lib.stark_memcpy_h2d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.stark_memcpy_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.stark_ctx_synchronize.argtypes = [ctypes.c_void_p]
        lib.stark_lde_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, u64p, u64p, ctypes.c_void_p]
        ctx = ctypes.c_void_p()
        assert lib.stark_ctx_create(0, ctypes.byref(ctx)) == 0
        src, work, out = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        for b, sz in ((src, n * batch * 32), (work, n * batch * 32), (out, 8 * n * batch * 32)):
            assert lib.stark_dev_alloc(ctx, sz, ctypes.byref(b)) == 0
        lib.stark_memcpy_h2d(ctx, src, host.ctypes.data, n * batch * 32)

        def step():  # (d_values is transformed in place; the digest is taken after the first call)
            assert lib.stark_lde_dev(ctx, work, out, log_steps, 3, batch, g1.ctypes.data_as(u64p),
                                     g2.ctypes.data_as(u64p), None) == 0
        lib.stark_memcpy_h2d(ctx, work, host.ctypes.data, n * batch * 32)
        step()
        lib.stark_ctx_synchronize(ctx)
        back = np.empty((8 * n * batch, 4), dtype=np.uint64)
        lib.stark_memcpy_d2h(ctx, back.ctypes.data, out, back.nbytes)
        lib.stark_ctx_synchronize(ctx)
        dig = hashlib.sha256(back.tobytes()).hexdigest()[:16]
        for _ in range(3):
            step()
        lib.stark_ctx_synchronize(ctx)
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        lib.stark_ctx_synchronize(ctx)
        ms = (time.perf_counter() - t0) * 1000 / reps
        print(f"{path}: LDE 2^{log_steps} x {batch} -> 2^{log_steps + 3}: {ms:.3f} ms  out {dig}", flush=True)


if __name__ == "__main__":
    main()
