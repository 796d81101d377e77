#!/bin/bash
# round-4 batch 17: Zb2 / Zb3 stored as Zb R^-1 so their batch inverses are Montgomery images (two products
# fewer per point in the constraint kernel, no to_mont pass in circuit_lde): variants/mz.so = in-tree, against
# variants/zb3.so (the shared-column library before it); prover / verifier / distributed GPU tests first.
mkdir -p gpurun_out/r4s
(while true; do date > gpurun_out/r4s/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_dprove.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4s/tests.log 2>&1 || exit 1
V="variants/mz.so variants/zb3.so variants/zb3.so variants/mz.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --reps 8 > gpurun_out/r4s/ab_2_20.log 2>&1 || exit 2
timeout -k 10 200 python tools/time_r1cs_libs.py $V --reps 30 --fixture pedersen_test > gpurun_out/r4s/ab_ped.log 2>&1 || exit 3
