#!/bin/bash
# round-4 batch 18: 1 / Zb2 by partial fractions over a shared 1 / (x - 1) table (no batch inverse over the
# domain in a cold proof; variants/pf.so = in-tree) against variants/mz.so; prover / verifier / distributed /
# large GPU tests first.
mkdir -p gpurun_out/r4t
(while true; do date > gpurun_out/r4t/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 800 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_dprove.py tests/test_gpu_large.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4t/tests.log 2>&1 || exit 1
V="variants/pf.so variants/mz.so variants/mz.so variants/pf.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --reps 8 > gpurun_out/r4t/ab_2_20.log 2>&1 || exit 2
timeout -k 10 200 python tools/time_r1cs_libs.py $V --reps 30 --fixture pedersen_test > gpurun_out/r4t/ab_ped.log 2>&1 || exit 3
