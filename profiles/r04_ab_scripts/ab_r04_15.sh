#!/bin/bash
# round-4 batch 15: F0 shared extension (variants/f0.so), + the shared 1/Zb3 column (variants/zb3.so = in-tree): prover / verifier / distributed GPU tests,
# then the cold 2^20-step proof, pedersen and the verifier against fin4, alternating order.
mkdir -p gpurun_out/r4q
(while true; do date > gpurun_out/r4q/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_dprove.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4q/tests.log 2>&1 || exit 1
V="variants/zb3.so variants/f0.so variants/fin4.so variants/fin4.so variants/f0.so variants/zb3.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --reps 6 > gpurun_out/r4q/ab_2_20.log 2>&1 || exit 2
timeout -k 10 200 python tools/time_r1cs_libs.py $V --reps 30 --fixture pedersen_test > gpurun_out/r4q/ab_ped.log 2>&1 || exit 3
timeout -k 10 400 python tools/time_verify_libs.py $V --reps 30 --synth > gpurun_out/r4q/ab_verify.log 2>&1 || exit 4
