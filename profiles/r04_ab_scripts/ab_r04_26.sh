#!/bin/bash
# round-4 batch 26: the record walk in 8 pieces (variants/walk.so = in-tree) against variants/base5.so after
# the prover GPU tests: cold 2^20-step proof, pedersen, the cold verifier and the trace head's phase time.
mkdir -p gpurun_out/r4ac
(while true; do date > gpurun_out/r4ac/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ac/tests.log 2>&1 || exit 1
V="variants/walk.so variants/base5.so variants/base5.so variants/walk.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --reps 8 > gpurun_out/r4ac/ab_2_20.log 2>&1 || exit 2
timeout -k 10 200 python tools/time_r1cs_libs.py $V --reps 30 --fixture pedersen_test > gpurun_out/r4ac/ab_ped.log 2>&1 || exit 3
timeout -k 10 400 python tools/time_verify_libs.py $V --reps 20 --synth > gpurun_out/r4ac/ab_verify.log 2>&1 || exit 4
for L in variants/base5.so variants/walk.so; do
  STARK_PROFILE=1 timeout -k 10 200 python tools/time_r1cs_libs.py $L --reps 4 > gpurun_out/r4ac/phases_$(basename $L .so).log 2>&1 || exit 5
done
