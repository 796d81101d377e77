#!/bin/bash
# round-4 batch 23: the record walk in 8 pieces on the host workers beside the staged upload
# (variants/walk.so = in-tree) against variants/base5.so; r1cs / verify / dprove / large GPU tests first.
mkdir -p gpurun_out/r4z
(while true; do date > gpurun_out/r4z/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 800 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_dprove.py tests/test_gpu_large.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4z/tests.log 2>&1 || exit 1
V="variants/walk.so variants/base5.so variants/base5.so variants/walk.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --reps 8 > gpurun_out/r4z/ab_2_20.log 2>&1 || exit 2
timeout -k 10 200 python tools/time_r1cs_libs.py $V --reps 30 --fixture pedersen_test > gpurun_out/r4z/ab_ped.log 2>&1 || exit 3
timeout -k 10 400 python tools/time_verify_libs.py $V --reps 20 --synth > gpurun_out/r4z/ab_verify.log 2>&1 || exit 4
for L in variants/base5.so variants/walk.so; do
  STARK_PROFILE=1 timeout -k 10 200 python tools/time_r1cs_libs.py $L --reps 4 > gpurun_out/r4z/phases_$(basename $L .so).log 2>&1 || exit 5
done
