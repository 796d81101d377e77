#!/bin/bash
# round-4 batch 21: the host record walk with a 4 KB software prefetch (variants/pfw.so) against the
# library before it (variants/base5.so): cold 2^20-step proof and pedersen, alternating order, and the
# trace head's phase time.
mkdir -p gpurun_out/r4x
(while true; do date > gpurun_out/r4x/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
V="variants/pfw.so variants/base5.so variants/base5.so variants/pfw.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --reps 8 > gpurun_out/r4x/ab_2_20.log 2>&1 || exit 1
timeout -k 10 200 python tools/time_r1cs_libs.py $V --reps 30 --fixture pedersen_test > gpurun_out/r4x/ab_ped.log 2>&1 || exit 2
for L in variants/base5.so variants/pfw.so; do
  STARK_PROFILE=1 timeout -k 10 200 python tools/time_r1cs_libs.py $L --reps 4 > gpurun_out/r4x/phases_$(basename $L .so).log 2>&1 || exit 3
done
