#!/bin/bash
# round-4 batch 14: 2^20 as two radix-2^10 passes (variants/r10.so, generic Shoup steps, B = 1 tiles,
# two workgroups per CU: no 1.33-round tail) against (8, 4, 8) (fin4); dense 2^20 and the 2^17 -> 2^20 LDE.
mkdir -p gpurun_out/r4p
(while true; do date > gpurun_out/r4p/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
V="variants/fin4.so variants/r10.so variants/fin4.so variants/r10.so"
LOG_N=20 REPS=500 WARM=50 timeout -k 10 120 python tools/time_ntt.py $V > gpurun_out/r4p/ab20.log 2>&1 || exit 1
LOG_STEPS=17 BATCH=8 REPS=100 timeout -k 10 120 python tools/time_lde.py $V > gpurun_out/r4p/lde17.log 2>&1 || exit 2
# (then batch 15 in the same call)
./tools/ab_r04_15.sh || exit $((10 + $?))
