#!/bin/bash
# round-4 batch 11: prepared-verify phases, round-start library (head) vs final (fin4), alternating.
mkdir -p gpurun_out/r4m
(while true; do date > gpurun_out/r4m/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
V="variants/fin4.so variants/head.so variants/fin4.so variants/head.so"
timeout -k 10 300 python tools/time_verify_libs.py $V --reps 60 > gpurun_out/r4m/ab_verify.log 2>&1 || exit 1
STARK_PROFILE=1 timeout -k 10 200 python tools/time_verify_libs.py variants/head.so variants/fin4.so --reps 5 > gpurun_out/r4m/phases.log 2>&1 || exit 2
