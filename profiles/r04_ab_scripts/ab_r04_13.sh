#!/bin/bash
# round-4 batch 13: the verifier's cold circuit build without the Zb inverses (nozb = in-tree) against fin4.
mkdir -p gpurun_out/r4o
(while true; do date > gpurun_out/r4o/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4o/tests.log 2>&1 || exit 1
V="variants/nozb.so variants/fin4.so variants/fin4.so variants/nozb.so"
timeout -k 10 400 python tools/time_verify_libs.py $V --reps 40 --synth > gpurun_out/r4o/ab_verify.log 2>&1 || exit 2
