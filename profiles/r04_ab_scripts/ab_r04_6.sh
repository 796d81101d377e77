#!/bin/bash
# round-4 A/B batch 6: small-proof host work (side-thread head JSON, one-buffer branch JSON; no trace
# read-back, one pack launch for the proof's inputs, the last FRI layer's download folded into the
# gather, running sums loaded eight terms ahead) -- every GPU test, then the A/B and the phase profile.
mkdir -p gpurun_out/r4h
(while true; do date > gpurun_out/r4h/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4h/tests.log 2>&1 || exit 1
V="variants/head.so variants/side.so variants/new.so variants/head.so variants/side.so variants/new.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture pedersen_test --reps 40 > gpurun_out/r4h/ab_pedersen.log 2>&1 || exit 2
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture poseidon3_test --reps 40 > gpurun_out/r4h/ab_poseidon3.log 2>&1 || exit 3
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture compute --reps 40 > gpurun_out/r4h/ab_compute.log 2>&1 || exit 4
timeout -k 10 300 python tools/time_r1cs_libs.py $V --steps 20 --reps 6 > gpurun_out/r4h/ab_2_20.log 2>&1 || exit 5
bash tools/prof_small_proofs.sh || exit 6
