#!/bin/bash
# round-4 A/B batch 5: small-proof host overlap (proof head JSON on the side thread beside the FRI finish,
# branch JSON rendered into one buffer) -- prover GPU tests, pedersen / poseidon3 / 2^20-step A/B, phases.
mkdir -p gpurun_out/r4g
(while true; do date > gpurun_out/r4g/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "r1cs or verify or merkle_fri or abi" > gpurun_out/r4g/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/time_r1cs_libs.py variants/head.so variants/side.so variants/head.so variants/side.so --fixture pedersen_test --reps 40 > gpurun_out/r4g/ab_pedersen.log 2>&1 || exit 2
timeout -k 10 300 python tools/time_r1cs_libs.py variants/head.so variants/side.so variants/head.so variants/side.so --fixture poseidon3_test --reps 40 > gpurun_out/r4g/ab_poseidon3.log 2>&1 || exit 3
timeout -k 10 300 python tools/time_r1cs_libs.py variants/head.so variants/side.so variants/head.so variants/side.so --steps 20 --reps 6 > gpurun_out/r4g/ab_2_20.log 2>&1 || exit 4
bash tools/prof_small_proofs.sh || exit 5
