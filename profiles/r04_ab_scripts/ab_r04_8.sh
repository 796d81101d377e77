#!/bin/bash
# round-4 A/B batch 8: which of the batch-7 changes cost time (fin = all; fin2 = without the fused small FRI
# layers; fin3 = fin2 with the head JSON on 16 threads), and a kernel trace of the cold 2^20-step proof.
mkdir -p gpurun_out/r4j
(while true; do date > gpurun_out/r4j/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
V="variants/new.so variants/fin.so variants/fin2.so variants/fin3.so variants/new.so variants/fin.so variants/fin2.so variants/fin3.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture pedersen_test --reps 40 > gpurun_out/r4j/ab_pedersen.log 2>&1 || exit 1
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture poseidon3_test --reps 40 > gpurun_out/r4j/ab_poseidon3.log 2>&1 || exit 2
timeout -k 10 400 python tools/time_r1cs_libs.py $V --steps 20 --reps 8 > gpurun_out/r4j/ab_2_20.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4j/trace20 -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs.py --fixtures "" --synth 20 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r4j/trace20.log 2>&1 || exit 4
