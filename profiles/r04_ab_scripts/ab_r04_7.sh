#!/bin/bash
# round-4 A/B batch 7: the small FRI layers fused into one launch, one host round trip for the cold proof's
# two batch inverses, 16-term running-sum prefetch -- every GPU test, smoke, the proof A/B, the bench line.
mkdir -p gpurun_out/r4i
(while true; do date > gpurun_out/r4i/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4i/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4i/smoke.log 2>&1 || exit 2
V="variants/head.so variants/new.so variants/fin.so variants/head.so variants/new.so variants/fin.so"
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture pedersen_test --reps 40 > gpurun_out/r4i/ab_pedersen.log 2>&1 || exit 3
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture poseidon3_test --reps 40 > gpurun_out/r4i/ab_poseidon3.log 2>&1 || exit 4
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture compute --reps 40 > gpurun_out/r4i/ab_compute.log 2>&1 || exit 5
timeout -k 10 300 python tools/time_r1cs_libs.py $V --steps 20 --reps 6 > gpurun_out/r4i/ab_2_20.log 2>&1 || exit 6
timeout -k 10 600 python bench.py > gpurun_out/r4i/bench.json 2> gpurun_out/r4i/bench.err || exit 7
bash tools/prof_small_proofs.sh || exit 8
