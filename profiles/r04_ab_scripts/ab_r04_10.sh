#!/bin/bash
# round-4 batch 10: the final library (fin4) -- every GPU test, smoke, proof and verifier A/B against the
# round's starting library (head), the bench line.
mkdir -p gpurun_out/r4l
(while true; do date > gpurun_out/r4l/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4l/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l/smoke.log 2>&1 || exit 2
V="variants/head.so variants/fin4.so variants/head.so variants/fin4.so"
timeout -k 10 300 python tools/time_verify_libs.py $V --reps 30 > gpurun_out/r4l/ab_verify.log 2>&1 || exit 3
for f in pedersen_test poseidon3_test compute; do
  timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture $f --reps 40 > gpurun_out/r4l/ab_$f.log 2>&1 || exit 4
done
timeout -k 10 300 python tools/time_r1cs_libs.py $V --steps 20 --reps 8 > gpurun_out/r4l/ab_2_20.log 2>&1 || exit 5
timeout -k 10 600 python bench.py > gpurun_out/r4l/bench.json 2> gpurun_out/r4l/bench.err || exit 6
