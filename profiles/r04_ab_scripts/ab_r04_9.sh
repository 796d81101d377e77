#!/bin/bash
# round-4 batch 9: the library without the fused FRI tail, with the verifier's one-launch path check --
# every GPU test, smoke, the verifier A/B (fin3 = host path checks), the proof A/B, the bench line.
mkdir -p gpurun_out/r4k
(while true; do date > gpurun_out/r4k/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4k/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k/smoke.log 2>&1 || exit 2
V="variants/head.so variants/fin3.so variants/ver.so variants/ver2.so variants/head.so variants/fin3.so variants/ver.so variants/ver2.so"
timeout -k 10 300 python tools/time_verify_libs.py $V --reps 30 > gpurun_out/r4k/ab_verify.log 2>&1 || exit 3
timeout -k 10 300 python tools/time_r1cs_libs.py $V --fixture pedersen_test --reps 40 > gpurun_out/r4k/ab_pedersen.log 2>&1 || exit 4
timeout -k 10 600 python bench.py > gpurun_out/r4k/bench.json 2> gpurun_out/r4k/bench.err || exit 5
STARK_PROFILE=1 timeout -k 10 120 python tools/time_verify.py > gpurun_out/r4k/verify_phases.log 2>&1 || exit 6
