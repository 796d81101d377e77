#!/bin/bash
# round-4 GPU pass after the 2^26 plan change: every GPU test, smoke(), the default bench line, and
# the small proofs' phase / gap profile
mkdir -p gpurun_out/r4f
(while true; do date > gpurun_out/r4f/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
if ls variants/skip0.so > /dev/null 2>&1; then
  V="variants/head.so variants/skip0.so variants/head.so variants/skip0.so"
  REPS=200 WARM=20 timeout -k 10 200 python tools/time_ntt.py $V > gpurun_out/r4f/skip0_24.log 2>&1 || exit 5
  LOG_N=20 REPS=500 WARM=50 timeout -k 10 200 python tools/time_ntt.py $V > gpurun_out/r4f/skip0_20.log 2>&1 || exit 6
  LOG_N=23 REPS=200 WARM=20 timeout -k 10 200 python tools/time_ntt.py $V > gpurun_out/r4f/skip0_23.log 2>&1 || exit 7
  LOG_STEPS=20 REPS=30 timeout -k 10 200 python tools/time_lde.py $V > gpurun_out/r4f/skip0_lde.log 2>&1 || exit 8
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/r4f/bench.json 2> gpurun_out/r4f/bench.err || exit 3
bash tools/prof_small_proofs.sh || exit 4
