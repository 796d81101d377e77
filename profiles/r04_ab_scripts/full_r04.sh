#!/bin/bash
# round-4 GPU pass: the persistent-pass A/B, then every GPU test, smoke(), the default bench line
mkdir -p gpurun_out/r4c
(while true; do date > gpurun_out/r4c/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
if ls variants/*.so > /dev/null 2>&1; then
  REPS=200 WARM=20 timeout -k 10 200 python tools/time_ntt.py variants/head.so variants/base.so variants/persist.so variants/head.so variants/base.so variants/persist.so > gpurun_out/r4c/ab24.log 2>&1 || exit 4
  LOG_N=23 REPS=200 WARM=20 timeout -k 10 200 python tools/time_ntt.py variants/head.so variants/base.so variants/persist.so variants/head.so variants/base.so variants/persist.so > gpurun_out/r4c/ab23.log 2>&1 || exit 5
  LOG_STEPS=20 REPS=30 timeout -k 10 200 python tools/time_lde.py variants/head.so variants/base.so variants/persist.so variants/head.so variants/base.so variants/persist.so > gpurun_out/r4c/ablde.log 2>&1 || exit 6
fi
timeout -k 10 200 python tools/time_strided.py > gpurun_out/r4c/strided.log 2>&1 || exit 7
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/r4c/bench.json 2> gpurun_out/r4c/bench.err || exit 3
