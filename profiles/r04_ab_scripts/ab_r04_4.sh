#!/bin/bash
# Round-4 A/B batch 4: 2^26 / 2^25 plans (second batch) and the LDS-table digit-basis twiddle prototype
# (variants/twdb64.so: timing only, wrong digests by construction) at several LDS sizes per workgroup.
mkdir -p gpurun_out/r4e
(while true; do date > gpurun_out/r4e/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
V="variants/base.so variants/d.so variants/f.so variants/g.so variants/h.so variants/i.so variants/j.so variants/k.so"
LOG_N=26 REPS=30 WARM=5 timeout -k 10 300 python tools/time_ntt.py $V $V > gpurun_out/r4e/ab26.log 2>&1 || exit 5
LOG_N=25 REPS=60 WARM=10 timeout -k 10 300 python tools/time_ntt.py $V $V > gpurun_out/r4e/ab25.log 2>&1 || exit 6
T="variants/base.so variants/twdb64.so variants/tw.so variants/tw77.so variants/base.so variants/twdb64.so variants/tw.so variants/tw77.so"
LOG_N=24 REPS=200 WARM=20 timeout -k 10 120 python tools/time_ntt.py $T > gpurun_out/r4e/tw_pad0.log 2>&1 || exit 7
for pad in 3128 3285 3300 3744; do
  STARK_LDS_PAD=$pad LOG_N=24 REPS=200 WARM=20 timeout -k 10 120 python tools/time_ntt.py $T > gpurun_out/r4e/tw_pad$pad.log 2>&1 || exit 8
done
LOG_N=20 REPS=500 WARM=50 timeout -k 10 120 python tools/time_ntt.py $T > gpurun_out/r4e/tw20.log 2>&1 || exit 9
LOG_N=23 REPS=200 WARM=20 timeout -k 10 120 python tools/time_ntt.py variants/base.so variants/tw.so variants/tw77.so variants/base.so variants/tw.so variants/tw77.so > gpurun_out/r4e/tw23.log 2>&1 || exit 10
LOG_N=26 REPS=30 WARM=5 timeout -k 10 200 python tools/time_ntt.py variants/d.so variants/tw.so variants/d.so variants/tw.so > gpurun_out/r4e/tw26.log 2>&1 || exit 11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt or large or field or lde" > gpurun_out/r4e/gpu_tests.log 2>&1 || exit 12
bash tools/prof_small_proofs.sh || exit 13
echo done
