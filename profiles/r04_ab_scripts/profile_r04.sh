#!/bin/bash
# round-4 evidence on the final library: rocprofv3 kernel stats + HBM bytes of the bench's timed NTT,
# the full bench's kernel stats, the NTT and Merkle counter passes, and the bench line of the same box.
mkdir -p gpurun_out/r4d
(while true; do date > gpurun_out/r4d/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
if ls variants/*.so > /dev/null 2>&1; then
  V="variants/base.so variants/a.so variants/b.so variants/c.so variants/d.so variants/e.so"
  LOG_N=26 REPS=30 WARM=5 timeout -k 10 300 python tools/time_ntt.py $V $V > gpurun_out/r4d/ab26.log 2>&1 || exit 5
  LOG_N=25 REPS=60 WARM=10 timeout -k 10 300 python tools/time_ntt.py $V $V > gpurun_out/r4d/ab25.log 2>&1 || exit 6
fi
bash tools/profile_round.sh r04 > gpurun_out/r4d/profile_round.log 2>&1 || exit 1
bash tools/pmc_round.sh r04 ntt > gpurun_out/r4d/pmc_ntt.log 2>&1 || exit 2
bash tools/pmc_round.sh r04m merkle32 > gpurun_out/r4d/pmc_merkle.log 2>&1 || exit 3
timeout -k 10 600 python bench.py > gpurun_out/r4d/bench_profiled_box.json 2> gpurun_out/r4d/bench.err || exit 4
