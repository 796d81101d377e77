#!/bin/bash
# round-4 A/B: pass plans at 2^20-2^22 (dense transforms and the prover's LDE shapes)
mkdir -p gpurun_out/ab3
(while true; do date > gpurun_out/ab3/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
V="variants/base.so variants/a.so variants/b.so variants/c.so variants/d.so"
for ln in 20 21 22; do
  LOG_N=$ln REPS=1000 WARM=50 timeout -k 10 200 python tools/time_ntt.py $V $V > gpurun_out/ab3/ntt$ln.log 2>&1 || exit 1
done
for ls in 17 18 19 20; do
  LOG_STEPS=$ls REPS=50 timeout -k 10 200 python tools/time_lde.py $V $V > gpurun_out/ab3/lde$ls.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
LOG_N=20 REPS=300 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab3/prof20 -o run -- python3 $GRAFT_REPO_ROOT/tools/time_ntt.py $GRAFT_REPO_ROOT/variants/base.so $GRAFT_REPO_ROOT/variants/a.so > $GRAFT_REPO_ROOT/gpurun_out/ab3/prof20.log 2>&1 || exit 3
