#!/bin/bash
# Where a small proof's wall-clock goes (pedersen_test, poseidon3_test, compute): host phase times
# (STARK_PROFILE=1) and a kernel trace whose idle gaps show the GPU waiting on the host.
OUT=gpurun_out/small
mkdir -p $OUT
STARK_PROFILE=1 timeout -k 10 120 python tools/time_r1cs.py --fixtures pedersen_test,poseidon3_test,compute --synth "" --reps 10 > $OUT/phases.log 2>&1 || exit 1
STARK_PROFILE=1 timeout -k 10 120 python tools/time_verify.py > $OUT/verify_phases.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs.py --fixtures pedersen_test --synth "" --reps 10 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit 2
cd $GRAFT_REPO_ROOT
python3 tools/trace_gaps.py $(ls $OUT/trace/*kernel_trace.csv $OUT/trace/*/*kernel_trace.csv 2>/dev/null | head -1) --window-ms 2.5 > $OUT/gaps.txt 2>&1 || exit 3
