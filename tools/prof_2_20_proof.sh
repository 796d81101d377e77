#!/bin/bash
# Where the cold 2^20-step proof's time goes: STARK_PROFILE=1 host phases, then a rocprofv3 kernel trace
# (stats + the idle gaps) of 6 cold proofs.
OUT=gpurun_out/p20
mkdir -p $OUT
STARK_PROFILE=1 timeout -k 10 180 python tools/time_r1cs.py --fixtures "" --synth 20 --reps 4 > $OUT/phases.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs.py --fixtures "" --synth 20 --reps 6 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit 2
cd $GRAFT_REPO_ROOT
F=$(ls $OUT/trace/*kernel_trace.csv $OUT/trace/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/trace_gaps.py $F --window-ms 14 > $OUT/gaps.txt 2>&1 || exit 3
python3 tools/trace_seq.py $F --window-ms 14 > $OUT/seq.txt 2>&1 || exit 3
