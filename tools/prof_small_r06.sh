#!/bin/bash
# kernel trace of back-to-back compute and pedersen proofs (current library): per-kernel totals and gaps
# (tools/trace_gaps.py) and the last proof's kernel sequence (tools/trace_seq.py)
OUT=$GRAFT_REPO_ROOT/gpurun_out/${SMALL_OUT:-small6}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for fx in compute pedersen_test; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$fx -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs.py --fixtures $fx --synth "" --reps 12 > $OUT/trace_$fx.log 2>&1 || exit 2
done
cd $GRAFT_REPO_ROOT
for fx in compute pedersen_test; do
  f=$(ls $OUT/trace_$fx/*kernel_trace.csv $OUT/trace_$fx/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/trace_gaps.py $f --window-ms 1.5 --top 40 > $OUT/gaps_$fx.txt 2>&1 || exit 3
  python3 tools/trace_seq.py $f --window-ms ${SEQ_MS:-2.5} > $OUT/seq_$fx.txt 2>&1 || exit 3
done
STARK_PROFILE=1 timeout -k 10 120 python tools/time_r1cs.py --fixtures compute,pedersen_test --synth "" --reps 6 > $OUT/phases.log 2>&1 || exit 1
