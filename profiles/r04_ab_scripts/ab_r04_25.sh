#!/bin/bash
# round-4 batch 25: the world-8 proofs with torch's empty tensors poisoned (a read of an unwritten tensor
# shows), cold and prepared, then cold and prepared alternating with the parent holding a GPU context.
mkdir -p gpurun_out/r4ab
(while true; do date > gpurun_out/r4ab/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
DIAG_POISON_TORCH=1 timeout -k 10 300 python -u tools/diag_dprove.py 8 3 1 > gpurun_out/r4ab/poison_prep.log 2>&1 || exit 1
DIAG_POISON_TORCH=1 timeout -k 10 300 python -u tools/diag_dprove.py 8 3 0 > gpurun_out/r4ab/poison_cold.log 2>&1 || exit 2
DIAG_ALTERNATE=1 DIAG_PARENT_GPU=1 timeout -k 10 600 python -u tools/diag_dprove.py 8 8 1 > gpurun_out/r4ab/alternate.log 2>&1 || exit 3
